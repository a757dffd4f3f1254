"""Client for the kubelet pod-resources API (``v1.PodResourcesLister``) — which devices of which
device-plugin resource (``amd.com/gpu``) the kubelet assigned to which pod container.

This is the supported way for a node agent to attribute GPUs to pods (the same API the AMD
device-metrics exporter and DCGM-style exporters use).  It is served on the kubelet's unix
socket ``/var/lib/kubelet/pod-resources/kubelet.sock``.

The messages are tiny, so they are (de)serialised here with a hand-written protobuf wire
codec rather than generated stubs (``grpcio`` is present, ``grpcio-tools`` is not)::

    message ListPodResourcesResponse { repeated PodResources pod_resources = 1; }
    message PodResources { string name = 1; string namespace = 2; repeated ContainerResources containers = 3; }
    message ContainerResources { string name = 1; repeated ContainerDevices devices = 2; ... }
    message ContainerDevices { string resource_name = 1; repeated string device_ids = 2; TopologyInfo topology = 3; }

The reference has no counterpart: its culler only asks Jupyter
(``kf/controllers/culling_controller.go:161-196,243-273``).
"""

from __future__ import annotations

import asyncio
import os
from dataclasses import dataclass, field
from typing import Iterator, List, Tuple

DEFAULT_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
LIST_METHOD = "/v1.PodResourcesLister/List"


@dataclass
class ContainerDevices:
    resource_name: str
    device_ids: List[str] = field(default_factory=list)


@dataclass
class ContainerResources:
    name: str
    devices: List[ContainerDevices] = field(default_factory=list)


@dataclass
class PodResources:
    name: str
    namespace: str
    containers: List[ContainerResources] = field(default_factory=list)

    def device_ids(self, resource: str) -> List[str]:
        return [i for c in self.containers for d in c.devices if d.resource_name == resource for i in d.device_ids]


# ------------------------------------------------------------------ protobuf wire codec (varint + length-delimited)


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated varint")
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _fields(buf: bytes) -> Iterator[Tuple[int, int, object]]:
    """Yield ``(field_number, wire_type, value)``; unknown wire types 1/5 are skipped by size."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
            yield num, wt, v
        elif wt == 2:
            n, i = _read_varint(buf, i)
            if i + n > len(buf):
                raise ValueError("truncated field")
            yield num, wt, buf[i:i + n]
            i += n
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")


def _ld(num: int, payload: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(payload)) + payload


def _s(num: int, s: str) -> bytes:
    return _ld(num, s.encode())


def encode_list_response(pods: List[PodResources]) -> bytes:
    out = bytearray()
    for p in pods:
        pb = _s(1, p.name) + _s(2, p.namespace)
        for c in p.containers:
            cb = _s(1, c.name)
            for d in c.devices:
                db = _s(1, d.resource_name) + b"".join(_s(2, x) for x in d.device_ids)
                cb += _ld(2, db)
            pb += _ld(3, cb)
        out += _ld(1, pb)
    return bytes(out)


def decode_list_response(buf: bytes) -> List[PodResources]:
    pods = []
    for num, wt, v in _fields(buf):
        if num != 1 or wt != 2:
            continue
        p = PodResources("", "")
        for pn, pw, pv in _fields(v):
            if pw != 2:
                continue
            if pn == 1:
                p.name = pv.decode()
            elif pn == 2:
                p.namespace = pv.decode()
            elif pn == 3:
                c = ContainerResources("")
                for cn, cw, cv in _fields(pv):
                    if cw != 2:
                        continue  # cpu_ids (packed/varint) and the rest are not needed
                    if cn == 1:
                        c.name = cv.decode()
                    elif cn == 2:
                        d = ContainerDevices("")
                        for dn, dw, dv in _fields(cv):
                            if dw == 2 and dn == 1:
                                d.resource_name = dv.decode()
                            elif dw == 2 and dn == 2:
                                d.device_ids.append(dv.decode())
                        c.devices.append(d)
                p.containers.append(c)
        pods.append(p)
    return pods


# ------------------------------------------------------------------ client


class PodResourcesClient:
    """Blocking gRPC ``List`` over the kubelet unix socket, run on a worker thread."""

    def __init__(self, socket_path: str = DEFAULT_SOCKET, timeout_s: float = 2.0):
        self.socket_path = socket_path
        self.timeout_s = timeout_s
        self._channel = None
        self._list = None
        self.calls = 0

    def available(self) -> bool:
        return os.path.exists(self.socket_path)

    def _stub(self):
        if self._list is None:
            import grpc

            self._channel = grpc.insecure_channel(f"unix://{self.socket_path}")
            self._list = self._channel.unary_unary(LIST_METHOD, request_serializer=lambda _req: b"",
                                                   response_deserializer=decode_list_response)
        return self._list

    def list_sync(self) -> List[PodResources]:
        self.calls += 1
        return self._stub()(None, timeout=self.timeout_s)

    async def list(self) -> List[PodResources]:
        return await asyncio.to_thread(self.list_sync)

    def close(self) -> None:
        if self._channel is not None:
            self._channel.close()
            self._channel = None
            self._list = None
