"""Pod → GPU attribution on a real MI355X node, without any pod annotation.

Three independent sources, merged (a pod is attributed the union of what they report):

1. **kubelet pod-resources API** (:mod:`.podresources`): the devices of ``amd.com/gpu`` the
   kubelet assigned to each pod container, keyed by namespace/name.  The supported API.
2. **device-manager checkpoint** (:mod:`.checkpoint`): the same allocations from the
   kubelet's on-disk checkpoint, keyed by pod UID.  Fallback when the socket is not mounted.
3. **KFD per-process sysfs** (native, ``ops/csrc/gpu_telemetry.cpp:odh_tel_kfd_procs``): every
   process holding VRAM on a GPU (``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>``), joined with
   its pod cgroup (``/proc/<pid>/cgroup`` → pod UID).  This also sees GPUs a pod uses without
   having been allocated them (e.g. a privileged pod), and it is the only source of
   **per-pod VRAM** when several pods share a device.

Every refresh re-checks each source (a pod-resources socket that appears after the agent
started is used from then on, one that disappears is reported), and concurrent lookups
share one in-flight refresh.  Per-source health is exported on the agent's ``/metrics``.

Device IDs from 1 and 2 are what the AMD device plugin advertises: the PCI address of a
whole GPU (``0000:c1:00.0``), matched against the KFD topology's ``domain``/``location_id``;
all KFD nodes of that GPU (CPX/DPX partitions) are returned.  ``renderD<minor>``,
``card<n>`` and a bare index are accepted too.

Replaces the reference's Jupyter-only activity lookup
(``kf/controllers/culling_controller.go:161-196,243-273``) with a node-local one.
"""

from __future__ import annotations

import asyncio
import logging
import re
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set, Tuple

from .checkpoint import read_checkpoint

log = logging.getLogger("nodeagent.attribution")

GPU_RESOURCE = "amd.com/gpu"
_BDF = re.compile(r"^(?:([0-9a-fA-F]{1,8}):)?([0-9a-fA-F]{1,2}):([0-9a-fA-F]{1,2})\.([0-7])$")


@dataclass
class PodGpus:
    devices: List[int]  # telemetry device indices
    vram_bytes: Dict[int, int] = field(default_factory=dict)  # index -> bytes held by the pod's processes (KFD)
    sources: List[str] = field(default_factory=list)

    @property
    def pod_vram_bytes(self) -> Optional[int]:
        return sum(self.vram_bytes.values()) if self.vram_bytes else None


@dataclass
class Snapshot:
    taken_at: float
    by_name: Dict[Tuple[str, str], Set[int]] = field(default_factory=dict)
    by_uid: Dict[str, Set[int]] = field(default_factory=dict)
    kfd: Dict[str, Dict[int, int]] = field(default_factory=dict)  # pod uid -> index -> vram bytes
    sources: Dict[str, str] = field(default_factory=dict)  # source -> "ok" | "unavailable" | error
    unresolved: Set[str] = field(default_factory=set)  # device IDs matching no local GPU


class DeviceResolver:
    """Device-plugin device ID → telemetry indices, from the KFD topology the sampler read."""

    def __init__(self, devices):
        self.devices = list(devices)
        self.by_bdf: Dict[Tuple[int, int, int], List[int]] = {}
        self.by_minor: Dict[int, int] = {}
        self.by_gpu_id: Dict[int, int] = {}
        for d in self.devices:
            loc = d.location_id
            self.by_bdf.setdefault((d.domain, (loc >> 8) & 0xFF, loc & 0xFF), []).append(d.index)
            self.by_minor[d.render_minor] = d.index
            if d.gpu_id:
                self.by_gpu_id[d.gpu_id] = d.index

    def resolve(self, dev_id: str) -> List[int]:
        s = dev_id.strip()
        mt = _BDF.match(s)
        if mt:
            dom = int(mt.group(1) or "0", 16)
            bus, dev, fn = int(mt.group(2), 16), int(mt.group(3), 16), int(mt.group(4))
            return list(self.by_bdf.get((dom, bus, dev << 3 | fn), []))
        if s.startswith("renderD") and s[7:].isdigit():
            i = self.by_minor.get(int(s[7:]))
            return [] if i is None else [i]
        if s.startswith("card") and s[4:].isdigit():
            i = self.by_minor.get(128 + int(s[4:]))
            return [] if i is None else [i]
        if s.isdigit() and int(s) < len(self.devices):
            return [int(s)]
        return []


class Attributor:
    def __init__(self, telemetry, pod_resources=None, checkpoint_path: Optional[str] = None,
                 proc_root: Optional[str] = None, resource: str = GPU_RESOURCE, ttl_s: float = 1.0):
        self.telemetry = telemetry
        self.pod_resources = pod_resources
        self.checkpoint_path = checkpoint_path
        self.proc_root = proc_root
        self.resource = resource
        self.ttl_s = ttl_s
        self.resolver = DeviceResolver(telemetry.devices())
        self._snap: Optional[Snapshot] = None
        self._inflight: Optional[asyncio.Future] = None
        self.refreshes = 0

    def _resolve_all(self, ids, snap: Snapshot) -> Set[int]:
        out: Set[int] = set()
        for i in ids:
            r = self.resolver.resolve(i)
            if not r:
                snap.unresolved.add(i)
            out.update(r)
        return out

    async def refresh(self) -> Snapshot:
        snap = Snapshot(time.monotonic())
        if self.pod_resources is not None and not self.pod_resources.available():
            # the kubelet socket is not mounted (yet): probed again on the next refresh
            snap.sources["podresources"] = "unavailable"
        elif self.pod_resources is not None:
            try:
                for p in await self.pod_resources.list():
                    ids = p.device_ids(self.resource)
                    if ids:
                        snap.by_name[(p.namespace, p.name)] = self._resolve_all(ids, snap)
                snap.sources["podresources"] = "ok"
            except Exception as e:  # the socket is optional: a failing source is reported, not fatal
                snap.sources["podresources"] = f"error: {type(e).__name__}"
        if self.checkpoint_path:
            cp = read_checkpoint(self.checkpoint_path, self.resource)
            if cp is None:
                snap.sources["checkpoint"] = "unavailable"
            else:
                for uid, ids in cp.items():
                    snap.by_uid[uid] = self._resolve_all(ids, snap)
                snap.sources["checkpoint"] = "ok"
        if self.proc_root:
            try:
                for p in self.telemetry.kfd_processes(self.proc_root):
                    idx = self.resolver.by_gpu_id.get(p.gpu_id)
                    if p.pod_uid is None or idx is None or p.vram_bytes <= 0:
                        continue
                    per = snap.kfd.setdefault(p.pod_uid, {})
                    per[idx] = per.get(idx, 0) + p.vram_bytes
                snap.sources["kfd"] = "ok"
            except Exception as e:
                snap.sources["kfd"] = f"error: {type(e).__name__}"
        self._snap = snap
        self.refreshes += 1
        return snap

    async def snapshot(self) -> Snapshot:
        """The attribution tables, refreshed when older than ``ttl_s``.  Lookups that find the
        tables stale while a refresh is already running wait for that one (one pod-resources
        List, one checkpoint read and one KFD scan however many culler queries arrive)."""
        if self._snap is not None and time.monotonic() - self._snap.taken_at < self.ttl_s:
            return self._snap
        if self._inflight is None:
            self._inflight = asyncio.ensure_future(self.refresh())
            self._inflight.add_done_callback(self._clear_inflight)
        return await asyncio.shield(self._inflight)

    def _clear_inflight(self, fut: asyncio.Future) -> None:
        if self._inflight is fut:
            self._inflight = None
        if not fut.cancelled():
            fut.exception()  # retrieved: a failed refresh is re-raised to its awaiters only

    def source_health(self) -> Dict[str, int]:
        """source → 1 when the last refresh read it, 0 when it was unavailable or failed."""
        snap = self._snap
        return {k: int(v == "ok") for k, v in (snap.sources.items() if snap else [])}

    async def lookup(self, uid: Optional[str] = None, namespace: Optional[str] = None,
                     name: Optional[str] = None) -> Optional[PodGpus]:
        snap = await self.snapshot()
        devs: Set[int] = set()
        sources = []
        if namespace and name and (namespace, name) in snap.by_name:
            devs |= snap.by_name[(namespace, name)]
            sources.append("podresources")
        if uid and uid in snap.by_uid:
            devs |= snap.by_uid[uid]
            sources.append("checkpoint")
        vram = dict(snap.kfd.get(uid, {})) if uid else {}
        if vram:
            devs |= set(vram)
            sources.append("kfd")
        if not devs:
            return None
        return PodGpus(sorted(devs), vram, sources)

    async def all_pods(self) -> dict:
        snap = await self.snapshot()
        return {"by_name": {f"{ns}/{n}": sorted(v) for (ns, n), v in snap.by_name.items()},
                "by_uid": {u: sorted(v) for u, v in snap.by_uid.items()},
                "kfd_vram_bytes": {u: {str(i): b for i, b in v.items()} for u, v in snap.kfd.items()},
                "sources": snap.sources, "unresolved_device_ids": sorted(snap.unresolved)}
