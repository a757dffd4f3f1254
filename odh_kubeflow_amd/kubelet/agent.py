"""MI355X node agent: the per-node process that owns GPUs (``amd.com/gpu`` device plugin
half + kubelet stand-in + amdgpu telemetry endpoint).

Responsibilities:

* register / refresh the ``Node`` object: capacity ``amd.com/gpu`` = number of MI355X,
  AMD node-labeller labels, ``amd.com/gpu-activity-port`` annotation;
* run :class:`~odh_kubeflow_amd.kubelet.node.GpuRuntime` for its devices: start pods
  allocated to them, gate Ready on the MI355X start-up probe (``ops/gpu.py``: MFMA GEMM
  checked bit-exactly + HBM3E sweep), report pod status;
* serve ``GET /gpu/activity?devices=0,3&window=60`` (mean/max busy %, VRAM) from the
  native sysfs sampler (``ops/csrc/gpu_telemetry.cpp``) for the culler's ``amdgpu``
  signal, plus ``/gpu/devices`` and ``/healthz``.

One agent per GPU process is the MI355X layout used by the benchmark (rank r owns
GPU r); one agent for the whole node is the DaemonSet layout.
"""

from __future__ import annotations

import logging
from typing import Callable, Dict, List, Optional, Sequence

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_already_exists
from .node import GpuRuntime, make_node

log = logging.getLogger("kubelet.agent")


def pci_bus_index_map(telemetry, local_bus_ids: Dict[int, int]) -> Dict[int, int]:
    """node-GPU index → telemetry index, matching PCI bus numbers (``location_id >> 8``)."""
    by_bus = {}
    for d in telemetry.devices():
        by_bus.setdefault((d.location_id >> 8) & 0xFF, d.index)
    return {g: by_bus[b] for g, b in local_bus_ids.items() if b in by_bus}


class TelemetryEndpoint:
    def __init__(self, telemetry, index_of: Optional[Callable[[int], Optional[int]]] = None,
                 host: str = "0.0.0.0", port: int = 0):
        self.telemetry = telemetry
        self.index_of = index_of or (lambda d: d)
        self.host = host
        self.port = port
        self._runner = None
        self.queries = 0

    async def start(self) -> "TelemetryEndpoint":
        from aiohttp import web

        from ..controllers.culling import aggregate_windows

        async def activity(req):
            self.queries += 1
            try:
                devs = [int(x) for x in (req.query.get("devices") or "").split(",") if x.strip() != ""]
                window = float(req.query.get("window") or 60)
            except ValueError:
                return web.json_response({"error": "bad query"}, status=400)
            if self.telemetry is None:
                return web.json_response({"n": 0})
            agg = aggregate_windows(self.telemetry, [self.index_of(d) for d in devs], window)
            return web.json_response(agg or {"n": 0})

        async def devices(_req):
            if self.telemetry is None:
                return web.json_response([])
            return web.json_response([d.__dict__ for d in self.telemetry.devices()])

        async def healthz(_req):
            return web.Response(text="ok")

        app = web.Application()
        app.router.add_get("/gpu/activity", activity)
        app.router.add_get("/gpu/devices", devices)
        app.router.add_get("/healthz", healthz)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None


class NodeAgent:
    def __init__(self, mgr, node_name: str, devices: Sequence[int], node_gpus: int = 8, runtime=None,
                 startup_probe=None, telemetry=None, telemetry_index: Optional[Callable[[int], Optional[int]]] = None,
                 register_node: bool = True, owns_cpu_pods: bool = True, address: str = "127.0.0.1",
                 activity_port: int = 0):
        self.mgr = mgr
        self.node_name = node_name
        self.devices = list(devices)
        self.node_gpus = node_gpus
        self.register_node = register_node
        self.address = address
        self.endpoint = TelemetryEndpoint(telemetry, telemetry_index, port=activity_port) if telemetry is not None \
            else None
        self.runtimes: List[GpuRuntime] = []
        for i, d in enumerate(self.devices):
            g = GpuRuntime(mgr.client, mgr.reader, mgr.get_event_recorder_for("kubelet"), node_name, [d],
                           runtime=runtime, startup_probe=startup_probe, owns_cpu_pods=owns_cpu_pods and i == 0,
                           host_ip=address)
            g.setup_with_manager(mgr, name=f"kubelet-{node_name}-gpu{d}")
            self.runtimes.append(g)
        mgr.add(self, needs_leader=False)

    async def start(self) -> None:
        if self.endpoint is not None:
            await self.endpoint.start()
        if self.register_node:
            node = make_node(self.node_name, self.node_gpus, address=self.address,
                             activity_port=self.endpoint.port if self.endpoint else 0)
            try:
                await self.mgr.client.create(node)
            except ApiError as e:
                if not is_already_exists(e):
                    raise
                if self.endpoint is not None:
                    await self.mgr.client.patch(kinds.NODE, {"metadata": {"annotations": {
                        "amd.com/gpu-activity-port": str(self.endpoint.port)}}}, name=self.node_name)

    async def stop(self) -> None:
        for g in self.runtimes:
            await g.close()
        if self.endpoint is not None:
            await self.endpoint.stop()

    @property
    def probe_results(self) -> List[dict]:
        return [p for g in self.runtimes for p in g.probe_results]
