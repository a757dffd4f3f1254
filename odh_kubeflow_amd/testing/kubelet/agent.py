"""Fake kubelet agent of one (or a few) GPUs — TEST HARNESS / BENCHMARK ONLY.

It plays the node-side platform pieces a real MI355X node already has, so the control
plane can be exercised without a cluster:

* registers the ``Node`` (capacity ``amd.com/gpu``, AMD node-labeller labels) — the kubelet's job;
* runs :class:`~odh_kubeflow_amd.testing.kubelet.node.GpuRuntime` for its devices (run init
  containers — the MI355X start-up probe as a real process when the runtime executes init
  containers —, start pods, report pod status) — the kubelet's job;
* publishes GPU allocations through a :class:`~odh_kubeflow_amd.testing.kubelet.node.FakeDeviceManager`
  (device-plugin checkpoint file) — the kubelet device manager's job;
* optionally hosts the **production** node agent
  (:class:`~odh_kubeflow_amd.nodeagent.server.NodeTelemetryAgent`) next to it, which attributes
  GPUs to pods from that checkpoint exactly as it does on a real node.

The shipped DaemonSet (``config/node-agent``) runs ``cmd/node_agent.py`` — the production
agent alone, which has no apiserver client.  Nothing here is deployed.
"""

from __future__ import annotations

import os
import tempfile
from typing import Callable, Dict, List, Optional, Sequence

from ...models.errors import ApiError, is_already_exists
from .node import FakeDeviceManager, GpuRuntime, make_node


def pci_bus_index_map(telemetry, local_bus_ids: Dict[int, int]) -> Dict[int, int]:
    """node-GPU index → telemetry index, matching PCI bus numbers (``location_id >> 8``)."""
    by_bus = {}
    for d in telemetry.devices():
        by_bus.setdefault((d.location_id >> 8) & 0xFF, d.index)
    return {g: by_bus[b] for g, b in local_bus_ids.items() if b in by_bus}


def default_device_id_of(telemetry=None) -> Callable[[int], str]:
    """Device-plugin IDs for node GPU indices: the PCI address of the telemetry device with
    that index when there is one, else the synthetic-tree address."""
    from ...ops.telemetry import fake_bdf

    devs = telemetry.devices() if telemetry is not None else []

    def of(i: int) -> str:
        return devs[i].pci_bdf if i < len(devs) else fake_bdf(i)
    return of


class FakeKubeletAgent:
    def __init__(self, mgr, node_name: str, devices: Sequence[int], node_gpus: int = 8, runtime=None,
                 telemetry=None, register_node: bool = True, owns_cpu_pods: bool = True,
                 address: str = "127.0.0.1", activity_port: int = 0, checkpoint_path: Optional[str] = None,
                 device_id_of: Optional[Callable[[int], str]] = None, one_runtime: bool = False):
        from ...nodeagent.checkpoint import CheckpointWriter

        self.mgr = mgr
        self.node_name = node_name
        self.devices = list(devices)
        self.node_gpus = node_gpus
        self.register_node = register_node
        self.address = address
        self._tmp = None
        if checkpoint_path is None:
            # memory-backed when the host has /dev/shm: the stand-in rewrites the file per pod
            shm = "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None
            self._tmp = tempfile.TemporaryDirectory(prefix="odh-kubelet-", dir=shm)
            checkpoint_path = os.path.join(self._tmp.name, "device-plugins", "kubelet_internal_checkpoint")
        self.checkpoint_path = checkpoint_path
        self.device_manager = FakeDeviceManager(device_id_of or default_device_id_of(telemetry),
                                                checkpoint=CheckpointWriter(checkpoint_path))
        self.telemetry_agent = None
        if telemetry is not None:
            from ...nodeagent.attribution import Attributor
            from ...nodeagent.server import NodeTelemetryAgent

            self.telemetry_agent = NodeTelemetryAgent(
                telemetry, Attributor(telemetry, checkpoint_path=checkpoint_path, ttl_s=0.0),
                host=address, port=activity_port)
        self.runtimes: List[GpuRuntime] = []
        # one_runtime: one kubelet loop for all the node's GPUs (a real kubelet is one process);
        # otherwise one per GPU (a rank owning its GPU)
        groups = [self.devices] if one_runtime else [[d] for d in self.devices]
        for i, devs in enumerate(groups):
            g = GpuRuntime(mgr.client, mgr.reader, mgr.get_event_recorder_for("kubelet"), node_name, devs,
                           runtime=runtime, owns_cpu_pods=owns_cpu_pods and i == 0,
                           host_ip=address, device_manager=self.device_manager)
            g.setup_with_manager(mgr, name=f"kubelet-{node_name}-gpu{'-'.join(map(str, devs))}")
            self.runtimes.append(g)
        mgr.add(self, needs_leader=False)

    async def start(self) -> None:
        if self.telemetry_agent is not None:
            await self.telemetry_agent.start()
        if self.register_node:
            try:
                await self.mgr.client.create(make_node(self.node_name, self.node_gpus, address=self.address))
            except ApiError as e:
                if not is_already_exists(e):
                    raise

    async def stop(self) -> None:
        for g in self.runtimes:
            await g.close()
        if self.telemetry_agent is not None:
            await self.telemetry_agent.stop()
        if self._tmp is not None:
            self._tmp.cleanup()
            self._tmp = None

    @property
    def probe_results(self) -> List[dict]:
        return [p for g in self.runtimes for p in g.probe_results]

