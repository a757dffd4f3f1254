"""Fake node (TEST HARNESS ONLY — never deployed): scheduler + ``amd.com/gpu`` device
manager + per-GPU container runtimes, standing in for kube-scheduler, the kubelet and the
AMD device plugin the way envtest stands in for kube-apiserver.

The production node-side component is :mod:`odh_kubeflow_amd.nodeagent` (read-only
telemetry + pod→GPU attribution); the shipped DaemonSet runs that, not this module.

The split follows the MI355X rule "one process per GPU":

* :class:`SchedulerController` (control-plane side) binds pending pods to a Node that
  has room (cpu / memory / ``amd.com/gpu``) and, acting as the kubelet device manager,
  allocates concrete GPU indices in the same write (annotation ``amd.com/gpu-ids``),
  so a pod needs exactly one bind+allocate round trip.  Unschedulable pods get the
  ``PodScheduled=False/Unschedulable`` condition the reference status test expects
  (``kf/controllers/notebook_controller_test.go`` "unschedulablePod").
* :class:`GpuRuntime` runs in the process that owns a GPU (one per rank in the
  multi-GPU bench).  It watches pods allocated to its device(s), runs the container
  runtime — by default an in-process Jupyter-API notebook server plus an MI355X
  start-up probe (HIP kernels, see ``ops/``) — and reports pod status.
* :class:`FakeDeviceManager` records each allocation where a real kubelet does — the
  device-manager checkpoint file and the pod-resources gRPC API — with the PCI-address
  device IDs the AMD device plugin advertises, so the production node agent attributes
  GPUs to pods through exactly the code path it uses on a real node.  (The
  ``amd.com/gpu-ids`` annotation is internal to this fake scheduler/kubelet pair; no
  production component reads it.)
"""

from __future__ import annotations

import asyncio
import logging
import time
from typing import Awaitable, Callable, Dict, Iterable, List, Optional, Sequence, Set

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_conflict, is_not_found
from ..models.notebook import GPU_IDS_ANNOTATION, GPU_RESOURCE, gpu_request

GPU_INDEX_LABEL = "amd.com/gpu-index"
# Namespace label naming the GPU index(es) whose node agent runs in the same control-plane
# shard as the namespace's controllers (``parallel/shard.py``).  The device allocator tries
# those GPUs first, so a shard's pods start inside the shard's own process instead of
# waiting on another rank's event loop; a busy preferred GPU falls back to bin-packing.
GPU_AFFINITY_LABEL = "amd.com/gpu-affinity"
NAMESPACE_CACHE_WAIT_S = 0.5
PROBE_CONDITION = "amd.com/GPUProbe"
from ..runtime.controller import Request, Result, pred_funcs
from ..utils.quantity import parse_quantity
from ..utils.timeutil import rfc3339

log = logging.getLogger(__name__)

NODE_LABELS_MI355X = {
    # AMD GPU node-labeller keys (amd.com/gpu.*); the product label is what notebooks select on
    "amd.com/gpu.family": "AI",
    "amd.com/gpu.product-name": "AMD_Instinct_MI355X",
    "amd.com/gpu.device-id": "75a3",
    "amd.com/gpu.vram": "288G",
    "amd.com/gpu.compute-units": "256",
}


def make_node(name: str, gpus: int = 8, cpu: str = "256", memory: str = "3Ti", address: str = "127.0.0.1") -> dict:
    cap = {"cpu": cpu, "memory": memory, "pods": "250", GPU_RESOURCE: str(gpus)}
    labels = {"kubernetes.io/hostname": name, "kubernetes.io/os": "linux", **NODE_LABELS_MI355X}
    node = {
        "apiVersion": "v1", "kind": "Node",
        "metadata": {"name": name, "labels": labels, "annotations": {}},
        "spec": {},
        "status": {"capacity": dict(cap), "allocatable": dict(cap),
                   "addresses": [{"type": "InternalIP", "address": address}, {"type": "Hostname", "address": name}],
                   "conditions": [{"type": "Ready", "status": "True", "reason": "KubeletReady",
                                   "lastHeartbeatTime": rfc3339(), "lastTransitionTime": rfc3339()}],
                   "daemonEndpoints": {"kubeletEndpoint": {"Port": 10250}}}}
    return node


def _pod_requests(pod: dict) -> Dict[str, float]:
    cpu = mem = 0.0
    for c in (pod.get("spec") or {}).get("containers") or []:
        req = ((c.get("resources") or {}).get("requests") or {})
        lim = ((c.get("resources") or {}).get("limits") or {})
        if req.get("cpu") or lim.get("cpu"):
            cpu += float(parse_quantity(req.get("cpu") or lim.get("cpu")).value)
        if req.get("memory") or lim.get("memory"):
            mem += float(parse_quantity(req.get("memory") or lim.get("memory")).value)
    return {"cpu": cpu, "memory": mem, "gpu": gpu_request(pod.get("spec") or {})}


def _tolerates(pod: dict, node: dict) -> bool:
    taints = (node.get("spec") or {}).get("taints") or []
    tols = (pod.get("spec") or {}).get("tolerations") or []
    for t in taints:
        if t.get("effect") not in ("NoSchedule", "NoExecute"):
            continue
        ok = any((tol.get("key") == t.get("key") and (tol.get("operator") == "Exists" or tol.get("value") == t.get("value")))
                 or (not tol.get("key") and tol.get("operator") == "Exists") for tol in tols)
        if not ok:
            return False
    return True


class SchedulerController:
    """Binds pods to nodes and allocates GPU device indices.

    Policy: the GPUs named by the pod namespace's ``amd.com/gpu-affinity`` label first (if
    free), then bin-packing by lowest free index.
    """

    def __init__(self, client, reader, recorder, scheduler_name: str = "default-scheduler"):
        self.client = client
        self.reader = reader
        self.recorder = recorder
        self.scheduler_name = scheduler_name
        self.bound = 0
        self._lock = asyncio.Lock()
        # "assumed" bindings (kube-scheduler's assume cache): a bind is visible to the
        # next scheduling decision before the informer has observed it, so two pods can
        # never be given the same GPU however far the cache lags behind the apiserver.
        self._assumed: Dict[str, tuple] = {}  # pod uid -> (node, cpu, mem, gpu ids)
        self._ns_wait: Dict[str, float] = {}  # pod uid -> first time its namespace was missing from the cache

    def _used(self, node_name: str) -> Dict[str, object]:
        cpu = mem = 0.0
        gpus: Set[int] = set()
        seen = set()
        for p in self.reader.list(kinds.POD, fields=f"spec.nodeName={node_name}"):
            if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                continue
            seen.add(m.uid(p))
            r = _pod_requests(p)
            cpu += r["cpu"]
            mem += r["memory"]
            ids = m.annotations(p).get(GPU_IDS_ANNOTATION)
            if ids:
                gpus.update(int(x) for x in ids.split(",") if x != "")
        for uid, (node, acpu, amem, aids) in list(self._assumed.items()):
            if node != node_name or uid in seen:
                continue
            cpu += acpu
            mem += amem
            gpus.update(aids)
        return {"cpu": cpu, "memory": mem, "gpus": gpus}

    def _preferred_gpus(self, namespace: str) -> List[int]:
        ns = self.reader.get(kinds.NAMESPACE, namespace)
        val = m.labels(ns).get(GPU_AFFINITY_LABEL) if ns is not None else None
        if not val:
            return []
        out = []
        for x in val.replace("_", ",").split(","):
            if x.strip().isdigit():
                out.append(int(x))
        return out

    def forget(self, pod: dict) -> None:
        self._assumed.pop(m.uid(pod), None)
        self._ns_wait.pop(m.uid(pod), None)

    async def reconcile(self, req: Request) -> Result:
        pod = self.reader.get(kinds.POD, req.name, req.namespace)
        if pod is None or m.is_deleting(pod) or (pod.get("spec") or {}).get("nodeName"):
            return Result()
        if m.uid(pod) in self._assumed:
            return Result()  # bound already; the cache has not caught up yet
        if self.reader.get(kinds.NAMESPACE, req.namespace) is None and gpu_request(pod.get("spec") or {}):
            # the namespace (and its gpu-affinity label) has not reached this cache yet: a
            # pod cannot outlive its namespace's creation by much, so wait briefly for it
            first = self._ns_wait.setdefault(m.uid(pod), time.monotonic())
            if time.monotonic() - first < NAMESPACE_CACHE_WAIT_S:
                return Result(requeue_after=0.002)
        self._ns_wait.pop(m.uid(pod), None)
        async with self._lock:  # allocation decisions must not race each other
            return await self._schedule(pod)

    async def _schedule(self, pod: dict) -> Result:
        need = _pod_requests(pod)
        sel = (pod.get("spec") or {}).get("nodeSelector") or {}
        reasons: List[str] = []
        nodes = self.reader.list(kinds.NODE)
        for node in nodes:
            if any(m.labels(node).get(k) != v for k, v in sel.items()):
                reasons.append("node(s) didn't match Pod's node affinity/selector")
                continue
            if not _tolerates(pod, node):
                reasons.append("node(s) had untolerated taint")
                continue
            alloc = (node.get("status") or {}).get("allocatable") or {}
            used = self._used(m.name(node))
            ngpu = int(alloc.get(GPU_RESOURCE, "0") or 0)
            free = [i for i in range(ngpu) if i not in used["gpus"]]
            if need["gpu"] > len(free):
                reasons.append(f"Insufficient {GPU_RESOURCE}")
                continue
            if alloc.get("cpu") and used["cpu"] + need["cpu"] > float(parse_quantity(alloc["cpu"]).value):
                reasons.append("Insufficient cpu")
                continue
            if alloc.get("memory") and used["memory"] + need["memory"] > float(parse_quantity(alloc["memory"]).value):
                reasons.append("Insufficient memory")
                continue
            if need["gpu"]:
                pref = self._preferred_gpus(m.namespace(pod))
                if pref:
                    free = [i for i in pref if i in free] + [i for i in free if i not in pref]
            ids = free[: need["gpu"]]
            patch = {"spec": {"nodeName": m.name(node)}}
            if ids:
                # the allocation (device-plugin style) plus a selectable label naming the
                # first GPU, so a per-GPU node agent can watch just its own pods
                patch["metadata"] = {"annotations": {GPU_IDS_ANNOTATION: ",".join(map(str, ids))},
                                     "labels": {GPU_INDEX_LABEL: str(ids[0])}}
            try:
                await self.client.patch(kinds.POD, patch, name=m.name(pod), namespace=m.namespace(pod))
            except ApiError as e:
                if is_not_found(e):
                    return Result()
                raise
            self.bound += 1
            self._assumed[m.uid(pod)] = (m.name(node), need["cpu"], need["memory"], tuple(ids))
            self.recorder.event(pod, "Normal", "Scheduled",
                                f"Successfully assigned {m.namespace(pod)}/{m.name(pod)} to {m.name(node)}")
            return Result()
        # unschedulable
        counts: Dict[str, int] = {}
        for r in reasons:
            counts[r] = counts.get(r, 0) + 1
        msg = f"0/{len(nodes)} nodes are available: " + ", ".join(f"{v} {k}" for k, v in sorted(counts.items())) + "."
        cond = {"type": "PodScheduled", "status": "False", "reason": "Unschedulable", "message": msg,
                "lastProbeTime": None, "lastTransitionTime": rfc3339()}
        st = pod.get("status") or {}
        cur = [c for c in st.get("conditions") or [] if c.get("type") == "PodScheduled"]
        if not cur or cur[0].get("message") != msg:
            try:
                await self.client.patch(kinds.POD, {"status": {"phase": "Pending", "conditions": [cond]}},
                                        name=m.name(pod), namespace=m.namespace(pod), subresource="status")
            except ApiError as e:
                if not is_not_found(e):
                    raise
            self.recorder.event(pod, "Warning", "FailedScheduling", msg)
        return Result(requeue_after=1.0)

    def setup_with_manager(self, mgr, max_concurrent: int = 1):
        unbound = pred_funcs(create=lambda o: not (o.get("spec") or {}).get("nodeName"),
                             update=lambda o, old: not (o.get("spec") or {}).get("nodeName"),
                             delete=lambda o: False)

        def pods_released(obj):  # a deleted pod frees capacity: retry pending pods
            self.forget(obj)
            return [Request(m.namespace(p), m.name(p)) for p in self.reader.list(kinds.POD)
                    if not (p.get("spec") or {}).get("nodeName")]

        return (mgr.builder().named("scheduler").for_(kinds.POD, [unbound])
                .watches(kinds.POD, pods_released, [pred_funcs(create=lambda o: False, update=lambda o, old: False,
                                                               delete=lambda o: True)])
                # namespaces carry the gpu-affinity label: synced before the first decision
                .watches(kinds.NAMESPACE, lambda o: [], [lambda et, o, old: False])
                .with_options(max_concurrent_reconciles=max_concurrent).complete(self))


# ------------------------------------------------------------------ container runtime


class ContainerHandle:
    def __init__(self, pod_key: str, devices: Sequence[int], ip: str = "127.0.0.1", port: int = 0, info=None):
        self.pod_key = pod_key
        self.devices = list(devices)
        self.ip = ip
        self.port = port
        self.info = info or {}
        self.started_at = time.time()


class ContainerRuntime:
    """CRI-ish interface: start/stop the containers of one pod."""

    async def start(self, pod: dict, devices: Sequence[int]) -> ContainerHandle:
        return ContainerHandle(m.key(pod), devices)

    async def stop(self, handle: ContainerHandle) -> None:
        return None

    async def close(self) -> None:
        return None


class FakeContainerRuntime(ContainerRuntime):
    def __init__(self, start_delay: float = 0.0):
        self.start_delay = start_delay

    async def start(self, pod, devices):
        if self.start_delay:
            await asyncio.sleep(self.start_delay)
        return ContainerHandle(m.key(pod), devices)


StartupProbe = Callable[[Sequence[int]], Awaitable[dict]]


class FakeDeviceManager:
    """kubelet device-manager stand-in: publishes allocations through the device-plugin
    checkpoint (:class:`~odh_kubeflow_amd.nodeagent.checkpoint.CheckpointWriter`) and/or a
    pod-resources gRPC server (:class:`~odh_kubeflow_amd.nodeagent.podresources.FakePodResourcesServer`).

    ``device_id_of(index)`` gives the device-plugin ID of node GPU ``index`` (the PCI
    address; :func:`~odh_kubeflow_amd.ops.telemetry.fake_bdf` for synthetic sysfs trees).
    """

    def __init__(self, device_id_of: Callable[[int], str], checkpoint=None, pod_resources=None):
        self.device_id_of = device_id_of
        self.checkpoint = checkpoint
        self.pod_resources = pod_resources

    def allocate(self, pod: dict, devices: Sequence[int]) -> None:
        containers = (pod.get("spec") or {}).get("containers") or [{}]
        cname = next((c.get("name", "") for c in containers
                      if ((c.get("resources") or {}).get("limits") or {}).get(GPU_RESOURCE)),
                     containers[0].get("name", ""))
        ids = [self.device_id_of(d) for d in devices]
        if self.checkpoint is not None:
            self.checkpoint.allocate(m.uid(pod), cname, ids)
        if self.pod_resources is not None:
            self.pod_resources.assign(m.namespace(pod), m.name(pod), cname, GPU_RESOURCE, ids)

    def release(self, uid: str, namespace: str, name: str) -> None:
        if self.checkpoint is not None:
            self.checkpoint.release(uid)
        if self.pod_resources is not None:
            self.pod_resources.release(namespace, name)


class GpuRuntime:
    """Per-GPU kubelet half: runs pods allocated to ``devices`` on ``node_name``.

    ``devices=None`` makes this runtime also own pods that request no GPU.
    ``startup_probe`` (e.g. :func:`odh_kubeflow_amd.ops.gpu.startup_probe`) must pass before
    a GPU pod is reported Ready; its result is recorded as the pod condition
    ``amd.com/GPUProbe``.
    """

    def __init__(self, client, reader, recorder, node_name: str, devices: Optional[Iterable[int]],
                 runtime: Optional[ContainerRuntime] = None, startup_probe: Optional[StartupProbe] = None,
                 owns_cpu_pods: bool = True, host_ip: str = "127.0.0.1",
                 device_manager: Optional[FakeDeviceManager] = None):
        self.client = client
        self.reader = reader
        self.recorder = recorder
        self.node_name = node_name
        self.devices = set(devices) if devices is not None else None
        self.runtime = runtime or FakeContainerRuntime()
        self.startup_probe = startup_probe
        self.owns_cpu_pods = owns_cpu_pods
        self.host_ip = host_ip
        self.device_manager = device_manager
        self.handles: Dict[str, ContainerHandle] = {}
        self.started = 0
        self.probe_results: List[dict] = []

    def _mine(self, pod: dict) -> bool:
        if (pod.get("spec") or {}).get("nodeName") != self.node_name:
            return False
        ids = m.annotations(pod).get(GPU_IDS_ANNOTATION)
        if gpu_request(pod.get("spec") or {}) > 0:
            if not ids:
                return False  # not allocated yet
            devs = {int(x) for x in ids.split(",") if x != ""}
            return self.devices is None or bool(devs & self.devices) and min(devs) in self.devices
        return self.owns_cpu_pods

    async def reconcile(self, req: Request) -> Result:
        key = f"{req.namespace}/{req.name}"
        pod = self.reader.get(kinds.POD, req.name, req.namespace)
        h = self.handles.get(key)
        if pod is None or m.is_deleting(pod):
            if h is not None:
                self.handles.pop(key, None)
                await self._stop(h, req)
            return Result()
        if h is not None and h.info.get("uid") != m.uid(pod):
            # same name, new incarnation (restart annotation / rolling update)
            self.handles.pop(key, None)
            await self._stop(h, req)
            h = None
        if not self._mine(pod):
            return Result()
        if h is not None:
            if not h.info.get("reported"):
                # started, but the Ready status write failed (connection dropped): report it
                # now instead of leaving the pod Pending behind a running container
                await self._set_status(pod, ready=True, handle=h, probe=h.info.get("probe"))
                h.info["reported"] = True
            return Result()
        ids = m.annotations(pod).get(GPU_IDS_ANNOTATION) or ""
        devices = [int(x) for x in ids.split(",") if x != ""]
        probe = None
        if devices and self.startup_probe is not None:
            probe = await self.startup_probe(devices)
            self.probe_results.append(probe)
            if not probe.get("ok", False):
                await self._set_status(pod, ready=False, reason="GPUProbeFailed", message=str(probe.get("error")))
                self.recorder.event(pod, "Warning", "GPUProbeFailed", f"MI355X start-up probe failed: {probe}")
                return Result(requeue_after=5.0)
        h = await self.runtime.start(pod, devices)
        h.info["uid"] = m.uid(pod)
        if devices and self.device_manager is not None:
            self.device_manager.allocate(pod, devices)
        if probe is not None:
            h.info["probe"] = probe
        self.handles[key] = h
        self.started += 1
        await self._set_status(pod, ready=True, handle=h, probe=probe)
        h.info["reported"] = True
        self.recorder.event(pod, "Normal", "Started", "Started container " + ",".join(
            c.get("name", "") for c in (pod.get("spec") or {}).get("containers") or []))
        return Result()

    async def _stop(self, h: ContainerHandle, req: Request) -> None:
        if h.devices and self.device_manager is not None:
            self.device_manager.release(h.info.get("uid", ""), req.namespace, req.name)
        await self.runtime.stop(h)

    async def _set_status(self, pod: dict, ready: bool, handle: Optional[ContainerHandle] = None,
                          reason: str = "", message: str = "", probe: Optional[dict] = None) -> None:
        now = rfc3339()
        t = "True" if ready else "False"
        conds = [
            {"type": "PodReadyToStartContainers", "status": "True", "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "Initialized", "status": "True", "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "Ready", "status": t, "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "ContainersReady", "status": t, "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "PodScheduled", "status": "True", "lastProbeTime": None, "lastTransitionTime": now},
        ]
        for c in conds:
            if not ready and c["type"] in ("Ready", "ContainersReady"):
                c["reason"] = reason or "ContainersNotReady"
                if message:
                    c["message"] = message
        statuses = []
        for c in (pod.get("spec") or {}).get("containers") or []:
            st = {"running": {"startedAt": now}} if ready else {"waiting": {"reason": reason or "ContainerCreating"}}
            statuses.append({"name": c.get("name", ""), "image": c.get("image", ""), "imageID": "",
                             "ready": ready, "restartCount": 0, "started": ready, "state": st})
        if probe is not None:
            # a custom pod condition (the readiness-gate mechanism) instead of an annotation:
            # the kubelet writes status only, so Ready costs one write, not two
            ok = bool(probe.get("ok"))
            r0 = (probe.get("results") or [{}])[0]
            links = probe.get("links") or []
            msg = f"bf16 MFMA {r0.get('gemm_tflops', 0):.0f} TFLOP/s, HBM {r0.get('hbm_gbps', 0):.0f} GB/s"
            if links:  # multi-GPU pod: the xGMI ring over its GPUs was read and verified too
                msg += f", xGMI {len(links)} links min {min(lk.get('gbps', 0) for lk in links):.0f} GB/s"
            conds.append({"type": PROBE_CONDITION, "status": "True" if ok else "False",
                          "reason": "MFMAAndHBMVerified" if ok else "GPUProbeFailed",
                          "message": msg if ok else str(probe.get("error")),
                          "lastProbeTime": None, "lastTransitionTime": now})
        status = {"phase": "Running" if ready else "Pending", "conditions": conds, "containerStatuses": statuses,
                  "hostIP": self.host_ip, "podIP": handle.ip if handle else self.host_ip, "startTime": now}
        if handle is not None and handle.port:
            status["podIPs"] = [{"ip": handle.ip}]
        patch_ann = {}
        if handle is not None and handle.port:
            patch_ann["amd.com/notebook-endpoint"] = f"{handle.ip}:{handle.port}"
        try:
            if patch_ann:
                await self.client.patch(kinds.POD, {"metadata": {"annotations": patch_ann}},
                                        name=m.name(pod), namespace=m.namespace(pod))
            await self.client.patch(kinds.POD, {"status": status}, name=m.name(pod), namespace=m.namespace(pod),
                                    subresource="status")
        except ApiError as e:
            if not (is_not_found(e) or is_conflict(e)):
                raise

    async def close(self) -> None:
        for h in list(self.handles.values()):
            await self.runtime.stop(h)
        self.handles.clear()
        await self.runtime.close()  # containers whose start was interrupted

    def setup_with_manager(self, mgr, max_concurrent: int = 8, name: Optional[str] = None):
        mine = pred_funcs(create=lambda o: (o.get("spec") or {}).get("nodeName") == self.node_name,
                          update=lambda o, old: (o.get("spec") or {}).get("nodeName") == self.node_name,
                          delete=lambda o: True)
        return (mgr.builder().named(name or f"kubelet-{self.node_name}-{sorted(self.devices) if self.devices else 'all'}")
                .for_(kinds.POD, [mine]).with_options(max_concurrent_reconciles=max_concurrent).complete(self))
