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
* :class:`GpuRuntime` is the kubelet half of one or more GPUs.  It watches pods allocated
  to its device(s), runs their init containers — the MI355X start-up probe
  (``odh-gpu-probe``) as a real process on the pod's GPUs when the runtime executes init
  containers — then the container runtime (nothing, a Jupyter-API stand-in, or a real
  PyTorch-ROCm workbench process), and reports pod status the way a kubelet does
  (``Initialized`` / ``initContainerStatuses`` / ``Ready``).
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
import os
import tempfile
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Set

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_conflict, is_not_found
from ...models.notebook import GPU_IDS_ANNOTATION, GPU_RESOURCE, gpu_request

GPU_INDEX_LABEL = "amd.com/gpu-index"
INIT_BACKOFF_S = 10.0  # kubelet's first CrashLoopBackOff step for a failed init container
from ...runtime.controller import Request, Result, pred_funcs
from ...utils.quantity import parse_quantity
from ...utils.timeutil import rfc3339

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

    Policy: the device plugin's — the lowest free indices of the node (first free).  Nothing
    about the pod's namespace or controller steers the choice, as with kube-scheduler plus the
    AMD device plugin.
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
        # kube-scheduler's NodeInfo cache: what the pods bound to each node request, kept up to
        # date from the pod watch (:meth:`_on_pod`) so a decision costs O(1) in the pods already
        # running — with hundreds resident, re-summing them per decision set the pace
        self._pods: Dict[str, tuple] = {}  # pod uid -> (node, cpu, mem, gpu ids)
        self._sums: Dict[str, List[float]] = {}  # node -> [cpu, mem]
        self._gpu_pods: Dict[str, Dict[str, tuple]] = {}  # node -> {uid: gpu ids}
        self._unbound: Dict[str, tuple] = {}  # uid -> (namespace, name) of pods waiting for a node
        self._tracking = False

    def _on_pod(self, etype: str, pod: dict, old: Optional[dict]) -> None:
        uid = m.uid(pod)
        spec = pod.get("spec") or {}
        node = spec.get("nodeName")
        gone = etype == "DELETED" or (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed")
        if gone or node or m.is_deleting(pod):
            self._unbound.pop(uid, None)
        else:
            self._unbound[uid] = (m.namespace(pod), m.name(pod))
        if node and uid in self._assumed:
            # the informer has seen the binding: the assumption is confirmed (kube-scheduler's
            # FinishBinding), so decisions stop walking it — it lives on as a cached pod
            self._assumed.pop(uid, None)
        cur = self._pods.get(uid)
        ids = m.annotations(pod).get(GPU_IDS_ANNOTATION)
        want = None
        if not gone and node:
            if cur is not None and cur[0] == node and cur[4] == ids:
                return  # requests are immutable: nothing this cache keeps changed
            r = _pod_requests(pod)
            want = (node, r["cpu"], r["memory"], tuple(int(x) for x in ids.split(",") if x != "") if ids else (), ids)
        if cur is not None:
            sums = self._sums[cur[0]]
            sums[0] -= cur[1]
            sums[1] -= cur[2]
            self._gpu_pods.get(cur[0], {}).pop(uid, None)
            del self._pods[uid]
        if want is not None:
            self._pods[uid] = want
            sums = self._sums.setdefault(node, [0.0, 0.0])
            sums[0] += want[1]
            sums[1] += want[2]
            if want[3]:
                self._gpu_pods.setdefault(node, {})[uid] = want[3]

    def _used(self, node_name: str) -> Dict[str, object]:
        if not self._tracking:
            return self._used_scan(node_name)
        cpu, mem = self._sums.get(node_name, (0.0, 0.0))
        gpus: Set[int] = set()
        for ids in self._gpu_pods.get(node_name, {}).values():
            gpus.update(ids)
        for uid, (node, acpu, amem, aids) in list(self._assumed.items()):
            seen = self._pods.get(uid)
            if node != node_name or (seen is not None and seen[0] == node_name):
                continue
            cpu += acpu
            mem += amem
            gpus.update(aids)
        return {"cpu": cpu, "memory": mem, "gpus": gpus}

    def _used_scan(self, node_name: str) -> Dict[str, object]:
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

    def forget(self, pod: dict) -> None:
        self._assumed.pop(m.uid(pod), None)

    async def reconcile(self, req: Request) -> Result:
        pod = self.reader.get(kinds.POD, req.name, req.namespace)
        if pod is None or m.is_deleting(pod) or (pod.get("spec") or {}).get("nodeName"):
            return Result()
        if m.uid(pod) in self._assumed:
            return Result()  # bound already; the cache has not caught up yet
        async with self._lock:  # scheduling cycle: allocation decisions must not race each other
            bind = await self._schedule(pod)
        if isinstance(bind, Result):
            return bind
        # binding cycle, outside the lock (kube-scheduler binds asynchronously): the
        # assumption already holds the pod's devices, so the next pod is decided meanwhile
        node_name, patch, ids = bind
        try:
            await self.client.patch(kinds.POD, patch, name=m.name(pod), namespace=m.namespace(pod))
        except ApiError as e:
            self.forget(pod)  # unreserve
            if is_not_found(e):
                return Result()
            raise
        except BaseException:
            self.forget(pod)
            raise
        self.bound += 1
        self.recorder.event(pod, "Normal", "Scheduled",
                            f"Successfully assigned {m.namespace(pod)}/{m.name(pod)} to {node_name}")
        return Result()

    async def _schedule(self, pod: dict):
        """Pick a node and devices; on success assume the pod there and return
        ``(node name, bind patch, device ids)``, else report it unschedulable (a Result)."""
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
            ids = free[: need["gpu"]]
            patch = {"spec": {"nodeName": m.name(node)}}
            if ids:
                # the allocation (device-plugin style) plus a selectable label naming the
                # first GPU, so a per-GPU node agent can watch just its own pods
                patch["metadata"] = {"annotations": {GPU_IDS_ANNOTATION: ",".join(map(str, ids))},
                                     "labels": {GPU_INDEX_LABEL: str(ids[0])}}
            self._assumed[m.uid(pod)] = (m.name(node), need["cpu"], need["memory"], tuple(ids))
            return m.name(node), patch, ids
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

    def setup_with_manager(self, mgr, max_concurrent: int = 8):
        unbound = pred_funcs(create=lambda o: not (o.get("spec") or {}).get("nodeName"),
                             update=lambda o, old: not (o.get("spec") or {}).get("nodeName"),
                             delete=lambda o: False)

        src = getattr(mgr, "cache", None) or mgr.reader
        if hasattr(src, "subscribe"):  # the NodeInfo cache follows every pod event
            src.subscribe(kinds.POD, self._on_pod)
            self._tracking = True

        def pods_released(obj):  # a deleted pod frees capacity: retry pending pods
            self.forget(obj)
            if self._tracking:
                return [Request(ns, nm) for ns, nm in list(self._unbound.values())]
            return [Request(m.namespace(p), m.name(p)) for p in self.reader.list(kinds.POD)
                    if not (p.get("spec") or {}).get("nodeName")]

        return (mgr.builder().named("scheduler").for_(kinds.POD, [unbound])
                .watches(kinds.POD, pods_released, [pred_funcs(create=lambda o: False, update=lambda o, old: False,
                                                               delete=lambda o: True)])
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


def is_gpu_probe(container: dict) -> bool:
    """The MI355X start-up probe init container (``controllers/notebook.py``
    ``gpu_probe_init_container``): its command is the ``odh-gpu-probe`` program."""
    cmd = container.get("command") or []
    return bool(cmd) and os.path.basename(str(cmd[0])) == "odh-gpu-probe"


async def run_gpu_probe_container(container: dict, visible: Sequence[int], timeout_s: float = 120.0) -> dict:
    """Run the probe init container the way a kubelet would: as its own process, seeing only
    the pod's GPUs (``HIP_VISIBLE_DEVICES``, the device plugin's job), its
    ``/dev/termination-log`` a file whose content becomes the termination message.  Only the
    image is missing: the in-tree ``odh-gpu-probe`` binary stands in for it."""
    from ...ops import probe_main

    fd, term = tempfile.mkstemp(prefix="odh-termination-log-")
    os.close(fd)
    args = [term if a == "/dev/termination-log" else str(a) for a in container.get("args") or []]
    env = {k: v for k, v in os.environ.items() if not k.startswith(("HIP_VISIBLE", "ROCR_VISIBLE", "CUDA_VISIBLE"))}
    env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in dict.fromkeys(visible))
    for e in container.get("env") or []:
        if "value" in e:
            env[e["name"]] = str(e["value"])
    env["ODH_PROBE_T0_NS"] = str(time.time_ns())  # the probe reports its exec + link time against it
    t0 = time.perf_counter()
    proc = await asyncio.create_subprocess_exec(*probe_main.command(args), env=env, stdout=asyncio.subprocess.PIPE,
                                                stderr=asyncio.subprocess.PIPE)
    try:
        out, err = await asyncio.wait_for(proc.communicate(), timeout_s)
        rc = proc.returncode
    except asyncio.TimeoutError:
        proc.kill()
        out, err = await proc.communicate()
        rc = 137
    wall_ms = (time.perf_counter() - t0) * 1e3
    try:
        with open(term) as f:
            msg = f.read()
    finally:
        os.unlink(term)
    if not msg and container.get("terminationMessagePolicy") == "FallbackToLogsOnError" and rc != 0:
        msg = ((out or b"") + (err or b"")).decode(errors="replace")[-4096:]
    return {"exitCode": rc, "message": msg[:4096], "wall_ms": wall_ms, "result": probe_main.parse_result(msg)}


class ContainerRuntime:
    """CRI-ish interface: run a pod's init containers, start/stop its app containers.

    ``exec_init`` makes :meth:`run_init` execute the init containers this node can run
    without an image — the MI355X start-up probe (``odh-gpu-probe``) — as real processes on the
    pod's GPUs; every other init container (and every init container when ``exec_init`` is
    off) completes at once, as app containers do in the fake runtimes.  ``visible_device``
    maps a node GPU index to the HIP device the process should see (a one-GPU box hosts all
    eight node GPUs on its device 0)."""

    exec_init: bool = False
    visible_device: Optional[Callable[[int], int]] = None

    async def run_init(self, pod: dict, container: dict, devices: Sequence[int]) -> dict:
        if self.exec_init and devices and is_gpu_probe(container):
            vis = self.visible_device or (lambda d: d)
            return await run_gpu_probe_container(container, [vis(d) for d in devices])
        return {"exitCode": 0, "message": "", "wall_ms": 0.0, "result": None}

    async def start(self, pod: dict, devices: Sequence[int]) -> ContainerHandle:
        return ContainerHandle(m.key(pod), devices)

    async def stop(self, handle: ContainerHandle) -> None:
        return None

    async def close(self) -> None:
        return None


class FakeContainerRuntime(ContainerRuntime):
    def __init__(self, start_delay: float = 0.0, exec_init: bool = False,
                 visible_device: Optional[Callable[[int], int]] = None):
        self.start_delay = start_delay
        self.exec_init = exec_init
        self.visible_device = visible_device

    async def start(self, pod, devices):
        if self.start_delay:
            await asyncio.sleep(self.start_delay)
        return ContainerHandle(m.key(pod), devices)


class FakeDeviceManager:
    """kubelet device-manager stand-in: publishes allocations through the device-plugin
    checkpoint (:class:`~odh_kubeflow_amd.nodeagent.checkpoint.CheckpointWriter`) and/or a
    pod-resources gRPC server (:class:`~odh_kubeflow_amd.testing.kubelet.podresources_server.FakePodResourcesServer`).

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


def _terminated_status(container: dict, r: dict) -> dict:
    """``initContainerStatuses[]`` entry of an init container that ran to completion."""
    ok = r["exitCode"] == 0
    term = {"exitCode": r["exitCode"], "reason": "Completed" if ok else "Error", "startedAt": rfc3339(),
            "finishedAt": rfc3339()}
    if r.get("message"):
        term["message"] = r["message"]
    return {"name": container.get("name", ""), "image": container.get("image", ""), "imageID": "", "ready": ok,
            "restartCount": 0, "started": False, "state": {"terminated": term}}


class GpuRuntime:
    """Per-GPU kubelet half: runs pods allocated to ``devices`` on ``node_name``.

    ``devices=None`` makes this runtime also own pods that request no GPU.  A pod's init
    containers run first, in order (:meth:`ContainerRuntime.run_init`); one that fails keeps
    the pod Pending with ``Initialized=False`` and is retried after a back-off, as the kubelet
    does for ``restartPolicy: Always`` pods.  Ready is gated on nothing a real kubelet would
    not gate it on: init containers, then the containers themselves.
    """

    def __init__(self, client, reader, recorder, node_name: str, devices: Optional[Iterable[int]],
                 runtime: Optional[ContainerRuntime] = None, owns_cpu_pods: bool = True, host_ip: str = "127.0.0.1",
                 device_manager: Optional[FakeDeviceManager] = None):
        self.client = client
        self.reader = reader
        self.recorder = recorder
        self.node_name = node_name
        self.devices = set(devices) if devices is not None else None
        self.runtime = runtime or FakeContainerRuntime()
        self.owns_cpu_pods = owns_cpu_pods
        self.host_ip = host_ip
        self.device_manager = device_manager
        self.handles: Dict[str, ContainerHandle] = {}
        self.started = 0
        self.probe_results: List[dict] = []  # GPU probe init containers run: exit code, wall time, verdict
        self.init_backoff_s = INIT_BACKOFF_S
        self._backoff: Dict[str, tuple] = {}  # pod key -> (uid, monotonic time its failed init may rerun)

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
            self._backoff.pop(key, None)
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
                await self._set_status(pod, ready=True, handle=h, init_statuses=h.info.get("init_statuses"))
                h.info["reported"] = True
            return Result()
        ids = m.annotations(pod).get(GPU_IDS_ANNOTATION) or ""
        devices = [int(x) for x in ids.split(",") if x != ""]
        uid, until = self._backoff.get(key, (None, 0.0))
        if uid == m.uid(pod) and time.monotonic() < until:
            # CrashLoopBackOff: our own status write (and any other pod event) must not rerun
            # the failed init container before the back-off has passed
            return Result(requeue_after=until - time.monotonic())
        self._backoff.pop(key, None)
        init_statuses = []
        for c in (pod.get("spec") or {}).get("initContainers") or []:
            r = await self.runtime.run_init(pod, c, devices)
            if is_gpu_probe(c):
                self.probe_results.append({"pod": key, **r})
            init_statuses.append(_terminated_status(c, r))
            if r["exitCode"] != 0:
                await self._set_status(pod, ready=False, reason="PodInitializing", init_statuses=init_statuses,
                                       failed_init=c.get("name", ""))
                self.recorder.event(pod, "Warning", "BackOff", f"Back-off restarting failed container {c.get('name')} "
                                    f"in pod {m.name(pod)}: exit code {r['exitCode']}")
                self._backoff[key] = (m.uid(pod), time.monotonic() + self.init_backoff_s)
                return Result(requeue_after=self.init_backoff_s)
        h = await self.runtime.start(pod, devices)
        h.info["uid"] = m.uid(pod)
        h.info["init_statuses"] = init_statuses
        self.handles[key] = h
        self.started += 1
        await self._set_status(pod, ready=True, handle=h, init_statuses=init_statuses)
        h.info["reported"] = True
        if devices and self.device_manager is not None:
            # the device-manager checkpoint / pod-resources record (what the node agent reads):
            # a file rewrite, kept off the Ready status write the pod is waiting for
            self.device_manager.allocate(pod, devices)
        self.recorder.event(pod, "Normal", "Started", "Started container " + ",".join(
            c.get("name", "") for c in (pod.get("spec") or {}).get("containers") or []))
        return Result()

    async def _stop(self, h: ContainerHandle, req: Request) -> None:
        if h.devices and self.device_manager is not None:
            self.device_manager.release(h.info.get("uid", ""), req.namespace, req.name)
        await self.runtime.stop(h)

    async def _set_status(self, pod: dict, ready: bool, handle: Optional[ContainerHandle] = None,
                          reason: str = "", message: str = "", init_statuses: Optional[List[dict]] = None,
                          failed_init: str = "") -> None:
        now = rfc3339()
        t = "True" if ready else "False"
        initialized = not failed_init
        conds = [
            {"type": "PodReadyToStartContainers", "status": "True", "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "Initialized", "status": "True" if initialized else "False", "lastProbeTime": None,
             "lastTransitionTime": now},
            {"type": "Ready", "status": t, "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "ContainersReady", "status": t, "lastProbeTime": None, "lastTransitionTime": now},
            {"type": "PodScheduled", "status": "True", "lastProbeTime": None, "lastTransitionTime": now},
        ]
        for c in conds:
            if not initialized and c["type"] == "Initialized":
                c["reason"] = "ContainersNotInitialized"
                c["message"] = f"containers with incomplete status: [{failed_init}]"
            if not ready and c["type"] in ("Ready", "ContainersReady"):
                c["reason"] = reason or "ContainersNotReady"
                if message:
                    c["message"] = message
        statuses = []
        for c in (pod.get("spec") or {}).get("containers") or []:
            st = {"running": {"startedAt": now}} if ready else {"waiting": {"reason": reason or "ContainerCreating"}}
            statuses.append({"name": c.get("name", ""), "image": c.get("image", ""), "imageID": "",
                             "ready": ready, "restartCount": 0, "started": ready, "state": st})
        status = {"phase": "Running" if ready else "Pending", "conditions": conds, "containerStatuses": statuses,
                  "hostIP": self.host_ip, "podIP": handle.ip if handle else self.host_ip, "startTime": now}
        if init_statuses:
            status["initContainerStatuses"] = init_statuses
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
