"""The node around the control plane in the benchmark: ONE set of platform stand-ins per node.

An 8×MI355X node has one kubelet, one kube-scheduler (+ the AMD device plugin choosing
devices) and one kube-controller-manager, however many control-plane replicas run against
the cluster.  :class:`NodePlatform` is that, for the benchmark and the multi-shard tests:

* ``scheduler`` — :mod:`odh_kubeflow_amd.testing.cmd.scheduler`: binds pods and allocates
  ``amd.com/gpu`` first-free (the device plugin's policy; nothing steers a pod to a GPU by
  namespace or shard);
* ``controller_manager`` — the same program with ``--controllers statefulset``:
  kube-controller-manager's StatefulSet controller;
* ``kubelet`` — :mod:`odh_kubeflow_amd.testing.cmd.fake_kubelet` for all the node's GPUs:
  registers the Node, runs each pod's init containers (with ``exec_init`` the MI355X start-up
  probe ``odh-gpu-probe`` as a real process on the pod's GPU) and reports pod status.

``workers`` > 1 runs the StatefulSet controller and the kubelet as that many processes each,
worker i of both serving the namespaces claimed for i (least-loaded first,
:class:`~odh_kubeflow_amd.testing.kubelet.statefulset.NamespaceClaimer`; ``--partition
i/W``).  That is the concurrency kube-controller-manager and the kubelet have in their
goroutines and one Python event loop has not: at 4 ranks a single StatefulSet controller
process was ≈80 % busy, so at 8 it would set the pace.  Device allocation stays with the one
scheduler (first free, written on the pod), so the workers never disagree about GPUs.

``process=True`` (the benchmark) runs both as child processes of rank 0; ``process=False``
runs the same controllers in this process (tests).  GC runs in the native apiserver.
"""

from __future__ import annotations

import asyncio
import os
import subprocess
import sys
from typing import Dict, List, Optional, Sequence

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


async def _in_thread(fn, *a):
    return await asyncio.get_running_loop().run_in_executor(None, fn, *a)


async def start_child(module: str, args: List[str], what: str, timeout: float = 120.0,
                      env: Optional[Dict[str, str]] = None, python_args: Sequence[str] = ()) -> subprocess.Popen:
    """``python [python_args] -m module args…`` with the repo on PYTHONPATH; waits for its
    ``ready`` line."""
    if env is None:
        env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    from ..utils.procutil import child_env

    import tempfile

    # the child's stderr goes to an unlinked temporary file: nothing accumulates, and a child
    # that fails to start says why in the exception.  ODH_CHILD_STDERR_DIR (diagnostics, e.g.
    # with PYTHONASYNCIODEBUG=1 to log every event-loop callback over 100 ms) keeps each
    # child's stderr as <dir>/<what>.<pid>.log instead
    keep = os.environ.get("ODH_CHILD_STDERR_DIR")
    if keep:
        os.makedirs(keep, exist_ok=True)
        err = tempfile.NamedTemporaryFile(dir=keep, prefix="".join(ch if ch.isalnum() else "_" for ch in what) + ".",
                                          suffix=".log", delete=False)
    else:
        err = tempfile.TemporaryFile()
    proc = subprocess.Popen([sys.executable, *python_args, "-m", module, *args], cwd=ROOT, env=child_env(env),
                            stdout=subprocess.PIPE, stderr=err, text=True)
    try:
        line = await asyncio.wait_for(_in_thread(proc.stdout.readline), timeout)
    except asyncio.TimeoutError:
        line = ""
    if line.strip() != "ready":
        proc.kill()
        proc.wait()
        err.seek(0)
        tail = err.read()[-2000:].decode(errors="replace").strip()
        err.close()
        raise RuntimeError(f"{what} did not start (rc={proc.poll()})" + (f": {tail}" if tail else ""))
    err.close()  # the child keeps writing to the unlinked file; it goes when the child does
    return proc


async def stop_child(proc: Optional[subprocess.Popen]) -> None:
    if proc is None:
        return
    proc.terminate()
    try:
        await asyncio.wait_for(_in_thread(proc.wait), 10)
    except asyncio.TimeoutError:
        proc.kill()


class NodePlatform:
    def __init__(self, apiserver_url: str, node_name: str = "mi355x-node-0", gpus: int = 8, process: bool = True,
                 exec_init: bool = False, hip_devices: int = 0, max_concurrent: int = 8, workers: int = 1,
                 pull_secret_delay_ms: float = -1.0, jupyter_proxy: bool = False):
        self.url = apiserver_url
        self.node_name = node_name
        self.gpus = gpus
        self.process = process
        self.exec_init = exec_init
        self.hip_devices = hip_devices
        self.max_concurrent = max_concurrent
        self.workers = max(1, int(workers))
        # >= 0: OpenShift's ServiceAccount pull-secret controller, adding each SA's dockercfg
        # secret this many ms after the SA appears (testing/kubelet/openshift.py)
        self.pull_secret_delay_ms = float(pull_secret_delay_ms)
        # the culler's DEV-mode kubectl proxy in front of every notebook's Jupyter API
        # (testing/cmd/jupyter_proxy.py): the resident-population benchmark's idle notebooks
        self.jupyter_proxy = jupyter_proxy
        self.jupyter_proxy_url: Optional[str] = None
        self.procs: Dict[str, subprocess.Popen] = {}
        self.managers = []
        self.agent = None
        self._rest = None
        self._caches = []

    async def start(self) -> "NodePlatform":
        if self.process:
            prof = os.environ.get("ODH_PLATFORM_PROFILE")  # cProfile output prefix (profiling runs)

            def pre(name):
                return ["-m", "cProfile", "-o", f"{prof}.{name}"] if prof else []
            ctrls = "scheduler" + (",pull-secrets" if self.pull_secret_delay_ms >= 0 else "")
            self.procs["scheduler"] = await start_child(
                "odh_kubeflow_amd.testing.cmd.scheduler",
                ["--master", self.url, "--controllers", ctrls,
                 "--pull-secret-delay-ms", f"{max(0.0, self.pull_secret_delay_ms):g}"],
                "scheduler", python_args=pre("scheduler"))
            w = self.workers
            for i in range(w):
                name = "controller_manager" if w == 1 else f"controller_manager_{i}"
                self.procs[name] = await start_child(
                    "odh_kubeflow_amd.testing.cmd.scheduler",
                    ["--master", self.url, "--controllers", "statefulset", "--partition", f"{i}/{w}"],
                    "StatefulSet controller", python_args=pre(name))
            for i in range(w):
                name = "kubelet" if w == 1 else f"kubelet_{i}"
                args = ["--master", self.url, "--node-name", self.node_name, "--node-gpus", str(self.gpus),
                        "--devices", ",".join(str(i) for i in range(self.gpus)), "--ready-line",
                        "--partition", f"{i}/{w}"]
                if self.exec_init:
                    args += ["--exec-init", "--hip-devices", str(self.hip_devices)]
                self.procs[name] = await start_child("odh_kubeflow_amd.testing.cmd.fake_kubelet", args, "kubelet",
                                                     python_args=pre(name))
            if self.jupyter_proxy:
                from .shard import free_port

                port = free_port()
                self.procs["jupyter_proxy"] = await start_child("odh_kubeflow_amd.testing.cmd.jupyter_proxy",
                                                                ["--port", str(port)], "Jupyter proxy")
                self.jupyter_proxy_url = f"http://127.0.0.1:{port}"
            return self
        from ..models import kinds
        from ..runtime.informer import InformerCache
        from ..runtime.manager import Manager
        from ..runtime.rest import RestClient, RestConfig
        from ..testing.kubelet.agent import FakeKubeletAgent
        from ..testing.kubelet.node import FakeContainerRuntime, SchedulerController
        from ..testing.kubelet.statefulset import StatefulSetController

        self._rest = RestClient(RestConfig(host=self.url))
        cache = InformerCache(self._rest)
        self._caches.append(cache)
        shared = (self._rest, cache)
        kcm = Manager.remote(None, name="kube-controller-manager", default_max_concurrent=self.max_concurrent,
                             shared=shared)
        StatefulSetController(kcm.client, kcm.reader, kcm.get_event_recorder_for("statefulset-controller")) \
            .setup_with_manager(kcm)
        SchedulerController(kcm.client, kcm.reader, kcm.get_event_recorder_for("default-scheduler")) \
            .setup_with_manager(kcm)
        if self.pull_secret_delay_ms >= 0:
            from ..testing.kubelet.openshift import PullSecretController

            self.pull_secrets = PullSecretController(kcm.client, kcm.reader, self.pull_secret_delay_ms / 1e3)
            self.pull_secrets.setup_with_manager(kcm)
        kl = Manager.remote(None, name=f"kubelet-{self.node_name}", default_max_concurrent=self.max_concurrent,
                            shared=shared)
        vis = (lambda d: d % self.hip_devices) if self.hip_devices else None
        rt = FakeContainerRuntime(exec_init=self.exec_init, visible_device=vis)
        self.agent = FakeKubeletAgent(kl, self.node_name, list(range(self.gpus)), node_gpus=self.gpus, runtime=rt,
                                      one_runtime=True)
        self.managers = [kcm, kl]
        for mgr in self.managers:
            await mgr.start()
        await cache.wait_synced([kinds.POD, kinds.STATEFUL_SET])
        return self

    def pids(self) -> Dict[str, int]:
        return {k: p.pid for k, p in self.procs.items()}

    @property
    def probe_results(self) -> List[dict]:
        return self.agent.probe_results if self.agent is not None else []

    def idle(self) -> bool:
        return all(m.idle() for m in self.managers)

    async def stop(self) -> None:
        for k in [*[k for k in self.procs if k.startswith(("kubelet", "controller_manager", "jupyter"))], "scheduler"]:
            await stop_child(self.procs.pop(k, None))
        for mgr in reversed(self.managers):
            await mgr.stop()
        for c in self._caches:
            await c.stop()
        if self._rest is not None:
            await self._rest.close()
