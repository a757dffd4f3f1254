"""One namespace shard of the benchmark: the shipped control-plane process + platform stand-ins.

The reference runs one notebook-controller and one odh-notebook-controller replica for
the whole cluster (``kf/main.go:87-98``, ``odh/main.go:155-192``; one worker each).  The
MI355X deployment (``config/overlays/mi355x-sharded``) runs N shards of
``cmd/control_plane.py`` — one per MI355X of the node, replica k owning the namespaces
labelled ``notebooks.amd.com/shard=k`` — against the cluster's apiserver.  A benchmark
shard is exactly that deployment unit plus the platform it would find on a node:

* **the product** — ``python -m odh_kubeflow_amd.cmd.control_plane --shard r …`` as a
  child process (``process=True``, what ``bench.py`` runs), or the same
  :func:`~odh_kubeflow_amd.cmd.control_plane.build` inside this process (tests, tools):
  kf reconciler + event re-emitter, odh reconciler and the odh mutating webhook (HTTPS,
  registered by this shard's MutatingWebhookConfiguration with a ``namespaceSelector``
  on the shard label), one informer cache over the shard's namespaces;
* **the platform stand-ins** (what kube-controller-manager and the kubelet do on a real
  cluster; never deployed) — the StatefulSet controller for the shard's namespace and the
  fake kubelet of GPU ``r`` (pods labelled ``amd.com/gpu-index=r``; it gates Ready on the
  MI355X start-up probe).  The shard's namespace is labelled ``amd.com/gpu-affinity=r`` so
  the scheduler stand-in (``cmd/scheduler.py``) gives its pods GPU ``r``;
* the bootstrap shard (rank 0) also registers the Node.  GC runs in the apiserver.
"""

from __future__ import annotations

import asyncio
import os
import shutil
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..controllers.setup import SHARD_LABEL
from ..models import kinds
from ..models import meta as m
from ..runtime.manager import Manager

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class ShardConfig:
    apiserver_url: str
    namespace: str
    gpu: int
    shard: Optional[str] = None  # default: str(gpu)
    node_name: str = "mi355x-node-0"
    node_gpus: int = 8
    controller_namespace: str = "opendatahub"
    bootstrap: bool = False
    # the bootstrap shard hosts the scheduler unless it runs as its own process
    # (``cmd/scheduler.py``, as kube-scheduler does); the node agent then watches only
    # its GPU's pods on every shard, bootstrap included (no CPU-only pods in that mode)
    run_scheduler: bool = True
    odh: bool = True
    webhook: bool = True
    startup_probe: Optional[Callable] = None
    reference_emulation: bool = False
    max_concurrent: int = 8
    env: Dict[str, str] = field(default_factory=dict)
    kube_rbac_proxy_image: str = "quay.io/brancz/kube-rbac-proxy:v0.18.1"
    process: bool = False  # run the control plane as its own process (cmd/control_plane.py)


class ControlPlaneShard:
    def __init__(self, cfg: ShardConfig):
        self.cfg = cfg
        self.shard = cfg.shard if cfg.shard is not None else str(cfg.gpu)
        self.env = {**os.environ, **cfg.env}
        self.managers: List[Manager] = []
        self.control_plane: Optional[Manager] = None  # in-process mode
        self.proc: Optional[subprocess.Popen] = None  # process mode
        self.metrics_url: Optional[str] = None
        self.agent = None
        self._caches = []
        self._waiters = None
        self._certs = None

    # ------------------------------------------------------------------ build

    def _cp_args(self, webhook_port: int, metrics_port: int, probe_port: int) -> List[str]:
        cfg = self.cfg
        ctrls = ["kf"] + (["odh"] if cfg.odh else []) + (["webhook"] if cfg.odh and cfg.webhook else [])
        a = ["--master", cfg.apiserver_url, "--shard", self.shard, "--controllers", ",".join(ctrls),
             "--kube-rbac-proxy-image", cfg.kube_rbac_proxy_image,
             "--webhook-cert-dir", self._certs.cert_dir, "--webhook-host", "127.0.0.1",
             "--webhook-port", str(webhook_port),
             "--metrics-bind-address", f"127.0.0.1:{metrics_port}" if metrics_port else "0",
             "--health-probe-bind-address", f"127.0.0.1:{probe_port}" if probe_port else "0",
             "--max-concurrent-reconciles", str(cfg.max_concurrent)]
        if cfg.reference_emulation:
            a.append("--reference-emulation")
        return a

    def _cp_env(self) -> Dict[str, str]:
        return {**self.env, "K8S_NAMESPACE": self.cfg.controller_namespace}

    async def start(self) -> "ControlPlaneShard":
        from ..kubelet.agent import FakeKubeletAgent
        from ..kubelet.node import GPU_AFFINITY_LABEL, GPU_INDEX_LABEL, SchedulerController
        from ..kubelet.statefulset import StatefulSetController
        from ..runtime.informer import InformerCache
        from ..runtime.rest import RestClient, RestConfig
        from ..webhook.certs import generate

        cfg = self.cfg
        self.rest_config = RestConfig(host=cfg.apiserver_url)
        self.rest = RestClient(self.rest_config)
        self.admin = self.rest
        if cfg.bootstrap:
            for ns in ("default", cfg.controller_namespace):
                await self.ensure_namespace(ns)
        # the shard owns the namespace; its pods prefer this rank's GPU
        await self.ensure_namespace(cfg.namespace, {SHARD_LABEL: self.shard, GPU_AFFINITY_LABEL: str(cfg.gpu)})

        # ---- the product: cmd/control_plane.py --shard <shard>
        self._certs = generate(("127.0.0.1", "localhost"))
        if cfg.process:
            wport, mport = free_port(), free_port()
            self.metrics_url = f"http://127.0.0.1:{mport}/metrics"
            prof = self.env.get("ODH_CONTROL_PLANE_PROFILE")  # cProfile output path (profiling runs)
            pre = ["-m", "cProfile", "-o", f"{prof}.{self.shard}"] if prof else []
            self.proc = subprocess.Popen(
                [sys.executable, *pre, "-m", "odh_kubeflow_amd.cmd.control_plane", *self._cp_args(wport, mport, 0)],
                cwd=ROOT, env={**self._cp_env(), "PYTHONPATH": ROOT + os.pathsep + self.env.get("PYTHONPATH", "")},
                stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
            line = await asyncio.wait_for(asyncio.get_running_loop().run_in_executor(None, self.proc.stdout.readline),
                                          120)
            if line.strip() != "ready":
                self.proc.kill()
                raise RuntimeError(f"control plane shard {self.shard} did not start (rc={self.proc.poll()})")
        else:
            from ..cmd import control_plane

            args = control_plane.parse(self._cp_args(0, 0, 0))
            self.control_plane = control_plane.build(args, self._cp_env())
            await self.control_plane.start()
            await self.control_plane.elected.wait()
            wport = self.control_plane.webhook_server.port if self.control_plane.webhook_server else 0
        if cfg.webhook and cfg.odh:
            await self._register_webhook(wport)

        # ---- platform stand-ins: StatefulSet controller + this GPU's kubelet (+ scheduler)
        self.cache = InformerCache(self.rest, namespaces=[cfg.namespace])
        self._caches.append(self.cache)
        shared = (self.rest, self.cache)
        kube = self._mgr("kube-controller-manager", shared)
        StatefulSetController(kube.client, kube.reader, kube.get_event_recorder_for("statefulset-controller")) \
            .setup_with_manager(kube)
        schedules = cfg.bootstrap and cfg.run_scheduler
        if schedules:
            node_cache = InformerCache(self.rest)
        else:
            node_cache = InformerCache(self.rest, selectors={kinds.POD: f"{GPU_INDEX_LABEL}={cfg.gpu}"})
        self._caches.append(node_cache)
        kl = self._mgr(f"kubelet-gpu{cfg.gpu}", (self.rest, node_cache))
        if schedules:
            SchedulerController(kl.client, kl.reader, kl.get_event_recorder_for("default-scheduler")) \
                .setup_with_manager(kl)
        self.agent = FakeKubeletAgent(kl, cfg.node_name, [cfg.gpu], node_gpus=cfg.node_gpus,
                                      startup_probe=cfg.startup_probe, register_node=cfg.bootstrap,
                                      owns_cpu_pods=schedules)
        for mgr in self.managers:
            await mgr.start()
        await self.cache.wait_synced([kinds.NOTEBOOK, kinds.POD, kinds.STATEFUL_SET])
        return self

    def _mgr(self, name: str, shared) -> Manager:
        mgr = Manager.remote(None, name=name, default_max_concurrent=self.cfg.max_concurrent, shared=shared)
        self.managers.append(mgr)
        return mgr

    async def _register_webhook(self, port: int) -> None:
        """This shard's MutatingWebhookConfiguration (what the overlay ships per shard, with a
        URL instead of the per-shard Service since the apiserver here runs on the host)."""
        from ..models.errors import ApiError, is_already_exists
        from ..webhook.server import mutating_webhook_configuration

        mwc = mutating_webhook_configuration(
            self._certs.ca_bundle_b64, url=f"https://127.0.0.1:{port}/mutate-notebook-v1",
            name=f"odh-notebook-webhook-shard-{self.shard}",
            namespace_selector={"matchLabels": {SHARD_LABEL: self.shard}})
        try:
            await self.admin.create(mwc)
        except ApiError as e:
            if not is_already_exists(e):
                raise
            cur = await self.admin.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, m.name(mwc))
            mwc["metadata"]["resourceVersion"] = m.resource_version(cur)
            await self.admin.update(mwc)

    # ------------------------------------------------------------------ helpers

    async def ensure_namespace(self, ns: str, labels: Optional[Dict[str, str]] = None) -> None:
        from ..models.errors import ApiError, is_already_exists

        meta = {"name": ns, **({"labels": dict(labels)} if labels else {})}
        try:
            await self.rest.create({"apiVersion": "v1", "kind": "Namespace", "metadata": meta})
        except ApiError as e:
            if not is_already_exists(e):
                raise
            if labels:
                await self.rest.patch(kinds.NAMESPACE, {"metadata": {"labels": dict(labels)}}, name=ns)

    def peek(self, kind, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        return self.cache.get(kind, name, namespace)

    def notebook_ready(self, name: str) -> bool:
        nb = self.cache.get(kinds.NOTEBOOK, name, self.cfg.namespace)
        if nb is None:
            return False
        st = nb.get("status") or {}
        if st.get("readyReplicas") != 1:
            return False
        return any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])

    def gone(self, name: str) -> bool:
        ns = self.cfg.namespace
        return self.cache.get(kinds.NOTEBOOK, name, ns) is None and self.cache.get(kinds.POD, f"{name}-0", ns) is None

    # -------------------------------------------------------------- control-plane counters

    async def scrape(self) -> Dict[str, Dict[tuple, float]]:
        """Process mode: the control plane's ``/metrics`` → {sample name: {sorted labels: value}}."""
        import aiohttp
        from prometheus_client.parser import text_string_to_metric_families

        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=10)) as s:
            async with s.get(self.metrics_url) as r:
                text = await r.text()
        out: Dict[str, Dict[tuple, float]] = {}
        for fam in text_string_to_metric_families(text):
            for smp in fam.samples:
                out.setdefault(smp.name, {})[tuple(sorted(smp.labels.items()))] = smp.value
        return out

    async def reconcile_breakdown(self) -> dict:
        """controller → {trigger → reconciles} of the notebook controllers (the culler and the
        namespace assigner are not part of a notebook's create→Ready path)."""
        skip = ("Culler", "shard-assigner")
        if self.control_plane is not None:
            return {k: v for k, v in self.control_plane.reconcile_breakdown().items() if k not in skip}
        out: dict = {}
        for labels, v in (await self.scrape()).get("odh_controller_reconcile_trigger_total", {}).items():
            d = dict(labels)
            if d.get("controller") in skip:
                continue
            out.setdefault(d["controller"], {})[d["trigger"]] = int(v)
        return out

    async def reconcile_count(self) -> int:
        return sum(sum(t.values()) for t in (await self.reconcile_breakdown()).values())

    def control_plane_pid(self) -> Optional[int]:
        return self.proc.pid if self.proc is not None else None

    # ------------------------------------------------------------------ waiting

    async def _cp_idle(self, last: list) -> bool:
        """Process mode: every workqueue of the control plane empty, no worker active, and the
        reconcile total unchanged since the previous poll (read from its ``/metrics``)."""
        samples = await self.scrape()
        busy = sum(samples.get("workqueue_depth", {}).values()) + \
            sum(samples.get("controller_runtime_active_workers", {}).values())
        total = sum(samples.get("controller_runtime_reconcile_total", {}).values())
        quiet = busy == 0 and last and last[0] == total
        last[:] = [total]
        return bool(quiet)

    async def settle(self, timeout: float = 10.0) -> bool:
        """Platform stand-ins and the control plane idle, three polls in a row."""
        mgrs = self.managers + ([self.control_plane] if self.control_plane is not None else [])
        deadline = time.monotonic() + timeout
        quiet = 0
        last: list = []
        while time.monotonic() < deadline:
            idle = all(mgr.idle() for mgr in mgrs)
            if idle and self.proc is not None:
                idle = await self._cp_idle(last)
            if idle:
                quiet += 1
                if quiet >= 3:
                    return True
            else:
                quiet = 0
            await asyncio.sleep(0.002 if self.proc is None else 0.01)
        return False

    async def wait_until(self, pred: Callable[[], bool], timeout: float = 10.0) -> bool:
        """Event-driven wait: ``pred`` is re-checked on every Notebook / Pod event of the
        shard's namespace (after the cache applied it) instead of on a polling timer."""
        if pred():
            return True
        if self._waiters is None:
            self._waiters = set()

            def on_event(etype, obj, old):
                for w in list(self._waiters):
                    fut, p = w
                    if not fut.done() and p():
                        fut.set_result(True)
            for k in (kinds.NOTEBOOK, kinds.POD):
                self.cache.subscribe(k, on_event, namespace=self.cfg.namespace)
        fut = asyncio.get_running_loop().create_future()
        w = (fut, pred)
        self._waiters.add(w)
        try:
            return await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            return pred()
        finally:
            self._waiters.discard(w)

    async def wait_for(self, pred: Callable[[], bool], timeout: float = 10.0, interval: float = 0.0005) -> bool:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if pred():
                return True
            await asyncio.sleep(interval)
        return pred()

    @property
    def probe_results(self) -> List[dict]:
        return self.agent.probe_results if self.agent is not None else []

    async def stop(self) -> None:
        for mgr in reversed(self.managers):
            await mgr.stop()
        if self.control_plane is not None:
            await self.control_plane.stop()
        if self.proc is not None:
            self.proc.terminate()
            try:
                await asyncio.wait_for(asyncio.get_running_loop().run_in_executor(None, self.proc.wait), 10)
            except asyncio.TimeoutError:
                self.proc.kill()
        for c in self._caches:
            await c.stop()
        await self.rest.close()
        if self._certs is not None:
            shutil.rmtree(self._certs.cert_dir, ignore_errors=True)
