"""Namespace-sharded control plane: one shard per MI355X rank against one apiserver.

The reference runs one notebook-controller and one odh-notebook-controller replica for
the whole cluster (``kf/main.go``, ``odh/main.go``; leader election, 1 worker each).  Its
throughput is bounded by that one process.  On an 8×MI355X node we scale the control
plane the way the node is scaled — one process per GPU — by sharding it on namespaces:

* the apiserver (native C++, multi-threaded; ``native/apiserver``) is shared;
* shard ``r`` runs the kf NotebookReconciler + event re-emitter, the odh reconciler, the
  odh mutating webhook (its own HTTPS server, registered by a per-shard
  MutatingWebhookConfiguration with a ``namespaceSelector``), the StatefulSet
  controller and the node agent of GPU ``r``;
* every manager of a shard shares ONE REST connection pool and ONE informer cache
  restricted to the shard's namespaces (+ the controller namespace), with HTTPRoutes
  (which live in the controller namespace) selected by their ``notebook-namespace``
  label — a shard receives only the watch events of the objects it owns, so per-shard
  work stays constant as shards are added;
* the node agent of GPU ``r`` watches only pods labelled ``amd.com/gpu-index=r`` (set by
  the scheduler together with the ``amd.com/gpu-ids`` allocation); the shard labels its
  namespace ``amd.com/gpu-affinity=r`` so the allocator gives its pods GPU ``r`` while it
  is free — pod start-up then stays inside the shard's own process;
* the bootstrap shard (rank 0) also registers the Node and, unless the scheduler runs as
  its own process (``cmd/scheduler.py``, what the multi-GPU benchmark does), schedules
  pods (``amd.com/gpu`` allocation).  GC runs in the apiserver.
"""

from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..models import kinds
from ..models import meta as m
from ..runtime.manager import Manager


@dataclass
class ShardConfig:
    apiserver_url: str
    namespace: str
    gpu: int
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


class ControlPlaneShard:
    def __init__(self, cfg: ShardConfig):
        import os

        self.cfg = cfg
        self.env = {**os.environ, **cfg.env}
        self.managers: List[Manager] = []
        self.kf: Optional[Manager] = None
        self.odh: Optional[Manager] = None
        self.agent = None
        self.webhook_server = None
        self._caches = []
        self._waiters = None

    # ------------------------------------------------------------------ build

    def _mgr(self, name: str, shared, **kw) -> Manager:
        mgr = Manager.remote(None, name=name, default_max_concurrent=self.cfg.max_concurrent, shared=shared, **kw)
        self.managers.append(mgr)
        return mgr

    async def start(self) -> "ControlPlaneShard":
        from ..controllers.notebook import NotebookEventReemitter, NotebookReconciler
        from ..controllers.metrics import NotebookMetrics
        from ..kubelet.agent import FakeKubeletAgent
        from ..kubelet.node import GPU_AFFINITY_LABEL, GPU_INDEX_LABEL, SchedulerController
        from ..kubelet.statefulset import StatefulSetController
        from ..runtime.informer import InformerCache
        from ..runtime.rest import RestClient, RestConfig

        cfg = self.cfg
        self.rest_config = RestConfig(host=cfg.apiserver_url)
        self.rest = RestClient(self.rest_config)
        self.admin = self.rest
        if cfg.bootstrap:
            for ns in ("default", cfg.controller_namespace):
                await self.ensure_namespace(ns)
        # the namespace's pods prefer this rank's GPU (its node agent lives in this process)
        await self.ensure_namespace(cfg.namespace, {GPU_AFFINITY_LABEL: str(cfg.gpu)})
        # The reference keeps ConfigMaps/Secrets out of its (cluster-wide) cache to bound
        # memory and reads them live.  A shard's cache spans two namespaces, so it caches
        # them in full and the webhook / odh reconciler read them locally.
        self.cache = InformerCache(
            self.rest, namespaces=[cfg.namespace, cfg.controller_namespace],
            selectors={kinds.HTTP_ROUTE: f"notebook-namespace={cfg.namespace}"})
        self._caches.append(self.cache)
        shared = (self.rest, self.cache)

        kube = self._mgr("kube-controller-manager", shared)
        StatefulSetController(kube.client, kube.reader, kube.get_event_recorder_for("statefulset-controller")) \
            .setup_with_manager(kube)

        # node agent of this rank's GPU (+ the cluster-wide scheduler on the bootstrap shard)
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

        if cfg.webhook and cfg.odh:
            await self._start_webhook(shared)
        self._build_kf(shared, NotebookReconciler, NotebookEventReemitter, NotebookMetrics)
        if cfg.odh:
            from ..controllers.odh.reconciler import OpenshiftNotebookReconciler

            odh = self.odh = self._mgr("odh-notebook-controller", shared)
            emu = cfg.reference_emulation
            r = OpenshiftNotebookReconciler(odh.client, odh.reader, cfg.controller_namespace, env=self.env,
                                            recorder=odh.get_event_recorder_for("odh-notebook-controller"),
                                            blocking_lock_removal=emu)
            r.setup_with_manager(odh, max_concurrent=1 if emu else None)
        for mgr in self.managers:
            await mgr.start()
        await self.cache.wait_synced([kinds.NOTEBOOK, kinds.POD, kinds.STATEFUL_SET])
        return self

    def _build_kf(self, shared, NotebookReconciler, NotebookEventReemitter, NotebookMetrics) -> None:
        kf = self.kf = self._mgr("notebook-controller", shared)
        metrics = NotebookMetrics(kf.reader, kf.registry)
        emu = self.cfg.reference_emulation
        r = NotebookReconciler(kf.client, kf.reader, kf.get_event_recorder_for("notebook-controller"), metrics,
                               env=self.env, unconditional_status=emu, owner_index=not emu)
        r.setup_with_manager(kf, max_concurrent=1 if emu else None)
        e = NotebookEventReemitter(kf.client, kf.reader, kf.get_event_recorder_for("notebook-controller"))
        e.setup_with_manager(kf, max_concurrent=1 if emu else None)

    async def _start_webhook(self, shared) -> None:
        from ..models.errors import ApiError, is_already_exists
        from ..webhook.certs import generate
        from ..webhook.notebook_webhook import NotebookWebhook
        from ..webhook.server import WebhookServer, mutating_webhook_configuration

        cfg = self.cfg
        wh_mgr = self._mgr("odh-webhook", shared)
        self.webhook = NotebookWebhook(wh_mgr.client, cfg.controller_namespace,
                                       kube_rbac_proxy_image=cfg.kube_rbac_proxy_image, env=self.env)
        certs = generate(("127.0.0.1", "localhost"))
        self.webhook_server = await WebhookServer(self.webhook, certs.cert_dir, "127.0.0.1", 0).start()
        mwc = mutating_webhook_configuration(
            certs.ca_bundle_b64, url=f"https://127.0.0.1:{self.webhook_server.port}/mutate-notebook-v1",
            name=f"odh-notebook-webhook-{cfg.namespace}",
            namespace_selector={"matchLabels": {"kubernetes.io/metadata.name": cfg.namespace}})
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

    def reconcile_count(self) -> int:
        return sum(mgr.reconcile_count() for mgr in (self.kf, self.odh) if mgr is not None)

    def reconcile_breakdown(self) -> dict:
        out: dict = {}
        for mgr in (self.kf, self.odh):
            if mgr is not None:
                out.update(mgr.reconcile_breakdown())
        return out

    async def settle(self, timeout: float = 10.0) -> bool:
        deadline = time.monotonic() + timeout
        quiet = 0
        while time.monotonic() < deadline:
            if all(mgr.idle() for mgr in self.managers):
                quiet += 1
                if quiet >= 3:
                    return True
            else:
                quiet = 0
            await asyncio.sleep(0.002)
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
        if self.webhook_server is not None:
            await self.webhook_server.stop()
        for c in self._caches:
            await c.stop()
        await self.rest.close()
