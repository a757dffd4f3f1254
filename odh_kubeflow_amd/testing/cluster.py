"""In-process cluster assembly: fake apiserver + the three controllers + fake node(s).

Used by the tests (the envtest-equivalent substrate), ``bench.py`` and the smoke test.
Every piece is the production component; only the apiserver, kube-controller-manager
(StatefulSet controller, scheduler, optional GC) and kubelet are stand-ins.
"""

from __future__ import annotations

import asyncio
import os
import tempfile
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from .apiserver.inprocess import in_process_manager
from .apiserver.store import ObjectStore
from ..models import kinds
from ..runtime.manager import Manager


@dataclass
class ClusterConfig:
    gc: bool = True
    gpus_per_node: int = 8
    nodes: int = 1
    kf: bool = True
    culler: bool = False
    odh: bool = False
    webhook: bool = False
    event_reemit: bool = True
    controller_namespace: str = "opendatahub"
    max_concurrent: int = 8
    env: Dict[str, str] = field(default_factory=dict)
    kube_rbac_proxy_image: str = "quay.io/brancz/kube-rbac-proxy:v0.18.1"
    runtime_factory: Optional[Callable[[int], object]] = None  # device -> ContainerRuntime
    # run the MI355X start-up probe init container (``amd.com/gpu-probe``) as a real process on
    # the pod's GPU; ``probe_visible_device`` maps node GPU index -> HIP device of this box
    exec_gpu_probe: bool = False
    probe_visible_device: Optional[Callable[[int], int]] = None
    gpu_runtimes_in_process: bool = True  # False: rank processes host GPU runtimes (multi-GPU bench)
    reference_emulation: bool = False  # reproduce the reference's serialising behaviour for comparison
    activity_source: Optional[object] = None
    # amdgpu telemetry (ops.telemetry.Telemetry) for the nodes: each node then runs the
    # production node agent (nodeagent/), which attributes GPUs to pods from the fake
    # kubelet's device-plugin checkpoint; the culler queries it over HTTP
    telemetry: Optional[object] = None
    device_id_of: Optional[Callable[[int], str]] = None  # node GPU index -> device-plugin ID (PCI address)
    openshift: bool = False  # serve the OpenShift APIs (image/config/route/oauth) like an OCP cluster
    # "inprocess": managers share the store directly; "http": the store is served by the REST
    # apiserver and the kf / odh managers, the webhook (HTTPS, MutatingWebhookConfiguration)
    # and the node agents talk to it over HTTP exactly as they would to kube-apiserver
    transport: str = field(default_factory=lambda: os.environ.get("ODH_CLUSTER_TRANSPORT", "inprocess"))
    remote_kubelets: bool = True  # with transport="http": node agents use REST clients too
    # Gateway API implementation stand-in (HTTPRoute ResolvedRefs status); default: with odh
    gateway: Optional[bool] = None
    # the reference envtest suite's debug aids (odh/controllers/suite_test.go:125-155): an
    # apiserver audit log (network transports) and a kubeconfig for poking at the test
    # apiserver with kubectl / the REST client while a test runs
    audit_log_path: Optional[str] = field(default_factory=lambda: os.environ.get("DEBUG_WRITE_AUDITLOG"))
    kubeconfig_path: Optional[str] = field(default_factory=lambda: os.environ.get("DEBUG_WRITE_KUBECONFIG"))
    audit_policy: Optional[object] = None  # apiserver.audit.AuditPolicy (default: config/debug/audit-policy.yaml)


OPENSHIFT_CRDS = (kinds.IMAGE_STREAM, kinds.PROXY, kinds.ROUTE, kinds.OAUTH_CLIENT)


def write_kubeconfig(path: str, server: str, user: str = "MasterOfTheSystems") -> None:
    """A kubeconfig for the test apiserver (``DEBUG_WRITE_KUBECONFIG``; the reference writes a
    ``system:masters`` user's kubeconfig for its envtest apiserver).  The test apiservers do
    not authenticate, so the user carries no credentials."""
    import yaml

    doc = {"apiVersion": "v1", "kind": "Config", "current-context": "odh-test",
           "clusters": [{"name": "odh-test", "cluster": {"server": server}}],
           "users": [{"name": user, "user": {}}],
           "contexts": [{"name": "odh-test", "context": {"cluster": "odh-test", "user": user}}]}
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        yaml.safe_dump(doc, f, sort_keys=False)


class LocalCluster:
    def __init__(self, cfg: Optional[ClusterConfig] = None, store: Optional[ObjectStore] = None):
        self.cfg = cfg or ClusterConfig()
        self.env = {**os.environ, **self.cfg.env}
        self.native = None
        if self.cfg.transport == "native":
            self.store = None  # a StoreView over an informer cache, set in start()
        else:
            self.store = store or ObjectStore(gc=self.cfg.gc)
            if not self.cfg.openshift and store is None:
                for crd in OPENSHIFT_CRDS:
                    self.store.uninstall_crd(crd)
        self.managers: List[Manager] = []
        self.kube: Optional[Manager] = None
        self.kf: Optional[Manager] = None
        self.odh: Optional[Manager] = None
        self.kubelets: List[Manager] = []
        self.gpu_runtimes = []
        self.device_managers = {}  # node name -> FakeDeviceManager
        self.node_agents = {}  # node name -> production NodeTelemetryAgent
        self._tmpdirs = []
        self.reconcilers: Dict[str, object] = {}
        self.webhook = None
        self.apiserver = None
        self.webhook_server = None
        self.rest_config = None

    # ------------------------------------------------------------------ build

    def _mgr(self, name: str, remote: bool = False, **kw) -> Manager:
        if (remote or self.cfg.transport == "native") and self.rest_config is not None:
            mgr = Manager.remote(self.rest_config, name=name, default_max_concurrent=self.cfg.max_concurrent,
                                 shared=self._shared(), **kw)
        else:
            mgr = in_process_manager(self.store, name=name, default_max_concurrent=self.cfg.max_concurrent, **kw)
        self.managers.append(mgr)
        return mgr

    def _shared(self):
        """One REST pool + informer cache for every remote manager of this process."""
        if getattr(self, "_shared_pair", None) is None:
            from ..runtime.informer import InformerCache, strip_data
            from ..runtime.rest import RestClient

            rest = RestClient(self.rest_config)
            self._shared_pair = (rest, InformerCache(rest, transforms={kinds.CONFIG_MAP: strip_data,
                                                                       kinds.SECRET: strip_data}))
        return self._shared_pair

    async def _start_apiserver(self) -> None:
        from .apiserver.http import ApiServer
        from ..runtime.rest import RestConfig

        audit = None
        if self.cfg.audit_log_path:
            from .apiserver.audit import DEFAULT_POLICY, AuditLogger, AuditPolicy

            audit = AuditLogger(self.cfg.audit_log_path, self.cfg.audit_policy or AuditPolicy.load(DEFAULT_POLICY))
        self.apiserver = await ApiServer(self.store, audit=audit).start("127.0.0.1", 0)
        self.rest_config = RestConfig(host=self.apiserver.url)

    async def start(self) -> "LocalCluster":
        from .kubelet.agent import default_device_id_of
        from .kubelet.node import FakeContainerRuntime, FakeDeviceManager, GpuRuntime, SchedulerController, make_node
        from .kubelet.statefulset import StatefulSetController
        from ..nodeagent.checkpoint import CheckpointWriter

        cfg = self.cfg
        if cfg.transport == "http":
            await self._start_apiserver()
        if cfg.transport == "native":
            from .apiserver.native import NativeApiServer, StoreView
            from ..runtime.informer import InformerCache
            from ..runtime.rest import RestClient, RestConfig

            self.native = await NativeApiServer(() if cfg.openshift else OPENSHIFT_CRDS, gc=cfg.gc,
                                                audit_log_path=cfg.audit_log_path, audit_policy=cfg.audit_policy).start()
            self.rest_config = RestConfig(host=self.native.url)
            admin = RestClient(self.rest_config)
            self._view_cache = InformerCache(admin)
            self.store = StoreView(self._view_cache)
            await self._view_cache.wait_synced(
                [k for k in (kinds.NAMESPACE, kinds.NODE, kinds.NOTEBOOK, kinds.STATEFUL_SET, kinds.POD,
                             kinds.SERVICE, kinds.EVENT, kinds.CONFIG_MAP, kinds.SECRET, kinds.SERVICE_ACCOUNT,
                             kinds.NETWORK_POLICY, kinds.ROLE_BINDING, kinds.CLUSTER_ROLE_BINDING, kinds.HTTP_ROUTE,
                             kinds.REFERENCE_GRANT, kinds.VIRTUAL_SERVICE, kinds.LEASE)])
        else:
            admin = in_process_manager(self.store, name="admin").client
        self.admin = admin
        if cfg.kubeconfig_path and self.rest_config is not None:
            write_kubeconfig(cfg.kubeconfig_path, self.rest_config.host)
        for ns in ("default", cfg.controller_namespace):
            await self.ensure_namespace(ns)

        # fake kube-controller-manager + scheduler
        kube = self.kube = self._mgr("kube-controller-manager", remote=cfg.transport == "native")
        StatefulSetController(kube.client, kube.reader, kube.get_event_recorder_for("statefulset-controller")) \
            .setup_with_manager(kube)
        SchedulerController(kube.client, kube.reader, kube.get_event_recorder_for("default-scheduler")) \
            .setup_with_manager(kube)
        if cfg.gateway or (cfg.gateway is None and cfg.odh):
            from .kubelet.gateway import GatewayRouteResolver

            GatewayRouteResolver(kube.client, kube.reader).setup_with_manager(kube)

        # nodes + per-GPU runtimes
        for n in range(cfg.nodes):
            node_name = f"mi355x-node-{n}"
            await admin.create(make_node(node_name, cfg.gpus_per_node))
            tmp = tempfile.TemporaryDirectory(prefix=f"odh-{node_name}-")
            self._tmpdirs.append(tmp)
            cp_path = os.path.join(tmp.name, "device-plugins", "kubelet_internal_checkpoint")
            dm = self.device_managers[node_name] = FakeDeviceManager(
                cfg.device_id_of or default_device_id_of(cfg.telemetry), checkpoint=CheckpointWriter(cp_path))
            if cfg.telemetry is not None:
                from ..nodeagent.attribution import Attributor
                from ..nodeagent.server import NodeTelemetryAgent

                # the production agent over HTTPS, as the DaemonSet serves it
                self.node_agents[node_name] = await NodeTelemetryAgent(
                    cfg.telemetry, Attributor(cfg.telemetry, checkpoint_path=cp_path, ttl_s=0.0),
                    host="127.0.0.1", port=0, tls_cert_dir=self._agent_cert_dir(node_name)).start()
            if cfg.gpu_runtimes_in_process:
                kl = self._mgr(f"kubelet-{node_name}", remote=cfg.remote_kubelets)
                self.kubelets.append(kl)
                for d in range(cfg.gpus_per_node):
                    rt = cfg.runtime_factory(d) if cfg.runtime_factory else None
                    if rt is None and cfg.exec_gpu_probe:
                        rt = FakeContainerRuntime(exec_init=True, visible_device=cfg.probe_visible_device)
                    g = GpuRuntime(kl.client, kl.reader, kl.get_event_recorder_for("kubelet"), node_name, [d],
                                   runtime=rt, owns_cpu_pods=(d == 0), device_manager=dm)
                    g.setup_with_manager(kl, name=f"kubelet-{node_name}-gpu{d}")
                    self.gpu_runtimes.append(g)

        if cfg.webhook:
            await self._start_webhook()
        if cfg.kf:
            self._build_kf()
        if cfg.odh:
            self._build_odh()
        for mgr in self.managers:
            await mgr.start()
        return self

    def _agent_ca_dir(self) -> str:
        """The node agents' CA (``ca.crt`` / ``ca.key``), as the signer keeps it."""
        if getattr(self, "_agent_ca", None) is None:
            from ..webhook.certs import generate_ca

            tmp = tempfile.TemporaryDirectory(prefix="odh-agent-ca-")
            self._tmpdirs.append(tmp)
            generate_ca(tmp.name)
            self._agent_ca = tmp.name
        return self._agent_ca

    def _agent_cert_dir(self, node: str) -> str:
        """Node ``node``'s own agent identity — a key of its own and a certificate naming the
        node, as ``nodeagent/identity.py``'s signer issues it for that node's agent pod."""
        from ..nodeagent.identity import LEAF_VALIDITY_S, new_key_and_csr, sign_leaf

        ca = self._agent_ca_dir()
        d = os.path.join(ca, node)
        os.makedirs(d, exist_ok=True)
        key, csr = new_key_and_csr(node, "127.0.0.1")
        with open(os.path.join(ca, "ca.crt")) as f, open(os.path.join(ca, "ca.key")) as g:
            crt = sign_leaf(csr, f.read(), g.read(), node, "127.0.0.1", LEAF_VALIDITY_S)
        for name, pem in (("tls.key", key), ("tls.crt", crt)):
            with open(os.path.join(d, name), "w") as f:
                f.write(pem)
        return d

    def _build_kf(self) -> None:
        from ..controllers.setup import setup_kf

        kf = self.kf = self._mgr("notebook-controller", remote=True)
        culling = bool(self.cfg.culler or self.env.get("ENABLE_CULLING") == "true")
        activity = self.cfg.activity_source
        if culling and activity is None and self.node_agents:
            from ..controllers.culling import NodeAgentActivity

            # every fake node's pods report hostIP 127.0.0.1: route by node name instead
            ports = {n: a.port for n, a in self.node_agents.items()}
            activity = NodeAgentActivity(endpoint_for=lambda pod: "127.0.0.1:%d" % ports[
                (pod.get("spec") or {}).get("nodeName")] if (pod.get("spec") or {}).get("nodeName") in ports
                else None, ca_file=os.path.join(self._agent_ca_dir(), "ca.crt"))
        out = setup_kf(kf, self.env, culling=culling, activity=activity, event_reemit=self.cfg.event_reemit,
                       reference_emulation=self.cfg.reference_emulation)
        self.kf_metrics = out["metrics"]
        for k in ("notebook", "events", "culler"):
            if k in out:
                self.reconcilers[k] = out[k]

    def _build_odh(self) -> None:
        from ..controllers.setup import setup_odh

        odh = self.odh = self._mgr("odh-notebook-controller", remote=True, uncached=(kinds.CONFIG_MAP, kinds.SECRET))
        self.reconcilers["odh"] = setup_odh(odh, self.cfg.controller_namespace, self.env,
                                            reference_emulation=self.cfg.reference_emulation)

    async def _start_webhook(self) -> None:
        from ..webhook.notebook_webhook import NotebookWebhook, register_in_process

        if self.rest_config is not None:
            from ..webhook.certs import generate  # noqa: F811
            from ..webhook.server import WebhookServer, mutating_webhook_configuration

            wh_mgr = self._mgr("odh-webhook", remote=True, uncached=(kinds.CONFIG_MAP, kinds.SECRET))
            self.webhook = NotebookWebhook(wh_mgr.client, self.cfg.controller_namespace,
                                           kube_rbac_proxy_image=self.cfg.kube_rbac_proxy_image, env=self.env)
            certs = generate(("127.0.0.1", "localhost"))
            self.webhook_server = await WebhookServer(self.webhook, certs.cert_dir, "127.0.0.1", 0).start()
            await self.admin.create(mutating_webhook_configuration(
                certs.ca_bundle_b64, url=f"https://127.0.0.1:{self.webhook_server.port}/mutate-notebook-v1"))
            return
        wh_mgr = in_process_manager(self.store, name="odh-webhook", uncached=(kinds.CONFIG_MAP, kinds.SECRET))
        self.webhook = NotebookWebhook(wh_mgr.client, self.cfg.controller_namespace,
                                       kube_rbac_proxy_image=self.cfg.kube_rbac_proxy_image, env=self.env)
        register_in_process(self.store, self.webhook)

    # ------------------------------------------------------------------ helpers

    async def ensure_namespace(self, ns: str) -> None:
        if self.store.peek(kinds.NAMESPACE, ns) is None:
            from ..models.errors import ApiError, is_already_exists

            try:
                await self.admin.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            except ApiError as e:
                if not is_already_exists(e):
                    raise

    async def edit(self, kind, name: str, namespace: Optional[str], fn: Callable[[dict], None]) -> dict:
        """A user's read-modify-write of one object (``kubectl edit``): re-read and retried
        on a Conflict, as controllers (and stand-ins such as the gateway's status writer) may
        write the object between the read and the write."""
        from ..runtime.retry import retry_on_conflict

        async def attempt():
            cur = await self.admin.get(kind, name, namespace)
            fn(cur)
            return await self.admin.update(cur)
        return await retry_on_conflict(attempt)

    async def stop(self) -> None:
        for mgr in reversed(self.managers):
            await mgr.stop()
        for g in self.gpu_runtimes:
            await g.close()
        for a in self.node_agents.values():
            await a.stop()
        for t in self._tmpdirs:
            t.cleanup()
        if self.webhook_server is not None:
            await self.webhook_server.stop()
        if self.apiserver is not None:
            await self.apiserver.stop()
        if getattr(self, "_shared_pair", None) is not None:
            await self._shared_pair[1].stop()
            await self._shared_pair[0].close()
        if self.native is not None:
            await self._view_cache.stop()
            await self.admin.close()
            await self.native.stop()

    async def settle(self, timeout: float = 10.0) -> bool:
        """Wait until every controller in every manager is idle (twice, to catch cascades)."""
        deadline = time.monotonic() + timeout
        quiet = 0
        while time.monotonic() < deadline:
            if all(mgr.idle() for mgr in self.managers):
                quiet += 1
                if quiet >= 3:
                    for mgr in self.managers:
                        for rec in mgr._recorders.values():
                            await rec.flush()
                    return True
            else:
                quiet = 0
            await asyncio.sleep(0.002)
        return False

    async def wait_for(self, pred: Callable[[], bool], timeout: float = 10.0, interval: float = 0.002) -> bool:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if pred():
                return True
            await asyncio.sleep(interval)
        return pred()

    def notebook_ready(self, name: str, namespace: str) -> bool:
        nb = self.store.peek(kinds.NOTEBOOK, name, namespace)
        if nb is None:
            return False
        st = nb.get("status") or {}
        if st.get("readyReplicas") != 1:
            return False
        return any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])

    def reconcile_count(self) -> int:
        return sum(mgr.reconcile_count() for mgr in (self.kf, self.odh) if mgr is not None)

    def reconcile_breakdown(self) -> dict:
        out: dict = {}
        for mgr in (self.kf, self.odh):
            if mgr is not None:
                out.update(mgr.reconcile_breakdown())
        return out

    async def __aenter__(self):
        return await self.start()

    async def __aexit__(self, *exc):
        await self.stop()
