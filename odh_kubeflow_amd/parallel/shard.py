"""One rank of the benchmark: the shipped control-plane process(es) + this rank's notebook driver.

The reference runs one notebook-controller and one odh-notebook-controller replica for the
whole cluster (``kf/main.go:87-98``, ``odh/main.go:155-192``; one worker each).  Two
deployable topologies are measured, both exactly as the manifests run them:

* ``arch="sharded"`` (``config/overlays/mi355x-sharded``) — every rank r starts its shard
  pod's three processes, ``python -m odh_kubeflow_amd.cmd.control_plane --shard r
  --controllers kf`` (kf reconciler + event re-emitter), ``… --controllers odh`` (odh
  reconciler) and ``… --controllers webhook`` (the odh mutating webhook), each with an informer cache over the
  namespaces labelled ``notebooks.amd.com/shard=r``, the webhook registered by its shard's
  MutatingWebhookConfiguration with a ``namespaceSelector`` on that label (``split=False``:
  one process with all three);
* ``arch="unsharded"`` (``config/overlays/mi355x``, the reference's two-process layout) —
  rank 0 starts ``cmd/kf_manager.py`` and ``cmd/odh_manager.py`` (+ its webhook, one MWC for
  every namespace); the other ranks only drive notebooks into them.

Each rank drives its namespaces (``bench-r``; with ``namespaces``, M of them — labelled by the
shipped :class:`~odh_kubeflow_amd.controllers.sharding.NamespaceShardAssigner` when ``assign``)
through an informer cache of its own.  The node
around them — scheduler + device allocator, StatefulSet controller, kubelet — is ONE
:class:`~odh_kubeflow_amd.parallel.platform.NodePlatform` for all ranks, as on a real node.

``process=False`` builds the same managers inside this process (tests, tools).
"""

from __future__ import annotations

import asyncio
import json
import os
import shutil
import subprocess
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..controllers.setup import SHARD_LABEL
from ..models import kinds
from ..models import meta as m

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DRIVEN_LABEL = "bench.odh-kubeflow-amd/driven"


def notebook_is_ready(nb: Optional[dict]) -> bool:
    """The Notebook's status mirrors a Ready pod (``readyReplicas`` 1 and the Ready condition)."""
    if nb is None:
        return False
    st = nb.get("status") or {}
    if st.get("readyReplicas") != 1:
        return False
    return any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])


def driven(nb: dict) -> dict:
    """Label a Notebook the benchmark driver times (``ShardConfig.driven_only``)."""
    nb.setdefault("metadata", {}).setdefault("labels", {})[DRIVEN_LABEL] = "true"
    return nb


def free_port() -> int:
    from ..utils.procutil import listen_port

    return listen_port()


@dataclass
class ShardConfig:
    apiserver_url: str
    namespace: str
    shard: Optional[str] = "0"  # sharded: this rank's shard id
    arch: str = "sharded"  # "sharded" | "unsharded"
    launch: bool = True  # start the control plane (unsharded: rank 0 only; the others just drive)
    controller_namespace: str = "opendatahub"
    bootstrap: bool = False  # create the cluster-wide namespaces (rank 0)
    odh: bool = True
    webhook: bool = True
    reference_emulation: bool = False
    max_concurrent: int = 8
    env: Dict[str, str] = field(default_factory=dict)
    kube_rbac_proxy_image: str = "quay.io/brancz/kube-rbac-proxy:v0.18.1"
    process: bool = False  # run the control plane as its own process(es), as deployed
    split: bool = True  # sharded, process mode: the shard pod's containers as processes (kf | odh | webhook)
    webhook_process: bool = True  # sharded, split: the webhook in a process of its own (False: odh + webhook)
    culler_process: bool = False  # sharded, split: culler + event re-emitter apart (notebook | culler,events)
    # sharded: flags added to every process that leads something (e.g. --leader-elect and the lease
    # timings; tools/bench_failover.py runs standby replicas next to them)
    leader_elect_args: List[str] = field(default_factory=list)
    cluster_watch: bool = False  # --cluster-wide-watches on every control-plane process
    workers: int = 1  # unsharded: --workers of the kf and odh managers (runtime/workers.py)
    kf_split_workers: bool = False  # unsharded with workers: the kf manager's --split-workers
    webhook_replicas: int = 1  # unsharded with workers: --webhook-replicas of the odh manager
    cache_configmaps: bool = False  # unsharded: --cache-configmaps-secrets=true on the odh manager
    # the user namespaces this rank drives (default: just ``namespace``); with ``assign`` they
    # are created unlabelled and the shipped NamespaceShardAssigner (``--assign-namespaces``,
    # run by every shard's kf process) labels each ``crc32(name) % shard_count``
    namespaces: List[str] = field(default_factory=list)
    assign: bool = False
    shard_count: int = 1
    assign_policy: str = "hash"  # NamespaceShardAssigner policy: hash | balanced
    # the driver's own cache selects only the notebooks (and their pods) it labelled DRIVEN_LABEL:
    # a resident population's culler heartbeats never reach the process that times new ones
    driven_only: bool = False

    @property
    def user_namespaces(self) -> List[str]:
        return list(self.namespaces) or [self.namespace]


class _Proc:
    """One launched control-plane process and its debug endpoint."""

    def __init__(self, name: str, proc: subprocess.Popen, metrics_port: int):
        self.name = name
        self.proc = proc
        self.base = f"http://127.0.0.1:{metrics_port}"


class ControlPlaneShard:
    def __init__(self, cfg: ShardConfig):
        self.cfg = cfg
        self.shard = cfg.shard if cfg.arch == "sharded" else None
        self.env = {**os.environ, **cfg.env}
        self.procs: List[_Proc] = []  # process mode
        self.managers = []  # in-process mode
        self.control_plane = None  # in-process sharded: the control_plane Manager
        self._caches = []
        self._waiters = None
        self._certs = None
        self._http = None
        self.worker_pids: Dict[str, int] = {}  # --workers: the managers' worker processes
        self.labels: Dict[str, str] = {}  # assign: namespace → the shard label it was given

    # ------------------------------------------------------------------ build

    def _common_flags(self) -> List[str]:
        return ["--master", self.cfg.apiserver_url, "--max-concurrent-reconciles", str(self.cfg.max_concurrent),
                "--enable-debug-endpoints", *(["--cluster-wide-watches"] if self.cfg.cluster_watch else [])]

    def _specs(self, webhook_port: int, split: Optional[bool] = None):
        """(name, module, argv, metrics flag) of the processes this rank launches."""
        cfg = self.cfg
        wh = ["--kube-rbac-proxy-image", cfg.kube_rbac_proxy_image, "--webhook-cert-dir", self._certs.cert_dir,
              "--webhook-host", "127.0.0.1", "--webhook-port", str(webhook_port)]
        if cfg.arch == "sharded":
            # the shard pod of config/overlays/mi355x-sharded: the control plane split into a
            # kf process, an odh process and a webhook process (cmd/control_plane.py docstring)
            sets = [["notebook"], ["culler", "events"]] \
                if cfg.culler_process and (cfg.split if split is None else split) else [["kf"]]
            if cfg.odh:
                if cfg.webhook and cfg.webhook_process:
                    sets += [["odh"], ["webhook"]]
                else:
                    sets.append(["odh"] + (["webhook"] if cfg.webhook else []))
            if not (cfg.split if split is None else split):
                sets = [[c for cs in sets for c in cs]]
            names = {"notebook": "kf"}  # the kf process keeps its name without the culler
            out = []
            for cs in sets:
                a = ["--shard", self.shard, "--controllers", ",".join(cs), "--health-probe-bind-address", "0"]
                if "odh" in cs or "webhook" in cs:
                    a += wh
                if cfg.assign and ("kf" in cs or "notebook" in cs):
                    a += ["--assign-namespaces", "--shard-count", str(cfg.shard_count),
                          "--assign-policy", cfg.assign_policy]
                if cfg.reference_emulation:
                    a.append("--reference-emulation")
                if cs != ["webhook"]:
                    a += cfg.leader_elect_args
                name = "control_plane" if len(sets) == 1 else f"control_plane_{names.get(cs[0], cs[0])}"
                out.append((name, "odh_kubeflow_amd.cmd.control_plane", a, "--metrics-bind-address"))
            return out
        wk = ["--workers", str(cfg.workers)] if cfg.workers > 1 else []
        kf_split = ["--split-workers"] if cfg.workers > 1 and cfg.kf_split_workers else []
        out = [("kf_manager", "odh_kubeflow_amd.cmd.kf_manager", ["--probe-addr", "0", *wk, *kf_split],
                "--metrics-addr")]
        if cfg.odh:
            rep = ["--webhook-replicas", str(cfg.webhook_replicas)] if cfg.workers > 1 and cfg.webhook_replicas > 1 \
                else []
            if cfg.cache_configmaps:
                rep.append("--cache-configmaps-secrets=true")
            out.append(("odh_manager", "odh_kubeflow_amd.cmd.odh_manager",
                        [*wh, "--health-probe-bind-address", "0", *wk, *rep], "--metrics-bind-address"))
        return out

    def _cp_env(self) -> Dict[str, str]:
        return {**self.env, "K8S_NAMESPACE": self.cfg.controller_namespace}

    async def start(self) -> "ControlPlaneShard":
        from ..runtime.informer import InformerCache
        from ..runtime.rest import RestClient, RestConfig
        from ..webhook.certs import generate

        cfg = self.cfg
        self.rest = RestClient(RestConfig(host=cfg.apiserver_url))
        self.admin = self.rest
        if cfg.bootstrap:
            for ns in ("default", cfg.controller_namespace):
                await self.ensure_namespace(ns)
        own = {SHARD_LABEL: self.shard} if self.shard is not None and not cfg.assign else None
        for ns in cfg.user_namespaces:
            await self.ensure_namespace(ns, own)
        if cfg.launch:
            self._certs = generate(("127.0.0.1", "localhost"))
            wport = free_port()
            if cfg.process:
                await self._launch_processes(wport)
            else:
                wport = await self._build_in_process()
            if cfg.webhook and cfg.odh:
                await self._register_webhook(wport)
        # this rank's notebook driver: its namespaces' Notebooks and Pods (driven_only: those it
        # labelled; the STS generator copies a Notebook's labels to its pod)
        sel = {kinds.NOTEBOOK: f"{DRIVEN_LABEL}=true", kinds.POD: f"{DRIVEN_LABEL}=true"} if cfg.driven_only else None
        self.cache = InformerCache(self.rest, namespaces=cfg.user_namespaces, selectors=sel)
        self._caches.append(self.cache)
        for k in (kinds.NOTEBOOK, kinds.POD):
            await self.cache.ensure_informer(k)
        await self.cache.wait_synced([kinds.NOTEBOOK, kinds.POD])
        return self

    async def _launch_processes(self, webhook_port: int) -> None:
        from .platform import start_child

        env = {**self._cp_env(), "PYTHONPATH": ROOT + os.pathsep + self.env.get("PYTHONPATH", "")}
        prof = self.env.get("ODH_CONTROL_PLANE_PROFILE")  # cProfile output path (profiling runs)
        for name, module, argv, metrics_flag in self._specs(webhook_port):
            mport = free_port()
            args = [*self._common_flags(), metrics_flag, f"127.0.0.1:{mport}", *argv]
            pre = ["-m", "cProfile", "-o", f"{prof}.{name}.{self.shard or 'all'}"] if prof else []
            proc = await start_child(module, args, f"{name} (shard {self.shard})", env=env, python_args=pre)
            self.procs.append(_Proc(name, proc, mport))
        if self.cfg.workers > 1:  # the managers' worker (and webhook replica) processes
            for p in self.procs:
                d = await self._get_json(f"{p.base}/debug/reconciles")
                for k, pid in (d.get("worker_pids") or {}).items():
                    self.worker_pids[f"{p.name}_{k}"] = pid

    async def _build_in_process(self) -> int:
        cfg = self.cfg
        wport = 0
        if cfg.arch == "sharded":
            from ..cmd import control_plane

            (_name, _mod, argv, mflag), = self._specs(0, split=False)  # one manager: tests read its cache
            args = control_plane.parse([*self._common_flags(), mflag, "0", *argv])
            mgrs = [control_plane.build(args, self._cp_env())]
            self.control_plane = mgrs[0]
        else:
            from ..cmd import kf_manager, odh_manager

            specs = {n: (a, f) for n, _mod, a, f in self._specs(0)}
            a, f = specs["kf_manager"]
            mgrs = [kf_manager.build(kf_manager.parse([*self._common_flags(), f, "0", *a]), self._cp_env())]
            if "odh_manager" in specs:
                a, f = specs["odh_manager"]
                mgrs.append(odh_manager.build(odh_manager.parse([*self._common_flags(), f, "0", *a]),
                                              self._cp_env()))
        for mgr in mgrs:
            await mgr.start()
            await mgr.elected.wait()
            srv = getattr(mgr, "webhook_server", None)
            if srv is not None:
                wport = srv.port
        self.managers = mgrs
        return wport

    async def _register_webhook(self, port: int) -> None:
        """The MutatingWebhookConfiguration the overlay ships (with a URL instead of the
        Service, since the apiserver here runs on the host): per shard with a
        ``namespaceSelector`` on the shard label, or one for every namespace (unsharded)."""
        from ..models.errors import ApiError, is_already_exists
        from ..webhook.server import mutating_webhook_configuration

        kw = {}
        name = "odh-notebook-controller-mutating-webhook-configuration"
        if self.shard is not None:
            name = f"odh-notebook-webhook-shard-{self.shard}"
            kw["namespace_selector"] = {"matchLabels": {SHARD_LABEL: self.shard}}
        mwc = mutating_webhook_configuration(self._certs.ca_bundle_b64,
                                             url=f"https://127.0.0.1:{port}/mutate-notebook-v1", name=name, **kw)
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

    async def wait_assigned(self, timeout: float = 60.0) -> Dict[str, str]:
        """namespace → shard label of this rank's namespaces, once every one carries it
        (``assign``: labelled by the shards' assigners, which come up with their shards)."""
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        out: Dict[str, str] = {}
        while True:
            for ns in self.cfg.user_namespaces:
                if ns not in out:
                    lab = m.labels(await self.rest.get(kinds.NAMESPACE, ns)).get(SHARD_LABEL)
                    if lab is not None:
                        out[ns] = lab
            if len(out) == len(self.cfg.user_namespaces) or loop.time() > deadline:
                return out
            await asyncio.sleep(0.05)

    def notebook_ready(self, name: str, namespace: Optional[str] = None) -> bool:
        return notebook_is_ready(self.cache.get(kinds.NOTEBOOK, name, namespace or self.cfg.namespace))

    def gone(self, name: str, namespace: Optional[str] = None) -> bool:
        ns = namespace or self.cfg.namespace
        return self.cache.get(kinds.NOTEBOOK, name, ns) is None and self.cache.get(kinds.POD, f"{name}-0", ns) is None

    # -------------------------------------------------------------- control-plane counters

    async def _get_json(self, url: str) -> dict:
        import aiohttp

        if self._http is None:
            self._http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=60))
        async with self._http.get(url) as r:
            return json.loads(await r.text())

    async def reconcile_breakdown(self, include_all: bool = False) -> dict:
        """controller → {trigger → reconciles} of the notebook controllers this rank launched
        (the culler and the namespace assigner are not part of a notebook's create→Ready path;
        ``include_all``: them too)."""
        skip = () if include_all else ("Culler", "shard-assigner")
        parts = [mgr.reconcile_breakdown() for mgr in self.managers]
        if self.procs:
            parts += [d["reconciles"] for d in await asyncio.gather(
                *(self._get_json(f"{p.base}/debug/reconciles") for p in self.procs))]
        out: dict = {}
        for part in parts:
            for ctrl, trig in part.items():
                if ctrl in skip:
                    continue
                o = out.setdefault(ctrl, {})
                for k, v in trig.items():
                    o[k] = o.get(k, 0) + v
        return out

    async def io_counters(self) -> Dict[str, dict]:
        """process name → {"watch_events": {kind: n}, "requests": {verb: n}} of the control-plane
        processes this rank launched (in-process managers under "inprocess_<i>")."""
        out = {f"inprocess_{i}": mgr.io_counters() for i, mgr in enumerate(self.managers)}
        if self.procs:
            sfx = f"_{self.shard}" if self.shard is not None else ""
            docs = await asyncio.gather(*(self._get_json(f"{p.base}/debug/reconciles") for p in self.procs))
            for p, d in zip(self.procs, docs):
                out[f"{p.name}{sfx}"] = d.get("io") or {}
        return out

    async def webhook_timings(self, since: Optional[Dict[str, dict]] = None) -> Dict[str, dict]:
        """process name → {"served": n, "handle_ms": [...], "gets": n, "get_ms": [...]} of the
        launched processes that serve the odh webhook: handle times of the admissions, and the
        process's live GETs, after ``since[name]`` (a previous answer's counters)."""
        out = {}
        for p in self.procs:
            s0 = (since or {}).get(p.name) or {}
            q = f"since={s0.get('served', 0)}" + (f"&get_since={s0['gets']}" if "gets" in s0 else "")
            reps = sorted(((int(k.rsplit("_", 1)[1]), v) for k, v in (since or {}).items()
                           if k.startswith(f"{p.name}_webhook_replica_")))
            if reps:
                q += "&replica_since=" + ",".join(f"{v.get('served', 0)}:{v.get('gets', 0)}" for _i, v in reps)
            d = await self._get_json(f"{p.base}/debug/webhook?{q}")
            for i, rd in (d.pop("replicas", None) or {}).items():  # --webhook-replicas children
                name = f"{p.name}_webhook_replica_{i}"
                if rd.get("served") or name in (since or {}):
                    out[name] = rd
            if d.get("served") or p.name in (since or {}):
                out[p.name] = d
        for i, mgr in enumerate(self.managers):
            srv = getattr(mgr, "webhook_server", None)
            if srv is not None:
                n = max(0, min(srv.served - ((since or {}).get(f"inprocess_{i}") or {}).get("served", 0),
                               len(srv.handle_s)))
                out[f"inprocess_{i}"] = {"served": srv.served,
                                         "handle_ms": [x * 1e3 for x in list(srv.handle_s)[len(srv.handle_s) - n:]]}
        return out

    async def worker_assignments(self) -> Dict[str, Dict[str, List[str]]]:
        """process name → {worker index → namespaces} of the launched managers that run
        ``--workers`` (the supervisor's namespace assignment)."""
        out = {}
        for p in self.procs:
            a = (await self._get_json(f"{p.base}/debug/reconciles")).get("assignments")
            if a:
                out[p.name] = a
        return out

    async def gc_pauses(self, since: Optional[Dict[str, int]] = None) -> Dict[str, dict]:
        """process name → {"seq": n, "pauses": [[seq, generation, ms], ...]} of the launched
        control-plane processes (a manager's workers as ``<name>_worker_<i>``), the
        collections after ``since[name]`` (a previous answer's seq)."""
        out = {}
        sfx = f"_{self.shard}" if self.shard is not None else ""
        for p in self.procs:
            d = await self._get_json(f"{p.base}/debug/gc")
            for k, v in d.items():
                name = f"{p.name}{sfx}" if k == "self" else f"{p.name}_{k}"
                s0 = (since or {}).get(name, 0)
                out[name] = {"seq": v.get("seq", 0), "pauses": [x for x in v.get("pauses") or [] if x[0] > s0]}
        return out

    async def reconcile_count(self) -> int:
        return sum(sum(t.values()) for t in (await self.reconcile_breakdown()).values())

    def control_plane_pids(self) -> Dict[str, int]:
        sfx = f"_{self.shard}" if self.shard is not None else ""
        out = {f"{p.name}{sfx}": p.proc.pid for p in self.procs}
        out.update(self.worker_pids)
        return out

    # ------------------------------------------------------------------ waiting

    async def quiesce(self, quiet: float = 0.002, timeout: float = 10.0, timers: Optional[float] = None) -> bool:
        """Every control-plane process this rank launched idle: queues empty, no reconcile
        running, no watch event for ``quiet`` s (event-driven inside each process,
        :meth:`Manager.quiesce`; one request each, answered when they are quiet).  ``timers``:
        delayed requeues due later than that many seconds are not waited for."""
        res = [await mgr.quiesce(quiet, timeout, timers) for mgr in self.managers]
        if self.procs:
            q = f"/debug/quiesce?quiet_ms={quiet * 1e3:g}&timeout_s={timeout:g}"
            if timers is not None:
                q += f"&timers_ms={timers * 1e3:g}"
            res += [d["idle"] for d in await asyncio.gather(*(self._get_json(p.base + q) for p in self.procs))]
        return all(res)

    async def settle(self, timeout: float = 10.0) -> bool:
        return await self.quiesce(0.002, timeout)

    async def wait_until(self, pred: Callable[[], bool], timeout: float = 10.0) -> bool:
        """Event-driven wait: ``pred`` is re-checked on every Notebook / Pod event of the
        rank's namespaces (after the cache applied it) instead of on a polling timer."""
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
                self.cache.subscribe(k, on_event)  # the cache holds only this rank's namespaces
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
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        while loop.time() < deadline:
            if pred():
                return True
            await asyncio.sleep(interval)
        return pred()

    async def stop(self) -> None:
        from .platform import stop_child

        for mgr in reversed(self.managers):
            await mgr.stop()
        for p in self.procs:
            await stop_child(p.proc)
        for c in self._caches:
            await c.stop()
        if self._http is not None:
            await self._http.close()
        await self.rest.close()
        if self._certs is not None:
            shutil.rmtree(self._certs.cert_dir, ignore_errors=True)
