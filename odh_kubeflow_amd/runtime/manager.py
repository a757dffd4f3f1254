"""Controller manager (``ctrl.Manager`` analogue).

Owns the client/cache/event-source triple, the controllers and other runnables, the
Prometheus registry, the ``/metrics`` and ``/healthz``/``/readyz`` servers
(``kf/main.go:125-133``, ``odh/main.go:231-238``) and optional leader election
(``LeaderElectionID`` ``kubeflow-notebook-controller`` / ``odh-notebook-controller``).
Controllers only start once leadership is held; runnables that do not need
leadership (the webhook server) start immediately, as in controller-runtime.  Losing
leadership is fatal, as in controller-runtime (``leaderelection.LeaderCallbacks.OnStoppedLeading``
→ ``os.Exit(1)``): the controllers stop, ``/healthz`` fails and :meth:`run_until` returns
exit code 1 so the process ends and the kubelet restarts it as a new candidate.
"""

from __future__ import annotations

import asyncio
import logging
import time
from typing import Callable, Dict, List, Optional, Sequence

from prometheus_client import CollectorRegistry, generate_latest

from .client import CachedClient, Client, EventSource, Reader
from .controller import DEFAULT_MAX_CONCURRENT_RECONCILES, Builder, Controller
from .events import EventRecorder
from .metrics import RuntimeMetrics

log = logging.getLogger(__name__)


class Manager:
    def __init__(self, client: Client, reader: Reader, source: EventSource, name: str = "manager",
                 registry: Optional[CollectorRegistry] = None,
                 default_max_concurrent: int = DEFAULT_MAX_CONCURRENT_RECONCILES,
                 leader_elector=None, metrics_addr: Optional[str] = None, probe_addr: Optional[str] = None,
                 debug_endpoints: bool = False, warm_standby: bool = True):
        self.name = name
        # with leader election: a standby replica lists and watches what its controllers will
        # watch before it leads, so a takeover starts reconciling from a synced cache instead of
        # relisting every Notebook and child first (controller-runtime starts the controllers'
        # informers only once elected)
        self.warm_standby = warm_standby
        self.synced_at: Optional[float] = None  # monotonic: the controllers' kinds were synced
        self.elected_at: Optional[float] = None  # monotonic: this replica took the lead
        self.client = client
        self.reader = reader
        self.source = source
        self.registry = registry or CollectorRegistry()
        self.runtime_metrics = RuntimeMetrics(self.registry)
        from ..utils.gctune import PAUSES

        try:
            self.registry.register(PAUSES)
        except ValueError:  # a registry shared by several managers of one process has it already
            pass
        self.default_max_concurrent = default_max_concurrent
        self.controllers: List[Controller] = []
        self.runnables: List = []
        self.leader_runnables: List = []
        self.healthz: Dict[str, Callable[[], bool]] = {}
        self.readyz: Dict[str, Callable[[], bool]] = {}
        self.leader_elector = leader_elector
        self.metrics_addr = metrics_addr
        self.probe_addr = probe_addr
        self.debug_endpoints = debug_endpoints
        self._recorders: Dict[str, EventRecorder] = {}
        self._servers: List = []
        self._started = False
        self._leader_task: Optional[asyncio.Task] = None
        self.elected = None  # asyncio.Event, created inside the loop by start()
        self.fatal: Optional[str] = None  # set when the manager must exit (leadership lost)
        self._fatal_event: Optional[asyncio.Event] = None
        self._started_event: Optional[asyncio.Event] = None
        self.healthz["leader-election"] = lambda: self.fatal is None
        # ``--workers W`` (runtime/workers.py): the worker processes this manager supervises
        # (their /metrics and /debug answers are merged into this manager's), and, in a
        # worker, the filter that keeps its controllers to its namespace partition
        self.supervisor = None
        self.webhook_replicas = None  # WorkerSupervisor of webhook-only children (odh --webhook-replicas)
        self.request_filter = None

    # ------------------------------------------------------------------ construction

    @classmethod
    def remote(cls, config, name: str = "manager", uncached: Sequence = (), transforms=None,
               namespace: Optional[str] = None, shared=None, cache_options: Optional[dict] = None,
               **kw) -> "Manager":
        """Manager against a real (or out-of-process) apiserver: REST client + informer cache.

        ``shared=(rest, cache)`` makes several managers of one process share a single
        connection pool and informer cache (one watch per kind per process, as the
        controllers of kube-controller-manager do); the owner of ``shared`` closes it.
        """
        from .informer import InformerCache
        from .rest import RestClient

        if shared is not None:
            rest, cache = shared
            mgr = cls(CachedClient(cache, rest, uncached), cache, cache, name=name, **kw)
            return mgr
        rest = RestClient(config)
        cache = InformerCache(rest, namespace=namespace, transforms=transforms, **(cache_options or {}))
        client = CachedClient(cache, rest, uncached)
        mgr = cls(client, cache, cache, name=name, **kw)
        mgr.rest = rest
        mgr.cache = cache
        return mgr

    def builder(self) -> Builder:
        return Builder(self)

    def add_controller(self, c: Controller) -> None:
        self.controllers.append(c)

    def requeue(self, controller: str, req) -> None:
        """Queue ``req`` again in the controller named ``controller`` (an event that the
        client had provisionally taken for that controller's own write, but was not)."""
        for c in self.controllers:
            if c.name == controller:
                c.enqueue(req, "misclaim")

    def add(self, runnable, needs_leader: bool = True) -> None:
        (self.leader_runnables if needs_leader else self.runnables).append(runnable)

    def add_healthz_check(self, name: str, fn: Callable[[], bool] = lambda: True) -> None:
        self.healthz[name] = fn

    def add_readyz_check(self, name: str, fn: Callable[[], bool] = lambda: True) -> None:
        self.readyz[name] = fn

    def get_event_recorder_for(self, component: str) -> EventRecorder:
        r = self._recorders.get(component)
        if r is None:
            r = self._recorders[component] = EventRecorder(self.client, component)
        return r

    # ------------------------------------------------------------------ lifecycle

    def started_event(self) -> asyncio.Event:
        """Set once :meth:`start` has started the servers and leader-independent runnables
        (then :attr:`elected` is set once this replica leads and its controllers run)."""
        if self._started_event is None:
            self._started_event = asyncio.Event()
        return self._started_event

    async def start(self) -> None:
        if self._started:
            return
        self._started = True
        self.elected = asyncio.Event()
        self._fatal_event = asyncio.Event()
        await self._start_servers()
        for r in self.runnables:
            await r.start()
        self.started_event().set()
        if self.leader_elector is None:
            await self._become_leader()
        else:
            if self.warm_standby and self.controllers:
                kinds_ = list(dict.fromkeys(w.kind for c in self.controllers for w in c.watches))
                try:
                    await self.source.wait_synced(kinds_)
                    self.synced_at = time.monotonic()
                except Exception:  # noqa: BLE001 — the controllers sync them again when elected
                    log.warning("%s: warming the standby cache failed", self.name, exc_info=True)
            self._leader_task = asyncio.ensure_future(self.leader_elector.run(self._become_leader, self._lost_leader))

    async def _become_leader(self) -> None:
        self.elected_at = time.monotonic()
        for c in self.controllers:
            await c.start(self.source)
        if self.synced_at is None:
            self.synced_at = time.monotonic()
        for r in self.leader_runnables:
            await r.start()
        self.elected.set()

    async def _lost_leader(self) -> None:
        log.error("%s: leader election lost; stopping controllers and exiting", self.name)
        self.fatal = "leader election lost"
        for c in self.controllers:
            await c.stop()
        if self._fatal_event is not None:
            self._fatal_event.set()

    async def stop(self) -> None:
        if self._leader_task is not None:
            self._leader_task.cancel()
            try:
                await self._leader_task
            except (asyncio.CancelledError, Exception):
                pass
            if self.leader_elector is not None:
                await self.leader_elector.release()
        for c in self.controllers:
            await c.stop()
        for r in self.leader_runnables + self.runnables:
            try:
                await r.stop()
            except Exception:
                log.exception("runnable stop failed")
        for rec in self._recorders.values():
            await rec.flush()
        for s in self._servers:
            await s.cleanup()
        self._servers.clear()
        cache = getattr(self, "cache", None)
        if cache is not None:
            await cache.stop()
        rest = getattr(self, "rest", None)
        if rest is not None:
            await rest.close()
        self._started = False

    async def run_until(self, stop: asyncio.Event) -> int:
        """Run until ``stop`` is set (exit code 0) or the manager hits a fatal condition such
        as losing leadership (exit code 1)."""
        await self.start()
        from ..utils import gctune

        gctune.tune()  # long-running process: keep gen-2 pauses off the reconcile path
        waits = [asyncio.ensure_future(stop.wait()), asyncio.ensure_future(self._fatal_event.wait())]
        try:
            await asyncio.wait(waits, return_when=asyncio.FIRST_COMPLETED)
        finally:
            for w in waits:
                w.cancel()
            await self.stop()
        if self.fatal:
            log.error("%s: exiting: %s", self.name, self.fatal)
            return 1
        return 0

    # ------------------------------------------------------------------ test / bench helpers

    def idle(self, timers_within: Optional[float] = None) -> bool:
        return all(c.idle(timers_within) for c in self.controllers)

    async def wait_idle(self, timeout: float = 10.0, settle: float = 0.0) -> bool:
        """Wait until every controller queue is drained (ignores delayed requeues beyond ``timeout``)."""
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            busy = any(len(c.queue) or c.queue._processing or c.active for c in self.controllers)
            if not busy:
                for rec in self._recorders.values():
                    await rec.flush()
                if settle:
                    await asyncio.sleep(settle)
                    if not any(len(c.queue) or c.active for c in self.controllers):
                        return True
                    continue
                return True
            await asyncio.sleep(0.002)
        return False

    async def quiesce(self, quiet: float = 0.002, timeout: float = 10.0,
                      timers_within: Optional[float] = None) -> bool:
        """Event-driven idle: return once no controller has queued or running work and no
        watch event has reached this manager's cache for ``quiet`` seconds (the trailing
        reconciles of a deletion — GC'd children, the pod going away — arrive as watch events
        after the object itself is gone).  No fixed polling period and no minimum number of
        checks: it returns ``quiet`` after the last event, or at once if that is long past.
        ``timers_within``: delayed requeues due later than that many seconds do not count as
        work (the culler's next check of every notebook is a period away)."""
        src = getattr(self, "cache", None) or self.reader
        deadline = time.monotonic() + timeout
        while True:
            now = time.monotonic()
            since = now - getattr(src, "last_event", 0.0)
            if self.idle(timers_within) and since >= quiet:
                for rec in self._recorders.values():
                    await rec.flush()
                if self.idle(timers_within):
                    return True
                continue
            if now >= deadline:
                return False
            await asyncio.sleep(max(0.0002, quiet - since) if self.idle(timers_within) else 0.0002)

    def fail(self, reason: str) -> None:
        """End :meth:`run_until` with exit code 1 (the process must restart)."""
        log.error("%s: %s", self.name, reason)
        self.fatal = reason
        if self._fatal_event is not None:
            self._fatal_event.set()

    def set_supervisor(self, sup) -> None:
        """Run ``sup`` (a :class:`~odh_kubeflow_amd.runtime.workers.WorkerSupervisor`) while
        this manager leads; its workers' health, metrics and debug answers join this one's."""
        self.supervisor = sup
        self.add(sup, needs_leader=True)
        self.healthz["workers"] = lambda: not self.elected or not self.elected.is_set() or sup.alive()

    def add_webhook_replicas(self, sup) -> None:
        """Run ``sup``'s webhook-only children on every replica (webhooks serve whether or not
        this one leads); their health, metrics and debug answers join this one's."""
        self.webhook_replicas = sup
        self.add(sup, needs_leader=False)
        self.healthz["webhook-replicas"] = sup.alive

    def _children(self) -> list:
        return [s for s in (self.supervisor, self.webhook_replicas) if s is not None]

    def io_counters(self) -> Dict[str, Dict[str, int]]:
        """What this process received and sent: watch events per kind, REST requests per verb,
        and lists per kind (relists after a 410 Gone among them)."""
        cache = getattr(self, "cache", None) or self.reader
        rest = getattr(self, "rest", None)
        ev = cache.event_counts() if hasattr(cache, "event_counts") else {}
        lists = cache.relist_counts() if hasattr(cache, "relist_counts") else {}
        return {"watch_events": ev, "requests": dict(getattr(rest, "by_verb", {}) or {}), "lists": lists,
                "bytes_in": dict(getattr(rest, "bytes_in", {}) or {}),
                "cache_scans": dict(getattr(cache, "list_scans", {}) or {})}

    def reconcile_count(self) -> int:
        return sum(c.reconciles for c in self.controllers)

    def reconcile_breakdown(self) -> Dict[str, Dict[str, int]]:
        """controller name → {triggering watch kind (or "requeue") → reconciles}."""
        return {c.name: dict(c.reconciles_by_trigger) for c in self.controllers}

    # ------------------------------------------------------------------ servers

    async def _start_servers(self) -> None:
        from aiohttp import web

        async def serve(addr: str, app: web.Application) -> None:
            host, _, port = addr.rpartition(":")
            runner = web.AppRunner(app, access_log=None)
            await runner.setup()
            site = web.TCPSite(runner, host or "0.0.0.0", int(port))
            await site.start()
            self._servers.append(runner)

        if self.metrics_addr and self.metrics_addr not in ("0", ""):
            app = web.Application()

            async def metrics(_req):
                body = generate_latest(self.registry)
                if self._children():
                    from .workers import merge_metrics

                    texts = [t for sup in self._children() for t in await sup.metrics_texts()]
                    body = merge_metrics([body.decode(), *texts]).encode()
                return web.Response(body=body, content_type="text/plain", charset="utf-8")

            app.router.add_get("/metrics", metrics)
            if self.debug_endpoints:
                self._add_debug_routes(app)
            await serve(self.metrics_addr, app)
        if self.probe_addr and self.probe_addr not in ("0", ""):
            app = web.Application()

            def checker(checks):
                async def h(_req):
                    bad = [n for n, fn in checks.items() if not fn()]
                    if bad:
                        return web.Response(status=500, text="\n".join(f"[-]{n} failed" for n in bad))
                    return web.Response(text="ok")

                return h

            app.router.add_get("/healthz", checker(self.healthz))
            app.router.add_get("/readyz", checker(self.readyz))
            await serve(self.probe_addr, app)

    def _add_debug_routes(self, app) -> None:
        """``--enable-debug-endpoints`` (off in the shipped manifests; benchmarks and e2e use it):
        ``GET /debug/reconciles`` → reconciles per controller and trigger (JSON, cheaper than
        parsing ``/metrics``); ``GET /debug/quiesce?quiet_ms=2&timeout_s=10`` → waits for
        :meth:`quiesce`, then answers ``{"idle": …, "reconciles": …}``."""
        from aiohttp import web

        from .workers import merge_counts

        async def reconciles(_req):
            docs = await self.supervisor.debug("/debug/reconciles") if self.supervisor is not None else []
            reps = self.webhook_replicas
            rdocs = await reps.debug("/debug/reconciles") if reps is not None else []
            pids = dict(self.supervisor.pids()) if self.supervisor is not None else {}
            if reps is not None:
                pids.update({f"webhook_replica_{k.rsplit('_', 1)[1]}": v for k, v in reps.pids().items()})
            return web.json_response({"reconciles": merge_counts([self.reconcile_breakdown(),
                                                                  *(d.get("reconciles") for d in docs)]),
                                      "io": merge_counts([self.io_counters(), *(d.get("io") for d in docs + rdocs)]),
                                      "workers": len(docs),
                                      "worker_pids": pids,
                                      "leader": bool(self.elected is not None and self.elected.is_set()),
                                      "pending": sum(c.queue.pending() + c.active for c in self.controllers),
                                      "assignments": {str(i): nss for i, nss in self.supervisor.assignments().items()}
                                      if self.supervisor is not None else {}})

        async def quiesce(req):
            quiet = float(req.query.get("quiet_ms", "2")) / 1e3
            timeout = float(req.query.get("timeout_s", "10"))
            timers = float(req.query["timers_ms"]) / 1e3 if "timers_ms" in req.query else None
            sub = []
            if self.supervisor is not None:
                sub = [asyncio.ensure_future(self.supervisor.debug(req.path_qs, timeout + 5))]
            idle = await self.quiesce(quiet, timeout, timers)
            docs = (await sub[0]) if sub else []
            idle = idle and all(d.get("idle") for d in docs) and (
                self.supervisor is None or len(docs) == len(self.supervisor.workers))
            return web.json_response({"idle": idle,
                                      "reconciles": merge_counts([self.reconcile_breakdown(),
                                                                  *(d.get("reconciles") for d in docs)]),
                                      "io": merge_counts([self.io_counters(), *(d.get("io") for d in docs)])})

        async def webhook(req):
            srv = getattr(self, "webhook_server", None)
            if srv is None:
                return web.json_response({"served": 0, "handle_ms": []})
            since = int(req.query.get("since", "0"))
            n = max(0, min(srv.served - since, len(srv.handle_s)))
            recent = list(srv.handle_s)[len(srv.handle_s) - n:] if n else []
            rest = getattr(self, "rest", None)
            gets = getattr(rest, "by_verb", {}).get("GET", 0)
            gsince = int(req.query.get("get_since", str(gets)))
            g = list(getattr(rest, "get_ms", ()))
            k = max(0, min(gets - gsince, len(g)))
            out = {"served": srv.served, "handle_ms": [round(x * 1e3, 3) for x in recent],
                   "gets": gets, "get_ms": [round(x, 3) for x in g[len(g) - k:]] if k else [],
                   "heartbeats": getattr(srv.webhook, "heartbeats", 0),
                   "heartbeats_full": getattr(srv.webhook, "heartbeats_full", 0)}
            reps = self.webhook_replicas
            if reps is not None:  # each replica's own window: replica_since=served:gets,served:gets,...
                rs = [x.split(":") for x in req.query.get("replica_since", "").split(",") if x]

                def path(i):
                    s0, g0 = (rs[i] + ["0", "0"])[:2] if i < len(rs) else ("0", "0")
                    return f"/debug/webhook?since={int(s0)}&get_since={int(g0)}"
                out["replicas"] = {str(i): d for i, d in (await reps.debug_each(path)).items()}
            return web.json_response(out)

        async def gc_pauses(req):
            from ..utils.gctune import PAUSES

            since = int(req.query.get("since", "0"))
            out = {"self": PAUSES.since(since)}
            if self.supervisor is not None:  # the workers' own (each numbers its collections itself)
                for i, d in (await self.supervisor.debug_by_worker("/debug/gc")).items():
                    out[f"worker_{i}"] = d.get("self") or {}
            if self.webhook_replicas is not None:
                for i, d in (await self.webhook_replicas.debug_by_worker("/debug/gc")).items():
                    out[f"webhook_replica_{i}"] = d.get("self") or {}
            return web.json_response(out)

        app.router.add_get("/debug/webhook", webhook)
        app.router.add_get("/debug/gc", gc_pauses)
        app.router.add_get("/debug/reconciles", reconciles)
        app.router.add_get("/debug/quiesce", quiesce)
