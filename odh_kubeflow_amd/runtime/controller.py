"""Controllers, event handlers, predicates and the builder DSL.

Mirrors the controller-runtime surface the reference uses
(``ctrl.NewControllerManagedBy(mgr).For(..).Owns(..).Watches(.., handler.EnqueueRequestsFromMapFunc(..),
builder.WithPredicates(..)).Named(..).Complete(r)``; e.g.
``kf/controllers/notebook_controller.go:778-826``).  One deliberate difference:
``max_concurrent_reconciles`` defaults to 8, not 1 — the reference never calls
``WithOptions`` and therefore runs every reconciler single-threaded,
which serialises notebook start-up.  The work queue still guarantees a given object
is never reconciled by two workers at once.
"""

from __future__ import annotations

import asyncio
import inspect
import logging
import time
from dataclasses import dataclass
from typing import Awaitable, Callable, Dict, Iterable, List, NamedTuple, Optional, Sequence

from ..models import meta as m
from ..models.scheme import SCHEME
from .client import CURRENT_RECONCILE
from . import workqueue as _wq
from .workqueue import ShutDown, WorkQueue

log = logging.getLogger(__name__)


class Request(NamedTuple):
    namespace: str
    name: str

    def __str__(self) -> str:
        return f"{self.namespace}/{self.name}" if self.namespace else self.name


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


Reconcile = Callable[[Request], Awaitable[Optional[Result]]]
Predicate = Callable[[str, dict, Optional[dict]], bool]
MapFunc = Callable[[dict], Iterable[Request]]

DEFAULT_MAX_CONCURRENT_RECONCILES = 8


# ------------------------------------------------------------------ predicates


def pred_funcs(create=None, update=None, delete=None, generic=None, default: bool = True) -> Predicate:
    """``predicate.Funcs``: per event-type filters; unset entries default to ``default``."""

    def p(etype: str, obj: dict, old: Optional[dict]) -> bool:
        if etype == "MODIFIED":
            return default if update is None else update(obj, old)
        fn = create if etype == "ADDED" else delete if etype == "DELETED" else generic
        return default if fn is None else fn(obj)

    return p


def pred_new(fn: Callable[[dict], bool]) -> Predicate:
    """``predicate.NewPredicateFuncs``: apply ``fn`` to the (new) object for every event."""
    return lambda etype, obj, old: fn(obj)


def generation_changed(etype: str, obj: dict, old: Optional[dict]) -> bool:
    if etype != "MODIFIED" or old is None:
        return True
    return (obj.get("metadata") or {}).get("generation") != (old.get("metadata") or {}).get("generation")


def annotations_changed(etype: str, obj: dict, old: Optional[dict]) -> bool:
    if etype != "MODIFIED" or old is None:
        return True
    return m.annotations(obj) != m.annotations(old)


_MISSING = object()


def maps_differ(a: Optional[dict], b: Optional[dict], ignore: frozenset = frozenset()) -> bool:
    """``a != b`` for two string maps (labels, annotations), not counting the keys in ``ignore``."""
    if a == b:
        return False
    a, b = a or {}, b or {}
    if not ignore:
        return a != b
    for k in a.keys() | b.keys():
        if k not in ignore and a.get(k, _MISSING) != b.get(k, _MISSING):
            return True
    return False


def metadata_changed(ignore_annotations: Iterable[str] = ()) -> Predicate:
    """Skip pure status writes: pass spec (generation), labels, annotations, finalizers and
    deletion changes.  ``ignore_annotations``: annotation keys whose changes alone do not
    pass — bookkeeping another controller rewrites that the reconcile never reads (the
    culler's activity heartbeat, :data:`~odh_kubeflow_amd.models.notebook.CULLER_HEARTBEAT_ANNOTATIONS`)."""
    ignore = frozenset(ignore_annotations)

    def p(etype: str, obj: dict, old: Optional[dict]) -> bool:
        if etype != "MODIFIED" or old is None:
            return True
        om, nm = old.get("metadata") or {}, obj.get("metadata") or {}
        return (om.get("generation") != nm.get("generation") or om.get("labels") != nm.get("labels")
                or maps_differ(om.get("annotations"), nm.get("annotations"), ignore)
                or om.get("finalizers") != nm.get("finalizers")
                or om.get("deletionTimestamp") != nm.get("deletionTimestamp"))

    return p


generation_or_metadata_changed = metadata_changed()


def _path(obj: Optional[dict], path):
    """``path``: dotted string, or its parts already split."""
    cur = obj
    for part in (path.split(".") if isinstance(path, str) else path):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(part)
    return cur


def fields_changed(*paths: str) -> Predicate:
    """Pass creates and deletes; pass an update only if one of the dotted ``paths``
    (e.g. ``"status.readyReplicas"``, ``"metadata.labels"``) differs from the old object."""

    split = tuple(tuple(x.split(".")) for x in paths)

    def p(etype: str, obj: dict, old: Optional[dict]) -> bool:
        if etype != "MODIFIED" or old is None:
            return True
        for x in split:
            if _path(obj, x) != _path(old, x):
                return True
        return False

    return p


def controller_owner_alive(reader, owner_kind: str) -> Predicate:
    """For delete events of owned objects: pass only while the controlling owner still
    exists and is not being deleted.  Garbage collection of a deleted Notebook's children
    then queues nothing, while the deletion of a child of a live Notebook (drift) still
    triggers the repair.  Other event types pass."""
    info = SCHEME.resolve(owner_kind)

    def p(etype: str, obj: dict, old: Optional[dict]) -> bool:
        if etype != "DELETED":
            return True
        for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
            if r.get("controller") and r.get("kind") == info.kind:
                owner = reader.get(owner_kind, r.get("name", ""), m.namespace(obj))
                return owner is not None and not m.is_deleting(owner) and m.uid(owner) == r.get("uid")
        return True

    return p


# ------------------------------------------------------------------ handlers


def enqueue_for_object(obj: dict) -> List[Request]:
    return [Request(m.namespace(obj), m.name(obj))]


def enqueue_for_owner(owner_kind: str, owner_group: str, controller_only: bool = True) -> MapFunc:
    def fn(obj: dict) -> List[Request]:
        out = []
        for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
            if controller_only and not r.get("controller"):
                continue
            if r.get("kind") != owner_kind:
                continue
            if r.get("apiVersion", "").rpartition("/")[0] != owner_group:
                continue
            out.append(Request(m.namespace(obj), r.get("name", "")))
        return out

    return fn


@dataclass
class _Watch:
    kind: str
    map_fn: MapFunc
    predicates: Sequence[Predicate]


# ------------------------------------------------------------------ controller


class Controller:
    def __init__(self, name: str, reconcile: Reconcile, max_concurrent: int = DEFAULT_MAX_CONCURRENT_RECONCILES,
                 rate_limiter=None, metrics=None):
        self.name = name
        self.reconcile = reconcile
        self.max_concurrent = max(1, int(max_concurrent))
        self.metrics = metrics
        self.queue = WorkQueue(name, rate_limiter, metrics)
        self.watches: List[_Watch] = []
        self._tasks: List[asyncio.Task] = []
        self._unsubs: List[Callable[[], None]] = []
        self._map_tasks: set = set()
        self.started = False
        self.reconciles = 0
        self.errors = 0
        self.busy_time = 0.0
        self.active = 0
        self.on_reconcile: Optional[Callable[[str, Request, float, Optional[BaseException]], None]] = None
        # which watch caused each reconcile: the kind of the event that first queued the
        # request (later events for a queued request are deduplicated into the same run),
        # or "requeue" for Result.requeue / RequeueAfter / error backoff
        self._trigger: dict = {}
        self.reconciles_by_trigger: Dict[str, int] = {}
        # ``client.own_write`` of the manager's client: skip the watch echo of this
        # controller's own write for the request that made it (False = reconcile on every
        # event, as controller-runtime does; the reference-emulation runs use that)
        self.own_writes: Optional[Callable[[dict, str], Optional[Request]]] = None
        self.echoes_skipped = 0
        # a manager split into namespace-partitioned worker processes (runtime/workers.py):
        # requests for another worker's namespaces are dropped here
        self.request_filter: Optional[Callable[[Request], bool]] = None

    def watch(self, kind: str, map_fn: MapFunc, predicates: Sequence[Predicate] = ()) -> None:
        self.watches.append(_Watch(kind, map_fn, tuple(predicates)))

    def enqueue(self, req: Request, trigger: str = "manual") -> None:
        if self.request_filter is not None and not self.request_filter(req):
            return
        self._trigger.setdefault(req, trigger)
        self.queue.add(req)

    def _handler(self, w: _Watch):
        try:
            trig = SCHEME.resolve(w.kind).kind
        except Exception:
            trig = str(w.kind)

        def on_event(etype: str, obj: dict, old: Optional[dict]) -> None:
            for p in w.predicates:
                if not p(etype, obj, old):
                    return
            own = None
            if etype != "DELETED" and self.own_writes is not None:
                own = self.own_writes(obj, self.name)
            res = w.map_fn(obj)
            if res is not None and not isinstance(res, (list, tuple)) and inspect.isawaitable(res):
                t = asyncio.ensure_future(self._enqueue_async(res, trig))
                self._map_tasks.add(t)
                t.add_done_callback(self._map_tasks.discard)
                return
            for r in res or ():
                if own is not None and r == own:
                    self.echoes_skipped += 1
                    if self.metrics:
                        self.metrics.child(self.metrics.echoes_skipped, self.name).inc()
                    continue
                self.enqueue(r, trig)
            # on updates that move an object away from its previous owner, also map the old one
            if etype == "MODIFIED" and old is not None and w.map_fn is not enqueue_for_object:
                try:
                    olds = w.map_fn(old)
                    if not inspect.isawaitable(olds):
                        for r in olds or ():
                            if own is not None and r == own:
                                continue
                            self.enqueue(r, trig)
                except Exception:  # the new object's mapping was enqueued; report, do not drop the event
                    log.warning("%s: mapping the previous state of a %s failed", self.name, trig, exc_info=True)

        return on_event

    async def _enqueue_async(self, aw, trig: str) -> None:
        try:
            for r in (await aw) or ():
                self.enqueue(r, trig)
        except Exception:
            log.exception("%s: async map function failed", self.name)

    async def start(self, source) -> None:
        """Subscribe all watches on ``source`` (an EventSource) and start the workers."""
        if self.started:
            return
        self.started = True
        for w in self.watches:
            self._unsubs.append(source.subscribe(w.kind, self._handler(w)))
        # WaitForCacheSync: workers start only once every watched kind has listed
        await source.wait_synced([w.kind for w in self.watches])
        if self.metrics:
            self.metrics.max_concurrent.labels(self.name).set(self.max_concurrent)
        for i in range(self.max_concurrent):
            self._tasks.append(asyncio.ensure_future(self._worker()))

    async def stop(self) -> None:
        for u in self._unsubs:
            u()
        self._unsubs.clear()
        self.queue.shutdown()
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self._tasks.clear()

    async def _worker(self) -> None:
        q = self.queue
        while True:
            try:
                req = await q.get()
            except ShutDown:
                return
            self.active += 1
            trig = self._trigger.pop(req, "requeue")
            self.reconciles_by_trigger[trig] = self.reconciles_by_trigger.get(trig, 0) + 1
            if self.metrics:
                self.metrics.child(self.metrics.active_workers, self.name).set(self.active)
                self.metrics.child(self.metrics.reconcile_trigger, self.name, trig).inc()
            t0 = time.perf_counter()
            err: Optional[BaseException] = None
            res: Optional[Result] = None
            tok = CURRENT_RECONCILE.set((self.name, req))
            try:
                res = await self.reconcile(req)
            except asyncio.CancelledError:
                q.done(req)
                raise
            except Exception as e:  # controller-runtime recovers panics into errors
                err = e
            finally:
                CURRENT_RECONCILE.reset(tok)
            dt = time.perf_counter() - t0
            if _wq._STALL_MS and dt * 1e3 >= _wq._STALL_MS:
                _wq.stall_report(f"reconcile {self.name} {req} took {dt * 1e3:.1f} ms ({trig})")
            self.busy_time += dt
            self.reconciles += 1
            self.active -= 1
            try:
                if err is not None:
                    self.errors += 1
                    log.debug("%s: reconcile %s failed: %r", self.name, req, err)
                    q.add_rate_limited(req)
                    outcome = "error"
                elif res is not None and res.requeue_after and res.requeue_after > 0:
                    q.forget(req)
                    q.add_after(req, res.requeue_after)
                    outcome = "requeue_after"
                elif res is not None and res.requeue:
                    q.add_rate_limited(req)
                    outcome = "requeue"
                else:
                    q.forget(req)
                    outcome = "success"
            finally:
                q.done(req)
            if self.metrics:
                self.metrics.child(self.metrics.reconcile_total, self.name, outcome).inc()
                self.metrics.child(self.metrics.reconcile_time, self.name).observe(dt)
                self.metrics.child(self.metrics.active_workers, self.name).set(self.active)
                if err is not None:
                    self.metrics.child(self.metrics.reconcile_errors, self.name).inc()
            if self.on_reconcile is not None:
                self.on_reconcile(self.name, req, dt, err)

    def idle(self, timers_within: Optional[float] = None) -> bool:
        return self.queue.pending(timers_within) == 0 and self.active == 0


class Builder:
    """``ctrl.NewControllerManagedBy(mgr)`` — collects watches, then ``complete()`` registers."""

    def __init__(self, mgr):
        self.mgr = mgr
        self._name: Optional[str] = None
        self._for: Optional[str] = None
        self._for_preds: Sequence[Predicate] = ()
        self._watches: List[_Watch] = []
        self._max = None
        self._rate_limiter = None

    def named(self, name: str) -> "Builder":
        self._name = name
        return self

    def for_(self, kind: str, predicates: Sequence[Predicate] = ()) -> "Builder":
        self._for = kind
        self._for_preds = tuple(predicates)
        return self

    def owns(self, kind: str, predicates: Sequence[Predicate] = ()) -> "Builder":
        if self._for is None:
            raise ValueError("owns() requires for_() first")
        info = SCHEME.resolve(self._for)
        self._watches.append(_Watch(kind, enqueue_for_owner(info.kind, info.group), tuple(predicates)))
        return self

    def watches(self, kind: str, map_fn: MapFunc, predicates: Sequence[Predicate] = ()) -> "Builder":
        self._watches.append(_Watch(kind, map_fn, tuple(predicates)))
        return self

    def with_options(self, max_concurrent_reconciles: Optional[int] = None, rate_limiter=None) -> "Builder":
        if max_concurrent_reconciles is not None:
            self._max = max_concurrent_reconciles
        if rate_limiter is not None:
            self._rate_limiter = rate_limiter
        return self

    def complete(self, reconciler) -> Controller:
        fn = reconciler.reconcile if hasattr(reconciler, "reconcile") else reconciler
        name = self._name or (SCHEME.resolve(self._for).kind.lower() if self._for else "controller")
        maxc = self._max if self._max is not None else self.mgr.default_max_concurrent
        c = Controller(name, fn, maxc, self._rate_limiter, self.mgr.runtime_metrics)
        c.request_filter = getattr(self.mgr, "request_filter", None)
        if getattr(self.mgr, "skip_own_write_echoes", True):
            c.own_writes = getattr(self.mgr.client, "own_write", None)
            if c.own_writes is not None and getattr(self.mgr.client, "requeue", False) is None:
                self.mgr.client.requeue = self.mgr.requeue
        if self._for:
            c.watch(self._for, enqueue_for_object, self._for_preds)
        for w in self._watches:
            c.watch(w.kind, w.map_fn, w.predicates)
        self.mgr.add_controller(c)
        return c
