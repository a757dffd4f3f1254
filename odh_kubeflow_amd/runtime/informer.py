"""Shared informer cache over a :class:`~odh_kubeflow_amd.runtime.rest.RestClient`.

The controller-runtime cache the reference managers read from: one list+watch per kind
(started on first use), a local store with namespace and owner-UID indexes, per-kind
transforms applied before caching (the odh manager strips ``managedFields`` everywhere
and the ``data`` of ConfigMaps/Secrets, ``odh/main.go:81-101,165-185``), relist on
``410 Gone`` with synthetic ADDED/MODIFIED/DELETED events for the difference, and
reconnect with backoff on stream errors.

Implements :class:`~odh_kubeflow_amd.runtime.client.Reader` (zero-copy, read-only
objects) and :class:`~odh_kubeflow_amd.runtime.client.EventSource`.
"""

from __future__ import annotations

import asyncio
import logging
import random
import time
from typing import Callable, Dict, Iterable, List, Optional, Set, Tuple

from ..models import meta as m
from ..models.errors import ApiError, Gone, is_no_match
from ..models.scheme import SCHEME, ResourceInfo
from ..utils.selectors import field_matcher, match_labels, parse_field_selector, parse_label_selector, selector_from_dict
from .client import EventSource, Reader, WatchCallback

log = logging.getLogger("runtime.informer")

Transform = Callable[[dict], dict]

# labels the cache indexes (``client.MatchingLabels`` lookups by them cost the matches, not a
# scan of the namespace): ``notebook-name`` finds a notebook's HTTPRoutes among every notebook's
# in the central namespace (odh/controllers/notebook_route.go:155-165) and its pods
LABEL_INDEX_KEYS = ("notebook-name",)


def _rv_num(obj: dict) -> int:
    try:
        return int(m.resource_version(obj) or 0)
    except (TypeError, ValueError):
        return 0


def strip_managed_fields(obj: dict) -> dict:
    md = obj.get("metadata")
    if md and "managedFields" in md:
        md.pop("managedFields", None)
    return obj


def strip_data(obj: dict) -> dict:
    obj.pop("data", None)
    obj.pop("binaryData", None)
    obj.pop("stringData", None)
    return strip_managed_fields(obj)


def _one_event_batches(watch):
    async def batches(*args, **kw):
        async for ev in watch(*args, **kw):
            yield [ev]
    return batches


class _Informer:
    def __init__(self, cache: "InformerCache", info: ResourceInfo, version: str,
                 namespace: Optional[str] = None, label_selector: Optional[str] = None,
                 field_selector: Optional[str] = None):
        self.cache = cache
        self.info = info
        self.version = version
        self.namespace = namespace
        self.label_selector = label_selector
        self.field_selector = field_selector
        self._label_reqs = parse_label_selector(label_selector) if label_selector else None
        self.items: Dict[Tuple[str, str], dict] = {}
        self.by_ns: Dict[str, Set[Tuple[str, str]]] = {}
        self.by_owner: Dict[str, Set[Tuple[str, str]]] = {}
        # (label key, value) -> keys, for the cache's indexed label keys (LABEL_INDEX_KEYS)
        self.by_label: Dict[Tuple[str, str], Set[Tuple[str, str]]] = {}
        self._label_keys = cache.label_index_keys
        # a cluster-wide informer of a namespace-restricted cache (``cluster_watch``): objects of
        # namespaces this returns False for are dropped on arrival
        self.ns_filter: Optional[Callable[[str], bool]] = None
        self.handlers: Dict[int, Tuple[Optional[str], WatchCallback]] = {}
        self.synced = asyncio.Event()
        self.rv = ""
        self.task: Optional[asyncio.Task] = None
        self.relists = 0
        self.events = 0
        self.mutations = 0  # store changes: a derived view is current while this stands still
        self.missing_kind = False
        self._rv_waiters: List[Tuple[int, asyncio.Future]] = []
        self._fill_tombstones: Dict[str, Dict[Tuple[str, str], int]] = {}  # see fill_namespace

    def _rv_reached(self) -> None:
        """Resolve read-your-own-write waiters whose resourceVersion this stream has passed."""
        try:
            cur = int(self.rv)
        except (TypeError, ValueError):
            return
        keep = []
        for want, fut in self._rv_waiters:
            if fut.done():
                continue
            if cur >= want:
                fut.set_result(True)
            else:
                keep.append((want, fut))
        self._rv_waiters = keep

    # -------------------------------------------------------------- index maintenance

    def _put(self, obj: dict) -> Optional[dict]:
        k = (m.namespace(obj), m.name(obj))
        old = self.items.get(k)
        if old is not None:
            self._unindex(k, old)
        self.items[k] = obj
        self.mutations += 1
        self.by_ns.setdefault(k[0], set()).add(k)
        md = obj.get("metadata") or {}
        for r in md.get("ownerReferences") or []:
            if r.get("uid"):
                self.by_owner.setdefault(r["uid"], set()).add(k)
        labels = md.get("labels")
        if labels and self._label_keys:
            for lk in self._label_keys:
                v = labels.get(lk)
                if v is not None:
                    self.by_label.setdefault((lk, v), set()).add(k)
        return old

    def _unindex(self, k, obj) -> None:
        s = self.by_ns.get(k[0])
        if s is not None:
            s.discard(k)
        md = obj.get("metadata") or {}
        for r in md.get("ownerReferences") or []:
            s = self.by_owner.get(r.get("uid"))
            if s is not None:
                s.discard(k)
                if not s:
                    self.by_owner.pop(r.get("uid"), None)
        labels = md.get("labels")
        if labels and self._label_keys:
            for lk in self._label_keys:
                v = labels.get(lk)
                s = self.by_label.get((lk, v)) if v is not None else None
                if s is not None:
                    s.discard(k)
                    if not s:
                        self.by_label.pop((lk, v), None)

    def _delete(self, obj: dict) -> Optional[dict]:
        k = (m.namespace(obj), m.name(obj))
        old = self.items.pop(k, None)
        if old is not None:
            self._unindex(k, old)
            self.mutations += 1
        return old

    def _notify(self, etype: str, obj: dict, old: Optional[dict]) -> None:
        self.events += 1
        self.cache.last_event = time.monotonic()
        ns = m.namespace(obj)
        for hns, cb in list(self.handlers.values()):
            if hns and hns != ns:
                continue
            try:
                cb(etype, obj, old)
            except Exception:
                log.exception("informer handler failed")

    def _transform(self, obj: dict) -> dict:
        obj.setdefault("apiVersion", self.info.api_version(self.version))
        obj.setdefault("kind", self.info.kind)
        t = self.cache.transforms.get(self.info.key, strip_managed_fields)
        return t(obj) if t else obj

    # -------------------------------------------------------------- list / watch loop

    async def fill_namespace(self, ns: str) -> None:
        """A namespace joined a cluster-wide informer's filter: its objects, dropped until now,
        are listed once (events of it are kept from now on; a listed copy older than one an
        event already brought is not applied)."""
        # deletions the watch delivers while the list is in flight: key -> resourceVersion.  The
        # list may have been taken before such a deletion; an object it deleted is not stored
        # yet (nothing to compare against), so without the tombstone the listed copy would put
        # it back, a ghost reconciled until the next relist
        tombs = self._fill_tombstones.setdefault(ns, {})
        try:
            try:
                items, _rv = await self.cache.rest.list_rv(
                    f"{self.info.api_version(self.version)}/{self.info.kind}", ns, self.label_selector,
                    self.field_selector)
            except Exception:  # noqa: BLE001 — a relist of the whole kind (410 / reconnect) fills it later
                log.warning("%s: listing namespace %s failed", self.info.kind, ns, exc_info=True)
                return
            self.relists += 1
            if self.ns_filter is not None and not self.ns_filter(ns):
                return  # left again meanwhile
            for o in items:
                o = self._transform(o)
                k = (m.namespace(o), m.name(o))
                gone = tombs.get(k)
                if gone is not None and _rv_num(o) <= gone:
                    continue
                cur = self.items.get(k)
                if cur is not None and _rv_num(cur) >= _rv_num(o):
                    continue
                old = self._put(o)
                self._notify("ADDED" if old is None else "MODIFIED", o, old)
        finally:
            if self._fill_tombstones.get(ns) is tombs:
                del self._fill_tombstones[ns]

    def drop_namespace(self, ns: str) -> None:
        """A namespace left a cluster-wide informer's filter: to subscribers its objects are gone."""
        for k in list(self.by_ns.get(ns, ())):
            old = self.items.get(k)
            if old is not None:
                self._delete(old)
                self._notify("DELETED", old, old)

    async def _relist(self) -> None:
        items, rv = await self.cache.rest.list_rv(f"{self.info.api_version(self.version)}/{self.info.kind}",
                                                  self.namespace, self.label_selector, self.field_selector)
        self.relists += 1
        seen = set()
        nsf = self.ns_filter
        for o in items:
            if nsf is not None and not nsf(m.namespace(o)):
                continue
            o = self._transform(o)
            k = (m.namespace(o), m.name(o))
            seen.add(k)
            old = self._put(o)
            if old is None:
                self._notify("ADDED", o, None)
            elif m.resource_version(old) != m.resource_version(o):
                self._notify("MODIFIED", o, old)
        for k in [k for k in self.items if k not in seen]:
            old = self.items[k]
            self._delete(old)
            self._notify("DELETED", old, old)
        self.rv = rv
        self.missing_kind = False
        self.synced.set()
        if self._rv_waiters:
            self._rv_reached()

    def _tombstone(self, obj: dict) -> None:
        if self._fill_tombstones:
            tombs = self._fill_tombstones.get(m.namespace(obj))
            if tombs is not None:
                tombs[(m.namespace(obj), m.name(obj))] = _rv_num(obj)

    def _stored(self, namespace: str, name: str) -> Optional[dict]:
        return self.items.get((namespace if self.info.namespaced else "", name))

    def _apply(self, et: str, obj: dict) -> None:
        """One watch event into the store, then to the subscribers."""
        self.rv = m.resource_version(obj) or self.rv
        if et == "BOOKMARK":
            return
        if self.ns_filter is not None and not self.ns_filter(m.namespace(obj)):
            return  # a cluster-wide watch: another shard's (or worker's) namespace
        obj = self._transform(obj)
        if et != "DELETED" and self._label_reqs is not None and not match_labels(
                self._label_reqs, (obj.get("metadata") or {}).get("labels")):
            # the object left the selector: to this cache it is gone
            if (m.namespace(obj), m.name(obj)) not in self.items:
                self._tombstone(obj)
                return
            et = "DELETED"
        if et == "DELETED":
            self._tombstone(obj)
            old = self._delete(obj)
            self._notify("DELETED", obj, old)
        else:
            old = self._put(obj)
            self._notify("ADDED" if old is None else "MODIFIED", obj, old)

    async def run(self) -> None:
        ref = f"{self.info.api_version(self.version)}/{self.info.kind}"
        backoff = 0.05
        need_list = True
        started: Optional[float] = None
        while True:
            try:
                if need_list:
                    await self._relist()
                    need_list = False
                started = time.monotonic()
                rest = self.cache.rest
                batches = getattr(rest, "watch_batches", None)
                kw = {}
                if batches is None:  # a client without batched watches (test doubles)
                    batches = _one_event_batches(rest.watch)
                else:  # decoded against the stored object: unchanged subtrees are shared
                    kw["lookup"] = self._stored
                async for batch in batches(ref, self.namespace, self.rv, labels=self.label_selector,
                                           fields=self.field_selector, timeout_s=self.cache.watch_timeout_s,
                                           **kw):
                    backoff = 0.05
                    for et, obj in batch:
                        self._apply(et, obj)
                    if self._rv_waiters:
                        self._rv_reached()
            except asyncio.CancelledError:
                raise
            except Gone:
                need_list = True
            except ApiError as e:
                if is_no_match(e) or e.code == 404:
                    self.missing_kind = True
                    self.synced.set()  # an uninstalled CRD is an empty, synced cache
                    await asyncio.sleep(5.0)
                    need_list = True
                    continue
                log.warning("%s watch error: %r", self.info.kind, e)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 5.0)
            except Exception as e:  # connection reset, server restart
                log.debug("%s watch dropped: %r", self.info.kind, e)
                if started is not None and time.monotonic() - started > 1.0:
                    backoff = 0.05  # the stream was healthy for a while: a fresh drop, not a flapping server
                await asyncio.sleep(backoff * (1 + random.random()))
                backoff = min(backoff * 2, 5.0)


class _Group:
    """The informers of one kind: one cluster-wide informer, or one per cached namespace
    (the set follows the Namespace selector).  Watch handlers live here, shared by every
    informer of the kind, so a namespace that joins later feeds existing subscriptions."""

    def __init__(self, info: ResourceInfo, version: str):
        self.info = info
        self.version = version
        self.infs: Dict[Optional[str], _Informer] = {}
        self.handlers: Dict[int, Tuple[Optional[str], WatchCallback]] = {}

    def all(self) -> List[_Informer]:
        return list(self.infs.values())


class InformerCache(Reader, EventSource):
    """Shared informers keyed by kind (and namespace, for a namespace-restricted cache).

    ``namespace`` restricts namespaced kinds to one namespace; ``namespaces`` to a set of
    them (one list/watch per namespace, merged for readers — controller-runtime's
    ``cache.Options.DefaultNamespaces``).  ``namespace_selector`` makes that set dynamic:
    a label-selected Namespace watch adds a namespace's informers when it starts matching
    (a shard is assigned a namespace) and drops them, with DELETED events for what they
    held, when it stops matching; ``namespaces`` are then always-cached extras (the
    controller namespace).  ``namespace_filter`` (a predicate on the Namespace object)
    narrows the dynamic set (with no ``namespace_selector``: every namespace it admits) — one
    worker of a controller partitioned over processes watches only its partition's namespaces.
    ``selectors`` maps a kind to a label selector applied server-side to its list/watch
    (``cache.Options.ByObject[..].Label``) so a shard only ever receives the objects it owns;
    ``field_selectors`` likewise with a field selector (``ByObject[..].Field``; immutable fields
    only, e.g. an Event's ``involvedObject.kind``, so an object never moves out of it).
    ``namespace_labels`` maps a kind that lives outside the notebooks' namespaces (cluster-scoped,
    or in the controller namespace) to the label naming the namespace an object belongs to: a
    namespace-restricted cache then lists and watches only the objects of its namespaces
    (``<label> in (<its namespaces>)``, re-scoped as the set changes) — every shard or worker
    would otherwise decode every other one's ClusterRoleBindings and HTTPRoutes.
    """

    def __init__(self, rest, namespace: Optional[str] = None, transforms: Optional[Dict[str, Optional[Transform]]] = None,
                 watch_timeout_s: int = 300, namespaces: Optional[Iterable[str]] = None,
                 selectors: Optional[Dict[str, str]] = None, namespace_selector: Optional[str] = None,
                 namespace_filter: Optional[Callable[[dict], bool]] = None,
                 field_selectors: Optional[Dict[str, str]] = None,
                 label_index_keys: Optional[Iterable[str]] = None, cluster_watch: bool = False,
                 namespace_labels: Optional[Dict[str, str]] = None):
        self.rest = rest
        self.namespace = namespace
        nss = list(namespaces) if namespaces is not None else ([namespace] if namespace else None)
        self.static_namespaces: List[str] = list(nss or [])
        self.namespace_selector = namespace_selector
        self.namespace_filter = namespace_filter
        self._dynamic = bool(namespace_selector) or namespace_filter is not None
        # None = every namespace (cluster-wide informers)
        self.namespaces: Optional[Set[str]] = set(nss or ()) if (nss or self._dynamic) else None
        # ``cluster_watch``: a namespace-restricted cache that still opens ONE list/watch per kind,
        # cluster-wide, and drops the other namespaces' objects on arrival — one watch stream per
        # kind however many namespaces it serves, for every event of the kind decoded here
        self.cluster_watch = bool(cluster_watch) and self.namespaces is not None
        self.transforms: Dict[str, Optional[Transform]] = {}
        for k, fn in (transforms or {}).items():
            self.transforms[SCHEME.resolve(k).key] = fn
        self.selectors: Dict[str, str] = {SCHEME.resolve(k).key: v for k, v in (selectors or {}).items()}
        self.field_selectors: Dict[str, str] = {SCHEME.resolve(k).key: v for k, v in (field_selectors or {}).items()}
        self.namespace_labels: Dict[str, str] = {SCHEME.resolve(k).key: v
                                                 for k, v in (namespace_labels or {}).items()}
        self._rescope_pending = False
        self.rescopes = 0
        self.watch_timeout_s = watch_timeout_s
        self.label_index_keys = frozenset(LABEL_INDEX_KEYS if label_index_keys is None else label_index_keys)
        # kind -> cached objects list() examined: the scans an index did not narrow (io counters)
        self.list_scans: Dict[str, int] = {}
        self._groups: Dict[str, _Group] = {}
        self._by_ref: Dict[str, _Group] = {}
        self._hid = 0
        self._ns_informer: Optional[_Informer] = None
        self.namespace_changes = 0
        self.last_event = 0.0  # monotonic time of the last watch event delivered (Manager.quiesce)

    # -------------------------------------------------------------- namespace membership

    def _ensure_ns_informer(self) -> None:
        if not self._dynamic or self._ns_informer is not None:
            return
        info = SCHEME.resolve(kinds_namespace())
        inf = _Informer(self, info, info.storage_version, None, self.namespace_selector or None)
        inf.handlers = {0: (None, self._on_namespace)}
        self._ns_informer = inf
        inf.task = asyncio.ensure_future(inf.run())

    def _on_namespace(self, etype: str, obj: dict, old: Optional[dict]) -> None:
        ns = m.name(obj)
        if ns in self.static_namespaces:
            return
        # a Terminating namespace stays cached: its Notebooks' finalizers still need the
        # controllers; it leaves when it is gone or stops matching the selector (DELETED)
        if etype == "DELETED" or (self.namespace_filter is not None and not self.namespace_filter(obj)):
            if ns in self.namespaces:
                self.namespaces.discard(ns)
                self.namespace_changes += 1
                self._schedule_rescope()
                for g in self._groups.values():
                    if not g.info.namespaced:
                        continue
                    if self.cluster_watch:
                        for inf in g.infs.values():
                            inf.drop_namespace(ns)
                        continue
                    inf = g.infs.pop(ns, None)
                    if inf is not None:
                        self._retire(inf)
        elif ns not in self.namespaces:
            self.namespaces.add(ns)
            self.namespace_changes += 1
            self._schedule_rescope()
            for g in self._groups.values():
                if not g.info.namespaced:
                    continue
                if self.cluster_watch:
                    for inf in g.infs.values():
                        if inf.synced.is_set():  # else its first list, still to come, includes it
                            asyncio.ensure_future(inf.fill_namespace(ns))
                    continue
                self._start_informer(g, ns)

    def refresh_namespace(self, name: str) -> None:
        """Re-evaluate ``namespace_filter`` for one namespace (its answer changed: a worker was
        assigned or released the namespace, runtime/workers.py)."""
        inf = self._ns_informer
        obj = inf.items.get(("", name)) if inf is not None else None
        if obj is not None:
            self._on_namespace("MODIFIED", obj, obj)

    def _retire(self, inf: _Informer) -> None:
        """A namespace left the cache: stop its informer; to subscribers its objects are gone."""
        if inf.task is not None:
            inf.task.cancel()
        for k in list(inf.items):
            old = inf.items[k]
            inf._delete(old)
            inf._notify("DELETED", old, old)

    def _scoped_selector(self, key: str) -> Optional[str]:
        """``kind``'s label selector: the static one, or for a ``namespace_labels`` kind of a
        namespace-restricted cache the objects of its namespaces."""
        sel = self.selectors.get(key)
        label = self.namespace_labels.get(key)
        if sel or not label or self.namespaces is None:
            return sel
        # "-" names no namespace: an empty set selects nothing
        return f"{label} in ({','.join(sorted(self.namespaces)) or '-'})"

    def _schedule_rescope(self) -> None:
        if not self.namespace_labels or self._rescope_pending:
            return
        self._rescope_pending = True
        try:
            asyncio.get_running_loop().call_soon(self._rescope)
        except RuntimeError:  # no loop yet: the informers start with the current set
            self._rescope_pending = False

    def _rescope(self) -> None:
        """The namespace set changed (coalesced per loop turn): re-list the ``namespace_labels``
        kinds under the new selector.  In place — the relist applies only the difference, so
        objects still in scope raise no event."""
        self._rescope_pending = False
        for key in self.namespace_labels:
            g = self._groups.get(key)
            if g is None:
                continue
            sel = self._scoped_selector(key)
            for inf in g.infs.values():
                if inf.label_selector == sel:
                    continue
                inf.label_selector = sel
                inf._label_reqs = parse_label_selector(sel) if sel else None
                self.rescopes += 1
                if inf.task is not None:
                    inf.task.cancel()
                inf.task = asyncio.ensure_future(inf.run())

    def _start_informer(self, g: _Group, ns: Optional[str]) -> _Informer:
        inf = _Informer(self, g.info, g.version, ns, self._scoped_selector(g.info.key),
                        self.field_selectors.get(g.info.key))
        inf.handlers = g.handlers  # shared: subscriptions made earlier see this namespace too
        g.infs[ns] = inf
        inf.task = asyncio.ensure_future(inf.run())
        return inf

    def set_field_selector(self, kind, selector: str) -> bool:
        """Narrow ``kind``'s list/watch server-side before its informer starts (a controller
        that needs only part of a kind, at setup); False when the informer already runs."""
        key = SCHEME.resolve(kind).key
        if key in self._groups:
            return False
        self.field_selectors[key] = selector
        return True

    def covers(self, kind, namespace: Optional[str]) -> bool:
        """Whether reads of ``kind`` in ``namespace`` are served by this cache (False: the
        caller must read live — the namespace belongs to another shard)."""
        if self.namespaces is None or not namespace:
            return True
        if not SCHEME.resolve(kind).namespaced:
            return True
        return namespace in self.namespaces

    # -------------------------------------------------------------- groups

    def _group(self, kind) -> _Group:
        if type(kind) is str:
            hit = self._by_ref.get(kind)
            if hit is not None:
                return hit
        info = SCHEME.resolve(kind)
        g = self._groups.get(info.key)
        if g is None:
            from .client import _version_of

            self._ensure_ns_informer()
            g = self._groups[info.key] = _Group(info, _version_of(kind) or info.storage_version)
            if info.namespaced and self.namespaces is not None and not self.cluster_watch:
                for ns in sorted(self.namespaces):
                    self._start_informer(g, ns)
            else:
                inf = self._start_informer(g, None)
                if info.namespaced and self.cluster_watch:
                    inf.ns_filter = self.namespaces.__contains__
        if type(kind) is str:
            self._by_ref[kind] = g
        return g

    def _for_ns(self, kind, namespace: Optional[str]) -> List[_Informer]:
        g = self._group(kind)
        if namespace and g.info.namespaced and self.namespaces is not None and not self.cluster_watch:
            inf = g.infs.get(namespace)
            return [inf] if inf is not None else []
        return g.all()

    def watching(self, kind, namespace: Optional[str]) -> bool:
        """Whether a synced informer already holds ``kind`` in ``namespace`` — without
        starting one (CachedClient's resourceVersion-validated reads of live-read kinds)."""
        try:
            info = SCHEME.resolve(kind)
        except KeyError:
            return False
        g = self._groups.get(info.key)
        if g is None:
            return False
        if namespace and info.namespaced and self.namespaces is not None:
            if self.cluster_watch and namespace not in self.namespaces:
                return False
            inf = g.infs.get(None if self.cluster_watch else namespace)
            infs = [inf] if inf is not None else []
        else:
            infs = g.all()
        return bool(infs) and all(i.synced.is_set() and not i.missing_kind for i in infs)

    def event_counts(self) -> Dict[str, int]:
        """Watch events delivered per kind since start (relist differences included)."""
        out: Dict[str, int] = {}
        for g in self._groups.values():
            n = sum(inf.events for inf in g.infs.values())
            if n:
                out[g.info.kind] = out.get(g.info.kind, 0) + n
        return out

    def relist_counts(self) -> Dict[str, int]:
        """Lists per kind since start, the initial one of each informer included: a rise means
        a watch was answered 410 Gone (it fell behind the apiserver's bounded history)."""
        out: Dict[str, int] = {}
        for g in self._groups.values():
            n = sum(inf.relists for inf in g.infs.values())
            if n:
                out[g.info.kind] = out.get(g.info.kind, 0) + n
        return out

    def informer(self, kind) -> _Informer:
        """The (first) informer of ``kind`` — for single-namespace / cluster-wide caches."""
        return self._group(kind).all()[0]

    async def _ns_synced(self, timeout: float) -> None:
        self._ensure_ns_informer()
        if self._ns_informer is not None and not self._ns_informer.synced.is_set():
            await asyncio.wait_for(self._ns_informer.synced.wait(), timeout)

    async def ensure_informer(self, kind, timeout: float = 30.0) -> None:
        await self._ns_synced(timeout)
        infs = self._group(kind).all()
        for inf in infs:
            if not inf.synced.is_set():
                await asyncio.wait_for(inf.synced.wait(), timeout)
        if infs and all(inf.missing_kind for inf in infs):
            from ..models.errors import NoKindMatch

            raise NoKindMatch(infs[0].info.kind)

    # -------------------------------------------------------------- EventSource

    def subscribe(self, kind, callback, namespace=None):
        g = self._group(kind)
        self._hid += 1
        hid = self._hid
        for inf in self._for_ns(kind, namespace):
            for o in list(inf.items.values()):
                if namespace and m.namespace(o) != namespace:
                    continue
                callback("ADDED", o, None)
        g.handlers[hid] = (namespace, callback)

        def cancel():
            g.handlers.pop(hid, None)
        return cancel

    async def wait_synced(self, kinds: Iterable, timeout: float = 30.0) -> None:
        await self._ns_synced(timeout)

        async def one(inf):
            if not inf.synced.is_set():
                await asyncio.wait_for(inf.synced.wait(), timeout)

        await asyncio.gather(*(one(inf) for k in kinds for inf in self._group(k).all()))

    async def wait_for_rv(self, kind, namespace: Optional[str], want: int, timeout: float) -> bool:
        """Wait until the watch stream holding ``namespace``'s ``kind`` objects has delivered
        resourceVersion ``want`` (e.g. a write this process just made).  A write's watch event
        is emitted when it commits, before the write's response, so this is normally one
        event-loop turn — no request, where a read-through GET would be a round trip."""
        infs = self._for_ns(kind, namespace)
        if len(infs) != 1:
            return False
        inf = infs[0]
        try:
            if int(inf.rv) >= want:
                return True
        except (TypeError, ValueError):
            pass
        fut = asyncio.get_running_loop().create_future()
        inf._rv_waiters.append((want, fut))
        try:
            return await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            return False

    # -------------------------------------------------------------- Reader

    def get(self, kind, name, namespace=None):
        infs = self._for_ns(kind, namespace)
        if len(infs) != 1 or (infs[0].namespace and namespace and infs[0].namespace != namespace):
            return None  # namespace outside this cache
        inf = infs[0]
        return inf.items.get((namespace or "" if inf.info.namespaced else "", name))

    def store_version(self, kind) -> Optional[Tuple[Tuple[int, int], ...]]:
        """A token that changes whenever the cached objects of ``kind`` do (None: not cached):
        views derived from a whole-kind list are reused while it stands still."""
        infs = self._for_ns(kind, None)
        if not infs:
            return None
        return tuple((id(inf), inf.mutations) for inf in infs)

    def kind_version(self, kind) -> Optional[Tuple[Tuple[int, int, bool], ...]]:
        """:meth:`store_version` without starting an informer: ``None`` until every informer
        of ``kind`` has synced (an uninstalled kind counts as synced and empty — the token
        changes when it gets installed)."""
        try:
            info = SCHEME.resolve(kind)
        except KeyError:
            return None
        g = self._groups.get(info.key)
        infs = g.all() if g is not None else []
        if not infs or not all(i.synced.is_set() for i in infs):
            return None
        return tuple((id(i), i.mutations, i.missing_kind) for i in infs)

    def any(self, kind, namespace: Optional[str], pred) -> bool:
        """Whether some cached object of ``kind`` (in ``namespace``) satisfies ``pred`` — stopping
        at the first: "is another Notebook of this namespace alive" costs one or two looks, not
        a sorted copy of every Notebook in it (the odh reconciler asks it once per deletion)."""
        n = 0
        try:
            for inf in self._for_ns(kind, namespace):
                keys = inf.by_ns.get(namespace, ()) if namespace and inf.info.namespaced else inf.items.keys()
                for k in keys:
                    n += 1
                    o = inf.items.get(k)
                    if o is not None and pred(o):
                        return True
            return False
        finally:
            kk = SCHEME.resolve(kind).kind
            self.list_scans[kk] = self.list_scans.get(kk, 0) + n

    def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None) -> List[dict]:
        infs = self._for_ns(kind, namespace)
        if isinstance(labels, dict):
            reqs = selector_from_dict({"matchLabels": labels})
        elif isinstance(labels, str):
            reqs = parse_label_selector(labels)
        else:
            reqs = labels or []
        fm = field_matcher(parse_field_selector(fields)) if fields else None
        indexed = next(((k, vals[0]) for k, op, vals in reqs if op == "=" and k in self.label_index_keys), None) \
            if reqs and self.label_index_keys else None
        out = []
        scans = self.list_scans
        for inf in infs:
            if owner_uid is not None:
                keys = inf.by_owner.get(owner_uid, ())
            elif indexed is not None:
                # an equality on an indexed label: the candidates, not every object of the namespace
                # (the odh reconciler's HTTPRoutes, found by label in the one central namespace)
                keys = inf.by_label.get(indexed, ())
            elif namespace and inf.info.namespaced:
                keys = inf.by_ns.get(namespace, ())
            else:
                keys = inf.items.keys()
            keys = list(keys)
            scans[inf.info.kind] = scans.get(inf.info.kind, 0) + len(keys)
            for k in keys:
                o = inf.items.get(k)
                if o is None:
                    continue
                if namespace and inf.info.namespaced and m.namespace(o) != namespace:
                    continue
                if reqs and not match_labels(reqs, (o.get("metadata") or {}).get("labels")):
                    continue
                if fm is not None and not fm(o):
                    continue
                out.append(o)
        out.sort(key=lambda o: (m.namespace(o), m.name(o)))
        return out

    async def stop(self) -> None:
        infs = [inf for g in self._groups.values() for inf in g.infs.values()]
        if self._ns_informer is not None:
            infs.append(self._ns_informer)
        for inf in infs:
            if inf.task is not None:
                inf.task.cancel()
        for inf in infs:
            if inf.task is not None:
                try:
                    await inf.task
                except (asyncio.CancelledError, Exception):
                    pass
        self._groups.clear()
        self._by_ref.clear()
        self._ns_informer = None


def kinds_namespace():
    from ..models import kinds

    return kinds.NAMESPACE
