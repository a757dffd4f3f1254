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
from typing import Callable, Dict, Iterable, List, Optional, Set, Tuple

from ..models import meta as m
from ..models.errors import ApiError, Gone, is_no_match
from ..models.scheme import SCHEME, ResourceInfo
from ..utils.selectors import field_matcher, match_labels, parse_field_selector, parse_label_selector, selector_from_dict
from .client import EventSource, Reader, WatchCallback

log = logging.getLogger("runtime.informer")

Transform = Callable[[dict], dict]


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


class _Informer:
    def __init__(self, cache: "InformerCache", info: ResourceInfo, version: str,
                 namespace: Optional[str] = None, label_selector: Optional[str] = None):
        self.cache = cache
        self.info = info
        self.version = version
        self.namespace = namespace
        self.label_selector = label_selector
        self._label_reqs = parse_label_selector(label_selector) if label_selector else None
        self.items: Dict[Tuple[str, str], dict] = {}
        self.by_ns: Dict[str, Set[Tuple[str, str]]] = {}
        self.by_owner: Dict[str, Set[Tuple[str, str]]] = {}
        self.handlers: Dict[int, Tuple[Optional[str], WatchCallback]] = {}
        self.synced = asyncio.Event()
        self.rv = ""
        self.task: Optional[asyncio.Task] = None
        self.relists = 0
        self.events = 0
        self.missing_kind = False
        self._rv_waiters: List[Tuple[int, asyncio.Future]] = []

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
        self.by_ns.setdefault(k[0], set()).add(k)
        for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
            if r.get("uid"):
                self.by_owner.setdefault(r["uid"], set()).add(k)
        return old

    def _unindex(self, k, obj) -> None:
        s = self.by_ns.get(k[0])
        if s is not None:
            s.discard(k)
        for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
            s = self.by_owner.get(r.get("uid"))
            if s is not None:
                s.discard(k)
                if not s:
                    self.by_owner.pop(r.get("uid"), None)

    def _delete(self, obj: dict) -> Optional[dict]:
        k = (m.namespace(obj), m.name(obj))
        old = self.items.pop(k, None)
        if old is not None:
            self._unindex(k, old)
        return old

    def _notify(self, etype: str, obj: dict, old: Optional[dict]) -> None:
        self.events += 1
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

    async def _relist(self) -> None:
        items, rv = await self.cache.rest.list_rv(f"{self.info.api_version(self.version)}/{self.info.kind}",
                                                  self.namespace, self.label_selector)
        self.relists += 1
        seen = set()
        for o in items:
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

    async def run(self) -> None:
        ref = f"{self.info.api_version(self.version)}/{self.info.kind}"
        backoff = 0.05
        need_list = True
        while True:
            try:
                if need_list:
                    await self._relist()
                    need_list = False
                async for et, obj in self.cache.rest.watch(ref, self.namespace, self.rv, labels=self.label_selector,
                                                           timeout_s=self.cache.watch_timeout_s):
                    backoff = 0.05
                    if et == "BOOKMARK":
                        self.rv = m.resource_version(obj) or self.rv
                        continue
                    obj = self._transform(obj)
                    self.rv = m.resource_version(obj) or self.rv
                    if et != "DELETED" and self._label_reqs is not None and not match_labels(
                            self._label_reqs, (obj.get("metadata") or {}).get("labels")):
                        # the object left the selector: to this cache it is gone
                        if (m.namespace(obj), m.name(obj)) not in self.items:
                            continue
                        et = "DELETED"
                    if et == "DELETED":
                        old = self._delete(obj)
                        self._notify("DELETED", obj, old)
                    else:
                        old = self._put(obj)
                        self._notify("ADDED" if old is None else "MODIFIED", obj, old)
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
                await asyncio.sleep(backoff * (1 + random.random()))
                backoff = min(backoff * 2, 5.0)


class InformerCache(Reader, EventSource):
    """Shared informers keyed by kind (and namespace, for a namespace-restricted cache).

    ``namespace`` restricts namespaced kinds to one namespace; ``namespaces`` to a set of
    them (one list/watch per namespace, merged for readers — controller-runtime's
    ``cache.Options.DefaultNamespaces``).  ``selectors`` maps a kind to a label selector
    applied server-side to its list/watch (``cache.Options.ByObject[..].Label``) so a
    shard only ever receives the objects it owns.
    """

    def __init__(self, rest, namespace: Optional[str] = None, transforms: Optional[Dict[str, Optional[Transform]]] = None,
                 watch_timeout_s: int = 300, namespaces: Optional[Iterable[str]] = None,
                 selectors: Optional[Dict[str, str]] = None):
        self.rest = rest
        self.namespace = namespace
        nss = list(namespaces) if namespaces is not None else ([namespace] if namespace else None)
        self.namespaces: Optional[List[str]] = nss
        self.transforms: Dict[str, Optional[Transform]] = {}
        for k, fn in (transforms or {}).items():
            self.transforms[SCHEME.resolve(k).key] = fn
        self.selectors: Dict[str, str] = {SCHEME.resolve(k).key: v for k, v in (selectors or {}).items()}
        self.watch_timeout_s = watch_timeout_s
        self._informers: Dict[Tuple[str, Optional[str]], _Informer] = {}
        self._by_kind: Dict[str, List[_Informer]] = {}
        self._by_ref: Dict[str, List[_Informer]] = {}
        self._hid = 0

    def _group(self, kind) -> List[_Informer]:
        if type(kind) is str:
            hit = self._by_ref.get(kind)
            if hit is not None:
                return hit
        info = SCHEME.resolve(kind)
        infs = self._by_kind.get(info.key)
        if infs is None:
            from .client import _version_of

            version = _version_of(kind) or info.storage_version
            nss = self.namespaces if (info.namespaced and self.namespaces) else [None]
            infs = []
            for ns in nss:
                inf = _Informer(self, info, version, ns, self.selectors.get(info.key))
                self._informers[(info.key, ns)] = inf
                inf.task = asyncio.ensure_future(inf.run())
                infs.append(inf)
            self._by_kind[info.key] = infs
        if type(kind) is str:
            self._by_ref[kind] = infs
        return infs

    def _for_ns(self, kind, namespace: Optional[str]) -> List[_Informer]:
        infs = self._group(kind)
        if namespace and len(infs) > 1:
            return [i for i in infs if i.namespace == namespace]
        return infs

    def informer(self, kind) -> _Informer:
        """The (first) informer of ``kind`` — for single-namespace / cluster-wide caches."""
        return self._group(kind)[0]

    async def ensure_informer(self, kind, timeout: float = 30.0) -> None:
        infs = self._group(kind)
        for inf in infs:
            if not inf.synced.is_set():
                await asyncio.wait_for(inf.synced.wait(), timeout)
        if all(inf.missing_kind for inf in infs):
            from ..models.errors import NoKindMatch

            raise NoKindMatch(infs[0].info.kind)

    # -------------------------------------------------------------- EventSource

    def subscribe(self, kind, callback, namespace=None):
        infs = self._for_ns(kind, namespace)
        self._hid += 1
        hid = self._hid
        for inf in infs:
            for o in list(inf.items.values()):
                if namespace and m.namespace(o) != namespace:
                    continue
                callback("ADDED", o, None)
            inf.handlers[hid] = (namespace, callback)

        def cancel():
            for inf in infs:
                inf.handlers.pop(hid, None)
        return cancel

    async def wait_synced(self, kinds: Iterable, timeout: float = 30.0) -> None:
        async def one(inf):
            if not inf.synced.is_set():
                await asyncio.wait_for(inf.synced.wait(), timeout)

        await asyncio.gather(*(one(inf) for k in kinds for inf in self._group(k)))

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

    def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None) -> List[dict]:
        infs = self._for_ns(kind, namespace)
        if isinstance(labels, dict):
            reqs = selector_from_dict({"matchLabels": labels})
        elif isinstance(labels, str):
            reqs = parse_label_selector(labels)
        else:
            reqs = labels or []
        fm = field_matcher(parse_field_selector(fields)) if fields else None
        out = []
        for inf in infs:
            if owner_uid is not None:
                keys = inf.by_owner.get(owner_uid, ())
            elif namespace and inf.info.namespaced:
                keys = inf.by_ns.get(namespace, ())
            else:
                keys = inf.items.keys()
            for k in list(keys):
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
        for inf in self._informers.values():
            if inf.task is not None:
                inf.task.cancel()
        for inf in self._informers.values():
            if inf.task is not None:
                try:
                    await inf.task
                except (asyncio.CancelledError, Exception):
                    pass
        self._informers.clear()
        self._by_kind.clear()
        self._by_ref.clear()
