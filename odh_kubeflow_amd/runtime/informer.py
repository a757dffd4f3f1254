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
    def __init__(self, cache: "InformerCache", info: ResourceInfo, version: str):
        self.cache = cache
        self.info = info
        self.version = version
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
                                                  self.cache.namespace)
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

    async def run(self) -> None:
        ref = f"{self.info.api_version(self.version)}/{self.info.kind}"
        backoff = 0.05
        need_list = True
        while True:
            try:
                if need_list:
                    await self._relist()
                    need_list = False
                async for et, obj in self.cache.rest.watch(ref, self.cache.namespace, self.rv,
                                                           timeout_s=self.cache.watch_timeout_s):
                    backoff = 0.05
                    if et == "BOOKMARK":
                        self.rv = m.resource_version(obj) or self.rv
                        continue
                    obj = self._transform(obj)
                    self.rv = m.resource_version(obj) or self.rv
                    if et == "DELETED":
                        old = self._delete(obj)
                        self._notify("DELETED", obj, old)
                    else:
                        old = self._put(obj)
                        self._notify("ADDED" if old is None else "MODIFIED", obj, old)
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
    def __init__(self, rest, namespace: Optional[str] = None, transforms: Optional[Dict[str, Optional[Transform]]] = None,
                 watch_timeout_s: int = 300):
        self.rest = rest
        self.namespace = namespace
        self.transforms: Dict[str, Optional[Transform]] = {}
        for k, fn in (transforms or {}).items():
            self.transforms[SCHEME.resolve(k).key] = fn
        self.watch_timeout_s = watch_timeout_s
        self._informers: Dict[str, _Informer] = {}
        self._hid = 0

    def informer(self, kind) -> _Informer:
        info = SCHEME.resolve(kind)
        inf = self._informers.get(info.key)
        if inf is None:
            from .client import _version_of

            inf = self._informers[info.key] = _Informer(self, info, _version_of(kind) or info.storage_version)
            inf.task = asyncio.ensure_future(inf.run())
        return inf

    async def ensure_informer(self, kind, timeout: float = 30.0) -> None:
        inf = self.informer(kind)
        if not inf.synced.is_set():
            await asyncio.wait_for(inf.synced.wait(), timeout)
        if inf.missing_kind:
            from ..models.errors import NoKindMatch

            raise NoKindMatch(inf.info.kind)

    # -------------------------------------------------------------- EventSource

    def subscribe(self, kind, callback, namespace=None):
        inf = self.informer(kind)
        self._hid += 1
        hid = self._hid
        for o in list(inf.items.values()):
            if namespace and m.namespace(o) != namespace:
                continue
            callback("ADDED", o, None)
        inf.handlers[hid] = (namespace, callback)
        return lambda: inf.handlers.pop(hid, None)

    async def wait_synced(self, kinds: Iterable, timeout: float = 30.0) -> None:
        async def one(k):
            inf = self.informer(k)
            if not inf.synced.is_set():
                await asyncio.wait_for(inf.synced.wait(), timeout)

        await asyncio.gather(*(one(k) for k in kinds))

    # -------------------------------------------------------------- Reader

    def get(self, kind, name, namespace=None):
        inf = self.informer(kind)
        return inf.items.get((namespace or "" if inf.info.namespaced else "", name))

    def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None) -> List[dict]:
        inf = self.informer(kind)
        if owner_uid is not None:
            keys = inf.by_owner.get(owner_uid, ())
        elif namespace and inf.info.namespaced:
            keys = inf.by_ns.get(namespace, ())
        else:
            keys = inf.items.keys()
        if isinstance(labels, dict):
            reqs = selector_from_dict({"matchLabels": labels})
        elif isinstance(labels, str):
            reqs = parse_label_selector(labels)
        else:
            reqs = labels or []
        fm = field_matcher(parse_field_selector(fields)) if fields else None
        out = []
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
