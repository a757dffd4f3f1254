"""In-process access to the test platform's object store (envtest analogue).

:class:`StoreReader` (an always-synced zero-copy cache), :class:`StoreEventSource` and
:class:`InProcessClient` let a :class:`~odh_kubeflow_amd.runtime.manager.Manager` run
against :class:`~odh_kubeflow_amd.testing.apiserver.store.ObjectStore` in the test process,
the way controller-runtime's envtest suites run managers against a local apiserver
(``kf/controllers/suite_test.go:50-104``).  Production managers use
:meth:`Manager.remote` (REST + informer cache) only.
"""

from __future__ import annotations

from typing import Sequence

from ...models.scheme import SCHEME
from ...runtime.client import CachedClient, Client, EventSource, Reader, _refresh, _version_of
from ...runtime.manager import Manager
from .store import ObjectStore


class StoreReader(Reader):
    """Zero-copy reads straight from the in-process store (an always-synced cache)."""

    def __init__(self, store: ObjectStore):
        self.store = store

    def get(self, kind, name, namespace=None):
        return self.store.peek(kind, name, namespace)

    def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None):
        return self.store.list_nocopy(kind, namespace, labels, fields, owner_uid)

    def watching(self, kind, namespace=None) -> bool:
        return True  # the store itself: always synced, every namespace

    def kind_version(self, kind):
        return self.store.kind_version(kind)


class StoreEventSource(EventSource):
    def __init__(self, store: ObjectStore):
        self.store = store

    def subscribe(self, kind, callback, namespace=None):
        return self.store.watch(kind, callback, namespace=namespace, initial=True)


class InProcessClient(Client):
    """Client talking to an in-process :class:`ObjectStore`.

    ``user`` is recorded for audit/debugging only; the in-process path does no authz.
    """

    def __init__(self, store: ObjectStore, user: str = "system:admin"):
        self.store = store
        self.user = user
        self.reader = StoreReader(store)  # what a cache over this store would show: the store

    async def get(self, kind, name, namespace=None):
        return await self.store.get(kind, name, namespace, version=_version_of(kind))

    async def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None):
        items, _ = await self.store.list(kind, namespace, labels, fields, version=_version_of(kind),
                                         owner_uid=owner_uid)
        return items

    async def create(self, obj):
        return _refresh(obj, await self.store.create(obj))

    async def update(self, obj):
        return _refresh(obj, await self.store.update(obj))

    async def update_status(self, obj):
        return _refresh(obj, await self.store.update(obj, subresource="status"))

    async def patch(self, obj_or_kind, patch, patch_type="merge", name=None, namespace=None, subresource=None):
        if isinstance(obj_or_kind, dict):
            kind = obj_or_kind
            name = name or obj_or_kind["metadata"]["name"]
            namespace = namespace or obj_or_kind["metadata"].get("namespace")
        else:
            kind = obj_or_kind
        res = await self.store.patch(kind, name, namespace, patch, patch_type, subresource)
        v = _version_of(kind)
        if v:
            info = SCHEME.resolve(kind)
            res["apiVersion"] = info.api_version(v)
        if isinstance(obj_or_kind, dict):
            return _refresh(obj_or_kind, res)
        return res

    async def delete(self, obj_or_kind, name=None, namespace=None, preconditions=None, propagation="Background"):
        if isinstance(obj_or_kind, dict):
            name = name or obj_or_kind["metadata"]["name"]
            namespace = namespace or obj_or_kind["metadata"].get("namespace")
        return await self.store.delete(obj_or_kind, name, namespace, preconditions, propagation)


def in_process_manager(store: ObjectStore, name: str = "manager", uncached: Sequence = (), **kw) -> Manager:
    """A manager whose reads, writes and watches go straight to ``store``."""
    reader = StoreReader(store)
    writer = InProcessClient(store, user=f"system:serviceaccount:{name}")
    client = CachedClient(reader, writer, uncached)
    return Manager(client, reader, StoreEventSource(store), name=name, **kw)
