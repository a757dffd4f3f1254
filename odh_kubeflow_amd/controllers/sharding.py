"""Namespace → control-plane shard assignment.

The reference runs one notebook-controller and one odh-notebook-controller for the whole
cluster (``kf/main.go:87-98``, ``odh/main.go:155-192``).  The MI355X deployment
(``config/overlays/mi355x-sharded``) runs N shards of ``cmd/control_plane.py`` instead,
each owning the namespaces labelled ``notebooks.amd.com/shard=<k>``: its informers watch
only those namespaces (plus the controller namespace), and its admission webhook is
called only for them (one MutatingWebhookConfiguration per shard, ``namespaceSelector``
on the same label).

A namespace nobody labelled would belong to no shard, so every shard runs this assigner
for itself: shard k labels the unlabelled namespaces whose ``crc32(name) % N`` is k (stable
across restarts and replicas, so assigners never disagree, and a namespace waits only for
the shard that will own it).  Administrators pin a namespace to a shard —
e.g. to keep a team's notebooks on the shard co-located with its GPUs — by setting the
label themselves; an existing label is never changed.  Until the label lands, the
``…-unassigned`` webhook configuration (``DoesNotExist`` selector, served by every shard)
still admits the namespace's Notebooks, reading that namespace live.
"""

from __future__ import annotations

import logging
import zlib
from typing import Iterable, Optional

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_not_found
from ..runtime.controller import Request, Result, pred_funcs
from .setup import SHARD_LABEL

log = logging.getLogger("controllers.sharding")

# never labelled: system namespaces hold no Notebooks and churn on cluster upgrades
EXCLUDED_PREFIXES = ("kube-", "openshift")


def shard_for(namespace: str, shard_count: int) -> str:
    return str(zlib.crc32(namespace.encode()) % max(1, shard_count))


class NamespaceShardAssigner:
    """Labels unlabelled namespaces ``crc32(name) % shard_count``.

    ``only_shard=k``: label only the namespaces that hash to shard ``k``.  Every shard runs
    one of these for itself, so a namespace is claimed by the shard that will own it, and no
    single replica is needed to bring new namespaces under management (with one assigner on
    replica 0, a namespace created while replica 0 was down waited for it, whichever shard
    it hashed to).  ``None``: label every namespace (one assigner for all shards)."""

    def __init__(self, client, reader, shard_count: int, exclude: Iterable[str] = (),
                 only_shard: Optional[str] = None):
        self.client = client
        self.reader = reader
        self.shard_count = int(shard_count)
        self.exclude = set(exclude)
        self.only_shard = only_shard
        self.assigned = 0

    def wants(self, ns: dict) -> bool:
        name = m.name(ns)
        return (SHARD_LABEL not in m.labels(ns) and not m.is_deleting(ns) and name not in self.exclude
                and not name.startswith(EXCLUDED_PREFIXES)
                and (self.only_shard is None or shard_for(name, self.shard_count) == self.only_shard))

    async def reconcile(self, req: Request) -> Result:
        ns = self.reader.get(kinds.NAMESPACE, req.name)
        if ns is None or not self.wants(ns):
            return Result()
        shard = shard_for(req.name, self.shard_count)
        try:
            await self.client.patch(kinds.NAMESPACE, {"metadata": {"labels": {SHARD_LABEL: shard}}}, name=req.name)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            raise
        self.assigned += 1
        log.info("namespace %s assigned to control-plane shard %s", req.name, shard)
        return Result()

    def setup_with_manager(self, mgr):
        pred = pred_funcs(create=self.wants, update=lambda o, old: self.wants(o), delete=lambda o: False)
        return mgr.builder().named("shard-assigner").for_(kinds.NAMESPACE, [pred]).complete(self)
