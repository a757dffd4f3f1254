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
the shard that will own it).  A hash spreads a handful of namespaces unevenly (measured:
16 per shard over 4 shards came out 13/17/10/24, ``bench.py --namespaces-per-rank``), so
``policy="balanced"`` (the mi355x-sharded overlay's) gives a new namespace to the shard
that owns the fewest, ties going to the hash's shard (unlabelled namespaces planned in
creation order, :meth:`NamespaceShardAssigner.plan`): every assigner computes the same
answer from its Namespace cache and claims it only if it is its own, with a
resourceVersion-preconditioned update, so two assigners with different views cannot both
win; if the chosen shard is down, the hash's shard claims the namespace after ``grace_s``.  Administrators pin a namespace to a shard —
e.g. to keep a team's notebooks on the shard co-located with its GPUs — by setting the
label themselves; an existing label is never changed.  Until the label lands, the
``…-unassigned`` webhook configuration (``DoesNotExist`` selector, served by every shard)
still admits the namespace's Notebooks, reading that namespace live.
"""

from __future__ import annotations

import copy
import datetime
import logging
import zlib
from typing import Iterable, Optional

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_conflict, is_not_found
from ..runtime.controller import Request, Result, pred_funcs
from .setup import SHARD_LABEL

log = logging.getLogger("controllers.sharding")

# never labelled: system namespaces hold no Notebooks and churn on cluster upgrades
EXCLUDED_PREFIXES = ("kube-", "openshift")


def _age_s(obj: dict) -> Optional[float]:
    ts = (obj.get("metadata") or {}).get("creationTimestamp")
    try:
        t = datetime.datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=datetime.timezone.utc)
    except (TypeError, ValueError):
        return None
    return (datetime.datetime.now(datetime.timezone.utc) - t).total_seconds()


def shard_for(namespace: str, shard_count: int) -> str:
    return str(zlib.crc32(namespace.encode()) % max(1, shard_count))


class NamespaceShardAssigner:
    """Labels unlabelled namespaces ``crc32(name) % shard_count``.

    ``only_shard=k``: label only the namespaces that hash to shard ``k``.  Every shard runs
    one of these for itself, so a namespace is claimed by the shard that will own it, and no
    single replica is needed to bring new namespaces under management (with one assigner on
    replica 0, a namespace created while replica 0 was down waited for it, whichever shard
    it hashed to).  ``None``: label every namespace (one assigner for all shards)."""

    POLICIES = ("hash", "balanced")

    def __init__(self, client, reader, shard_count: int, exclude: Iterable[str] = (),
                 only_shard: Optional[str] = None, policy: str = "hash", grace_s: float = 5.0):
        if policy not in self.POLICIES:
            raise ValueError(f"unknown shard assignment policy {policy!r}")
        self.client = client
        self.reader = reader
        self.shard_count = int(shard_count)
        self.exclude = set(exclude)
        self.only_shard = only_shard
        self.policy = policy
        self.grace_s = float(grace_s)
        self.assigned = 0
        self.conflicts = 0  # balanced: another shard's assigner claimed it first
        self._plan: Optional[tuple] = None  # (Namespace store version, plan)
        self.plans = 0
        self.plan_hits = 0

    def _eligible(self, ns: dict) -> bool:
        name = m.name(ns)
        return (SHARD_LABEL not in m.labels(ns) and not m.is_deleting(ns) and name not in self.exclude
                and not name.startswith(EXCLUDED_PREFIXES))

    def wants(self, ns: dict) -> bool:
        if not self._eligible(ns):
            return False
        # balanced: any shard may be the target (decided in reconcile, from current loads)
        return (self.policy == "balanced" or self.only_shard is None
                or shard_for(m.name(ns), self.shard_count) == self.only_shard)

    def plan(self) -> dict:
        """balanced: name → shard of every unlabelled namespace, decided greedily in creation
        order (then name) on top of the labelled namespaces' per-shard counts.  Every assigner
        sees the same namespaces, so they agree on the plan even for namespaces created all at
        once (counts from labels alone would still read 0 everywhere and send each to its hash).

        The plan is a function of the Namespace cache alone, so it is kept until the cache's
        Namespace store changes (``store_version``): K namespaces created together and
        reconciled after they are all cached cost one scan of the cluster's namespaces, not K."""
        ver_of = getattr(self.reader, "store_version", None)
        ver = ver_of(kinds.NAMESPACE) if ver_of is not None else None
        if ver is not None and self._plan is not None and self._plan[0] == ver:
            self.plan_hits += 1
            return self._plan[1]
        out = self._compute_plan()
        if ver is not None:
            self._plan = (ver, out)
        return out

    def _compute_plan(self) -> dict:
        self.plans += 1
        n = max(1, self.shard_count)
        loads = [0] * n
        pending = []
        for ns in self.reader.list(kinds.NAMESPACE):
            lab = m.labels(ns).get(SHARD_LABEL, "")
            if lab.isdigit() and int(lab) < n:
                loads[int(lab)] += 1
            elif self._eligible(ns):
                pending.append(ns)
        pending.sort(key=lambda o: ((o.get("metadata") or {}).get("creationTimestamp") or "", m.name(o)))
        out = {}
        for o in pending:
            h = int(shard_for(m.name(o), n))
            k = min(range(n), key=lambda i: (loads[i], (i - h) % n))
            loads[k] += 1
            out[m.name(o)] = str(k)
        return out

    def target(self, name: str) -> str:
        if self.policy == "hash":
            return shard_for(name, self.shard_count)
        return self.plan().get(name) or shard_for(name, self.shard_count)

    async def reconcile(self, req: Request) -> Result:
        ns = self.reader.get(kinds.NAMESPACE, req.name)
        if ns is None or not self.wants(ns):
            return Result()
        shard = self.target(req.name)
        if self.only_shard is not None and shard != self.only_shard:
            # another shard's to claim; the hash's shard stands in if that one never does
            if shard_for(req.name, self.shard_count) != self.only_shard:
                return Result()
            age = _age_s(ns)
            if age is not None and age < self.grace_s:
                return Result(requeue_after=self.grace_s - age + 0.05)
            shard = self.only_shard
        try:
            if self.policy == "hash":
                await self.client.patch(kinds.NAMESPACE, {"metadata": {"labels": {SHARD_LABEL: shard}}},
                                        name=req.name)
            else:  # preconditioned: of two assigners with different views, one wins
                obj = copy.deepcopy(ns)
                obj["metadata"].setdefault("labels", {})[SHARD_LABEL] = shard
                await self.client.update(obj)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            if is_conflict(e):
                self.conflicts += 1
                return Result(requeue=True)  # re-read: labelled by the winner, or retry
            raise
        self.assigned += 1
        log.info("namespace %s assigned to control-plane shard %s (%s)", req.name, shard, self.policy)
        return Result()

    def setup_with_manager(self, mgr):
        pred = pred_funcs(create=self.wants, update=lambda o, old: self.wants(o), delete=lambda o: False)
        return mgr.builder().named("shard-assigner").for_(kinds.NAMESPACE, [pred]).complete(self)
