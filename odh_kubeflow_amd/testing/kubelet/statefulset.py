"""Fake kube-controller-manager StatefulSet controller.

envtest runs no controllers (``kf/controllers/notebook_controller_bdd_test.go:73-76``);
to measure create→Ready latency without a cluster ("fake
kubelet") this turns StatefulSets into ordinal pods ``<sts>-<i>``, rolls pods whose
template changed, scales down to ``replicas``, and maintains ``status``
(``replicas``/``readyReplicas``/``currentReplicas``/``availableReplicas``/
``observedGeneration``) from the pods it owns.
"""

from __future__ import annotations

import hashlib
import json
import logging
from typing import Optional

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_conflict, is_not_found
from ...runtime.controller import Request, Result, enqueue_for_owner
from ...utils.objutil import deepcopy_json

log = logging.getLogger(__name__)

REVISION_LABEL = "controller-revision-hash"
# which node-platform worker (StatefulSet controller + kubelet process pair) owns a
# namespace (NamespaceClaimer)
WORKER_LABEL = "testing.odh-kubeflow-amd/platform-worker"
# never claimed (cluster-lifetime namespaces, no notebooks): worker 0 owns them unlabelled
SYSTEM_NAMESPACES = ("default",)
SYSTEM_PREFIXES = ("kube-", "openshift")


def is_system_namespace(name: str) -> bool:
    return name in SYSTEM_NAMESPACES or name.startswith(SYSTEM_PREFIXES)


def worker_owns(ns: dict, index: int) -> bool:
    """Whether platform worker ``index`` serves the namespace ``ns`` (a Namespace object)."""
    md = ns.get("metadata") or {}
    w = (md.get("labels") or {}).get(WORKER_LABEL)
    if w is None:
        return index == 0 and is_system_namespace(md.get("name", ""))
    return w == str(index)


def template_hash(sts: dict) -> str:
    tmpl = (sts.get("spec") or {}).get("template") or {}
    h = hashlib.sha1(json.dumps(tmpl, sort_keys=True, separators=(",", ":")).encode(),
                    usedforsecurity=False).hexdigest()[:10]
    return f"{m.name(sts)}-{h}"


def pod_is_ready(pod: dict) -> bool:
    for c in ((pod.get("status") or {}).get("conditions") or []):
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False


class StatefulSetController:
    def __init__(self, client, reader, recorder):
        self.client = client
        self.reader = reader
        self.recorder = recorder
        self._created: set = set()  # (sts uid, ordinal) of pods this controller has created
        self._rev: dict = {}  # (sts uid, generation) -> template hash: the template changes only with generation
        self._status: dict = {}  # sts uid -> the status this controller last wrote

    def _pod_for(self, sts: dict, ordinal: int, rev: str) -> dict:
        tmpl = (sts.get("spec") or {}).get("template") or {}
        md = deepcopy_json(tmpl.get("metadata") or {})
        md["name"] = f"{m.name(sts)}-{ordinal}"
        md["namespace"] = m.namespace(sts)
        labels = md.setdefault("labels", {})
        labels[REVISION_LABEL] = rev
        labels["statefulset.kubernetes.io/pod-name"] = md["name"]
        labels["apps.kubernetes.io/pod-index"] = str(ordinal)
        md.setdefault("annotations", {})
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": deepcopy_json(tmpl.get("spec") or {}),
               "status": {"phase": "Pending"}}
        pod["spec"]["hostname"] = md["name"]
        m.set_controller_reference(sts, pod)
        return pod

    async def reconcile(self, req: Request) -> Result:
        sts = await self.client.get_or_none(kinds.STATEFUL_SET, req.name, req.namespace)
        if sts is None or m.is_deleting(sts):
            return Result()
        replicas = int((sts.get("spec") or {}).get("replicas", 1) or 0)
        key = (m.uid(sts), (sts.get("metadata") or {}).get("generation"))
        rev = self._rev.get(key)
        if rev is None:
            if len(self._rev) > 65536:
                self._rev.clear()
            rev = self._rev[key] = template_hash(sts)
        pods = [p for p in self.reader.list(kinds.POD, req.namespace, owner_uid=m.uid(sts)) if m.is_controlled_by(p, sts)]
        by_ord = {}
        for p in pods:
            try:
                by_ord[int(m.name(p).rsplit("-", 1)[1])] = p
            except (IndexError, ValueError):
                continue
        for i in range(replicas):
            p = by_ord.get(i)
            if p is None:
                if (m.uid(sts), i) in self._created and not await self._still_exists(sts):
                    # the pod went away because its StatefulSet was deleted (GC), and the STS
                    # DELETED event has not reached this cache yet: do not resurrect it
                    return Result()
                self._created.add((m.uid(sts), i))
                if len(self._created) > 65536:
                    self._created.clear()
                try:
                    await self.client.create(self._pod_for(sts, i, rev))
                    self.recorder.event(sts, "Normal", "SuccessfulCreate",
                                        f"create Pod {m.name(sts)}-{i} in StatefulSet {m.name(sts)} successful")
                except ApiError as e:
                    if not is_already_exists(e):
                        raise
            elif m.labels(p).get(REVISION_LABEL) != rev and not m.is_deleting(p):
                # RollingUpdate: replace pods built from an outdated template
                await self._delete_pod(sts, p)
        for i, p in by_ord.items():
            if i >= replicas and not m.is_deleting(p):
                await self._delete_pod(sts, p)
        await self._update_status(sts, rev)
        return Result()

    async def _still_exists(self, sts: dict) -> bool:
        from ...runtime.client import LIVE_READS

        tok = LIVE_READS.set(True)
        try:
            live = await self.client.get_or_none(kinds.STATEFUL_SET, m.name(sts), m.namespace(sts))
        finally:
            LIVE_READS.reset(tok)
        return live is not None and m.uid(live) == m.uid(sts) and not m.is_deleting(live)

    async def _delete_pod(self, sts: dict, p: dict) -> None:
        try:
            await self.client.delete(kinds.POD, m.name(p), m.namespace(p))
            self.recorder.event(sts, "Normal", "SuccessfulDelete",
                                f"delete Pod {m.name(p)} in StatefulSet {m.name(sts)} successful")
        except ApiError as e:
            if not is_not_found(e):
                raise

    async def _update_status(self, sts: dict, rev: str) -> None:
        pods = [p for p in self.reader.list(kinds.POD, m.namespace(sts), owner_uid=m.uid(sts))
                if m.is_controlled_by(p, sts) and not m.is_deleting(p)]
        ready = sum(1 for p in pods if pod_is_ready(p))
        current = sum(1 for p in pods if m.labels(p).get(REVISION_LABEL) == rev)
        st = {"replicas": len(pods), "readyReplicas": ready, "currentReplicas": current, "updatedReplicas": current,
              "availableReplicas": ready, "currentRevision": rev, "updateRevision": rev,
              "observedGeneration": (sts.get("metadata") or {}).get("generation", 1)}
        uid = m.uid(sts)
        if (sts.get("status") or {}) != st and self._status.get(uid) != st:
            # (the second test: the cache may not show our last write yet — pod events arrive
            # in bursts and each one reconciles the StatefulSet)
            if len(self._status) > 65536:
                self._status.clear()
            try:
                await self.client.patch(sts, [{"op": "add", "path": "/status", "value": st}], "json",
                                        subresource="status")
                self._status[uid] = st
            except ApiError as e:
                if not is_not_found(e):
                    raise

    def setup_with_manager(self, mgr, max_concurrent: Optional[int] = None):
        b = (mgr.builder().named("statefulset").for_(kinds.STATEFUL_SET)
             .watches(kinds.POD, enqueue_for_owner("StatefulSet", "apps")))
        if max_concurrent:
            b.with_options(max_concurrent_reconciles=max_concurrent)
        return b.complete(self)


class NamespaceClaimer:
    """Balances namespaces over W node-platform workers.

    kube-controller-manager is one Go process syncing StatefulSets concurrently, and a
    kubelet one Go process running pod workers concurrently; the Python stand-ins run W
    processes of each instead, worker i of both watching only the namespaces labelled
    ``WORKER_LABEL=i`` (``InformerCache(namespace_filter=…)``).  The StatefulSet workers
    claim.  A new namespace is
    claimed by the worker that owns the fewest (ties: the lowest index) — every worker
    computes the same answer from its Namespace cache and only that one writes, with the
    namespace's resourceVersion as precondition, so a worker whose cache lags cannot
    double-claim.  System namespaces (``default``, ``kube-*``, ``openshift*``) are never
    claimed and not counted: worker 0 serves them.  A hash of the name would be simpler, but
    over the handful of namespaces a node's notebooks live in it is lumpy (4 ``bench-r``
    names, W=2: all four on one worker)."""

    RECHECK_S = 0.05  # an unclaimed namespace another worker should take: look again
    TAKEOVER_S = 2.0  # ... still unclaimed after this (its worker is gone): any worker claims it

    def __init__(self, client, reader, index: int, workers: int):
        self.client = client
        self.reader = reader
        self.index = int(index)
        self.workers = int(workers)
        self.claimed = 0
        self._mine: set = set()  # claims of this worker its cache may not show yet
        self._waiting: dict = {}  # namespace -> monotonic time this worker first left it to another

    async def reconcile(self, req: Request) -> Result:
        ns = self.reader.get(kinds.NAMESPACE, req.name)
        if ns is None or m.is_deleting(ns) or WORKER_LABEL in m.labels(ns) or is_system_namespace(req.name):
            return Result()
        load = [0] * self.workers
        seen = set()
        for x in self.reader.list(kinds.NAMESPACE):
            w = m.labels(x).get(WORKER_LABEL)
            if w is not None and w.isdigit() and int(w) < self.workers:
                load[int(w)] += 1
                seen.add(m.name(x))
        self._mine &= {m.name(x) for x in self.reader.list(kinds.NAMESPACE)}
        load[self.index] += len(self._mine - seen)
        if min(range(self.workers), key=lambda i: (load[i], i)) != self.index:
            # the least-loaded worker claims it; should its cache lag behind claims this one
            # already sees (or the other way round), both decide again shortly — and should
            # that worker be gone, this one takes the namespace over after TAKEOVER_S
            import time

            first = self._waiting.setdefault(req.name, time.monotonic())
            if time.monotonic() - first < self.TAKEOVER_S:
                return Result(requeue_after=self.RECHECK_S)
        self._waiting.pop(req.name, None)
        self._mine.add(req.name)  # before the write: a concurrent decision must count it
        try:
            await self.client.patch(kinds.NAMESPACE, {"metadata": {
                "resourceVersion": m.resource_version(ns), "labels": {WORKER_LABEL: str(self.index)}}},
                "merge", name=m.name(ns))
            self.claimed += 1
        except ApiError as e:
            self._mine.discard(req.name)
            if is_conflict(e):  # claimed (or changed) meanwhile: decide again on the new version
                return Result(requeue=True)
            if not is_not_found(e):
                raise
        return Result()

    def setup_with_manager(self, mgr):
        # one decision at a time: each counts the claims before it
        return (mgr.builder().named("namespace-claimer").for_(kinds.NAMESPACE)
                .with_options(max_concurrent_reconciles=1).complete(self))
