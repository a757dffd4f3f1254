"""OpenDataHub notebook reconciler (reference ``odh/controllers/notebook_controller.go``).

Pipeline per Notebook (``Reconcile`` :178-497):

* **deleting** → legacy OAuthClient cleanup, HTTPRoute delete (central namespace),
  ReferenceGrant delete iff last notebook, auth ClusterRoleBinding delete; finalizers
  of the successful cleanups are removed even when others failed (partial progress),
  failures are retried (:195-321);
* ensure the ``httproute-cleanup`` / ``referencegrant-cleanup`` (+ ``kube-rbac-proxy-
  cleanup`` in auth mode) finalizers, then requeue (:323-369);
* trusted-CA bundle (+ un-mount when the bundle vanished), NetworkPolicies,
  runtime-images ConfigMap, [``SET_PIPELINE_RBAC``] RoleBinding,
  [``SET_PIPELINE_SECRET``] Elyra Secret, ReferenceGrant, then either the auth branch
  (SA, CRB, kube-rbac-proxy ConfigMap/Service/HTTPRoute) or the plain HTTPRoute, each
  after deleting the other mode's route;
* remove the webhook's reconciliation lock (``kubeflow-resource-stopped:
  odh-notebook-controller-lock``) so the kf controller scales the StatefulSet to 1.

**The lock removal does not sleep in the worker.**  The reference waits for the
notebook ServiceAccount's image-pull secret with a blocking 1 s + 5 s backoff
(:143-174) on a single worker, which serialises notebook start-up (≈6·k s for the
k-th of N simultaneous notebooks).  Here:

* the wait only happens where pull secrets are actually injected
  (``LOCK_WAIT_FOR_PULL_SECRET``: ``auto`` = only on OpenShift, i.e. when the
  ``image.openshift.io`` API is served; ``true`` / ``false`` force it);
* waiting is a ``RequeueAfter`` plus a watch on the owned ServiceAccount (the
  OpenShift token controller adding the pull secret re-triggers the reconcile at
  once), bounded by the reference's 6 s total budget, after which the lock is removed
  anyway (best effort, as in the reference);
* workers are concurrent (``max_concurrent_reconciles`` default 8).

``blocking_lock_removal=True`` reproduces the reference's blocking behaviour for
side-by-side benchmarks.
"""

from __future__ import annotations

import asyncio
import logging
import os
import time
from typing import Dict, List, Mapping, Optional

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_no_match, is_not_found
from ...runtime.controller import (Request, Result, controller_owner_alive, fields_changed,
                                   generation_or_metadata_changed)
from ...runtime.retry import retry_on_conflict
from ...tracing import get_tracer
from . import auth, certs, dspa_secret, network, oauth, rbac, route, runtime_images
from .constants import (ANNOTATION_VALUE_RECONCILIATION_LOCK, HTTPROUTE_FINALIZER, KUBE_RBAC_PROXY_FINALIZER,
                        ODH_CONFIGMAP_NAME, REFERENCE_GRANT_NAME, REFERENCEGRANT_FINALIZER, SELF_SIGNED_CONFIGMAP_NAME,
                        SERVICE_CA_CONFIGMAP_NAME, STOP_ANNOTATION, WORKBENCH_CA_CONFIGMAP_NAME)

log = logging.getLogger("controllers.odh")
tracer = get_tracer("odh_kubeflow_amd/controllers/odh/reconciler")

NOTEBOOK_KIND = kinds.NOTEBOOK_V1
LOCK_WAIT_BUDGET_S = 6.0  # the reference's 1 s + 5 s backoff
LOCK_POLL_S = 0.25


def env_true(env: Mapping[str, str], key: str) -> bool:
    return (env.get(key) or "").strip().lower() == "true"


def reconciliation_lock_enabled(nb: dict) -> bool:
    return m.annotations(nb).get(STOP_ANNOTATION) == ANNOTATION_VALUE_RECONCILIATION_LOCK


class OpenshiftNotebookReconciler:
    def __init__(self, client, reader, namespace: str, env: Optional[Mapping[str, str]] = None, recorder=None,
                 blocking_lock_removal: bool = False, store_info=None,
                 route_labels: Optional[Mapping[str, str]] = None):
        self.client = client
        self.route_labels = dict(route_labels or {})  # sharded control plane: the shard's label
        self.reader = reader
        self.namespace = namespace  # central (controller) namespace
        self.env = env if env is not None else os.environ
        self.recorder = recorder
        self.blocking_lock_removal = blocking_lock_removal
        self._lock_wait_start: Dict[str, float] = {}
        self.locks_removed = 0
        self._openshift: Optional[bool] = None

    # -------------------------------------------------------------- lock

    async def _is_openshift(self) -> bool:
        if self._openshift is None:
            try:
                await self.client.list(kinds.IMAGE_STREAM, self.namespace)
                self._openshift = True
            except ApiError as e:
                self._openshift = not is_no_match(e)
        return self._openshift

    async def _wait_for_pull_secret(self) -> bool:
        mode = (self.env.get("LOCK_WAIT_FOR_PULL_SECRET") or "auto").strip().lower()
        if mode in ("false", "0", "no"):
            return False
        if mode in ("true", "1", "yes"):
            return True
        return await self._is_openshift()

    @staticmethod
    def pod_service_account(nb: dict) -> str:
        spec = ((nb.get("spec") or {}).get("template") or {}).get("spec") or {}
        return spec.get("serviceAccountName") or spec.get("serviceAccount") or "default"

    async def _sa_has_pull_secret(self, nb: dict, sa_name: Optional[str] = None) -> bool:
        try:
            sa = await self.client.get(kinds.SERVICE_ACCOUNT, sa_name or m.name(nb), m.namespace(nb))
        except ApiError:
            return False
        return bool(sa.get("imagePullSecrets"))

    async def remove_reconciliation_lock(self, nb: dict) -> Optional[Result]:
        """Drop the lock annotation; returns a RequeueAfter while still waiting for the pull secret."""
        if self.blocking_lock_removal:
            # reference emulation: retry.OnError(Backoff{Steps:3, 1s, x5}) blocking the worker
            for delay in (1.0, 5.0, None):
                if await self._sa_has_pull_secret(nb):
                    break
                if delay is None:
                    break
                await asyncio.sleep(delay)
        elif await self._wait_for_pull_secret() and not await self._sa_has_pull_secret(
                nb, self.pod_service_account(nb)):
            # wait on the ServiceAccount the pod will actually run as (the reference checks
            # the SA named like the notebook, which does not exist outside auth mode)
            key = m.uid(nb)
            t0 = self._lock_wait_start.setdefault(key, time.monotonic())
            left = LOCK_WAIT_BUDGET_S - (time.monotonic() - t0)
            if left > 0:
                return Result(requeue_after=min(LOCK_POLL_S, left))
            log.info("pull secret not mounted in SA %s/%s after %.0fs; removing lock anyway",
                     m.namespace(nb), m.name(nb), LOCK_WAIT_BUDGET_S)
        self._lock_wait_start.pop(m.uid(nb), None)
        await self.client.patch(nb, {"metadata": {"annotations": {STOP_ANNOTATION: None}}}, "merge")
        self.locks_removed += 1
        return None

    # -------------------------------------------------------------- reconcile

    async def reconcile(self, req: Request) -> Result:
        with tracer.start_span("odh.reconcile", {"notebook": req.name, "namespace": req.namespace}):
            return await self._reconcile(req)

    async def _reconcile(self, req: Request) -> Result:
        try:
            nb = await self.client.get(NOTEBOOK_KIND, req.name, req.namespace)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            raise
        if m.is_deleting(nb):
            return await self._finalize(nb)

        want = [f for f in (HTTPROUTE_FINALIZER, REFERENCEGRANT_FINALIZER) if not m.contains_finalizer(nb, f)]
        if auth.kube_rbac_proxy_injection_enabled(nb) and not m.contains_finalizer(nb, KUBE_RBAC_PROXY_FINALIZER):
            want.append(KUBE_RBAC_PROXY_FINALIZER)
        if want:
            async def add():
                cur = await self.client.get(NOTEBOOK_KIND, req.name, req.namespace)
                if any([m.add_finalizer(cur, f) for f in want]):
                    await self.client.update(cur)
                return cur

            nb = await retry_on_conflict(add)
            if self.blocking_lock_removal:
                return Result(requeue=True)  # reference emulation: work happens on the next pass
            # The reference returns Requeue:true here and does the work on the next pass;
            # the finalizers are durable now, so carry on with the fresh object instead of
            # paying a second queue round-trip on the create→Ready path.

        await certs.create_notebook_cert_configmap(self.client, nb)
        if await certs.is_configmap_deleted(self.client, nb):
            await certs.unset_notebook_cert_config(self.client, nb)

        # The reference runs these sub-reconcilers one after another; they touch disjoint
        # objects, so here they run concurrently (one apiserver round trip of latency for
        # the whole fan-out instead of one per object).  Order is kept only where it
        # matters: the conflicting route goes before the new one.
        c, ns = self.client, self.namespace
        steps = [network.reconcile_all_network_policies(c, nb, ns),
                 runtime_images.sync_runtime_images_configmap(c, m.namespace(nb), ns)]
        if env_true(self.env, "SET_PIPELINE_RBAC"):
            steps.append(rbac.reconcile_role_bindings(c, nb))
        if env_true(self.env, "SET_PIPELINE_SECRET"):
            steps.append(dspa_secret.sync_elyra_runtime_config_secret(c, nb))
        steps.append(route.reconcile_reference_grant(c, nb, ns))
        if auth.kube_rbac_proxy_injection_enabled(nb):
            async def routes():
                await route.ensure_conflicting_httproute_absent(c, nb, ns, True)
                await route.reconcile_httproute(c, nb, ns, route.new_kube_rbac_proxy_httproute, self.env,
                                                self.route_labels)

            steps += [auth.reconcile_notebook_service_account(c, nb), auth.reconcile_kube_rbac_proxy_crb(c, nb),
                      auth.reconcile_kube_rbac_proxy_configmap(c, nb), auth.reconcile_kube_rbac_proxy_service(c, nb),
                      routes()]
        else:
            async def routes():
                await route.ensure_conflicting_httproute_absent(c, nb, ns, False)
                await route.reconcile_httproute(c, nb, ns, route.new_notebook_httproute, self.env,
                                                self.route_labels)

            steps += [auth.cleanup_kube_rbac_proxy_crb(c, nb), routes()]
        if self.blocking_lock_removal:  # reference emulation: strictly sequential
            for i, st in enumerate(steps):
                try:
                    await st
                except BaseException:
                    for rest in steps[i + 1:]:
                        rest.close()  # never started: no "coroutine was never awaited"
                    raise
        else:
            results = await asyncio.gather(*steps, return_exceptions=True)
            errs = [r for r in results if isinstance(r, BaseException)]
            if errs:
                raise errs[0]

        if reconciliation_lock_enabled(nb):
            res = await self.remove_reconciliation_lock(nb)
            if res is not None:
                return res
        return Result()

    async def _finalize(self, nb: dict) -> Result:
        if oauth.has_oauth_client_finalizer(nb):
            await oauth.delete_oauth_client(self.client, nb)
            await oauth.remove_oauth_client_finalizer(self.client, nb)
        done: List[str] = []
        errors: List[str] = []
        if m.contains_finalizer(nb, HTTPROUTE_FINALIZER):
            try:
                await route.delete_httproute_for_notebook(self.client, nb, self.namespace)
                done.append(HTTPROUTE_FINALIZER)
            except Exception as e:
                errors.append(str(e))
        if m.contains_finalizer(nb, REFERENCEGRANT_FINALIZER):
            try:
                await route.delete_reference_grant_if_last_notebook(self.client, nb)
                done.append(REFERENCEGRANT_FINALIZER)
            except Exception as e:
                errors.append(str(e))
        proxy_ok = True
        if auth.kube_rbac_proxy_injection_enabled(nb):
            try:
                await auth.cleanup_kube_rbac_proxy_crb(self.client, nb)
            except Exception as e:
                proxy_ok = False
                errors.append(str(e))
        if m.contains_finalizer(nb, KUBE_RBAC_PROXY_FINALIZER) and proxy_ok:
            done.append(KUBE_RBAC_PROXY_FINALIZER)
        if done:
            async def drop():
                try:
                    cur = await self.client.get(NOTEBOOK_KIND, m.name(nb), m.namespace(nb))
                except ApiError as e:
                    if is_not_found(e):
                        return
                    raise
                if any([m.remove_finalizer(cur, f) for f in done]):
                    try:
                        await self.client.update(cur)
                    except ApiError as e:
                        if not is_not_found(e):
                            raise

            await retry_on_conflict(drop)
        self._lock_wait_start.pop(m.uid(nb), None)
        if errors:
            if len(errors) == 1:
                raise RuntimeError(errors[0])
            raise RuntimeError(f"multiple cleanup failures ({len(errors)} errors): " + "; ".join(errors))
        return Result()

    # -------------------------------------------------------------- wiring

    def _first_notebook(self, namespace: str) -> List[Request]:
        """The reference maps namespace-wide objects to the namespace's first Notebook; a
        Notebook being deleted needs none of them (its finalizer is what deletes the
        shared ReferenceGrant), so the first live one is chosen."""
        for nb in self.reader.list(NOTEBOOK_KIND, namespace):
            if not m.is_deleting(nb):
                return [Request(namespace, m.name(nb))]
        return []

    def setup_with_manager(self, mgr, max_concurrent: Optional[int] = None):
        """``SetupWithManager`` (:707-855) — same watch fan-in, plus a status-write filter."""

        def map_route(o: dict):
            if m.namespace(o) != self.namespace:
                return []
            lb = m.labels(o)
            n, ns = lb.get("notebook-name"), lb.get("notebook-namespace")
            return [Request(ns, n)] if n and ns else []

        def map_refgrant(o: dict):
            if m.name(o) != REFERENCE_GRANT_NAME or m.namespace(o) == self.namespace:
                return []
            return self._first_notebook(m.namespace(o))

        def map_configmap(o: dict):
            name, ns = m.name(o), m.namespace(o)
            if name in (ODH_CONFIGMAP_NAME, SELF_SIGNED_CONFIGMAP_NAME, SERVICE_CA_CONFIGMAP_NAME):
                return self._first_notebook(ns)
            if name == WORKBENCH_CA_CONFIGMAP_NAME:
                return [Request(ns, m.name(nb)) for nb in self.reader.list(NOTEBOOK_KIND, ns)
                        if certs.notebook_uses_bundle(nb)]
            return []

        def map_sa(o: dict):  # pull secret landed on the SA a locked notebook's pod will use
            ns = m.namespace(o)
            return [Request(ns, m.name(nb)) for nb in self.reader.list(NOTEBOOK_KIND, ns)
                    if reconciliation_lock_enabled(nb) and self.pod_service_account(nb) == m.name(o)]

        alive, svc_preds, route_preds, nb_preds = [], [], [], [generation_or_metadata_changed]
        if not self.blocking_lock_removal:
            # a deleted Notebook's finalizers already ran: its DELETED event has nothing left
            nb_preds.append(lambda etype, o, old: etype != "DELETED")  # the reference-emulation runs keep every event
            # GC of a deleted Notebook's children queues nothing; a child deleted under a live
            # Notebook (drift) still does
            alive = [controller_owner_alive(self.reader, NOTEBOOK_KIND)]

            def proxy_service(etype, svc, old):  # not the kf Service <nb> the Notebook also controls
                return m.name(svc).endswith(auth.KUBE_RBAC_PROXY_SERVICE_SUFFIX)
            svc_preds = [proxy_service]

            def route_nb_alive(etype, o, old):  # routes are deleted by this controller's finalizer
                if etype != "DELETED":
                    return True
                lb = m.labels(o)
                nb = self.reader.get(NOTEBOOK_KIND, lb.get("notebook-name", ""), lb.get("notebook-namespace", ""))
                return nb is not None and not m.is_deleting(nb)
            # the Gateway implementation's status writes (ResolvedRefs, …) are not drift: the
            # reconcile compares spec + labels only
            route_preds = [route_nb_alive, fields_changed("spec", "metadata.labels")]

        b = (mgr.builder().named("odh-notebook-controller")
             .for_(NOTEBOOK_KIND, nb_preds)
             .owns(kinds.SERVICE_ACCOUNT, alive).owns(kinds.SERVICE, svc_preds + alive)
             .owns(kinds.SECRET, alive).owns(kinds.CONFIG_MAP, alive)
             .owns(kinds.NETWORK_POLICY, alive).owns(kinds.ROLE_BINDING, alive)
             .watches(kinds.SERVICE_ACCOUNT, map_sa)
             .watches(kinds.HTTP_ROUTE, map_route, route_preds)
             .watches(kinds.REFERENCE_GRANT, map_refgrant)
             .watches(kinds.CONFIG_MAP, map_configmap))
        if max_concurrent is not None:
            b.with_options(max_concurrent_reconciles=max_concurrent)
        return b.complete(self)
