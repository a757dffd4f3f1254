"""Controller wiring shared by every process that runs the controllers.

``cmd/kf_manager.py``, ``cmd/odh_manager.py``, ``cmd/control_plane.py`` (the sharded
process the MI355X overlay deploys and the headline benchmark runs) and the in-process
test cluster all register the reconcilers through these functions, so what is tested
and benchmarked is wired exactly as what is deployed.

Reference counterparts: ``kf/main.go:100-123`` (NotebookReconciler, optional
CullingReconciler when ``ENABLE_CULLING=true``) and ``odh/main.go:202-227``
(OpenshiftNotebookReconciler + the mutating webhook).

``reference_emulation`` reproduces the reference's serialising behaviour for
same-harness comparisons: one worker per controller, no watch predicates or own-write
echo suppression, an unconditional status write per reconcile, a namespace List to find
the StatefulSet, and the blocking 1 s + 5 s lock-removal backoff.
"""

from __future__ import annotations

import logging
import os
from typing import Dict, Mapping, Optional

log = logging.getLogger("setup")

SHARD_LABEL = "notebooks.amd.com/shard"


def setup_kf(mgr, env: Mapping[str, str] = os.environ, *, culling: Optional[bool] = None, activity=None,
             event_reemit: bool = True, reference_emulation: bool = False) -> Dict[str, object]:
    """kf manager controllers on ``mgr``: NotebookReconciler, the Pod/StatefulSet event
    re-emitter and (``ENABLE_CULLING=true``) the CullingReconciler."""
    from .metrics import NotebookMetrics
    from .notebook import NotebookEventReemitter, NotebookReconciler

    emu = reference_emulation
    mgr.skip_own_write_echoes = not emu
    one = 1 if emu else None
    out: Dict[str, object] = {}
    metrics = out["metrics"] = NotebookMetrics(mgr.reader, mgr.registry)
    r = out["notebook"] = NotebookReconciler(mgr.client, mgr.reader, mgr.get_event_recorder_for("notebook-controller"),
                                             metrics, env=env, unconditional_status=emu, owner_index=not emu,
                                             event_filters=not emu)
    r.setup_with_manager(mgr, max_concurrent=one)
    if event_reemit:
        e = out["events"] = NotebookEventReemitter(mgr.client, mgr.reader,
                                                   mgr.get_event_recorder_for("notebook-controller"))
        e.setup_with_manager(mgr, max_concurrent=one)
    if culling is None:
        culling = (env.get("ENABLE_CULLING") or "false") == "true"
    if culling:
        from .culling import CullingReconciler

        c = out["culler"] = CullingReconciler(mgr.client, mgr.reader, metrics, env=env, activity=activity)
        c.setup_with_manager(mgr, max_concurrent=one)
    else:
        log.info("Culling of idle Pods is Disabled. To enable it set the ENV Var 'ENABLE_CULLING=true'")
    return out


def setup_event_reemitter(mgr, *, reference_emulation: bool = False):
    """The Pod/StatefulSet event re-emitter alone (``--controllers events``; the reference runs it
    in the kf manager, ``kf/controllers/notebook_controller.go:778-826``).  Its work is one
    reconcile and one Event write per platform Event, none of it on a notebook's create→Ready
    path, so the shard pod runs it beside the culler — a process that already watches the
    Notebooks and Pods it maps Events with — rather than in the notebook reconciler's."""
    from .notebook import NotebookEventReemitter

    mgr.skip_own_write_echoes = not reference_emulation
    e = NotebookEventReemitter(mgr.client, mgr.reader, mgr.get_event_recorder_for("notebook-controller"))
    e.setup_with_manager(mgr, max_concurrent=1 if reference_emulation else None)
    return e


def setup_culler(mgr, env: Mapping[str, str] = os.environ, *, activity=None, reference_emulation: bool = False):
    """The CullingReconciler alone (``--controllers culler``: the culler in a process of its
    own, so its periodic checks of every resident notebook never queue a notebook's create→Ready
    work behind them).  Off unless ``ENABLE_CULLING=true``, as in the kf manager."""
    from .culling import CullingReconciler
    from .metrics import CullerMetrics

    if (env.get("ENABLE_CULLING") or "false") != "true":
        log.info("Culling of idle Pods is Disabled. To enable it set the ENV Var 'ENABLE_CULLING=true'")
        return None
    mgr.skip_own_write_echoes = not reference_emulation
    c = CullingReconciler(mgr.client, mgr.reader, CullerMetrics(mgr.registry), env=env, activity=activity)
    c.setup_with_manager(mgr, max_concurrent=1 if reference_emulation else None)
    return c


def setup_odh(mgr, namespace: str, env: Mapping[str, str] = os.environ, *, shard: Optional[str] = None,
              reference_emulation: bool = False):
    """The odh reconciler on ``mgr``.  ``shard``: label this shard's HTTPRoutes (they live in
    the shared controller namespace) so each shard's cache selects only its own."""
    from .odh.reconciler import OpenshiftNotebookReconciler

    emu = reference_emulation
    mgr.skip_own_write_echoes = not emu
    r = OpenshiftNotebookReconciler(mgr.client, mgr.reader, namespace, env=env,
                                    recorder=mgr.get_event_recorder_for("odh-notebook-controller"),
                                    blocking_lock_removal=emu,
                                    route_labels={SHARD_LABEL: shard} if shard is not None else None)
    r.setup_with_manager(mgr, max_concurrent=1 if emu else None)
    return r


# the Services each Notebook-owning reconciler reads: kf its <nb> Service (no labels,
# kf/controllers/notebook_controller.go:525-552), odh its <nb>-kube-rbac-proxy (labelled
# notebook-name, odh/controllers/notebook_kube_rbac_auth.go) — a process running one of them
# watches only those, instead of decoding the other's too
OWN_SERVICES = {"notebook": "!notebook-name", "odh": "notebook-name"}


def with_own_services(cache_options: dict, role: str) -> dict:
    """``cache_options`` with the Service label selector of ``role`` (``notebook`` / ``odh``)."""
    from ..models import kinds

    sel = OWN_SERVICES.get(role)
    if not sel:
        return cache_options
    return {**cache_options, "selectors": {**(cache_options.get("selectors") or {}), kinds.SERVICE: sel}}


def odh_namespace_labels() -> Dict[str, str]:
    """The odh reconciler's objects outside the notebooks' namespaces, by the label naming the
    notebook namespace they belong to: a namespace-restricted cache (a shard, a worker) lists
    and watches only its own (``InformerCache`` ``namespace_labels``)."""
    from ..models import kinds

    return {kinds.CLUSTER_ROLE_BINDING: "opendatahub.io/namespace",  # controllers/odh/auth.py
            kinds.HTTP_ROUTE: "notebook-namespace"}  # controllers/odh/route.py (central namespace)


def shard_cache_options(shard: Optional[str], controller_namespace: str, cluster_watch: bool = False) -> dict:
    """InformerCache keyword arguments for one shard: the namespaces labelled
    ``notebooks.amd.com/shard=<shard>`` (followed live) plus the controller namespace, with
    HTTPRoutes selected by the same label (``{}`` when not sharded: cluster-wide).
    ``cluster_watch``: one cluster-wide watch per kind filtered here, instead of one per namespace."""
    from ..models import kinds

    if shard is None:
        return {}
    sel = f"{SHARD_LABEL}={shard}"
    return {"namespace_selector": sel, "namespaces": [controller_namespace], "selectors": {kinds.HTTP_ROUTE: sel},
            "cluster_watch": cluster_watch, "namespace_labels": odh_namespace_labels()}
