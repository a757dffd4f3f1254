"""Gateway API routing: HTTPRoute in the central namespace + per-namespace ReferenceGrant.

Reference: ``odh/controllers/notebook_route.go`` and ``notebook_referencegrant.go``.

* HTTPRoute ``nb-<ns>-<name>`` lives in the **controller's** namespace (no ownerRef
  possible across namespaces), labelled ``notebook-name`` / ``notebook-namespace`` and
  found by those labels.  Names over 63 chars use ``generateName``
  ``nb-<ns[:10]>-<name[:10]>-`` (:50-74).  parentRef defaults to
  ``openshift-ingress/data-science-gateway`` (``NOTEBOOK_GATEWAY_NAME`` /
  ``NOTEBOOK_GATEWAY_NAMESPACE``).  PathPrefix ``/notebook/<ns>/<name>`` → Service
  ``<name>`` **port 80**.  Deliberate fix: the reference targets port 8888
  (``odh/controllers/notebook_route.go:120``), but the kf Service it routes to exposes
  only port 80 → targetPort 8888 (``kf/controllers/notebook_controller.go:49-50,525-552``),
  and a Gateway API backendRef's ``port`` is the *Service* port.  The reference's plain
  (non-auth) route therefore never resolves (``ResolvedRefs=False/BackendNotFound``;
  ``kubelet/gateway.py`` reproduces what implementations report; its e2e checks only
  the auth route, ``odh/e2e/notebook_creation_test.go:398-411``).  Routes a reference
  controller left at 8888 are recognised as the plain route and corrected to 80 by the
  drift check.
* In auth mode the backend is ``<name>-kube-rbac-proxy`` port 8443, and the route of
  the other mode is deleted on a switch (:269-324).
* ReferenceGrant ``notebook-httproute-access`` in the user namespace lets HTTPRoutes
  from the central namespace reference Services; it is deleted when the last
  non-deleting notebook in the namespace is finalised.
"""

from __future__ import annotations

import logging
import os
from typing import Callable, Mapping, Optional

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_not_found
from ...runtime.retry import retry_on_conflict
from ...models.notebook import DEFAULT_SERVING_PORT as NOTEBOOK_SERVICE_PORT  # the kf Service's port (80)
from .constants import (DEFAULT_GATEWAY_NAME, DEFAULT_GATEWAY_NAMESPACE, HTTPROUTE_SUBDOMAIN_MAX_LEN,
                        KUBE_RBAC_PROXY_PORT, KUBE_RBAC_PROXY_SERVICE_SUFFIX, NOTEBOOK_PORT, REFERENCE_GRANT_NAME)

log = logging.getLogger("controllers.odh.route")


def route_labels(nb: dict) -> dict:
    return {"notebook-name": m.name(nb), "notebook-namespace": m.namespace(nb)}


def new_notebook_httproute(nb: dict, central_namespace: str, env: Mapping[str, str] = os.environ,
                           extra_labels: Optional[Mapping[str, str]] = None) -> dict:
    """``extra_labels``: the owning shard's label when the control plane is sharded (routes
    live in the shared controller namespace; each shard watches only its own)."""
    ns, name = m.namespace(nb), m.name(nb)
    rname = f"nb-{ns}-{name}"
    labels = {**route_labels(nb), **(extra_labels or {})}
    if len(rname) > HTTPROUTE_SUBDOMAIN_MAX_LEN:
        md = {"generateName": f"nb-{ns[:10]}-{name[:10]}-", "namespace": central_namespace, "labels": labels}
    else:
        md = {"name": rname, "namespace": central_namespace, "labels": labels}
    gw_name = env.get("NOTEBOOK_GATEWAY_NAME") or DEFAULT_GATEWAY_NAME
    gw_ns = env.get("NOTEBOOK_GATEWAY_NAMESPACE") or DEFAULT_GATEWAY_NAMESPACE
    return {
        "apiVersion": "gateway.networking.k8s.io/v1", "kind": "HTTPRoute", "metadata": md,
        "spec": {
            "parentRefs": [{"name": gw_name, "namespace": gw_ns}],
            "rules": [{
                "matches": [{"path": {"type": "PathPrefix", "value": f"/notebook/{ns}/{name}"}}],
                "backendRefs": [{"name": name, "namespace": ns, "port": NOTEBOOK_SERVICE_PORT}],
            }],
        },
    }


def new_kube_rbac_proxy_httproute(nb: dict, central_namespace: str, env: Mapping[str, str] = os.environ,
                                  extra_labels: Optional[Mapping[str, str]] = None) -> dict:
    r = new_notebook_httproute(nb, central_namespace, env, extra_labels)
    br = r["spec"]["rules"][0]["backendRefs"][0]
    br["name"] = m.name(nb) + KUBE_RBAC_PROXY_SERVICE_SUFFIX
    br["port"] = KUBE_RBAC_PROXY_PORT
    return r


def _same_route(a: dict, b: dict) -> bool:
    return (m.labels(a) or {}) == (m.labels(b) or {}) and a.get("spec") == b.get("spec")


async def list_routes(client, nb: dict, central_namespace: str):
    return await client.list(kinds.HTTP_ROUTE, central_namespace, labels=route_labels(nb))


async def reconcile_httproute(client, nb: dict, central_namespace: str,
                              new_route: Callable[..., dict],
                              env: Mapping[str, str] = os.environ,
                              extra_labels: Optional[Mapping[str, str]] = None) -> None:
    desired = new_route(nb, central_namespace, env, extra_labels)
    items = await list_routes(client, nb, central_namespace)
    if len(items) > 1:
        raise RuntimeError("multiple HTTPRoutes found for notebook")
    if not items:
        try:
            await client.create(desired)
        except ApiError as e:
            if not is_already_exists(e):
                raise
        return
    found = items[0]
    if _same_route(desired, found):
        return

    async def update():
        cur = await client.get(kinds.HTTP_ROUTE, m.name(found), central_namespace)
        cur["spec"] = desired["spec"]
        cur["metadata"]["labels"] = dict(m.labels(desired))
        await client.update(cur)

    await retry_on_conflict(update)


async def delete_httproute_for_notebook(client, nb: dict, central_namespace: str) -> None:
    errors = []
    for r in await list_routes(client, nb, central_namespace):
        try:
            await client.delete(kinds.HTTP_ROUTE, m.name(r), central_namespace)
        except ApiError as e:
            if not is_not_found(e):
                errors.append(f"failed to delete HTTPRoute {m.name(r)}: {e}")
    if errors:
        raise RuntimeError(f"failed to delete some HTTPRoutes: {errors}")


async def ensure_conflicting_httproute_absent(client, nb: dict, central_namespace: str, auth_mode: bool) -> None:
    for r in await list_routes(client, nb, central_namespace):
        rules = (r.get("spec") or {}).get("rules") or []
        if not rules or not rules[0].get("backendRefs"):
            continue
        br = rules[0]["backendRefs"][0]
        bname, bport = br.get("name"), br.get("port")
        is_proxy = bname == m.name(nb) + KUBE_RBAC_PROXY_SERVICE_SUFFIX or bport == KUBE_RBAC_PROXY_PORT
        is_regular = bname == m.name(nb) or bport in (NOTEBOOK_SERVICE_PORT, NOTEBOOK_PORT)
        if (auth_mode and is_regular) or (not auth_mode and is_proxy):
            log.info("deleting conflicting HTTPRoute %s (auth_mode=%s)", m.name(r), auth_mode)
            try:
                await client.delete(kinds.HTTP_ROUTE, m.name(r), central_namespace)
            except ApiError as e:
                if not is_not_found(e):
                    raise


# ------------------------------------------------------------------ ReferenceGrant


def new_reference_grant(namespace: str, central_namespace: str) -> dict:
    return {
        "apiVersion": "gateway.networking.k8s.io/v1beta1", "kind": "ReferenceGrant",
        "metadata": {"name": REFERENCE_GRANT_NAME, "namespace": namespace,
                     "labels": {"app.kubernetes.io/managed-by": "odh-notebook-controller",
                                "opendatahub.io/component": "notebook-controller"}},
        "spec": {"from": [{"group": "gateway.networking.k8s.io", "kind": "HTTPRoute", "namespace": central_namespace}],
                 "to": [{"group": "", "kind": "Service"}]},
    }


async def reconcile_reference_grant(client, nb: dict, central_namespace: str) -> None:
    desired = new_reference_grant(m.namespace(nb), central_namespace)
    try:
        found = await client.get(kinds.REFERENCE_GRANT, REFERENCE_GRANT_NAME, m.namespace(nb))
    except ApiError as e:
        if not is_not_found(e):
            raise
        try:
            await client.create(desired)
        except ApiError as e2:
            if not is_already_exists(e2):
                raise
        return
    if _same_route(desired, found):
        return
    found["spec"] = desired["spec"]
    found["metadata"]["labels"] = dict(m.labels(desired))
    await client.update(found)


async def is_last_notebook_in_namespace(client, nb: dict) -> bool:
    from ...runtime.client import any_readonly

    name = m.name(nb)
    return not await any_readonly(client, kinds.NOTEBOOK, m.namespace(nb),
                                  lambda other: m.name(other) != name and not m.is_deleting(other))


async def delete_reference_grant_if_last_notebook(client, nb: dict) -> Optional[bool]:
    if not await is_last_notebook_in_namespace(client, nb):
        return False
    try:
        await client.delete(kinds.REFERENCE_GRANT, REFERENCE_GRANT_NAME, m.namespace(nb))
    except ApiError as e:
        if not is_not_found(e):
            raise
    return True
