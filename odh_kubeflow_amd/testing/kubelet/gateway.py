"""Gateway API implementation stand-in — TEST HARNESS ONLY (never deployed).

What a Gateway implementation (OpenShift's data-science gateway, Istio, Envoy Gateway)
reports for an HTTPRoute: per parent, ``Accepted`` and ``ResolvedRefs`` conditions in
``status.parents[]`` (Gateway API v1, ``RouteConditionResolvedRefs``).  A backendRef
resolves when

* its kind is a core ``Service`` (the default),
* a cross-namespace reference is allowed by a ReferenceGrant in the Service's namespace
  (``from`` HTTPRoutes of the route's namespace, ``to`` Services — optionally by name),
* the Service exists, and
* ``port`` is one of the **Service's** ports: Gateway API defines a Service backendRef's
  port as the service port, not the target port.

Otherwise ``ResolvedRefs`` is False with reason ``InvalidKind``, ``RefNotPermitted`` or
``BackendNotFound``, and the implementation answers that rule with HTTP 500.

The odh controller's routes are checked against this: the reference points the
non-auth route at port 8888 (``odh/controllers/notebook_route.go:120``) while the kf
Service listens on 80 (``kf/controllers/notebook_controller.go:49-50,525-552``), so the
reference's plain route never resolves; see ``controllers/odh/route.py``.
"""

from __future__ import annotations

import logging
from typing import List, Optional

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_not_found
from ...runtime.controller import Request, Result
from ...utils.timeutil import rfc3339

log = logging.getLogger("gateway")

CONTROLLER_NAME = "gateway.amd.com/stand-in"


def _grant_allows(grants: List[dict], route_ns: str, svc_name: str) -> bool:
    for g in grants:
        spec = g.get("spec") or {}
        frm = any(f.get("group") == "gateway.networking.k8s.io" and f.get("kind") == "HTTPRoute"
                  and f.get("namespace") == route_ns for f in spec.get("from") or [])
        to = any((t.get("group") or "") == "" and t.get("kind") == "Service"
                 and (not t.get("name") or t.get("name") == svc_name) for t in spec.get("to") or [])
        if frm and to:
            return True
    return False


def resolve_backend(reader, route: dict, br: dict) -> Optional[tuple]:
    """None when ``br`` resolves, else ``(reason, message)``."""
    if (br.get("group") or "") != "" or (br.get("kind") or "Service") != "Service":
        return "InvalidKind", f"backendRef {br.get('group')}/{br.get('kind')} is not a core Service"
    route_ns = m.namespace(route)
    ns, name = br.get("namespace") or route_ns, br.get("name", "")
    if ns != route_ns and not _grant_allows(reader.list(kinds.REFERENCE_GRANT, ns), route_ns, name):
        return "RefNotPermitted", f"no ReferenceGrant in {ns} allows HTTPRoutes from {route_ns} to Service {name}"
    svc = reader.get(kinds.SERVICE, name, ns)
    if svc is None:
        return "BackendNotFound", f"Service {ns}/{name} not found"
    ports = [p.get("port") for p in (svc.get("spec") or {}).get("ports") or []]
    if br.get("port") not in ports:
        return "BackendNotFound", f"port {br.get('port')} is not a port of Service {ns}/{name} (ports {ports})"
    return None


class GatewayRouteResolver:
    def __init__(self, client, reader):
        self.client = client
        self.reader = reader

    async def reconcile(self, req: Request) -> Result:
        route = self.reader.get(kinds.HTTP_ROUTE, req.name, req.namespace)
        if route is None or m.is_deleting(route):
            return Result()
        bad = None
        for rule in (route.get("spec") or {}).get("rules") or []:
            for br in rule.get("backendRefs") or []:
                bad = bad or resolve_backend(self.reader, route, br)
        gen = (route.get("metadata") or {}).get("generation")
        prev = {(p.get("parentRef", {}).get("name"), c.get("type")): c
                for p in (route.get("status") or {}).get("parents") or [] for c in p.get("conditions") or []}
        parents = []
        for pr in (route.get("spec") or {}).get("parentRefs") or []:
            conds = [("Accepted", "True", "Accepted", "Route is accepted"),
                     ("ResolvedRefs", "False", *bad) if bad else
                     ("ResolvedRefs", "True", "ResolvedRefs", "All references resolved")]
            out = []
            for typ, status, reason, msg in conds:
                old = prev.get((pr.get("name"), typ))
                ltt = old["lastTransitionTime"] if old and old.get("status") == status else rfc3339()
                out.append({"type": typ, "status": status, "reason": reason, "message": msg,
                            "observedGeneration": gen, "lastTransitionTime": ltt})
            parents.append({"parentRef": pr, "controllerName": CONTROLLER_NAME, "conditions": out})
        status = {"parents": parents}
        if status == (route.get("status") or {}):
            return Result()
        try:
            await self.client.patch(kinds.HTTP_ROUTE, [{"op": "add", "path": "/status", "value": status}], "json",
                                    name=req.name, namespace=req.namespace, subresource="status")
        except ApiError as e:
            if not is_not_found(e):
                raise
        return Result()

    def setup_with_manager(self, mgr):
        def routes_to(ns: str, name: Optional[str] = None) -> List[Request]:
            out = []
            for r in self.reader.list(kinds.HTTP_ROUTE):
                for rule in (r.get("spec") or {}).get("rules") or []:
                    if any((br.get("namespace") or m.namespace(r)) == ns and (name is None or br.get("name") == name)
                           for br in rule.get("backendRefs") or []):
                        out.append(Request(m.namespace(r), m.name(r)))
                        break
            return out

        return (mgr.builder().named("gateway-route-resolver").for_(kinds.HTTP_ROUTE)
                .watches(kinds.SERVICE, lambda s: routes_to(m.namespace(s), m.name(s)))
                .watches(kinds.REFERENCE_GRANT, lambda g: routes_to(m.namespace(g)))
                .complete(self))
