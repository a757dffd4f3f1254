"""HTTPRoute backendRefs resolved the way a Gateway API implementation resolves them.

The reference points the plain (non-auth) HTTPRoute at Service port 8888
(``odh/controllers/notebook_route.go:120``) while the kf Service exposes only port 80
(``kf/controllers/notebook_controller.go:49-50,525-552``); Gateway API defines a Service
backendRef's ``port`` as the service port.  The test platform's Gateway stand-in
(``kubelet/gateway.py``) reports ``ResolvedRefs`` like an implementation would: the
routes this controller writes resolve in both modes, the reference's 8888 route does not,
and a reference-era 8888 route is corrected by the drift check.
"""

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook

CENTRAL = "opendatahub"
ENV = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}


def _route(cl, nb):
    rs = [r for r in cl.store.list_nocopy(kinds.HTTP_ROUTE, CENTRAL) if m.labels(r).get("notebook-name") == nb]
    return rs[0] if rs else None


def _resolved(cl, nb):
    r = _route(cl, nb)
    for p in ((r or {}).get("status") or {}).get("parents") or []:
        for c in p.get("conditions") or []:
            if c["type"] == "ResolvedRefs":
                return c["status"], c["reason"], c["message"]
    return None


def test_routes_resolve_in_both_modes_and_reference_port_does_not(run):
    async def go():
        async with LocalCluster(ClusterConfig(odh=True, webhook=True, env=ENV)) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("plain", "user"))
            await cl.admin.create(notebook("authed", "user",
                                           annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
            for nb in ("plain", "authed"):
                assert await cl.wait_for(lambda: cl.notebook_ready(nb, "user"), 10)
                assert await cl.wait_for(lambda: (_resolved(cl, nb) or ("",))[0] == "True", 10), _resolved(cl, nb)
            assert _route(cl, "plain")["spec"]["rules"][0]["backendRefs"][0]["port"] == 80
            assert _route(cl, "authed")["spec"]["rules"][0]["backendRefs"][0]["port"] == 8443

            # the reference's plain route (port 8888): the Service has no such port.  Written
            # with a foreign label set so the controller does not claim it.
            ref = {"apiVersion": "gateway.networking.k8s.io/v1", "kind": "HTTPRoute",
                   "metadata": {"name": "reference-style", "namespace": CENTRAL, "labels": {"notebook-name": "ref"}},
                   "spec": {"parentRefs": [{"name": "data-science-gateway", "namespace": "openshift-ingress"}],
                            "rules": [{"backendRefs": [{"name": "plain", "namespace": "user", "port": 8888}]}]}}
            await cl.admin.create(ref)
            assert await cl.wait_for(lambda: _resolved(cl, "ref") is not None, 10)
            status, reason, msg = _resolved(cl, "ref")
            assert (status, reason) == ("False", "BackendNotFound") and "port 8888" in msg

            # a reference-era route of a managed notebook is moved to the Service port
            await cl.edit(kinds.HTTP_ROUTE, m.name(_route(cl, "plain")), CENTRAL,
                          lambda r: r["spec"]["rules"][0]["backendRefs"][0].__setitem__("port", 8888))
            assert await cl.wait_for(lambda: _route(cl, "plain")["spec"]["rules"][0]["backendRefs"][0]["port"] == 80)
            assert await cl.wait_for(lambda: (_resolved(cl, "plain") or ("",))[0] == "True", 10)
    run(go())


def test_cross_namespace_backend_needs_the_reference_grant(run):
    async def go():
        async with LocalCluster(ClusterConfig(odh=True, webhook=True, env=ENV)) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user"))
            assert await cl.wait_for(lambda: (_resolved(cl, "nb") or ("",))[0] == "True", 10)
            # without the grant the gateway may not reach across namespaces
            rg = await cl.admin.get(kinds.REFERENCE_GRANT, "notebook-httproute-access", "user")
            rg["spec"]["from"][0]["namespace"] = "elsewhere"
            await cl.admin.update(rg)
            # the controller restores its grant (drift), and the route resolves again
            assert await cl.wait_for(lambda: cl.store.peek(kinds.REFERENCE_GRANT, "notebook-httproute-access", "user")
                                     ["spec"]["from"][0]["namespace"] == CENTRAL, 10)
            assert await cl.wait_for(lambda: (_resolved(cl, "nb") or ("",))[0] == "True", 10)
            # without any grant the gateway may not reach across namespaces: the resolver says so
            from odh_kubeflow_amd.testing.kubelet.gateway import resolve_backend

            class NoGrants:
                def list(self, kind, ns=None):
                    return [] if kind == kinds.REFERENCE_GRANT else cl.store.list_nocopy(kind, ns)

                def get(self, kind, name, ns=None):
                    return cl.store.peek(kind, name, ns)
            r = _route(cl, "nb")
            assert resolve_backend(NoGrants(), r, r["spec"]["rules"][0]["backendRefs"][0])[0] == "RefNotPermitted"
    run(go())
