"""ODH reconciler integration tests on the in-process apiserver (envtest analogue).

Scenario list follows odh/controllers/notebook_controller_test.go: HTTPRoute create /
drift-restore / recreate / delete (:59-179), ReferenceGrant lifecycle and sharing
(:181-362), RoleBinding behind SET_PIPELINE_RBAC (:365-430), CA bundle with real
certificates (:433-534), long names (:537-677), NetworkPolicies (:789-955),
kube-rbac-proxy lifecycle incl. lock removal (:957-1358), mode switching (:1360-1530),
DSPA secret (:1532-1791).  envtest has no GC, so "deleted with the Notebook" is asserted
through ownerReferences (:1316-1328), except where the cluster runs with GC.
"""

import asyncio
import base64
import json
import os
import shutil
import subprocess

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.controllers.odh import certs, dspa_secret
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook

CENTRAL = "opendatahub"
AUTH = {"notebooks.opendatahub.io/inject-auth": "true"}


def cfg(**env):
    # the reference's Makefile runs the whole suite with SET_PIPELINE_RBAC=false and =true
    # (odh/Makefile:106-115); `make test-matrix` does the same through this variable
    base = {"SET_PIPELINE_RBAC": os.environ.get("ODH_TEST_SET_PIPELINE_RBAC", "false"), "SET_PIPELINE_SECRET": "false"}
    base.update(env)
    return ClusterConfig(odh=True, webhook=True, gc=False, env=base)


def route_for(cl, name, ns="user"):
    return [r for r in cl.store.list_nocopy(kinds.HTTP_ROUTE, CENTRAL)
            if m.labels(r).get("notebook-name") == name and m.labels(r).get("notebook-namespace") == ns]


async def create_nb(cl, name, ns="user", **kw):
    await cl.ensure_namespace(ns)
    await cl.admin.create(notebook(name, ns, **kw))


def test_httproute_lifecycle(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await create_nb(cl, "nb")
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1)
            r = route_for(cl, "nb")[0]
            assert m.name(r) == "nb-user-nb"
            assert r["spec"]["parentRefs"] == [{"name": "data-science-gateway", "namespace": "openshift-ingress"}]
            rule = r["spec"]["rules"][0]
            assert rule["matches"] == [{"path": {"type": "PathPrefix", "value": "/notebook/user/nb"}}]
            assert rule["backendRefs"] == [{"name": "nb", "namespace": "user", "port": 80}]
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "user")
            assert {"notebook.opendatahub.io/httproute-cleanup",
                    "notebook.opendatahub.io/referencegrant-cleanup"} <= set(m.finalizers(nb))
            # lock removed without waiting (vanilla Kubernetes: no pull-secret injection)
            assert await cl.wait_for(lambda: "kubeflow-resource-stopped" not in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, "nb", "user")))
            # drift is restored
            await cl.edit(kinds.HTTP_ROUTE, "nb-user-nb", CENTRAL,
                          lambda r: r["spec"]["rules"][0]["backendRefs"][0].__setitem__("port", 9999))
            assert await cl.wait_for(lambda: route_for(cl, "nb")[0]["spec"]["rules"][0]["backendRefs"][0]["port"] == 80)
            # deleted route is recreated
            await cl.admin.delete(kinds.HTTP_ROUTE, "nb-user-nb", CENTRAL)
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1)
            # notebook deletion removes it (finalizer) and the notebook goes away
            await cl.admin.delete(kinds.NOTEBOOK, "nb", "user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "nb", "user") is None)
            assert route_for(cl, "nb") == []
    run(go())


def test_gateway_env_override_and_long_name(run):
    async def go():
        async with LocalCluster(cfg(NOTEBOOK_GATEWAY_NAME="gw", NOTEBOOK_GATEWAY_NAMESPACE="gw-ns")) as cl:
            long_name = "a-very-long-notebook-name-that-exceeds-the-limit-of-routes"
            await create_nb(cl, long_name, ns="long-namespace-for-routes")
            assert await cl.wait_for(lambda: len(route_for(cl, long_name, "long-namespace-for-routes")) == 1)
            r = route_for(cl, long_name, "long-namespace-for-routes")[0]
            assert m.name(r).startswith("nb-long-names-a-very-lon-") and len(m.name(r)) <= 63
            assert r["spec"]["parentRefs"] == [{"name": "gw", "namespace": "gw-ns"}]
            # drift correction works through the label lookup
            await cl.edit(kinds.HTTP_ROUTE, m.name(r), CENTRAL, lambda cur: cur["spec"].__setitem__("parentRefs", []))
            assert await cl.wait_for(lambda: route_for(cl, long_name, "long-namespace-for-routes")[0]["spec"]
                                     ["parentRefs"] == [{"name": "gw", "namespace": "gw-ns"}])
            await cl.admin.delete(kinds.NOTEBOOK, long_name, "long-namespace-for-routes")
            assert await cl.wait_for(lambda: route_for(cl, long_name, "long-namespace-for-routes") == [])
    run(go())


def test_reference_grant_shared_and_deleted_with_last_notebook(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await create_nb(cl, "nb1")
            await create_nb(cl, "nb2")
            rg = lambda: cl.store.peek(kinds.REFERENCE_GRANT, "notebook-httproute-access", "user")  # noqa: E731
            assert await cl.wait_for(lambda: rg() is not None and len(route_for(cl, "nb2")) == 1)
            g = rg()
            assert g["spec"] == {"from": [{"group": "gateway.networking.k8s.io", "kind": "HTTPRoute",
                                           "namespace": CENTRAL}], "to": [{"group": "", "kind": "Service"}]}
            assert m.labels(g) == {"app.kubernetes.io/managed-by": "odh-notebook-controller",
                                   "opendatahub.io/component": "notebook-controller"}
            assert len(cl.store.list_nocopy(kinds.REFERENCE_GRANT, "user")) == 1
            # modified spec and labels are restored; deleted grant is recreated
            cur = await cl.admin.get(kinds.REFERENCE_GRANT, "notebook-httproute-access", "user")
            cur["spec"]["to"] = [{"group": "", "kind": "Secret"}]
            cur["metadata"]["labels"] = {"x": "y"}
            await cl.admin.update(cur)
            assert await cl.wait_for(lambda: rg()["spec"]["to"] == [{"group": "", "kind": "Service"}]
                                     and m.labels(rg()).get("opendatahub.io/component") == "notebook-controller")
            await cl.admin.delete(kinds.REFERENCE_GRANT, "notebook-httproute-access", "user")
            assert await cl.wait_for(lambda: rg() is not None)
            # deleting one notebook keeps it, deleting the last removes it
            await cl.admin.delete(kinds.NOTEBOOK, "nb1", "user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "nb1", "user") is None)
            assert rg() is not None
            await cl.admin.delete(kinds.NOTEBOOK, "nb2", "user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "nb2", "user") is None)
            assert rg() is None
    run(go())


def test_network_policies(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await create_nb(cl, "nb")
            np = lambda n: cl.store.peek(kinds.NETWORK_POLICY, n, "user")  # noqa: E731
            assert await cl.wait_for(lambda: np("nb-ctrl-np") is not None and np("nb-kube-rbac-proxy-np") is not None)
            ctrl = np("nb-ctrl-np")
            assert ctrl["spec"] == {
                "podSelector": {"matchLabels": {"notebook-name": "nb"}},
                "ingress": [{"ports": [{"protocol": "TCP", "port": 8888}],
                             "from": [{"namespaceSelector": {"matchLabels": {"kubernetes.io/metadata.name": CENTRAL}}}]}],
                "policyTypes": ["Ingress"]}
            assert np("nb-kube-rbac-proxy-np")["spec"]["ingress"] == [{"ports": [{"protocol": "TCP", "port": 8443}]}]
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "user")
            for n in ("nb-ctrl-np", "nb-kube-rbac-proxy-np"):
                assert m.is_controlled_by(np(n), nb)
            cur = await cl.admin.get(kinds.NETWORK_POLICY, "nb-ctrl-np", "user")
            cur["spec"]["policyTypes"] = ["Egress"]
            await cl.admin.update(cur)
            assert await cl.wait_for(lambda: np("nb-ctrl-np")["spec"]["policyTypes"] == ["Ingress"])
            await cl.admin.delete(kinds.NETWORK_POLICY, "nb-kube-rbac-proxy-np", "user")
            assert await cl.wait_for(lambda: np("nb-kube-rbac-proxy-np") is not None)
    run(go())


def test_kube_rbac_proxy_full_lifecycle(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await create_nb(cl, "nb", annotations=AUTH)
            get = lambda k, n, ns="user": cl.store.peek(k, n, ns)  # noqa: E731
            assert await cl.wait_for(lambda: all((
                get(kinds.SERVICE_ACCOUNT, "nb"), get(kinds.SERVICE, "nb-kube-rbac-proxy"),
                get(kinds.CONFIG_MAP, "nb-kube-rbac-proxy-config"),
                get(kinds.CLUSTER_ROLE_BINDING, "nb-rbac-user-auth-delegator", None), route_for(cl, "nb"))))
            nb = get(kinds.NOTEBOOK, "nb")
            assert "notebook.opendatahub.io/kube-rbac-proxy-cleanup" in m.finalizers(nb)
            # sidecar in the notebook and therefore in the StatefulSet the kf controller generated
            assert await cl.wait_for(lambda: get(kinds.STATEFUL_SET, "nb") is not None and "kube-rbac-proxy" in [
                c["name"] for c in get(kinds.STATEFUL_SET, "nb")["spec"]["template"]["spec"]["containers"]])
            svc = get(kinds.SERVICE, "nb-kube-rbac-proxy")
            assert svc["spec"]["ports"] == [{"name": "kube-rbac-proxy", "port": 8443, "targetPort": "kube-rbac-proxy",
                                             "protocol": "TCP"}]
            assert m.annotations(svc)["service.beta.openshift.io/serving-cert-secret-name"] == "nb-kube-rbac-proxy-tls"
            cm = get(kinds.CONFIG_MAP, "nb-kube-rbac-proxy-config")
            assert "name: nb" in cm["data"]["config-file.yaml"] and "namespace: user" in cm["data"]["config-file.yaml"]
            crb = get(kinds.CLUSTER_ROLE_BINDING, "nb-rbac-user-auth-delegator", None)
            assert crb["roleRef"]["name"] == "system:auth-delegator"
            assert crb["subjects"] == [{"kind": "ServiceAccount", "name": "nb", "namespace": "user"}]
            r = route_for(cl, "nb")[0]
            assert r["spec"]["rules"][0]["backendRefs"] == [{"name": "nb-kube-rbac-proxy", "namespace": "user",
                                                             "port": 8443}]
            # the lock is removed and the pod comes up
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user"), 10)
            # owned objects carry the controller reference (GC substitute)
            for k, n in ((kinds.SERVICE_ACCOUNT, "nb"), (kinds.SERVICE, "nb-kube-rbac-proxy"),
                         (kinds.CONFIG_MAP, "nb-kube-rbac-proxy-config")):
                assert m.is_controlled_by(get(k, n), get(kinds.NOTEBOOK, "nb"))
            # recreated when deleted; ConfigMap data drift restored
            await cl.admin.delete(kinds.SERVICE_ACCOUNT, "nb", "user")
            await cl.admin.delete(kinds.CONFIG_MAP, "nb-kube-rbac-proxy-config", "user")
            assert await cl.wait_for(lambda: get(kinds.SERVICE_ACCOUNT, "nb") and
                                     get(kinds.CONFIG_MAP, "nb-kube-rbac-proxy-config"))
            # deleting the notebook removes the cluster-scoped CRB and the route
            await cl.admin.delete(kinds.NOTEBOOK, "nb", "user")
            assert await cl.wait_for(lambda: get(kinds.NOTEBOOK, "nb") is None)
            assert get(kinds.CLUSTER_ROLE_BINDING, "nb-rbac-user-auth-delegator", None) is None
            assert route_for(cl, "nb") == []
    run(go())


class _LaggingNotebookReads:
    """The reconciler's client with an informer that has not caught up: cached Notebook reads
    answer ``stale`` (a pre-deletion copy); live reads and everything else pass through."""

    def __init__(self, inner, stale):
        self._inner, self._stale = inner, stale

    def __getattr__(self, name):
        return getattr(self._inner, name)

    async def get(self, kind, name, namespace=None):
        from odh_kubeflow_amd.runtime.client import LIVE_READS
        from odh_kubeflow_amd.utils.objutil import deepcopy_json

        if not LIVE_READS.get() and kind == kinds.NOTEBOOK_V1 and name == m.name(self._stale):
            return deepcopy_json(self._stale)
        return await self._inner.get(kind, name, namespace)


@pytest.mark.parametrize("auth_mode", [True, False])
def test_stale_notebook_after_finalize_recreates_no_exposure_child(run, auth_mode):
    """A reconcile that reads a pre-deletion Notebook from a lagging cache after the finalize
    pass ran must not recreate the finalizer-managed children — the cluster-scoped
    auth-delegator binding, the central-namespace HTTPRoute, the ReferenceGrant — which
    nothing would delete again (odh/controllers/notebook_controller.go:195-321)."""
    from odh_kubeflow_amd.runtime.controller import Request

    async def go():
        async with LocalCluster(cfg()) as cl:
            await create_nb(cl, "nb", annotations=AUTH if auth_mode else None)
            crb = lambda: cl.store.peek(kinds.CLUSTER_ROLE_BINDING, "nb-rbac-user-auth-delegator")  # noqa: E731
            rg = lambda: cl.store.peek(kinds.REFERENCE_GRANT, "notebook-httproute-access", "user")  # noqa: E731
            assert await cl.wait_for(lambda: route_for(cl, "nb") and rg() is not None
                                     and (crb() is not None or not auth_mode))
            assert await cl.wait_for(lambda: "kubeflow-resource-stopped" not in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, "nb", "user")))
            stale = json.loads(json.dumps(cl.store.peek(kinds.NOTEBOOK, "nb", "user")))
            await cl.admin.delete(kinds.NOTEBOOK, "nb", "user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "nb", "user") is None)
            assert crb() is None and rg() is None and route_for(cl, "nb") == []
            r = cl.reconcilers["odh"]
            await cl.odh.stop()  # nothing else reconciles from here on
            real = r.client
            r.client = _LaggingNotebookReads(real, stale)
            try:
                await r.reconcile(Request("user", "nb"))
            finally:
                r.client = real
            assert crb() is None and rg() is None and route_for(cl, "nb") == []
            assert r.stale_reads == 1
    run(go())


def test_mode_switching(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await create_nb(cl, "nb")
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1)
            assert route_for(cl, "nb")[0]["spec"]["rules"][0]["backendRefs"][0]["port"] == 80
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": AUTH}}, name="nb", namespace="user")
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1 and route_for(cl, "nb")[0]["spec"]["rules"]
                                     [0]["backendRefs"][0]["port"] == 8443)
            assert await cl.wait_for(lambda: cl.store.peek(kinds.CLUSTER_ROLE_BINDING, "nb-rbac-user-auth-delegator")
                                     is not None)
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                "notebooks.opendatahub.io/inject-auth": "false"}}}, name="nb", namespace="user")
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1 and route_for(cl, "nb")[0]["spec"]["rules"]
                                     [0]["backendRefs"][0]["port"] == 80)
            assert await cl.wait_for(lambda: cl.store.peek(kinds.CLUSTER_ROLE_BINDING, "nb-rbac-user-auth-delegator")
                                     is None)
    run(go())


def test_role_binding_behind_env(run):
    async def go():
        async with LocalCluster(cfg(SET_PIPELINE_RBAC="true")) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                                   "metadata": {"name": "ds-pipeline-user-access-dspa", "namespace": "user"},
                                   "rules": []})
            await create_nb(cl, "nb")
            rb = lambda: cl.store.peek(kinds.ROLE_BINDING, "elyra-pipelines-nb", "user")  # noqa: E731
            assert await cl.wait_for(lambda: rb() is not None)
            assert rb()["roleRef"] == {"kind": "Role", "name": "ds-pipeline-user-access-dspa",
                                       "apiGroup": "rbac.authorization.k8s.io"}
            assert rb()["subjects"] == [{"kind": "ServiceAccount", "name": "nb", "namespace": "user"}]
            assert m.is_controlled_by(rb(), cl.store.peek(kinds.NOTEBOOK, "nb", "user"))
            cur = await cl.admin.get(kinds.ROLE_BINDING, "elyra-pipelines-nb", "user")
            cur["subjects"] = []
            await cl.admin.update(cur)
            assert await cl.wait_for(lambda: rb()["subjects"] == [{"kind": "ServiceAccount", "name": "nb",
                                                                   "namespace": "user"}])
        async with LocalCluster(cfg(SET_PIPELINE_RBAC="false")) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                                   "metadata": {"name": "ds-pipeline-user-access-dspa", "namespace": "user"}})
            await create_nb(cl, "nb")
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1)
            assert await cl.settle()
            assert cl.store.peek(kinds.ROLE_BINDING, "elyra-pipelines-nb", "user") is None
    run(go())


def _openssl_cert(tmp, cn):
    key, crt = os.path.join(tmp, cn + ".key"), os.path.join(tmp, cn + ".crt")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "ed25519", "-nodes", "-keyout", key, "-out", crt,
                    "-subj", f"/CN={cn}", "-days", "2"], check=True, capture_output=True)
    return open(crt).read()


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI missing")
def test_ca_bundle_concatenates_valid_certs_and_unmounts_when_deleted(run, tmp_path):
    c1, c2, c3 = (_openssl_cert(str(tmp_path), n) for n in ("odh", "odh2", "kube"))
    assert certs.is_valid_certificate(c1) and not certs.is_valid_certificate("-----BEGIN CERTIFICATE-----\nAAAA\n"
                                                                              "-----END CERTIFICATE-----")

    async def go():
        async with LocalCluster(cfg()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": "odh-trusted-ca-bundle", "namespace": "user"},
                                   "data": {"ca-bundle.crt": c1, "odh-ca-bundle.crt": c2 + "\n"}})
            await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": "kube-root-ca.crt", "namespace": "user"},
                                   "data": {"ca.crt": c3}})
            await create_nb(cl, "nb")
            wb = lambda: cl.store.peek(kinds.CONFIG_MAP, "workbench-trusted-ca-bundle", "user")  # noqa: E731
            want = "\n".join(x.strip() for x in (c1, c2, c3))
            assert await cl.wait_for(lambda: wb() is not None and wb()["data"]["ca-bundle.crt"] == want)
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "user")
            assert any(v["name"] == "trusted-ca" for v in nb["spec"]["template"]["spec"]["volumes"])
            # invalid certificate content is skipped
            cur = await cl.admin.get(kinds.CONFIG_MAP, "kube-root-ca.crt", "user")
            cur["data"]["ca.crt"] = "garbage"
            await cl.admin.update(cur)
            want2 = "\n".join(x.strip() for x in (c1, c2))
            assert await cl.wait_for(lambda: wb()["data"]["ca-bundle.crt"] == want2)
            # odh bundle gone + workbench bundle deleted while mounted → volume, mount and env removed
            await cl.admin.delete(kinds.CONFIG_MAP, "odh-trusted-ca-bundle", "user")
            await cl.admin.delete(kinds.CONFIG_MAP, "workbench-trusted-ca-bundle", "user")

            def unmounted():
                spec = cl.store.peek(kinds.NOTEBOOK, "nb", "user")["spec"]["template"]["spec"]
                c = spec["containers"][0]
                return (not any(v["name"] == "trusted-ca" for v in spec.get("volumes") or [])
                        and not any(e["name"] == "SSL_CERT_FILE" for e in c.get("env") or [])
                        and not any(vm["name"] == "trusted-ca" for vm in c.get("volumeMounts") or []))
            assert await cl.wait_for(unmounted)
    run(go())


def test_dspa_secret_created_and_mounted(run):
    async def go():
        async with LocalCluster(cfg(SET_PIPELINE_SECRET="true")) as cl:
            await cl.ensure_namespace("user")
            await cl.ensure_namespace("openshift-ingress")
            await cl.admin.create({"apiVersion": "v1", "kind": "Secret",
                                   "metadata": {"name": "cos", "namespace": "user"},
                                   "data": {"ak": base64.b64encode(b"user").decode(),
                                            "sk": base64.b64encode(b"pass").decode()}})
            dspa = await cl.admin.create({
                "apiVersion": "datasciencepipelinesapplications.opendatahub.io/v1",
                "kind": "DataSciencePipelinesApplication", "metadata": {"name": "dspa", "namespace": "user"},
                "spec": {"objectStorage": {"externalStorage": {
                    "host": "s3.example.com", "bucket": "b",
                    "s3CredentialsSecret": {"secretName": "cos", "accessKey": "ak", "secretKey": "sk"}}}}})
            dspa["status"] = {"components": {"apiServer": {"externalUrl": "https://ds-pipeline.example"}}}
            await cl.admin.update_status(dspa)
            gw = await cl.admin.create({"apiVersion": "gateway.networking.k8s.io/v1", "kind": "Gateway",
                                        "metadata": {"name": "data-science-gateway", "namespace": "openshift-ingress"},
                                        "spec": {"listeners": [{"name": "https", "hostname": "apps.example.com"}]}})
            assert gw
            await create_nb(cl, "nb")
            sec = lambda: cl.store.peek(kinds.SECRET, "ds-pipeline-config", "user")  # noqa: E731
            assert await cl.wait_for(lambda: sec() is not None)
            s = sec()
            payload = json.loads(base64.b64decode(s["data"]["odh_dsp.json"]))
            assert payload["display_name"] == "Pipeline" and payload["schema_name"] == "kfp"
            md = payload["metadata"]
            assert md["api_endpoint"] == "https://ds-pipeline.example"
            assert md["cos_endpoint"] == "https://s3.example.com" and md["cos_bucket"] == "b"
            assert md["cos_username"] == "user" and md["cos_password"] == "pass" and md["cos_secret"] == "cos"
            assert md["public_api_endpoint"] == "https://apps.example.com/external/elyra/user"
            assert m.labels(s) == {"opendatahub.io/managed-by": "workbenches"}
            assert s["metadata"]["ownerReferences"][0]["kind"] == "DataSciencePipelinesApplication"
            vol = {"name": "elyra-dsp-details", "secret": {"secretName": "ds-pipeline-config", "optional": True}}
            spec = lambda: ((cl.store.peek(kinds.NOTEBOOK, "nb", "user") or {}).get("spec", {})  # noqa: E731
                            .get("template", {}).get("spec", {}))
            # the Secret and the Notebook arrive on different watches: no cross-kind ordering
            assert await cl.wait_for(lambda: vol in spec().get("volumes", []))
            spec = spec()
            assert {"name": "elyra-dsp-details", "mountPath": "/opt/app-root/runtimes"} in \
                spec["containers"][0]["volumeMounts"]
    run(go())


def test_dspa_hostname_route_fallback(run):
    async def go():
        async with LocalCluster(ClusterConfig(odh=False, webhook=False, kf=False, openshift=True)) as cl:
            c = cl.admin
            await cl.ensure_namespace("openshift-ingress")
            gw = {"metadata": {"ownerReferences": [{"kind": "GatewayConfig", "name": "default-gateway"}]},
                  "spec": {"listeners": [{"name": "x"}]}}
            assert await dspa_secret.hostname_for_public_endpoint(c, None) == ""
            assert await dspa_secret.hostname_for_public_endpoint(c, gw) == ""
            await c.create({"apiVersion": "route.openshift.io/v1", "kind": "Route",
                            "metadata": {"name": "r", "namespace": "openshift-ingress",
                                         "ownerReferences": [{"apiVersion": "x/v1", "kind": "GatewayConfig",
                                                              "name": "default-gateway", "uid": "1"}]},
                            "spec": {"host": "route.example.com"}})
            assert await dspa_secret.hostname_for_public_endpoint(c, gw) == "route.example.com"
            gw["spec"]["listeners"][0]["hostname"] = "gw.example.com"
            assert await dspa_secret.hostname_for_public_endpoint(c, gw) == "gw.example.com"
            assert dspa_secret.gateway_config_owner_name({"metadata": {"ownerReferences": [
                {"kind": "Other", "name": "a"}, {"kind": "GatewayConfig", "name": "b"}]}}) == "b"
    run(go())


def test_openshift_lock_waits_for_pull_secret_without_blocking_workers(run):
    async def go():
        async with LocalCluster(ClusterConfig(odh=True, webhook=True, gc=False, openshift=True,
                                              env={"SET_PIPELINE_RBAC": "false"})) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create({"apiVersion": "v1", "kind": "ServiceAccount",
                                   "metadata": {"name": "default", "namespace": "user"}})
            await create_nb(cl, "slow")
            await create_nb(cl, "other", ns="user2")
            await cl.admin.create({"apiVersion": "v1", "kind": "ServiceAccount",
                                   "metadata": {"name": "default", "namespace": "user2"},
                                   "imagePullSecrets": [{"name": "default-dockercfg"}]})
            locked = lambda n, ns: "kubeflow-resource-stopped" in m.annotations(  # noqa: E731
                cl.store.peek(kinds.NOTEBOOK, n, ns))
            # the notebook whose SA already has a pull secret is unlocked at once...
            assert await cl.wait_for(lambda: not locked("other", "user2"), 2)
            assert locked("slow", "user")
            # ...and the waiting one is released by the SA watch as soon as the secret lands
            sa = await cl.admin.get(kinds.SERVICE_ACCOUNT, "default", "user")
            sa["imagePullSecrets"] = [{"name": "default-dockercfg"}]
            await cl.admin.update(sa)
            assert await cl.wait_for(lambda: not locked("slow", "user"), 2)
    run(go())


@pytest.mark.parametrize("transport", ["http", "native"])
def test_create_path_order_gating_children_then_one_unlock_write(run, tmp_path, transport):
    """New Notebook: the objects the pod mounts / runs as and its NetworkPolicies exist
    before the lock goes; finalizers and lock removal are ONE write; the finalizer-managed
    exposure children (ReferenceGrant, HTTPRoute, auth-delegator binding) come after it."""
    from odh_kubeflow_amd.testing.apiserver.audit import AuditPolicy

    log = tmp_path / "audit.log"

    async def go():
        c = cfg()
        c.transport, c.audit_log_path, c.audit_policy = transport, str(log), AuditPolicy([{"level": "Metadata"}])
        async with LocalCluster(c) as cl:
            await create_nb(cl, "nb", annotations=AUTH)
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user"), 15)
    run(go())
    evs = [json.loads(line) for line in log.read_text().splitlines()]
    writes = [(e["verb"], e["objectRef"]["resource"], e["objectRef"].get("name", ""), e["objectRef"].get("subresource", ""))
              for e in evs if e["stage"] == "ResponseComplete" and e["verb"] not in ("get", "list", "watch")
              and e["responseStatus"]["code"] < 300]
    nb_writes = [w for w in writes if w[1] == "notebooks" and w[2] == "nb" and w[3] == "" and w[0] != "create"]
    assert nb_writes == [("patch", "notebooks", "nb", "")], nb_writes  # finalizers + unlock: one write
    unlock = writes.index(nb_writes[0])

    def at(verb, res, name):
        return next(i for i, w in enumerate(writes) if w[:3] == (verb, res, name))

    for gating in (("create", "networkpolicies", "nb-ctrl-np"), ("create", "networkpolicies", "nb-kube-rbac-proxy-np"),
                   ("create", "serviceaccounts", "nb"), ("create", "configmaps", "nb-kube-rbac-proxy-config")):
        assert at(*gating) < unlock, gating
    for exposure in (("create", "referencegrants", "notebook-httproute-access"), ("create", "httproutes", "nb-user-nb"),
                     ("create", "clusterrolebindings", "nb-rbac-user-auth-delegator")):
        assert at(*exposure) > unlock, exposure
    # the kf controller scales the StatefulSet only after the unlock
    assert at("update", "statefulsets", "nb") > unlock


def test_lock_removal_never_drops_a_user_stop(run):
    """The unlock write tests the lock value: a user who stops the Notebook while it still
    waits for its pull secret keeps their stop annotation."""
    async def go():
        async with LocalCluster(ClusterConfig(odh=True, webhook=True, gc=False, openshift=True,
                                              env={"SET_PIPELINE_RBAC": "false"})) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create({"apiVersion": "v1", "kind": "ServiceAccount",
                                   "metadata": {"name": "default", "namespace": "user"}})
            await create_nb(cl, "nb")
            peek = lambda: cl.store.peek(kinds.NOTEBOOK, "nb", "user")  # noqa: E731
            # waiting for the pull secret: finalizers are already durable, the lock is still on
            # (peek is the test's watch mirror of the native server: it may not hold the notebook yet)
            assert await cl.wait_for(
                lambda: "notebook.opendatahub.io/httproute-cleanup" in m.finalizers(peek() or {}), 3)
            assert m.annotations(peek())["kubeflow-resource-stopped"] == "odh-notebook-controller-lock"
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                "kubeflow-resource-stopped": "2026-10-16T00:00:00Z"}}}, "merge", name="nb", namespace="user")
            sa = await cl.admin.get(kinds.SERVICE_ACCOUNT, "default", "user")
            sa["imagePullSecrets"] = [{"name": "default-dockercfg"}]
            await cl.admin.update(sa)
            await asyncio.sleep(0.5)  # the SA watch re-triggers the reconcile at once
            assert m.annotations(peek())["kubeflow-resource-stopped"] == "2026-10-16T00:00:00Z"
    run(go())
