"""More ODH reconciler + webhook scenarios, one per reference ``It`` block.

Scenarios from odh/controllers/notebook_controller_test.go not pinned by
test_odh_controller.py: updating a Notebook (:680-787, incl. the trusted-CA bundle
appearing after creation, with the reference's own ed25519 PEM fixtures), the long
name HTTPRoute recreate (:639-653), NetworkPolicies deleted with the Notebook
(:929-944, GC on), the kube-rbac-proxy HTTPRoute drift / recreate (:1155-1190), a
manually modified auth Notebook restored by admission (:1204-1265) and the
non-auth notebook (:1485-1530).
"""

import os
import copy

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.retry import retry_on_conflict

CENTRAL = "opendatahub"
AUTH = {"notebooks.opendatahub.io/inject-auth": "true"}

# ed25519 certificates from the reference test (notebook_controller_test.go:716-717)
REF_CERT_1 = ("-----BEGIN CERTIFICATE-----\nMIGrMF+gAwIBAgIBATAFBgMrZXAwADAeFw0yNDExMTMyMzI4MjZaFw0yNTExMTMy\n"
              "MzI4MjZaMAAwKjAFBgMrZXADIQD77pLvWIX0WmlkYthRZ79oIf7qrGO7yECf668T\nSB42vTAFBgMrZXADQQDs76j81LPh+lgn"
              "nf4L0ROUqB66YiBx9SyDTjm83Ya4KC+2\nLEP6Mw1//X2DX89f1chy7RxCpFS3eXb7U/p+GPwA\n-----END CERTIFICATE-----")
REF_CERT_2 = ("-----BEGIN CERTIFICATE-----\nMIGrMF+gAwIBAgIBATAFBgMrZXAwADAeFw0yNDExMTMyMzI4NDJaFw0yNTExMTMy\n"
              "MzI4NDJaMAAwKjAFBgMrZXADIQAw01381TUVSxaCvjQckcw3RTcg+bsVMgNZU8eF\nXa/f3jAFBgMrZXADQQBeJZHSiMOYqa/tXUrQ"
              "TfNIcklHuvieGyBRVSrX3bVUV2uM\nDBkZLsZt65rCk1A8NG+xkA6j3eIMAA9vBKJ0ht8F\n-----END CERTIFICATE-----")


def cfg(gc=False, **env):
    base = {"SET_PIPELINE_RBAC": os.environ.get("ODH_TEST_SET_PIPELINE_RBAC", "false"), "SET_PIPELINE_SECRET": "false"}
    base.update(env)
    return ClusterConfig(odh=True, webhook=True, gc=gc, env=base)


def route_for(cl, name, ns="user"):
    return [r for r in cl.store.list_nocopy(kinds.HTTP_ROUTE, CENTRAL)
            if m.labels(r).get("notebook-name") == name and m.labels(r).get("notebook-namespace") == ns]


def unlocked(cl, name, ns="user"):
    nb = cl.store.peek(kinds.NOTEBOOK, name, ns)
    return nb is not None and "kubeflow-resource-stopped" not in m.annotations(nb)


async def update_nb(cl, name, ns, fn):
    from odh_kubeflow_amd.runtime.retry import retry_on_conflict

    async def attempt():
        nb = await cl.admin.get(kinds.NOTEBOOK, name, ns)
        fn(nb)
        return await cl.admin.update(nb)
    return await retry_on_conflict(attempt)


def test_update_notebook_image_reaches_the_statefulset(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("test-notebook-update", "user"))
            assert await cl.wait_for(lambda: cl.notebook_ready("test-notebook-update", "user"))
            updated = "registry.redhat.io/ubi9/ubi:updated"

            def set_image(nb):
                nb["spec"]["template"]["spec"]["containers"][0]["image"] = updated
            out = await update_nb(cl, "test-notebook-update", "user", set_image)
            assert out["spec"]["template"]["spec"]["containers"][0]["image"] == updated
            assert "notebooks.opendatahub.io/update-pending" not in m.annotations(out)
            assert await cl.wait_for(lambda: cl.store.peek(kinds.STATEFUL_SET, "test-notebook-update", "user")
                                     ["spec"]["template"]["spec"]["containers"][0]["image"] == updated)
    run(go())


def test_update_mounts_trusted_ca_bundle_created_after_the_notebook(run, tmp_path):
    from tests.test_odh_controller import _openssl_cert

    kube_root = _openssl_cert(str(tmp_path), "kube-root")

    async def go():
        async with LocalCluster(cfg()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": "kube-root-ca.crt", "namespace": "user"},
                                   "data": {"ca.crt": kube_root}})
            await cl.admin.create(notebook("nb", "user"))
            assert await cl.wait_for(lambda: unlocked(cl, "nb"))
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "user")
            assert not any(v["name"] == "trusted-ca" for v in nb["spec"]["template"]["spec"].get("volumes") or [])
            await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": "odh-trusted-ca-bundle", "namespace": "user",
                                                "labels": {"config.openshift.io/inject-trusted-cabundle": "true"}},
                                   "data": {"ca-bundle.crt": REF_CERT_1, "odh-ca-bundle.crt": REF_CERT_2}})

            def set_image(o):
                o["spec"]["template"]["spec"]["containers"][0]["image"] = "registry.redhat.io/ubi9/ubi:updated"
            out = await update_nb(cl, "nb", "user", set_image)
            spec = out["spec"]["template"]["spec"]
            assert {"name": "trusted-ca", "mountPath": "/etc/pki/tls/custom-certs/ca-bundle.crt",
                    "subPath": "ca-bundle.crt", "readOnly": True} in spec["containers"][0]["volumeMounts"]
            assert {"name": "trusted-ca", "configMap": {"name": "workbench-trusted-ca-bundle", "optional": True,
                                                        "items": [{"key": "ca-bundle.crt",
                                                                   "path": "ca-bundle.crt"}]}} in spec["volumes"]
            env = {e["name"]: e.get("value") for e in spec["containers"][0]["env"]}
            for k in ("PIP_CERT", "REQUESTS_CA_BUNDLE", "SSL_CERT_FILE", "PIPELINES_SSL_SA_CERTS",
                      "KF_PIPELINES_SSL_SA_CERTS", "GIT_SSL_CAINFO"):
                assert env[k] == "/etc/pki/tls/custom-certs/ca-bundle.crt"

            def three_valid_certs():
                wb = cl.store.peek(kinds.CONFIG_MAP, "workbench-trusted-ca-bundle", "user")
                return wb is not None and wb["data"]["ca-bundle.crt"].count("BEGIN CERTIFICATE") == 3
            assert await cl.wait_for(three_valid_certs)
    run(go())


def test_long_name_route_recreated_when_deleted(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            ns = "long-namespace-for-routes"
            name = "a-very-long-notebook-name-that-exceeds-the-limit-of-routes"
            await cl.ensure_namespace(ns)
            await cl.admin.create(notebook(name, ns))
            assert await cl.wait_for(lambda: len(route_for(cl, name, ns)) == 1)
            first = m.name(route_for(cl, name, ns)[0])
            await cl.admin.delete(kinds.HTTP_ROUTE, first, CENTRAL)
            assert await cl.wait_for(lambda: len(route_for(cl, name, ns)) == 1 and
                                     m.name(route_for(cl, name, ns)[0]) != first)
            r = route_for(cl, name, ns)[0]
            assert m.name(r).startswith("nb-long-names-a-very-lon-") and len(m.name(r)) <= 63
            assert r["spec"]["rules"][0]["matches"] == [{"path": {"type": "PathPrefix", "value": f"/notebook/{ns}/{name}"}}]
    run(go())


def test_network_policies_deleted_with_the_notebook(run):
    async def go():
        async with LocalCluster(cfg(gc=True)) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user"))
            np = lambda n: cl.store.peek(kinds.NETWORK_POLICY, n, "user")  # noqa: E731
            assert await cl.wait_for(lambda: np("nb-ctrl-np") is not None and np("nb-kube-rbac-proxy-np") is not None)
            await cl.admin.delete(kinds.NOTEBOOK, "nb", "user")
            assert await cl.wait_for(lambda: np("nb-ctrl-np") is None and np("nb-kube-rbac-proxy-np") is None
                                     and cl.store.peek(kinds.NOTEBOOK, "nb", "user") is None)
    run(go())


def test_auth_route_drift_and_recreate(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user", annotations=AUTH))
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1)
            want = copy.deepcopy(route_for(cl, "nb")[0]["spec"])
            assert want["rules"][0]["backendRefs"] == [{"name": "nb-kube-rbac-proxy", "namespace": "user",
                                                        "port": 8443}]
            async def tamper():  # the route may still be written (status) while the test edits it
                cur = await cl.admin.get(kinds.HTTP_ROUTE, "nb-user-nb", CENTRAL)
                cur["spec"]["rules"][0]["backendRefs"][0]["name"] = "elsewhere"
                await cl.admin.update(cur)
            await retry_on_conflict(tamper)
            assert await cl.wait_for(lambda: route_for(cl, "nb")[0]["spec"] == want)
            await cl.admin.delete(kinds.HTTP_ROUTE, "nb-user-nb", CENTRAL)
            assert await cl.wait_for(lambda: len(route_for(cl, "nb")) == 1 and route_for(cl, "nb")[0]["spec"] == want)
    run(go())


def test_manually_modified_auth_notebook_is_restored_by_admission(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user", annotations=AUTH))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user"))
            orig = copy.deepcopy(cl.store.peek(kinds.NOTEBOOK, "nb", "user")["spec"]["template"]["spec"])
            assert orig["serviceAccountName"] == "nb"
            proxy_idx = [c["name"] for c in orig["containers"]].index("kube-rbac-proxy")

            def tamper(nb):
                s = nb["spec"]["template"]["spec"]
                s["serviceAccountName"] = "foo"
                s["containers"][proxy_idx]["image"] = "bar"
                vol = [v for v in s["volumes"] if v["name"] == "kube-rbac-proxy-config"][0]
                for k in list(vol):
                    if k != "name":
                        vol.pop(k)
            out = await update_nb(cl, "nb", "user", tamper)
            s = out["spec"]["template"]["spec"]
            assert s["serviceAccountName"] == "nb"
            assert s["containers"][proxy_idx]["image"] == orig["containers"][proxy_idx]["image"]
            assert s["volumes"] == orig["volumes"]
    run(go())


def test_notebook_without_auth_has_no_sidecar_and_an_unauthenticated_route(run):
    async def go():
        async with LocalCluster(cfg()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user"))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user") and len(route_for(cl, "nb")) == 1)
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "user")
            assert [c["name"] for c in nb["spec"]["template"]["spec"]["containers"]] == ["nb"]
            assert "notebook.opendatahub.io/kube-rbac-proxy-cleanup" not in m.finalizers(nb)
            assert route_for(cl, "nb")[0]["spec"]["rules"][0]["backendRefs"] == [
                {"name": "nb", "namespace": "user", "port": 80}]
            for k, n in ((kinds.SERVICE_ACCOUNT, "nb"), (kinds.SERVICE, "nb-kube-rbac-proxy"),
                         (kinds.CONFIG_MAP, "nb-kube-rbac-proxy-config")):
                assert cl.store.peek(k, n, "user") is None
    run(go())
