"""Elyra / DSP runtime Secret helpers against a fake client (in-process store).

Case list follows odh/controllers/notebook_dspa_secret_test.go:
``getGatewayConfigOwnerName`` (:34-98), ``getHostnameForPublicEndpoint`` (:100-336),
``getHostnameFromRoute`` (:338-493) and ``extractElyraRuntimeConfigInfo`` (:495-840).
Secret data is base64 in the JSON wire format; the reference's fake client holds the
raw bytes — both decode to the same credentials.
"""

import base64

import pytest

from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.controllers.odh import dspa_secret as ds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.testing.apiserver.inprocess import InProcessClient

NS = "test-namespace"
INGRESS = "openshift-ingress"


async def _client(*objs):
    store = ObjectStore()
    c = InProcessClient(store)
    for ns in (NS, INGRESS):
        await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    for o in objs:
        await c.create(o)
    return c


def gateway(hostname=None, listeners=True, owners=None):
    gw = {"apiVersion": "gateway.networking.k8s.io/v1", "kind": "Gateway",
          "metadata": {"name": "data-science-gateway", "namespace": INGRESS}, "spec": {"listeners": []}}
    if owners is not None:
        gw["metadata"]["ownerReferences"] = owners
    if listeners:
        lst = {"name": "https", "port": 443, "protocol": "HTTPS"}
        if hostname is not None:
            lst["hostname"] = hostname
        gw["spec"]["listeners"] = [lst]
    return gw


def gwc_owner(name="default-gateway"):
    return {"apiVersion": "services.platform.opendatahub.io/v1alpha1", "kind": "GatewayConfig",
            "name": name, "uid": "gwc-uid"}


def route(name, host, owners=()):
    return {"apiVersion": "route.openshift.io/v1", "kind": "Route",
            "metadata": {"name": name, "namespace": INGRESS, "ownerReferences": list(owners)},
            "spec": {"host": host, "to": {"kind": "Service", "name": "gw"}}}


# ------------------------------------------------------------------ getGatewayConfigOwnerName


@pytest.mark.parametrize("gw,want", [
    (None, ""),
    (gateway(), ""),                                              # no ownerReferences
    (gateway(owners=[{"kind": "Deployment", "name": "d", "apiVersion": "apps/v1", "uid": "u"}]), ""),
    (gateway(owners=[gwc_owner("my-gwc")]), "my-gwc"),
    (gateway(owners=[{"kind": "Deployment", "name": "d", "apiVersion": "apps/v1", "uid": "u"},
                     gwc_owner("second")]), "second"),            # among multiple owners
])
def test_gateway_config_owner_name(gw, want):
    assert ds.gateway_config_owner_name(gw) == want


# ------------------------------------------------------------------ getHostnameForPublicEndpoint


def test_hostname_nil_gateway(run):
    async def go():
        assert await ds.hostname_for_public_endpoint(await _client(), None) == ""
    run(go())


def test_hostname_from_gateway_listener(run):
    async def go():
        c = await _client(route("r", "route.example.com", [gwc_owner()]))
        gw = gateway("gateway.example.com", owners=[gwc_owner()])
        assert await ds.hostname_for_public_endpoint(c, gw) == "gateway.example.com"  # preferred over the Route
    run(go())


@pytest.mark.parametrize("gw", [
    gateway(listeners=False, owners=[gwc_owner()]),          # empty listeners
    gateway(hostname=None, owners=[gwc_owner()]),            # hostname unset
    gateway(hostname="", owners=[gwc_owner()]),              # hostname empty
], ids=["no-listeners", "nil-hostname", "empty-hostname"])
def test_hostname_route_fallback(run, gw):
    async def go():
        c = await _client(route("data-science-gateway", "fallback.example.com", [gwc_owner()]))
        assert await ds.hostname_for_public_endpoint(c, gw) == "fallback.example.com"
    run(go())


def test_hostname_empty_without_owner_or_hostname(run):
    async def go():
        c = await _client(route("r", "fallback.example.com", [gwc_owner()]))
        assert await ds.hostname_for_public_endpoint(c, gateway(hostname="")) == ""
    run(go())


def test_hostname_empty_when_route_fallback_finds_nothing(run):
    async def go():
        c = await _client(route("r", "x.example.com", [gwc_owner("another")]))
        assert await ds.hostname_for_public_endpoint(c, gateway(hostname="", owners=[gwc_owner()])) == ""
    run(go())


# ------------------------------------------------------------------ getHostnameFromRoute


@pytest.mark.parametrize("routes,gwc,want", [
    ([route("r", "h.example.com", [gwc_owner()])], "", ""),                               # no GatewayConfig name
    ([], "default-gateway", ""),                                                          # no routes
    ([route("r", "h.example.com", [gwc_owner()])], "default-gateway", "h.example.com"),   # matching owner
    ([route("r", "h.example.com", [gwc_owner("other")])], "default-gateway", ""),         # other GatewayConfig
    ([route("r", "h.example.com")], "default-gateway", ""),                               # no owners
    ([route("r", "h.example.com", [{"apiVersion": "apps/v1", "kind": "Deployment", "name": "default-gateway",
                                    "uid": "u"}])], "default-gateway", ""),               # owner not a GatewayConfig
    ([route("r", "", [gwc_owner()])], "default-gateway", ""),                             # matching owner, empty host
], ids=["no-name", "no-routes", "match", "other-gwc", "no-owner", "wrong-kind", "empty-host"])
def test_hostname_from_route(run, routes, gwc, want):
    async def go():
        c = await _client(*routes)
        assert await ds.hostname_from_route(c, gwc) == want
    run(go())


# ------------------------------------------------------------------ extractElyraRuntimeConfigInfo


def dspa(host="minio.example.com", bucket="my-bucket", secret="cos-secret", ak="accesskey", sk="secretkey",
         scheme=""):
    ext = {"host": host, "bucket": bucket,
           "s3CredentialsSecret": {"secretName": secret, "accessKey": ak, "secretKey": sk}}
    if scheme:
        ext["scheme"] = scheme
    return {"apiVersion": "datasciencepipelinesapplications.opendatahub.io/v1",
            "kind": "DataSciencePipelinesApplication", "metadata": {"name": "dspa", "namespace": NS},
            "spec": {"objectStorage": {"externalStorage": ext}},
            "status": {"components": {"apiServer": {"externalUrl": "https://api.example.com"}}}}


def cos_secret(keys=("accesskey", "secretkey")):
    vals = {"accesskey": b"myaccesskey", "secretkey": b"mysecretkey"}
    return {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "cos-secret", "namespace": NS},
            "data": {k: base64.b64encode(vals[k]).decode() for k in keys}}


@pytest.mark.parametrize("d,objs,msg", [
    (dspa(host=""), [cos_secret()], "missing or invalid 'host'"),
    (dspa(bucket=""), [cos_secret()], "missing or invalid 'bucket'"),
    (dspa(), [], "failed to get secret 'cos-secret'"),
    (dspa(), [cos_secret(keys=("secretkey",))], "missing key 'accesskey'"),
    (dspa(), [cos_secret(keys=("accesskey",))], "missing key 'secretkey'"),
], ids=["empty-host", "empty-bucket", "no-secret", "no-access-key", "no-secret-key"])
def test_extract_errors(run, d, objs, msg):
    async def go():
        c = await _client(*objs)
        with pytest.raises(ds.ElyraConfigError, match=msg):
            await ds.extract_elyra_runtime_config_info(c, None, d, notebook("notebook", NS))
    run(go())


@pytest.mark.parametrize("scheme,want", [("", "https://minio.example.com"), ("http", "http://minio.example.com")])
def test_extract_cos_scheme(run, scheme, want):
    async def go():
        c = await _client(cos_secret())
        info = await ds.extract_elyra_runtime_config_info(c, None, dspa(scheme=scheme), notebook("notebook", NS))
        assert info["metadata"]["cos_endpoint"] == want
    run(go())


def test_extract_public_endpoint_from_gateway(run):
    async def go():
        c = await _client(cos_secret())
        info = await ds.extract_elyra_runtime_config_info(c, gateway("gw.example.com"), dspa(),
                                                          notebook("notebook", NS))
        assert info["metadata"]["public_api_endpoint"] == f"https://gw.example.com/external/elyra/{NS}"
    run(go())


def test_extract_no_public_endpoint_without_gateway(run):
    async def go():
        c = await _client(cos_secret())
        info = await ds.extract_elyra_runtime_config_info(c, None, dspa(), notebook("notebook", NS))
        assert "public_api_endpoint" not in info["metadata"]
    run(go())


def test_extract_public_endpoint_from_route_fallback(run):
    async def go():
        c = await _client(cos_secret(), route("r", "route-host.example.com", [gwc_owner()]))
        info = await ds.extract_elyra_runtime_config_info(c, gateway(hostname="", owners=[gwc_owner()]), dspa(),
                                                          notebook("notebook", NS))
        assert info["metadata"]["public_api_endpoint"] == f"https://route-host.example.com/external/elyra/{NS}"
    run(go())


def test_extract_populates_every_elyra_field(run):
    async def go():
        c = await _client(cos_secret())
        info = await ds.extract_elyra_runtime_config_info(c, None, dspa(), notebook("notebook", NS))
        assert info["display_name"] == "Pipeline" and info["schema_name"] == "kfp"
        assert info["metadata"] == {
            "tags": [], "display_name": "Pipeline", "engine": "Argo", "runtime_type": "KUBEFLOW_PIPELINES",
            "auth_type": "KUBERNETES_SERVICE_ACCOUNT_TOKEN", "cos_auth_type": "KUBERNETES_SECRET",
            "api_endpoint": "https://api.example.com", "cos_endpoint": "https://minio.example.com",
            "cos_bucket": "my-bucket", "cos_username": "myaccesskey", "cos_password": "mysecretkey",
            "cos_secret": "cos-secret"}
    run(go())


# ------------------------------------------------------------------ sync + mount


def test_sync_without_dspa_creates_nothing_and_mount_is_noop(run):
    async def go():
        c = await _client()
        nb = notebook("notebook", NS)
        await ds.sync_elyra_runtime_config_secret(c, nb)
        from odh_kubeflow_amd.models import kinds
        assert await c.list(kinds.SECRET, NS) == []
        await ds.mount_elyra_runtime_config_secret(c, nb)
        assert "volumes" not in nb["spec"]["template"]["spec"]
    run(go())


def test_sync_updates_drifted_secret_and_mounts_on_every_container(run):
    async def go():
        from odh_kubeflow_amd.models import kinds

        c = await _client(cos_secret())
        d = await c.create({k: v for k, v in dspa().items() if k != "status"})
        d["status"] = dspa()["status"]
        await c.update_status(d)
        nb = notebook("notebook", NS)
        nb["spec"]["template"]["spec"]["containers"].append({"name": "sidecar", "image": "s"})
        await ds.sync_elyra_runtime_config_secret(c, nb)
        sec = await c.get(kinds.SECRET, "ds-pipeline-config", NS)
        want = sec["data"]
        sec["data"] = {"odh_dsp.json": base64.b64encode(b"{}").decode()}
        sec["metadata"]["labels"] = {}
        await c.update(sec)
        await ds.sync_elyra_runtime_config_secret(c, nb)
        sec = await c.get(kinds.SECRET, "ds-pipeline-config", NS)
        assert sec["data"] == want and sec["metadata"]["labels"] == {"opendatahub.io/managed-by": "workbenches"}
        await ds.mount_elyra_runtime_config_secret(c, nb)
        await ds.mount_elyra_runtime_config_secret(c, nb)  # idempotent
        spec = nb["spec"]["template"]["spec"]
        assert spec["volumes"] == [{"name": "elyra-dsp-details",
                                    "secret": {"secretName": "ds-pipeline-config", "optional": True}}]
        for ct in spec["containers"]:
            assert ct["volumeMounts"] == [{"name": "elyra-dsp-details", "mountPath": "/opt/app-root/runtimes"}]
    run(go())
