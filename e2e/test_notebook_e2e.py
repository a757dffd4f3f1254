"""The reference's e2e sequence (``odh/e2e/*.go``), runnable against a deployed cluster or
the local dev processes (``e2e/harness.py``).  Tests run in file order and share the
notebooks they create, as the reference's ``t.Run`` chain does
(``notebook_controller_setup_test.go:102-119``):

1. controllers deployed (``notebook_controller_test.go:11-52``);
2. per notebook — create → HTTPRoute → NetworkPolicies → StatefulSet 1/1 → auth sidecar →
   sidecar resources → Service connectivity → HTTPRoute configuration
   (``notebook_creation_test.go:31-415,520-607``);
3. culling of the first notebook: culler settings on, the controller rolled, the
   StatefulSet reaches 0 replicas, settings restored and the notebook resumed (:417-518);
4. update: a new image rolls the StatefulSet (``notebook_update_test.go:15-126``);
5. deletion, unless ``--skip-deletion``: every dependent goes
   (``notebook_deletion_test.go:21-128``).
"""

from __future__ import annotations

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.errors import ApiError
from odh_kubeflow_amd.utils.quantity import parse_quantity

AUTH = "notebooks.opendatahub.io/inject-auth"
STOP = "kubeflow-resource-stopped"
SIDECAR = "kube-rbac-proxy"
SIDECAR_DEFAULTS = {"requests": {"cpu": "100m", "memory": "64Mi"}, "limits": {"cpu": "100m", "memory": "64Mi"}}
RESOURCE_ANNOTATIONS = {
    ("requests", "cpu"): "notebooks.opendatahub.io/auth-sidecar-cpu-request",
    ("requests", "memory"): "notebooks.opendatahub.io/auth-sidecar-memory-request",
    ("limits", "cpu"): "notebooks.opendatahub.io/auth-sidecar-cpu-limit",
    ("limits", "memory"): "notebooks.opendatahub.io/auth-sidecar-memory-limit",
}


def minimal_rbac_notebook(ns: str, image: str) -> dict:
    """``setupThothMinimalRbacNotebook`` (helper_test.go:547-620)."""
    name = "thoth-minimal-rbac-notebook"
    base = f"/notebook/{ns}/{name}"
    return {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
            "metadata": {"name": name, "namespace": ns, "annotations": {AUTH: "true"}},
            "spec": {"template": {"spec": {"containers": [{
                "name": name, "image": image, "workingDir": "/opt/app-root/src",
                "ports": [{"name": "notebook-port", "containerPort": 8888, "protocol": "TCP"}],
                "env": [{"name": "JUPYTER_NOTEBOOK_PORT", "value": "8888"},
                        {"name": "NOTEBOOK_ARGS", "value": "--ServerApp.port=8888 --NotebookApp.token='' "
                                                           "--NotebookApp.password='' --ServerApp.base_url=" + base}],
                "resources": {"limits": {"cpu": "400m", "memory": "256Mi"},
                              "requests": {"cpu": "200m", "memory": "128Mi"}},
                "livenessProbe": {"httpGet": {"path": base + "/api", "port": "notebook-port", "scheme": "HTTP"},
                                  "initialDelaySeconds": 5, "timeoutSeconds": 1, "periodSeconds": 5,
                                  "successThreshold": 1, "failureThreshold": 3}}]}}}}


def custom_resources_notebook(ns: str, image: str) -> dict:
    """``setupThothRbacCustomResourcesNotebook`` (helper_test.go:622-690): sidecar
    resources from annotations."""
    name = "thoth-custom-resources-notebook"
    return {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
            "metadata": {"name": name, "namespace": ns, "annotations": {
                AUTH: "true",
                RESOURCE_ANNOTATIONS[("requests", "cpu")]: "0.2",  # = 200m
                RESOURCE_ANNOTATIONS[("requests", "memory")]: "128Mi",
                RESOURCE_ANNOTATIONS[("limits", "cpu")]: "400m",
                RESOURCE_ANNOTATIONS[("limits", "memory")]: "256Mi"}},
            "spec": {"template": {"spec": {"containers": [{
                "name": name, "image": image, "workingDir": "/opt/app-root/src",
                "ports": [{"name": "notebook-port", "containerPort": 8888, "protocol": "TCP"}],
                "env": [{"name": "JUPYTER_ENABLE_LAB", "value": "yes"}],
                "resources": {"limits": {"cpu": "500m", "memory": "384Mi"},
                              "requests": {"cpu": "250m", "memory": "192Mi"}}}]}}}}


@pytest.fixture(scope="module")
def notebooks(harness, opts):
    return [minimal_rbac_notebook(harness.nb_ns, opts.notebook_image),
            custom_resources_notebook(harness.nb_ns, opts.notebook_image)]


def _get(h, kind, name, ns=None):
    return h.run(h.client.get(kind, name, ns))


def _route(h, nb):
    async def find():
        for r in await h.client.list(kinds.HTTP_ROUTE, h.ctrl_ns):
            lb = m.labels(r)
            if lb.get("notebook-name") == m.name(nb) and lb.get("notebook-namespace") == m.namespace(nb):
                return r
        return None
    return h.eventually(find, what=f"HTTPRoute of {m.name(nb)}")


def _sts_ready(h, nb, replicas=1, image=None):
    async def ready():
        s = await h.client.get(kinds.STATEFUL_SET, m.name(nb), m.namespace(nb))
        st = s.get("status") or {}
        if image and s["spec"]["template"]["spec"]["containers"][0]["image"] != image:
            return None
        if replicas == 0:
            return s if s["spec"].get("replicas") == 0 and not st.get("readyReplicas") else None
        return s if (st.get("readyReplicas") == replicas and st.get("updatedReplicas", replicas) == replicas
                     and s["spec"].get("replicas") == replicas) else None
    return h.eventually(ready, timeout=h.cull_wait if replicas == 0 else None,
                        what=f"StatefulSet {m.name(nb)} at {replicas} ready replica(s)")


def _pods(h, nb):
    async def ls():
        return await h.client.list(kinds.POD, m.namespace(nb), labels={"statefulset": m.name(nb)})
    return h.run(ls())


# ------------------------------------------------------------------ 1. controllers


def test_controllers_deployed(harness):
    bad = [c for c in harness.controllers() if not c[1]]
    assert not bad, bad


# ------------------------------------------------------------------ 2. creation


def test_create_notebooks(harness, notebooks):
    async def create():
        for nb in notebooks:
            try:
                await harness.client.create(nb)
            except ApiError as e:
                if e.code != 409:  # AlreadyExists: a previous --skip-deletion run left it
                    raise
    harness.run(create())
    for nb in notebooks:
        _sts_ready(harness, nb)


@pytest.mark.parametrize("i", [0, 1])
def test_httproute(harness, notebooks, i):
    nb = notebooks[i]
    r = _route(harness, nb)
    rule = r["spec"]["rules"][0]
    assert rule["matches"][0]["path"] == {"type": "PathPrefix",
                                          "value": f"/notebook/{m.namespace(nb)}/{m.name(nb)}"}
    # auth mode: the route targets the kube-rbac-proxy Service's HTTPS port
    assert rule["backendRefs"] == [{"name": f"{m.name(nb)}-kube-rbac-proxy", "namespace": m.namespace(nb),
                                    "port": 8443}], rule["backendRefs"]
    assert r["spec"]["parentRefs"] and r["spec"]["parentRefs"][0]["name"]


@pytest.mark.parametrize("i", [0, 1])
def test_network_policies(harness, notebooks, i):
    nb = notebooks[i]
    name, ns = m.name(nb), m.namespace(nb)
    ctrl = _get(harness, kinds.NETWORK_POLICY, f"{name}-ctrl-np", ns)
    assert ctrl["spec"]["podSelector"]["matchLabels"] == {"notebook-name": name}
    assert ctrl["spec"]["policyTypes"] == ["Ingress"]
    ports = [p["port"] for p in ctrl["spec"]["ingress"][0]["ports"]]
    assert ports == [8888]
    # only the controller namespace may reach the notebook port
    assert ctrl["spec"]["ingress"][0]["from"][0]["namespaceSelector"]["matchLabels"] == {
        "kubernetes.io/metadata.name": harness.ctrl_ns}
    proxy = _get(harness, kinds.NETWORK_POLICY, f"{name}-kube-rbac-proxy-np", ns)
    assert [p["port"] for p in proxy["spec"]["ingress"][0]["ports"]] == [8443]


@pytest.mark.parametrize("i", [0, 1])
def test_auth_sidecar_and_resources(harness, notebooks, i):
    nb = notebooks[i]
    live = _get(harness, kinds.NOTEBOOK, m.name(nb), m.namespace(nb))
    names = [c["name"] for c in live["spec"]["template"]["spec"]["containers"]]
    assert names == [m.name(nb), SIDECAR], names
    pods = _pods(harness, nb)
    assert pods
    ann = m.annotations(live)
    for pod in pods:
        assert (pod.get("status") or {}).get("phase") == "Running", m.name(pod)
        side = [c for c in pod["spec"]["containers"] if c["name"] == SIDECAR]
        assert side, m.name(pod)
        res = side[0].get("resources") or {}
        for (section, res_name), key in RESOURCE_ANNOTATIONS.items():
            want = ann.get(key, SIDECAR_DEFAULTS[section][res_name]).strip()
            got = (res.get(section) or {}).get(res_name)
            assert got is not None and parse_quantity(got) == parse_quantity(want), (section, res_name, got, want)


@pytest.mark.parametrize("i", [0, 1])
def test_service_connectivity(harness, notebooks, i):
    """``testNotebookServiceConnectivity``: the kube-rbac-proxy Service (8443, selecting the
    notebook's pods) and a Running pod whose sidecar is Ready; where the runner can reach
    the notebook directly, its Jupyter API answers too."""
    nb = notebooks[i]
    svc = _get(harness, kinds.SERVICE, f"{m.name(nb)}-kube-rbac-proxy", m.namespace(nb))
    assert 8443 in [p["port"] for p in svc["spec"]["ports"]]
    assert svc["spec"]["selector"].get("statefulset") == m.name(nb)

    async def sidecar_ready():
        pods = await harness.client.list(kinds.POD, m.namespace(nb), labels={"notebook-name": m.name(nb)})
        return [p for p in pods if (p.get("status") or {}).get("phase") == "Running" and any(
            cs.get("name") == SIDECAR and cs.get("ready") for cs in (p.get("status") or {}).get("containerStatuses") or [])]
    assert harness.eventually(sidecar_ready, what=f"{m.name(nb)} sidecar Ready")
    code = harness.jupyter_kernels(nb)
    assert code in (None, 200), code


# ------------------------------------------------------------------ 3. culling


def test_culling(harness, notebooks):
    nb = notebooks[0]
    harness.enable_culling()
    try:
        _sts_ready(harness, nb, replicas=0)
        live = _get(harness, kinds.NOTEBOOK, m.name(nb), m.namespace(nb))
        stop = m.annotations(live).get(STOP)
        assert stop and stop != "odh-notebook-controller-lock", stop
    finally:
        harness.restore_culling()

    # resume (helper_test.go restartNotebook): drop the stop annotation
    async def resume():
        await harness.client.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {STOP: None}}}, "merge",
                                   name=m.name(nb), namespace=m.namespace(nb))
    harness.run(resume())
    _sts_ready(harness, nb)


# ------------------------------------------------------------------ 4. update


def test_update_rolls_statefulset(harness, notebooks, opts):
    nb = notebooks[0]

    async def update():
        # the controllers keep writing the Notebook (status, culler annotations): a stale
        # resourceVersion is retried on the latest, as kubectl / client-go RetryOnConflict do
        from odh_kubeflow_amd.runtime.retry import retry_on_conflict

        async def once():
            cur = await harness.client.get(kinds.NOTEBOOK, m.name(nb), m.namespace(nb))
            cur["spec"]["template"]["spec"]["containers"][0]["image"] = opts.updated_image
            await harness.client.update(cur)
        await retry_on_conflict(once)
    harness.run(update())
    _sts_ready(harness, nb, image=opts.updated_image)


# ------------------------------------------------------------------ 5. deletion


def test_delete_removes_dependents(harness, notebooks, opts):
    if opts.skip_deletion:
        pytest.skip("--skip-deletion")

    async def delete():
        for nb in notebooks:
            await harness.client.delete(kinds.NOTEBOOK, m.name(nb), m.namespace(nb))
    harness.run(delete())
    for nb in notebooks:
        name, ns = m.name(nb), m.namespace(nb)
        left = [(kinds.NOTEBOOK, name, ns), (kinds.STATEFUL_SET, name, ns), (kinds.SERVICE, name, ns),
                (kinds.SERVICE, f"{name}-kube-rbac-proxy", ns), (kinds.SERVICE_ACCOUNT, name, ns),
                (kinds.CONFIG_MAP, f"{name}-kube-rbac-proxy-config", ns), (kinds.NETWORK_POLICY, f"{name}-ctrl-np", ns),
                (kinds.NETWORK_POLICY, f"{name}-kube-rbac-proxy-np", ns),
                (kinds.CLUSTER_ROLE_BINDING, f"{name}-rbac-{ns}-auth-delegator", None)]

        async def gone():
            remaining = []
            for kind, n, nsp in left:
                try:
                    await harness.client.get(kind, n, nsp)
                    remaining.append(n)
                except ApiError as e:
                    if e.code != 404:
                        raise
            routes = [r for r in await harness.client.list(kinds.HTTP_ROUTE, harness.ctrl_ns)
                      if m.labels(r).get("notebook-name") == name and m.labels(r).get("notebook-namespace") == ns]
            return not remaining and not routes
        harness.eventually(gone, what=f"dependents of {name} deleted")
