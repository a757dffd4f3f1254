"""kube-apiserver defaulting in both fake apiservers (``models/defaults.py``, ``native/apiserver``
``api_defaults``) and the end of the reference's StatefulSet/Service write storm
(``common/reconcilehelper/util.go:107-134,166-195`` compares the raw desired pod template
with the defaulted live one, so every reconcile against a real apiserver issues an Update)."""

import asyncio
import copy

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import defaults, kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.controller import Request


def _sts():
    return {"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "s", "namespace": "d"},
            "spec": {"selector": {"matchLabels": {"a": "b"}}, "serviceName": "",
                     "template": {"metadata": {"labels": {"a": "b"}}, "spec": {
                         "containers": [{"name": "c", "image": "rocm/pytorch:latest",
                                         "ports": [{"containerPort": 8888, "name": "notebook-port"}],
                                         "env": [{"name": "POD", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}],
                                         "resources": {"limits": {"cpu": "0.5", "memory": "1024Mi", "amd.com/gpu": "1"},
                                                       "requests": {"cpu": "2000m", "memory": "1000"}},
                                         "readinessProbe": {"httpGet": {"port": 8888}}},
                                        {"name": "sidecar", "image": "quay.io/x/y:v1.2@sha256:abc"}],
                         "volumes": [{"name": "cm", "configMap": {"name": "x"}}, {"name": "sec", "secret": {"secretName": "y"}},
                                     {"name": "shm", "emptyDir": {"medium": "Memory", "sizeLimit": "16384Mi"}}],
                         "serviceAccountName": "nb"}}}}


def _svc():
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "s", "namespace": "d"},
            "spec": {"selector": {"a": "b"}, "ports": [{"name": "http", "port": 80, "targetPort": 8888},
                                                       {"name": "raw", "port": 9000}]}}


def test_defaults_rules_and_idempotence():
    s = defaults.apply("statefulsets.apps", _sts())
    sp = s["spec"]
    assert (sp["replicas"], sp["podManagementPolicy"], sp["revisionHistoryLimit"]) == (1, "OrderedReady", 10)
    assert sp["updateStrategy"] == {"type": "RollingUpdate", "rollingUpdate": {"partition": 0}}
    assert sp["persistentVolumeClaimRetentionPolicy"] == {"whenDeleted": "Retain", "whenScaled": "Retain"}
    ps = sp["template"]["spec"]
    assert (ps["restartPolicy"], ps["dnsPolicy"], ps["schedulerName"], ps["terminationGracePeriodSeconds"]) == \
        ("Always", "ClusterFirst", "default-scheduler", 30)
    assert ps["securityContext"] == {} and ps["serviceAccount"] == "nb" and ps["enableServiceLinks"] is True
    c0, c1 = ps["containers"]
    assert (c0["imagePullPolicy"], c1["imagePullPolicy"]) == ("Always", "IfNotPresent")
    assert c0["terminationMessagePath"] == "/dev/termination-log" and c0["terminationMessagePolicy"] == "File"
    assert c0["ports"][0]["protocol"] == "TCP" and c0["env"][0]["valueFrom"]["fieldRef"]["apiVersion"] == "v1"
    assert c0["resources"] == {"limits": {"cpu": "500m", "memory": "1Gi", "amd.com/gpu": "1"},
                               "requests": {"cpu": "2", "memory": "1k"}}
    assert c0["readinessProbe"] == {"httpGet": {"port": 8888, "path": "/", "scheme": "HTTP"}, "timeoutSeconds": 1,
                                    "periodSeconds": 10, "successThreshold": 1, "failureThreshold": 3}
    assert c1["resources"] == {}
    vols = {v["name"]: v for v in ps["volumes"]}
    assert vols["cm"]["configMap"]["defaultMode"] == 420 and vols["sec"]["secret"]["defaultMode"] == 420
    assert vols["shm"]["emptyDir"]["sizeLimit"] == "16Gi"
    assert sp["template"]["metadata"]["creationTimestamp"] is None
    assert defaults.apply("statefulsets.apps", copy.deepcopy(s)) == s
    v = defaults.apply("services", _svc())["spec"]
    assert (v["type"], v["sessionAffinity"], v["ipFamilies"], v["ipFamilyPolicy"], v["internalTrafficPolicy"]) == \
        ("ClusterIP", "None", ["IPv4"], "SingleStack", "Cluster")
    assert [p["targetPort"] for p in v["ports"]] == [8888, 9000] and {p["protocol"] for p in v["ports"]} == {"TCP"}
    p = defaults.apply("pods", {"spec": {"containers": [{"name": "c", "image": "i:1", "resources": {
        "limits": {"cpu": "1", "amd.com/gpu": "1"}, "requests": {"cpu": "500m"}}}]}})
    assert p["spec"]["containers"][0]["resources"]["requests"] == {"cpu": "500m", "amd.com/gpu": "1"}


def _strip(o):
    o = copy.deepcopy(o)
    for k in ("uid", "resourceVersion", "creationTimestamp", "generation", "managedFields"):
        o["metadata"].pop(k, None)
    o.get("spec", {}).pop("clusterIP", None)
    o.get("spec", {}).pop("clusterIPs", None)
    return o


def test_native_and_python_apiservers_default_identically(run):
    """The C++ apiserver's api_defaults must agree with models/defaults.py byte for byte."""
    async def go():
        results = {}
        for transport in ("inprocess", "native"):
            async with LocalCluster(ClusterConfig(kf=False, transport=transport)) as cl:
                await cl.ensure_namespace("d")
                out = []
                for obj in (_sts(), _svc(), {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"},
                                            "spec": copy.deepcopy(_sts()["spec"]["template"]["spec"])}):
                    out.append(_strip(await cl.admin.create(obj)))
                # an update that drops defaulted fields gets them back, clusterIP is kept
                svc = await cl.admin.get(kinds.SERVICE, "s", "d")
                ip = svc["spec"]["clusterIP"]
                for k in ("sessionAffinity", "clusterIP", "clusterIPs", "ipFamilies"):
                    svc["spec"].pop(k)
                svc = await cl.admin.update(svc)
                assert svc["spec"]["clusterIP"] == ip and svc["spec"]["sessionAffinity"] == "None"
                out.append(_strip(svc))
                results[transport] = out
        for a, b in zip(results["inprocess"], results["native"]):
            assert a == b
    run(go(), timeout=60)


@pytest.mark.parametrize("transport", ["inprocess", "http", "native"])
def test_no_statefulset_or_service_writes_in_steady_state(run, transport):
    """20 steady-state reconciles of a Ready GPU notebook against a defaulting apiserver:
    0 StatefulSet / Service updates, 0 status writes."""
    async def go():
        cfg = ClusterConfig(transport=transport)
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("u")
            nb = notebook("nb", "u", gpus=1, image="rocm/pytorch:latest")
            c = nb["spec"]["template"]["spec"]["containers"][0]
            c["resources"]["limits"].update(cpu="0.5", memory="65536Mi")
            c["readinessProbe"] = {"httpGet": {"port": 8888, "path": "/api"}}
            c["env"] = [{"name": "POD", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}]
            nb["spec"]["template"]["spec"]["volumes"] = [{"name": "shm", "emptyDir": {"medium": "Memory",
                                                                                    "sizeLimit": "16384Mi"}}]
            c["volumeMounts"] = [{"name": "shm", "mountPath": "/dev/shm"}]
            await cl.admin.create(nb)
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "u"), 20)
            assert await cl.settle(10)
            sts = cl.store.peek(kinds.STATEFUL_SET, "nb", "u")
            assert sts["spec"]["podManagementPolicy"] == "OrderedReady"  # the server defaulted it
            assert sts["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]["memory"] == "64Gi"
            writes = []
            client = cl.kf.client
            orig_update, orig_patch = client.update, client.patch

            async def update(obj, *a, **kw):
                writes.append(("update", obj.get("kind"), kw.get("subresource")))
                return await orig_update(obj, *a, **kw)

            async def patch(obj, *a, **kw):
                writes.append(("patch", obj if isinstance(obj, str) else obj.get("kind"), kw.get("subresource")))
                return await orig_patch(obj, *a, **kw)
            client.update, client.patch = update, patch
            ctl = next(x for x in cl.kf.controllers if x.name == "notebook-controller")
            n0 = ctl.reconciles
            for _ in range(20):
                ctl.queue.add(Request("u", "nb"))
                await asyncio.sleep(0)
                assert await cl.settle(10)
            assert ctl.reconciles - n0 >= 20
            assert writes == [], writes
            # a real spec change still goes through
            cur = await cl.admin.get(kinds.NOTEBOOK, "nb", "u")
            cur["spec"]["template"]["spec"]["containers"][0]["image"] = "rocm/pytorch:rocm7.0"
            await cl.admin.update(cur)
            assert await cl.wait_for(lambda: cl.store.peek(kinds.STATEFUL_SET, "nb", "u")["spec"]["template"]["spec"][
                "containers"][0]["image"] == "rocm/pytorch:rocm7.0", 10)
            assert [w for w in writes if w[1] == "StatefulSet"] == [("update", "StatefulSet", None)]
    run(go(), timeout=90)


def _random_pod_spec(rnd, name):
    """A notebook pod spec in the shapes users write: non-canonical quantities, partial
    probes / ports / env sources / volumes — everything the apiserver defaults or
    canonicalises."""
    q_cpu = ["0.5", "500m", "1", "2000m", "1.5", "100m"]
    q_mem = ["1Gi", "1024Mi", "65536Mi", "512M", "2G", "1e9"]
    c = {"name": name, "image": rnd.choice(["rocm/pytorch:latest", "quay.io/x/y:1", "img"])}
    res = {"limits": {"amd.com/gpu": "1"}}  # 8 notebooks fill the node's 8 GPUs
    if rnd.random() < 0.7:
        res["limits"]["cpu"] = rnd.choice(q_cpu)
        res["limits"]["memory"] = rnd.choice(q_mem)
    if rnd.random() < 0.5:
        res["requests"] = {"cpu": rnd.choice(q_cpu), "memory": rnd.choice(q_mem)}
    c["resources"] = res
    if rnd.random() < 0.6:
        c["ports"] = [dict({"containerPort": 8888, "name": "notebook-port"},
                           **({"protocol": "TCP"} if rnd.random() < 0.5 else {}))]
    probe = rnd.choice([None, {"httpGet": {"port": 8888, "path": "/api"}}, {"tcpSocket": {"port": 8888}},
                        {"exec": {"command": ["true"]}, "periodSeconds": 5}])
    if probe:
        c[rnd.choice(["readinessProbe", "livenessProbe"])] = probe
    env = []
    if rnd.random() < 0.5:
        env.append({"name": "POD", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}})
    if rnd.random() < 0.5:
        env.append({"name": "A", "value": "1"})
    if env:
        c["env"] = env
    spec = {"containers": [c]}
    vols = []
    if rnd.random() < 0.5:
        vols.append({"name": "shm", "emptyDir": {"medium": "Memory", "sizeLimit": rnd.choice(["16Gi", "16384Mi"])}})
        c["volumeMounts"] = [{"name": "shm", "mountPath": "/dev/shm"}]
    if rnd.random() < 0.4:
        vols.append({"name": "cfg", "configMap": {"name": "cfg"}})
    if vols:
        spec["volumes"] = vols
    if rnd.random() < 0.3:
        spec["tolerations"] = [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]
    if rnd.random() < 0.3:
        spec["securityContext"] = {"runAsUser": 1000}
    if rnd.random() < 0.3:
        spec["initContainers"] = [{"name": "init", "image": "busybox", "command": ["true"]}]
    return spec


@pytest.mark.parametrize("transport", ["inprocess", "native"])
def test_no_writes_in_steady_state_for_random_pod_specs(run, transport):
    """The write-storm guard over 8 randomly shaped notebooks (seeded): once each is Ready,
    3 more reconciles write nothing to its StatefulSet or Service."""
    import random

    rnd = random.Random(20261016)

    async def go():
        async with LocalCluster(ClusterConfig(transport=transport)) as cl:
            await cl.ensure_namespace("fz")
            names = [f"fz{i}" for i in range(8)]
            for n in names:
                nb = notebook(n, "fz", gpus=1)
                nb["spec"]["template"]["spec"] = _random_pod_spec(rnd, n)
                await cl.admin.create(nb)
            assert await cl.wait_for(lambda: all(cl.notebook_ready(n, "fz") for n in names), 60)
            assert await cl.settle(10)
            writes = []
            client = cl.kf.client
            orig_update, orig_patch = client.update, client.patch

            async def update(obj, *a, **kw):
                writes.append(("update", obj.get("kind"), (obj.get("metadata") or {}).get("name")))
                return await orig_update(obj, *a, **kw)

            async def patch(obj, *a, **kw):
                writes.append(("patch", obj if isinstance(obj, str) else obj.get("kind"), kw.get("name")))
                return await orig_patch(obj, *a, **kw)
            client.update, client.patch = update, patch
            ctl = next(x for x in cl.kf.controllers if x.name == "notebook-controller")
            for _ in range(3):
                for n in names:
                    ctl.queue.add(Request("fz", n))
                await asyncio.sleep(0)
                assert await cl.settle(10)
            assert [w for w in writes if w[1] in ("StatefulSet", "Service")] == [], writes
    run(go(), timeout=120)
