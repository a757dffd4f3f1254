"""kf NotebookReconciler: envtest-style integration tests (kf/controllers/*_test.go analogues)."""

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.controllers.notebook import (create_notebook_status, generate_service, generate_statefulset,
                                                   generate_virtual_service, nb_name_from_involved_object)
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.testing.apiserver.inprocess import StoreReader
from odh_kubeflow_amd.runtime.controller import Request


def test_generate_statefulset_shape():
    nb = notebook("nb1", "user", gpus=1, labels={"team": "a"},
                  annotations={"notebooks.kubeflow.org/x": "1", "kubectl.kubernetes.io/last": "x", "keep": "y"})
    sts = generate_statefulset(nb, False, env={})
    assert sts["metadata"]["name"] == "nb1"
    assert sts["spec"]["replicas"] == 1
    assert sts["spec"]["selector"] == {"matchLabels": {"statefulset": "nb1"}}
    tl = sts["spec"]["template"]["metadata"]["labels"]
    assert tl == {"statefulset": "nb1", "notebook-name": "nb1", "opendatahub.io/workbenches": "true", "team": "a"}
    # annotations containing "kubectl" or "notebook" are not copied to the pod (notebook_controller.go:488)
    assert sts["spec"]["template"]["metadata"]["annotations"] == {"keep": "y"}
    c = sts["spec"]["template"]["spec"]["containers"][0]
    assert c["workingDir"] == "/home/jovyan"
    assert c["ports"] == [{"containerPort": 8888, "name": "notebook-port", "protocol": "TCP"}]
    assert {"name": "NB_PREFIX", "value": "/notebook/user/nb1"} in c["env"]
    assert c["resources"]["limits"]["amd.com/gpu"] == "1"
    assert sts["spec"]["template"]["spec"]["securityContext"] == {"fsGroup": 100}


def test_generate_statefulset_stopped_generate_name_and_fsgroup_off():
    long = "n" * 53
    nb = notebook(long, "user", annotations={"kubeflow-resource-stopped": "odh-notebook-controller-lock"})
    sts = generate_statefulset(nb, True, env={"ADD_FSGROUP": "false"})
    assert sts["metadata"] == {"generateName": "nb-", "namespace": "user"}
    assert sts["spec"]["replicas"] == 0
    assert "securityContext" not in sts["spec"]["template"]["spec"]


def test_existing_nb_prefix_not_overwritten():
    nb = notebook("nb1", "user", extra_container={"env": [{"name": "NB_PREFIX", "value": "/custom"}]})
    c = generate_statefulset(nb, False, env={})["spec"]["template"]["spec"]["containers"][0]
    assert c["env"] == [{"name": "NB_PREFIX", "value": "/custom"}]


def test_generate_service_and_vs():
    nb = notebook("nb1", "user", extra_container={"ports": [{"containerPort": 9999, "name": "x"}]},
                  annotations={"notebooks.kubeflow.org/http-headers-request-set": '{"X-A": "b"}',
                               "notebooks.kubeflow.org/http-rewrite-uri": "/"})
    svc = generate_service(nb)
    assert svc["spec"]["ports"] == [{"name": "http-notebook", "port": 80, "targetPort": 9999, "protocol": "TCP"}]
    vs = generate_virtual_service(nb, env={"CLUSTER_DOMAIN": "c.local", "ISTIO_GATEWAY": "gw/g"})
    assert vs["metadata"]["name"] == "notebook-user-nb1"
    http = vs["spec"]["http"][0]
    assert http["headers"]["request"]["set"] == {"X-A": "b"}
    assert http["rewrite"]["uri"] == "/"
    assert http["match"][0]["uri"]["prefix"] == "/notebook/user/nb1/"
    assert http["route"][0]["destination"] == {"host": "nb1.user.svc.c.local", "port": {"number": 80}}
    assert vs["spec"]["gateways"] == ["gw/g"] and vs["spec"]["hosts"] == ["*"]
    bad = notebook("nb1", "user", annotations={"notebooks.kubeflow.org/http-headers-request-set": "not json"})
    assert generate_virtual_service(bad, env={})["spec"]["http"][0]["headers"]["request"]["set"] == {}
    # Go unmarshals into map[string]string: a number / object value fails the whole map, a
    # null value is the zero string
    # (kf/controllers/notebook_controller.go:605-613)
    for raw, want in (('{"X-A": 1}', {}), ('{"X-A": {"b": 1}}', {}), ('{"X-A": "1", "X-B": null}', {"X-A": "1", "X-B": ""}),
                      ('["X-A"]', {}), ("null", {}), ('{"X-A": "1", "X-B": "2"}', {"X-A": "1", "X-B": "2"})):
        odd = notebook("nb1", "user", annotations={"notebooks.kubeflow.org/http-headers-request-set": raw})
        assert generate_virtual_service(odd, env={})["spec"]["http"][0]["headers"]["request"]["set"] == want, raw


def test_create_notebook_status_table():
    # mirrors TestCreateNotebookStatus (kf/controllers/notebook_controller_test.go:94-291)
    nb = {"metadata": {"name": "test", "namespace": "kubeflow-user"}, "status": {}}
    assert create_notebook_status(nb, {}, {}) == {"conditions": [], "readyReplicas": 0, "containerState": {}}
    t = "2022-08-30T01:10:30Z"
    pod = {"status": {"conditions": [
        {"type": "Running", "lastProbeTime": t, "lastTransitionTime": t},
        {"type": "Waiting", "lastProbeTime": t, "lastTransitionTime": t, "reason": "PodInitializing"}]}}
    st = create_notebook_status(nb, {"status": {"readyReplicas": 1}}, pod)
    assert st == {"conditions": [{"type": "Running", "lastProbeTime": t, "lastTransitionTime": t},
                                 {"type": "Waiting", "lastProbeTime": t, "lastTransitionTime": t,
                                  "reason": "PodInitializing"}],
                  "readyReplicas": 1, "containerState": {}}
    t2 = "2022-04-21T01:10:30Z"
    pod = {"status": {"conditions": [{"type": "PodScheduled", "lastProbeTime": t2, "lastTransitionTime": t2,
                                      "message": "0/1 nodes are available: 1 Insufficient cpu.", "status": "false",
                                      "reason": "Unschedulable"}]}}
    st = create_notebook_status(nb, {"status": {}}, pod)
    assert st["conditions"][0]["reason"] == "Unschedulable" and st["readyReplicas"] == 0
    # zero timestamps are stamped with "now"
    st = create_notebook_status(nb, {}, {"status": {"conditions": [{"type": "Ready", "status": "True"}]}}, now=t)
    assert st["conditions"][0]["lastProbeTime"] == t and st["conditions"][0]["lastTransitionTime"] == t


def test_nb_name_from_involved_object(run):
    async def go():
        store = ObjectStore()
        from odh_kubeflow_amd.testing.apiserver.inprocess import InProcessClient
        c = InProcessClient(store)
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "test-notebook-0",
                        "namespace": "test-namespace", "labels": {"notebook-name": "test-notebook"}}, "spec": {}})
        r = StoreReader(store)
        assert nb_name_from_involved_object(r, {"kind": "Pod", "name": "test-notebook-0",
                                                "namespace": "test-namespace"}) == "test-notebook"
        assert nb_name_from_involved_object(r, {"kind": "StatefulSet", "name": "test-notebook",
                                                "namespace": "test-namespace"}) == "test-notebook"
        assert nb_name_from_involved_object(r, {"kind": "Deployment", "name": "x"}) is None
    run(go())


def test_notebook_to_ready_pod_with_gpu(run):
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
            sts = cl.store.peek(kinds.STATEFUL_SET, "nb1", "user")
            assert m.controller_of(sts)["kind"] == "Notebook"
            assert m.labels(sts) == {}  # notebook had no labels
            pod = cl.store.peek(kinds.POD, "nb1-0", "user")
            assert pod["spec"]["nodeName"] == "mi355x-node-0"
            assert m.annotations(pod)["amd.com/gpu-ids"] == "0"
            svc = cl.store.peek(kinds.SERVICE, "nb1", "user")
            assert svc["spec"]["ports"][0]["port"] == 80
            nb = cl.store.peek(kinds.NOTEBOOK, "nb1", "user")
            assert nb["status"]["containerState"].get("running")
            assert await cl.settle()
            # steady state: status is not rewritten when nothing changed
            writes = cl.reconcilers["notebook"].status_writes
            cl.kf.controllers[0].enqueue(Request("user", "nb1"))
            assert await cl.settle()
            assert cl.reconcilers["notebook"].status_writes == writes
            # events from the pod were re-emitted on the notebook
            evs = [e for e in cl.store.list_nocopy(kinds.EVENT, "user") if e["involvedObject"]["kind"] == "Notebook"]
            assert any(e["message"].startswith("Reissued from pod/nb1-0") for e in evs)
    run(go())


def test_stop_annotation_scales_to_zero_and_resume(run):
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"))
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {"kubeflow-resource-stopped": "now"}}},
                                 name="nb1", namespace="user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.POD, "nb1-0", "user") is None)
            assert cl.store.peek(kinds.STATEFUL_SET, "nb1", "user")["spec"]["replicas"] == 0
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "nb1", "user")["status"]["readyReplicas"] == 0)
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {"kubeflow-resource-stopped": None}}},
                                 name="nb1", namespace="user")
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"))
    run(go())


def test_eight_notebooks_fill_eight_gpus_ninth_unschedulable(run):
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            for i in range(9):
                await cl.admin.create(notebook(f"nb{i}", "user", gpus=1))
            assert await cl.wait_for(lambda: sum(cl.notebook_ready(f"nb{i}", "user") for i in range(9)) == 8, 10)
            ids = sorted(m.annotations(cl.store.peek(kinds.POD, f"nb{i}-0", "user")).get("amd.com/gpu-ids", "-")
                         for i in range(9))
            assert sorted(i for i in ids if i != "-") == [str(i) for i in range(8)]
            pending = [i for i in range(9) if not cl.notebook_ready(f"nb{i}", "user")][0]
            assert await cl.wait_for(lambda: any(
                c.get("reason") == "Unschedulable" for c in
                (cl.store.peek(kinds.NOTEBOOK, f"nb{pending}", "user").get("status") or {}).get("conditions") or []))
            # free one GPU: the pending notebook lands on it
            other = (pending + 1) % 9
            await cl.admin.delete(kinds.NOTEBOOK, f"nb{other}", "user")
            assert await cl.wait_for(lambda: cl.notebook_ready(f"nb{pending}", "user"), 10)
    run(go())


def test_gpu_allocation_is_first_free_whatever_the_namespace(run):
    """The device plugin's policy: lowest free indices; a namespace label steers nothing
    (the old ``amd.com/gpu-affinity`` steering is gone — no real scheduler honours it)."""
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.admin.create({"apiVersion": "v1", "kind": "Namespace",
                                   "metadata": {"name": "team", "labels": {"amd.com/gpu-affinity": "5_6"}}})
            await cl.ensure_namespace("other")
            await cl.admin.create(notebook("a", "team", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("a", "team"), 10)
            await cl.admin.create(notebook("b", "team", gpus=2))
            assert await cl.wait_for(lambda: cl.notebook_ready("b", "team"), 10)
            await cl.admin.create(notebook("c", "other", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("c", "other"), 10)

            def ids(nm, ns):
                return m.annotations(cl.store.peek(kinds.POD, f"{nm}-0", ns))["amd.com/gpu-ids"]
            assert ids("a", "team") == "0"
            assert ids("b", "team") == "1,2"
            assert ids("c", "other") == "3"
            assert m.labels(cl.store.peek(kinds.POD, "b-0", "team"))["amd.com/gpu-index"] == "1"
            # a released GPU is the next one handed out
            await cl.admin.delete(kinds.NOTEBOOK, "a", "team")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.POD, "a-0", "team") is None, 10)
            await cl.admin.create(notebook("d", "other", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("d", "other"), 10)
            assert ids("d", "other") == "0"
    run(go())


def test_restart_annotation_deletes_pod(run):
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user"))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"))
            uid0 = m.uid(cl.store.peek(kinds.POD, "nb1-0", "user"))
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                "notebooks.opendatahub.io/notebook-restart": "true"}}}, name="nb1", namespace="user")
            assert await cl.wait_for(lambda: (cl.store.peek(kinds.POD, "nb1-0", "user") or {}).get("metadata", {})
                                     .get("uid", uid0) != uid0)
            assert await cl.wait_for(lambda: "notebooks.opendatahub.io/notebook-restart" not in
                                     m.annotations(cl.store.peek(kinds.NOTEBOOK, "nb1", "user")))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"))
    run(go())


def test_istio_virtual_service_and_spec_drift(run):
    async def go():
        async with LocalCluster(ClusterConfig(env={"USE_ISTIO": "true"})) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user"))
            assert await cl.wait_for(lambda: cl.store.peek(kinds.VIRTUAL_SERVICE, "notebook-user-nb1", "user") is not None)
            vs = await cl.admin.get(kinds.VIRTUAL_SERVICE, "notebook-user-nb1", "user")
            vs["spec"]["hosts"] = ["evil"]
            await cl.admin.update(vs)
            assert await cl.wait_for(lambda: cl.store.peek(kinds.VIRTUAL_SERVICE, "notebook-user-nb1",
                                                           "user")["spec"]["hosts"] == ["*"])
            # STS drift is reverted too
            sts = await cl.admin.get(kinds.STATEFUL_SET, "nb1", "user")
            sts["spec"]["template"]["spec"]["containers"][0]["image"] = "other"
            await cl.admin.update(sts)
            assert await cl.wait_for(lambda: cl.store.peek(kinds.STATEFUL_SET, "nb1", "user")["spec"]["template"]
                                     ["spec"]["containers"][0]["image"] == "rocm/pytorch:latest")
    run(go())


def test_gpu_shm_sized_per_gpu_and_overridable():
    from odh_kubeflow_amd.controllers.notebook import generate_statefulset

    env = {"GPU_SHM_SIZE_PER_GPU": "16Gi"}
    sts = generate_statefulset(notebook("nb", "ns", gpus=4), False, env)
    spec = sts["spec"]["template"]["spec"]
    assert {"name": "dshm", "emptyDir": {"medium": "Memory", "sizeLimit": "64Gi"}} in spec["volumes"]
    assert {"name": "dshm", "mountPath": "/dev/shm"} in spec["containers"][0]["volumeMounts"]
    # annotation override, opt-out, CPU notebooks and user-provided /dev/shm are left alone
    sts = generate_statefulset(notebook("nb", "ns", gpus=2, annotations={"amd.com/shm-size": "100Gi"}), False, env)
    assert sts["spec"]["template"]["spec"]["volumes"][0]["emptyDir"]["sizeLimit"] == "100Gi"
    sts = generate_statefulset(notebook("nb", "ns", gpus=2, annotations={"amd.com/shm-size": "0"}), False, env)
    assert "volumes" not in sts["spec"]["template"]["spec"]
    assert "volumes" not in generate_statefulset(notebook("nb", "ns"), False, env)["spec"]["template"]["spec"]
    own = notebook("nb", "ns", gpus=1)
    own["spec"]["template"]["spec"]["containers"][0]["volumeMounts"] = [{"name": "mine", "mountPath": "/dev/shm"}]
    assert "volumes" not in generate_statefulset(own, False, env)["spec"]["template"]["spec"]
    # off unless configured (the reference copies the pod spec verbatim)
    assert "volumes" not in generate_statefulset(notebook("nb", "ns", gpus=1), False, {})["spec"]["template"]["spec"]


def test_multi_gpu_env_defaults():
    from odh_kubeflow_amd.controllers.notebook import generate_statefulset, parse_env_pairs

    assert parse_env_pairs(" A=1, B = x=y ,bad,,=v") == [("A", "1"), ("B", "x=y")]
    env = {"MULTI_GPU_ENV": "HSA_ENABLE_IPC_MODE_LEGACY=0,NB_PREFIX=/nope"}

    def env_of(nb):
        c = generate_statefulset(nb, False, env)["spec"]["template"]["spec"]["containers"][0]
        return {e["name"]: e.get("value") for e in c.get("env") or []}

    e = env_of(notebook("nb", "ns", gpus=2))
    assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert e["NB_PREFIX"] == "/notebook/ns/nb"  # a variable already set wins
    assert "HSA_ENABLE_IPC_MODE_LEGACY" not in env_of(notebook("nb", "ns", gpus=1))  # one GPU: no collectives
    assert "HSA_ENABLE_IPC_MODE_LEGACY" not in env_of(notebook("nb", "ns"))


def test_pod_ready_seconds_observed_on_ready_transitions(run):
    """``notebook_pod_ready_seconds`` (declared in round 1, never observed) is recorded once
    per transition to Ready — creation, then resume — and exported on /metrics."""
    from prometheus_client import generate_latest

    def count(cl):
        for line in generate_latest(cl.kf.registry).decode().splitlines():
            if line.startswith('notebook_pod_ready_seconds_count{namespace="user"}'):
                return float(line.split()[-1])
        return 0.0

    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
            assert await cl.settle()
            assert count(cl) == 1
            cl.kf.controllers[0].enqueue(Request("user", "nb1"))  # steady state: no new sample
            assert await cl.settle()
            assert count(cl) == 1
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {"kubeflow-resource-stopped": "t"}}},
                                 name="nb1", namespace="user")
            assert await cl.wait_for(lambda: not cl.notebook_ready("nb1", "user"))
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {"kubeflow-resource-stopped": None}}},
                                 name="nb1", namespace="user")
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
            assert await cl.settle()
            assert count(cl) == 2
    run(go())


def test_pod_ready_seconds_start_time_rule():
    from prometheus_client import CollectorRegistry

    from odh_kubeflow_amd.controllers.metrics import NotebookMetrics
    from odh_kubeflow_amd.utils.timeutil import parse_rfc3339

    mt = NotebookMetrics(type("R", (), {"list": lambda *a, **k: []})(), CollectorRegistry())
    nb = {"metadata": {"namespace": "u", "creationTimestamp": "2026-01-01T00:00:00Z"}}
    first = {"metadata": {"creationTimestamp": "2026-01-01T00:00:02Z"}}
    resumed = {"metadata": {"creationTimestamp": "2026-01-02T00:00:00Z"}}
    t0 = parse_rfc3339("2026-01-01T00:00:00Z")
    assert mt.observe_ready(nb, first, now=t0 + 30) == 30  # first pod: from the Notebook's creation
    assert mt.observe_ready(nb, resumed, now=t0 + 86400 + 7) == 7  # resumed: from the pod's creation


def test_scheduler_binds_concurrently_and_unreserves_a_failed_bind(run):
    """Scheduling decisions are serial (the allocator lock) but binds run concurrently: a
    slow bind does not hold the next pod's decision, the assumption keeps the two apart, and
    a bind that fails releases its devices (kube-scheduler's assume / unreserve)."""
    import asyncio

    from odh_kubeflow_amd.models.errors import ApiError
    from odh_kubeflow_amd.testing.kubelet.node import SchedulerController

    node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n0", "labels": {}},
            "status": {"allocatable": {"amd.com/gpu": "2"}}}

    def pod(name):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "u", "uid": "uid-" + name},
                "spec": {"containers": [{"name": "c", "resources": {"limits": {"amd.com/gpu": "1"}}}]}}

    pods = {p["metadata"]["name"]: p for p in (pod("a"), pod("b"), pod("c"))}

    class Reader:
        def get(self, kind, name, ns=None):
            return pods.get(name)

        def list(self, kind, fields=None, **_):
            return [node] if kind == kinds.NODE else []  # the cache has seen no bind yet

    gate = asyncio.Event()
    binds = []

    class Client:
        async def patch(self, kind, patch, name=None, namespace=None, **_):
            binds.append((name, patch["metadata"]["annotations"]["amd.com/gpu-ids"]))
            if name == "a":
                await gate.wait()  # a slow bind
            if name == "b":
                raise ApiError(409, "Conflict", "bind lost")

    class Recorder:
        def event(self, *a, **k):
            pass

    async def go():
        s = SchedulerController(Client(), Reader(), Recorder())
        ta = asyncio.create_task(s.reconcile(Request("u", "a")))
        await asyncio.sleep(0)
        with pytest.raises(ApiError):  # decided while a's bind is still in flight
            await asyncio.wait_for(s.reconcile(Request("u", "b")), 2)
        await asyncio.wait_for(s.reconcile(Request("u", "c")), 2)  # b's failed bind freed GPU 1
        gate.set()
        await ta
        assert binds == [("a", "0"), ("b", "1"), ("c", "1")]
        assert s.bound == 2 and set(s._assumed) == {"uid-a", "uid-c"}
    run(go())
