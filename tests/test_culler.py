"""Culler: reference unit tables (kf/controllers/culling_controller_test.go) + integration
with the Jupyter API over HTTP and with the amdgpu busy signal (native telemetry on a
synthetic sysfs tree)."""

import asyncio
import time

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.controllers import culling as c
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import (LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION,
                                              STOP_ANNOTATION, notebook)
from odh_kubeflow_amd.testing.notebook_server.jupyter import JupyterContainerRuntime
from odh_kubeflow_amd.utils import timeutil
from odh_kubeflow_amd.utils.timeutil import rfc3339


@pytest.fixture
def clock():
    offset = [0.0]
    timeutil.set_clock(lambda: time.time() + offset[0])
    yield offset
    timeutil.set_clock(None)


def nbmeta(ann=None):
    return {"metadata": {"name": "n", "namespace": "s", **({"annotations": ann} if ann is not None else {})}}


def test_set_and_detect_stop_annotation():
    for meta in (nbmeta(), nbmeta({}), nbmeta({STOP_ANNOTATION: rfc3339()})):
        c.set_stop_annotation(meta)
        assert STOP_ANNOTATION in meta["metadata"]["annotations"]
    assert not c.stop_annotation_is_set(nbmeta())
    assert not c.stop_annotation_is_set(nbmeta({}))
    assert c.stop_annotation_is_set(nbmeta({STOP_ANNOTATION: rfc3339()}))


def test_all_kernels_are_idle():
    assert c.all_kernels_are_idle([])
    assert c.all_kernels_are_idle([{"execution_state": "idle"}, {"execution_state": "idle"}])
    assert not c.all_kernels_are_idle([{"execution_state": "idle"}, {"execution_state": "busy"}])


@pytest.mark.parametrize("ann,idle_min,want", [
    (None, 1440, False),
    ({}, 1440, False),
    ({STOP_ANNOTATION: "now"}, 1440, False),
    ({LAST_ACTIVITY_ANNOTATION: "garbage"}, 1440, False),
    ({LAST_ACTIVITY_ANNOTATION: rfc3339(time.time() - 3600)}, 1440, False),
    ({LAST_ACTIVITY_ANNOTATION: rfc3339(time.time() - 3600)}, 30, True),
    ({LAST_ACTIVITY_ANNOTATION: rfc3339(time.time() - 60 * 60 * 25)}, 1440, True),
])
def test_notebook_is_idle(ann, idle_min, want):
    # the reference drives CULL_IDLE_TIME through os.Setenv + initGlobalVars
    cfg = c.CullerConfig.from_env({"CULL_IDLE_TIME": str(idle_min)})
    assert c.notebook_is_idle(nbmeta(ann), cfg.cull_idle_time_s) is want


def test_config_from_env():
    cfg = c.CullerConfig.from_env({})
    assert cfg.cull_idle_time_s == 1440 * 60 and cfg.check_period_s == 60 and not cfg.enable_culling
    assert cfg.cluster_domain == "cluster.local" and cfg.activity_source == "jupyter"
    assert c.CullerConfig.from_env({"CULL_IDLE_TIME": "abc"}).cull_idle_time_s == 1440 * 60
    with pytest.raises(ValueError):
        c.CullerConfig.from_env({"IDLENESS_CHECK_PERIOD": "x"})
    with pytest.raises(ValueError):
        c.CullerConfig.from_env({"CULLING_ACTIVITY_SOURCE": "vibes"})


def test_kernel_and_terminal_timestamp_updates():
    old = rfc3339(time.time() - 600)
    newer = rfc3339(time.time() - 60)
    nb = nbmeta({LAST_ACTIVITY_ANNOTATION: old})
    assert not c.update_from_kernels(nb, None) and not c.update_from_kernels(nb, [])
    assert c.update_from_kernels(nb, [{"execution_state": "idle", "last_activity": newer},
                                      {"execution_state": "idle", "last_activity": old}])
    assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == newer
    # an older resource time never moves the annotation backwards
    assert not c.update_from_terminals(nb, [{"last_activity": old}])
    # a busy kernel means "active now"
    c.update_from_kernels(nb, [{"execution_state": "busy", "last_activity": old}])
    assert c.annotation_not_after({"metadata": {"annotations": {LAST_ACTIVITY_ANNOTATION: newer}}},
                                  m.annotations(nb)[LAST_ACTIVITY_ANNOTATION])
    assert c.most_recent_time(["bad"]) == ""


def test_check_period(clock):
    nb = nbmeta({LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION: rfc3339()})
    assert not c.culling_check_period_has_passed(nb, 60)
    clock[0] = 61
    assert c.culling_check_period_has_passed(nb, 60)
    assert not c.culling_check_period_has_passed(nbmeta({}), 60)


def test_checks_land_on_a_per_notebook_phase_of_the_period(clock):
    """R notebooks reconciled at the same instant (a manager start) are next checked spread over
    the period — each on its own phase — not R at once every period; each wakes strictly past
    its period, and a notebook keeps its phase from check to check."""
    from odh_kubeflow_amd.runtime.controller import Request

    r = c.CullingReconciler(None, None, config=c.CullerConfig(check_period_s=60.0))
    clock[0] = 0.0

    def due(req, last):  # absolute time of the next check
        return timeutil.now() + r._next_check(req, last)

    t = float(int(timeutil.now()))
    when = [due(Request("ns", f"nb-{i}"), t) for i in range(1000)]
    assert all(t + 60.0 < d <= t + 120.0 + 0.01 for d in when)
    buckets = [0] * 6  # the 60 s after the first possible check, in 10 s buckets
    for d in when:
        buckets[min(5, int((d - t - 60.0) // 10))] += 1
    assert min(buckets) > 120 and max(buckets) < 220  # ~167 each: spread, not a burst
    req = Request("ns", "nb-7")
    first = due(req, t)
    clock[0] = first - time.time()  # the check runs at its slot and stamps its whole second
    assert abs(due(req, float(int(first))) - (first + 60.0)) < 0.01  # a period later, same phase


def test_start_up_time_is_not_idle_time():
    """A Pending pod (image pull, the odh-gpu-probe init container) is not checked, and the
    idle clock starts no earlier than the pod's Ready transition (the reference counts from
    the pod's first sighting, so a start-up slower than CULL_IDLE_TIME culls it unused)."""
    assert c.pod_is_starting({"status": {"phase": "Pending"}})
    assert not c.pod_is_starting({"status": {"phase": "Running"}}) and not c.pod_is_starting({})
    old, ready = rfc3339(time.time() - 600), rfc3339(time.time() - 60)
    pod = {"status": {"phase": "Running", "conditions": [
        {"type": "Ready", "status": "True", "lastTransitionTime": ready}]}}
    nb = nbmeta({LAST_ACTIVITY_ANNOTATION: old})
    c.update_from_pod_start(nb, pod)
    assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == ready
    later = rfc3339(time.time() - 1)
    nb = nbmeta({LAST_ACTIVITY_ANNOTATION: later})
    c.update_from_pod_start(nb, pod)  # never moved backwards
    assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == later
    pod["status"]["conditions"][0]["status"] = "False"
    nb = nbmeta({LAST_ACTIVITY_ANNOTATION: old})
    c.update_from_pod_start(nb, pod)
    assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == old


def test_ready_flaps_do_not_reset_the_idle_clock():
    """Once per pod: a readiness probe that flaps, or a container restart, is a new Ready
    transition of the same pod; the clock it started is not moved again.  A new pod of the
    notebook (restart annotation, resume) starts it once more."""
    born = rfc3339(time.time() - 3600)
    first_ready, stamp, flap = (rfc3339(time.time() - x) for x in (3500, 1800, 5))
    pod = {"metadata": {"creationTimestamp": born}, "status": {"phase": "Running", "conditions": [
        {"type": "Ready", "status": "True", "lastTransitionTime": flap}]}}
    nb = nbmeta({LAST_ACTIVITY_ANNOTATION: stamp})  # newer than the pod: its clock runs already
    c.update_from_pod_start(nb, pod)
    assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == stamp
    older = rfc3339(time.time() - 7200)  # left by the notebook's previous pod
    pod["status"]["conditions"][0]["lastTransitionTime"] = first_ready
    nb = nbmeta({LAST_ACTIVITY_ANNOTATION: older})
    c.update_from_pod_start(nb, pod)
    assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == first_ready


def test_stuck_start_detection():
    assert not c.pod_start_stuck({"status": {"phase": "Pending"}})
    assert not c.pod_start_stuck({"status": {"containerStatuses": [
        {"state": {"waiting": {"reason": "ContainerCreating"}}}]}})
    for reason in ("ImagePullBackOff", "ErrImagePull", "InvalidImageName", "CreateContainerConfigError"):
        assert c.pod_start_stuck({"status": {"containerStatuses": [{"state": {"waiting": {"reason": reason}}}]}})
    # an init container (amd-gpu-probe on a bad GPU) that failed: terminated non-zero, or in back-off
    assert c.pod_start_stuck({"status": {"initContainerStatuses": [{"state": {"terminated": {"exitCode": 1}}}]}})
    assert c.pod_start_stuck({"status": {"initContainerStatuses": [
        {"state": {"waiting": {"reason": "CrashLoopBackOff"}}, "lastState": {"terminated": {"exitCode": 1}}}]}})
    assert c.pod_start_stuck({"status": {"initContainerStatuses": [
        {"state": {"waiting": {"reason": "PodInitializing"}}, "lastState": {"terminated": {"exitCode": 2}}}]}})
    assert not c.pod_start_stuck({"status": {"initContainerStatuses": [{"state": {"terminated": {"exitCode": 0}}},
                                                                       {"state": {"running": {}}}]}})
    cfg = c.CullerConfig.from_env({})
    assert cfg.startup_allowance_s == 600
    assert c.CullerConfig.from_env({"CULL_STARTUP_ALLOWANCE_SECONDS": "2.5"}).startup_allowance_s == 2.5


# ------------------------------------------------------------------ integration


def _cfg(runtime, **env):
    base = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME": "60", "IDLENESS_CHECK_PERIOD_SECONDS": "0.05",
            "CULLER_USE_POD_ENDPOINT": "true"}
    base.update(env)
    return ClusterConfig(culler=True, env=base, runtime_factory=lambda d: runtime)


def test_culler_jupyter_busy_keeps_idle_culls(run, clock):
    rt = JupyterContainerRuntime()

    async def go():
        async with LocalCluster(_cfg(rt)) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("busy", "user", gpus=1))
            await cl.admin.create(notebook("idle", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("busy", "user") and cl.notebook_ready("idle", "user"))
            st_busy, st_idle = rt.state("user", "busy"), rt.state("user", "idle")
            kid = st_busy.start_kernel(busy=True)
            st_idle.start_kernel(busy=False)
            # annotations initialised and the busy kernel observed before time jumps
            assert await cl.wait_for(lambda: c.annotations_exist(cl.store.peek(kinds.NOTEBOOK, "busy", "user")))
            culler0 = cl.reconcilers["culler"]
            assert await cl.wait_for(lambda: any(r[1] == "user/busy" and r[3] and r[3][0]["execution_state"] == "busy"
                                                 for r in list(culler0.recent)), 10)
            n_seen = len(culler0.recent)
            assert await cl.wait_for(lambda: len(culler0.recent) >= n_seen + 2, 10)
            # two hours pass
            clock[0] += 7200
            idle_nb = lambda: cl.store.peek(kinds.NOTEBOOK, "idle", "user")  # noqa: E731
            assert await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(idle_nb()), 10)
            # culled → StatefulSet scaled to zero, pod gone, activity annotations stripped
            assert await cl.wait_for(lambda: cl.store.peek(kinds.POD, "idle-0", "user") is None, 10)
            assert cl.store.peek(kinds.STATEFUL_SET, "idle", "user")["spec"]["replicas"] == 0
            assert await cl.wait_for(lambda: LAST_ACTIVITY_ANNOTATION not in m.annotations(idle_nb()))
            busy = cl.store.peek(kinds.NOTEBOOK, "busy", "user")
            assert STOP_ANNOTATION not in m.annotations(busy), (list(cl.reconcilers["culler"].recent), st_busy.kernels)
            assert st_busy.requests >= 2  # the culler really polled over HTTP
            culler = cl.reconcilers["culler"]
            assert culler.culled == 1
            # culling metrics are exported (the reference forgets them)
            from prometheus_client import generate_latest
            text = generate_latest(cl.kf.registry).decode()
            assert 'notebook_culling_total{name="idle",namespace="user"} 1.0' in text
            assert "last_notebook_culling_timestamp_seconds" in text
            # busy kernel goes idle; later it is culled too
            st_busy.set_kernel_state(kid, "idle")
            n0 = len(culler.recent)
            # let an in-flight sample of the busy kernel land before time jumps
            assert await cl.wait_for(lambda: any(
                r[1] == "user/busy" and r[3] and r[3][0]["execution_state"] == "idle"
                for r in list(culler.recent)[n0:]), 10)
            clock[0] += 7200
            ok = await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, "busy", "user")), 10)
            assert ok, (m.annotations(cl.store.peek(kinds.NOTEBOOK, "busy", "user")), st_busy.kernels, rfc3339())
    run(go(), timeout=60)


class _FailingProbe:
    """Container runtime whose init containers exit 1: the amd-gpu-probe of a bad GPU."""

    exec_init = True
    visible_device = None

    def __init__(self):
        self.calls = 0

    async def run_init(self, pod, container, devices):
        self.calls += 1
        return {"exitCode": 1, "message": '{"ok": false, "error": "GPU 0: GEMM mismatches"}', "wall_ms": 1.0}

    async def start(self, pod, devices):
        raise AssertionError("containers must not start after a failed init container")

    async def stop(self, handle):
        return None

    async def close(self):
        return None


@pytest.mark.parametrize("stuck", [True, False])
def test_pod_that_cannot_start_is_culled_and_frees_its_gpu(run, clock, stuck):
    """a notebook pod that never leaves Pending — its amd-gpu-probe init container
    failing on a bad GPU and retried with back-off — holds its amd.com/gpu devices.  The culler
    checks it anyway (idle since the pod's creation) and the GPU is released; a Pending pod that
    is merely slow (no failure) is left alone until CULL_IDLE_TIME + CULL_STARTUP_ALLOWANCE."""
    from odh_kubeflow_amd.controllers.notebook import GPU_PROBE_ANNOTATION

    class _Slow(_FailingProbe):
        async def run_init(self, pod, container, devices):
            import asyncio

            self.calls += 1
            await asyncio.sleep(3600)  # an init container still working (a huge image, a slow probe)

    rts = []

    def factory(d):
        rts.append(_FailingProbe() if stuck else _Slow())
        return rts[-1]

    async def go():
        env = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME": "60", "IDLENESS_CHECK_PERIOD_SECONDS": "0.05",
               "CULL_STARTUP_ALLOWANCE": "30"}
        async with LocalCluster(ClusterConfig(culler=True, env=env, runtime_factory=factory)) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"}))
            pod = lambda: cl.store.peek(kinds.POD, "nb-0", "user")  # noqa: E731
            nbk = lambda: cl.store.peek(kinds.NOTEBOOK, "nb", "user")  # noqa: E731
            if stuck:
                assert await cl.wait_for(lambda: bool(pod() and (pod().get("status") or {}).get(
                    "initContainerStatuses")), 30)
            else:
                assert await cl.wait_for(lambda: bool(rts) and sum(r.calls for r in rts) >= 1, 30)
            assert pod()["status"]["phase"] == "Pending"
            culler = cl.reconcilers["culler"]
            clock[0] += 61 * 60  # past CULL_IDLE_TIME, inside CULL_IDLE_TIME + the allowance
            if stuck:
                assert await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(nbk()), 10)
                assert await cl.wait_for(lambda: pod() is None, 10)  # its GPU is free again
                assert cl.store.peek(kinds.STATEFUL_SET, "nb", "user")["spec"]["replicas"] == 0
                assert culler.culled == 1 and culler.cull_log[-1]["jupyter"] == "unreachable"
            else:
                n = culler.checks
                import asyncio

                await asyncio.sleep(0.5)  # ≈10 check periods: still starting, so never checked
                assert STOP_ANNOTATION not in m.annotations(nbk()) and culler.checks == n
                clock[0] += 30 * 60  # now older than CULL_IDLE_TIME + CULL_STARTUP_ALLOWANCE
                assert await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(nbk()), 10), (
                    m.annotations(nbk()), list(culler.recent), pod()["metadata"].get("creationTimestamp"), rfc3339())
    run(go(), timeout=60)


def test_culler_no_data_never_culls(run, clock):
    rt = JupyterContainerRuntime()

    async def go():
        cfg = _cfg(rt, CULLER_USE_POD_ENDPOINT="false", CLUSTER_DOMAIN="invalid.example")  # unreachable
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user"))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user"))
            assert await cl.wait_for(lambda: c.annotations_exist(cl.store.peek(kinds.NOTEBOOK, "nb", "user")))
            la = m.annotations(cl.store.peek(kinds.NOTEBOOK, "nb", "user"))[LAST_ACTIVITY_ANNOTATION]
            clock[0] += 30  # within CULL_IDLE_TIME: checks run, no data, nothing changes
            assert await cl.wait_for(lambda: cl.reconcilers["culler"].checks >= 1, 10)
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "user")
            assert m.annotations(nb)[LAST_ACTIVITY_ANNOTATION] == la and STOP_ANNOTATION not in m.annotations(nb)
    run(go(), timeout=60)


def _gpu_of_pods(cl, tel, ns, names):
    """telemetry index of each notebook's GPU, read back the way the node agent reads it:
    the fake kubelet's device-plugin checkpoint (PCI addresses), resolved via the KFD topology."""
    from odh_kubeflow_amd.nodeagent.attribution import DeviceResolver
    from odh_kubeflow_amd.nodeagent.checkpoint import read_checkpoint

    cp = read_checkpoint(cl.device_managers["mi355x-node-0"].checkpoint.path)
    res = DeviceResolver(tel.devices())
    out = {}
    for n in names:
        ids = cp[m.uid(cl.store.peek(kinds.POD, f"{n}-0", ns))]
        out[n] = res.resolve(ids[0])[0]
    return out


def test_culler_amdgpu_signal(run, clock, tmp_path):
    """GPU-busy culling through the production node agent: no pod carries an
    ``amd.com/gpu-ids`` annotation the culler could read; the agent attributes GPUs from
    the (fake) kubelet's device-plugin checkpoint and the culler asks it by pod UID."""
    from odh_kubeflow_amd.ops.telemetry import Telemetry, set_fake_counter, write_fake_sysfs

    minors = write_fake_sysfs(str(tmp_path), gpus=8)
    tel = Telemetry(str(tmp_path)).start(interval_ms=10, capacity=2000)
    rt = JupyterContainerRuntime()

    async def go():
        cfg = _cfg(rt, CULLING_ACTIVITY_SOURCE="amdgpu", IDLENESS_CHECK_PERIOD_SECONDS="0.2")
        cfg.telemetry = tel
        async with LocalCluster(cfg) as cl:
            culler = cl.reconcilers["culler"]
            assert isinstance(culler.gpu, c.NodeAgentActivity)
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("train", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("train", "user"))
            await cl.admin.create(notebook("idle", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("idle", "user"))
            for n in ("train", "idle"):  # strip the fake scheduler's internal annotation
                pod = cl.store.peek(kinds.POD, f"{n}-0", "user")
                await cl.admin.patch(kinds.POD, {"metadata": {"annotations": {"amd.com/gpu-ids": None}}},
                                     name=m.name(pod), namespace="user")
            gid = _gpu_of_pods(cl, tel, "user", ("train", "idle"))
            assert gid["train"] != gid["idle"]
            # "train" runs an MI355X job: its GPU is 97% busy; no kernel is busy in Jupyter
            set_fake_counter(str(tmp_path), minors[gid["train"]], busy=97)
            rt.state("user", "train").start_kernel(busy=False)
            assert await cl.wait_for(lambda: c.annotations_exist(cl.store.peek(kinds.NOTEBOOK, "train", "user")))
            import asyncio
            await asyncio.sleep(0.3)
            clock[0] += 7200
            assert await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, "idle", "user")), 10)
            assert STOP_ANNOTATION not in m.annotations(cl.store.peek(kinds.NOTEBOOK, "train", "user"))
            agent = cl.node_agents["mi355x-node-0"]
            assert agent.attributed_queries > 0 and culler.gpu.requests > 0
            # the job ends: GPU idle → culled after the idle time
            set_fake_counter(str(tmp_path), minors[gid["train"]], busy=0)
            await asyncio.sleep(0.5)
            clock[0] += 7200
            assert await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, "train", "user")), 10)
    try:
        run(go(), timeout=60)
    finally:
        tel.close()


def test_gpu_says_active_vram_policy():
    cfg = c.CullerConfig.from_env({})
    assert cfg.gpu_vram_active_bytes == 0 and cfg.gpu_agent_port == 9464
    held = {"n": 5, "busy_mean": 0.0, "busy_max": 0, "pod_vram_bytes": 200 * 10 ** 9}
    assert not c.gpu_says_active(held, cfg)  # default: resident HBM alone is not activity
    assert c.gpu_says_active({**held, "busy_mean": 40.0}, cfg)
    cfg = c.CullerConfig.from_env({"CULLING_GPU_VRAM_ACTIVE_BYTES": "1e9"})
    assert c.gpu_says_active(held, cfg)
    assert not c.gpu_says_active({**held, "pod_vram_bytes": 10 ** 6}, cfg)
    assert not c.gpu_says_active({**held, "pod_vram_bytes": None}, cfg)


def test_node_agent_endpoint_brackets_ipv6_host_ips():
    """IPv6 / dual-stack-v6 nodes: the node agent URL authority needs ``[addr]:port``; an
    unbracketed literal would make every query fail and culling silently fall back."""
    from odh_kubeflow_amd.controllers.culling import NodeAgentActivity

    a = NodeAgentActivity(port=9464)
    assert a.default_endpoint({"status": {"hostIP": "10.0.0.7"}}) == "10.0.0.7:9464"
    assert a.default_endpoint({"status": {"hostIP": "fd00:10:244::5"}}) == "[fd00:10:244::5]:9464"
    assert a.default_endpoint({"status": {"hostIP": "node-3.example"}}) == "node-3.example:9464"
    assert a.default_endpoint({"status": {}}) is None


class _NoCache:
    def get(self, kind, name, namespace):
        return None  # read through the client


class _PatchRecorder:
    """A client that records the culler's Notebook patches (``CullingReconciler._update``)."""

    def __init__(self, nb):
        self.nb, self.patches = nb, []

    async def get(self, kind, name, namespace):
        return self.nb

    async def patch(self, kind, body, ptype, name, namespace):
        self.patches.append(body)
        return self.nb


def test_culler_write_rules(run):
    """A notebook's first activity annotations go without a resourceVersion precondition
    (nobody else writes them: preconditioned, they conflicted with the notebook controller's
    status write of the same moment on every notebook); periodic checks and a stop keep it;
    a notebook being deleted is not written."""
    nb = notebook("n", "s")
    nb["metadata"]["resourceVersion"] = "7"
    cl = _PatchRecorder(nb)
    rec = c.CullingReconciler(cl, reader=_NoCache(), env={"ENABLE_CULLING": "true"})
    req = c.Request("s", "n")

    async def go():
        await rec._update(req, lambda cur: c.initialize_annotations(cur, None), precondition=False)
        await rec._update(req, lambda cur: c.update_check_timestamp(cur))  # a periodic check
        await rec._update(req, lambda cur: c.set_stop_annotation(cur, None), precondition=False)
        nb["metadata"]["deletionTimestamp"] = rfc3339()
        await rec._update(req, lambda cur: c.initialize_annotations(cur, None), precondition=False)
    run(go())
    first, check, stop = cl.patches
    assert set(first["metadata"]["annotations"]) == {LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION}
    assert "resourceVersion" not in first["metadata"]
    assert check["metadata"]["resourceVersion"] == "7"
    assert STOP_ANNOTATION in stop["metadata"]["annotations"] and stop["metadata"]["resourceVersion"] == "7"


def test_check_stamp_written_every_kth_check_when_nothing_else_changes(run):
    """CULL_CHECK_STAMP_EVERY=k: an idle notebook's check stamp is written on every k-th check
    only (the reference writes it on every check, :171-196; nothing but the culler's own
    schedule reads it).  The checks still run every period, the stamp stays RFC 3339 and at
    most k periods old, and an activity change is written at once."""
    rt = JupyterContainerRuntime()
    k, period = 3, 1.0

    async def go():
        async with LocalCluster(_cfg(rt, IDLENESS_CHECK_PERIOD_SECONDS=str(period),
                                     CULL_CHECK_STAMP_EVERY=str(k))) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user"))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user"), 20)
            st = rt.state("user", "nb")
            st.start_kernel(busy=False)
            nb = lambda: cl.store.peek(kinds.NOTEBOOK, "nb", "user")  # noqa: E731
            assert await cl.wait_for(lambda: c.annotations_exist(nb()), 10)
            culler = cl.reconcilers["culler"]
            c0, s0 = culler.checks, culler.stamps_skipped
            stamps, ages = set(), []
            t_end = time.monotonic() + 6.5 * period
            while time.monotonic() < t_end:
                a = m.annotations(nb())
                stamps.add(a[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION])
                ages.append(time.time() - timeutil.parse_rfc3339(a[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION]))
                await asyncio.sleep(0.05)
            checks, skipped = culler.checks - c0, culler.stamps_skipped - s0
            assert checks >= 5, checks
            assert skipped >= checks // 2, (checks, skipped)
            assert len(stamps) <= checks - skipped + 1
            assert max(ages) <= k * period + 1.5  # whole-second stamps
            # activity is written at once: a busy kernel moves last-activity on the next check
            la0 = m.annotations(nb())[LAST_ACTIVITY_ANNOTATION]
            st.start_kernel(busy=True)
            assert await cl.wait_for(lambda: m.annotations(nb())[LAST_ACTIVITY_ANNOTATION] != la0, 3 * period)
    run(go(), timeout=60)
