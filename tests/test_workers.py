"""``--workers W``: the kf and odh managers as one supervisor + W namespace-partitioned worker
processes (``runtime/workers.py``).

* unit: the assignment policy (least-loaded, sticky, system namespaces on worker 0 and not
  counted), the stdin protocol, the ``/metrics`` merge and the worker command lines;
* processes: ``kf_manager --workers 2`` + ``odh_manager --workers 2`` (webhook on the
  supervisor) against the native apiserver serve three namespaces; each notebook's objects are
  written by exactly one worker; the merged ``/metrics`` and ``/debug`` answers add up; a killed
  worker is restarted and its namespaces are served again.

Reference counterpart: none — the reference runs each manager as one process with one worker
per controller (``kf/main.go:87-98``, ``odh/main.go:155-192``).
"""

from __future__ import annotations

import asyncio
import io
import os
import signal

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime import workers as wk
from odh_kubeflow_amd.runtime.controller import Request


class _FakeProc:
    def __init__(self):
        self.stdin = io.StringIO()


def _sup(n=3, system=("opendatahub",)):
    s = wk.WorkerSupervisor("x", n, lambda i, a: [], system_namespaces=system)
    for w in s.workers:
        w.proc = _FakeProc()
    return s


def test_assignment_least_loaded_sticky_and_system_namespaces():
    s = _sup(3)
    for ns in ("default", "opendatahub", "kube-system", "openshift-ingress"):
        assert s.assign(ns) == 0  # system namespaces: worker 0, not counted as load
    got = [s.assign(f"team-{i}") for i in range(6)]
    assert got == [0, 1, 2, 0, 1, 2]  # least loaded, ties to the lowest index
    assert s.assign("team-1") == 1  # sticky
    s.release("team-0")
    s.release("team-3")
    assert s.assign("team-9") == 0  # worker 0 now has no user namespace
    assert "assign team-9" in s.workers[0].proc.stdin.getvalue()
    assert "release team-3" in s.workers[0].proc.stdin.getvalue()
    assert s.assignments()[1] == ["team-1", "team-4"]
    s._on_namespace("DELETED", {"metadata": {"name": "team-4"}}, None)
    assert s.assignments()[1] == ["team-1"]


def test_worker_side_protocol_filters_requests_and_refreshes_the_cache():
    a = wk.WorkerAssignments(1, 2)
    refreshed = []

    class Cache:
        def refresh_namespace(self, ns):
            refreshed.append(ns)
    a.cache = Cache()
    a.apply("assign team-a")
    a.apply("assign team-b")
    a.apply("release team-a")
    a.apply("bogus line")
    assert a.namespaces == {"team-b"} and refreshed == ["team-a", "team-b", "team-a"]
    assert a.request_filter(Request("team-b", "nb")) and not a.request_filter(Request("team-a", "nb"))
    assert a.request_filter(Request("", "cluster-scoped"))
    opts = a.cache_options(extra_namespaces=["opendatahub", ""])
    assert opts["namespaces"] == ["opendatahub"]
    assert opts["namespace_filter"]({"metadata": {"name": "team-b"}})
    assert not opts["namespace_filter"]({"metadata": {"name": "team-c"}})


def test_worker_reads_initial_set_then_follows_stdin(run):
    async def go():
        r, w = os.pipe()
        rf = os.fdopen(r, "rb", buffering=0)
        a = wk.WorkerAssignments(0, 1, stream=rf)
        lost = []
        a.on_lost = lambda: lost.append(True)
        os.write(w, b"assign ns-1\nassign ns-2\nsync\n")
        await asyncio.wait_for(a.start(), 5)
        assert a.namespaces == {"ns-1", "ns-2"}
        os.write(w, b"release ns-1\n")
        for _ in range(100):
            if a.namespaces == {"ns-2"}:
                break
            await asyncio.sleep(0.01)
        assert a.namespaces == {"ns-2"}
        os.close(w)  # the supervisor is gone
        for _ in range(100):
            if lost:
                break
            await asyncio.sleep(0.01)
        assert lost == [True]
        await a.stop()
    run(go())


_FAKE_WORKER = """
import os, sys, time
state = os.environ["FAKE_STATE"]
n = int(open(state).read()) if os.path.exists(state) else 0
open(state, "w").write(str(n + 1))
if os.environ.get("FAKE_FAIL_START") == str(n):
    sys.exit(3)  # dies before it reports ready
print("ready", flush=True)
for _line in sys.stdin:
    pass
"""


def test_failed_worker_restart_is_retried(run, tmp_path):
    """A worker that exits is restarted; when that restart fails (the new process never reports
    ready) the worker stays pending and a later pass brings it back (it was dropped
    for good, its namespaces unserved until the liveness probe killed the pod)."""
    import time

    (tmp_path / "fakeworker.py").write_text(_FAKE_WORKER)
    env = {**os.environ, "PYTHONPATH": str(tmp_path), "FAKE_STATE": str(tmp_path / "starts"), "FAKE_FAIL_START": "1"}

    async def go():
        s = wk.WorkerSupervisor("fakeworker", 1, lambda i, a: [], env=env, start_timeout=10,
                                restart_backoff=(0.05, 0.2))
        await s.start()
        try:
            w = s.workers[0]
            w.proc.kill()  # crash: start 1 fails, start 2 succeeds
            deadline = time.monotonic() + 30
            while time.monotonic() < deadline and not (w.restarts >= 2 and not w.pending and s.alive()):
                await asyncio.sleep(0.05)
            assert s.alive() and not w.pending
            assert w.restarts == 2 and (tmp_path / "starts").read_text() == "3"
        finally:
            await s.stop()
    run(go())


def test_merge_metrics_sums_samples_and_keeps_one_header():
    a = ("# HELP x_total Things.\n# TYPE x_total counter\nx_total{ns=\"a\"} 2.0\nx_created{ns=\"a\"} 100.0\n"
         "# HELP h Hist.\n# TYPE h histogram\nh_bucket{le=\"1.0\"} 1.0\nh_sum 0.5\nh_count 1.0\n")
    b = ("# HELP x_total Things.\n# TYPE x_total counter\nx_total{ns=\"a\"} 3.0\nx_total{ns=\"b\"} 1.0\n"
         "x_created{ns=\"a\"} 50.0\n# HELP h Hist.\n# TYPE h histogram\nh_bucket{le=\"1.0\"} 2.0\nh_sum 1.5\n"
         "h_count 2.0\n")
    out = wk.merge_metrics([a, b])
    assert out.count("# HELP x_total") == 1 and out.count("# TYPE h histogram") == 1
    assert 'x_total{ns="a"} 5.0' in out and 'x_total{ns="b"} 1.0' in out
    assert 'x_created{ns="a"} 50.0' in out  # a creation time: the earliest
    assert 'h_bucket{le="1.0"} 3.0' in out and "h_sum 2.0" in out and "h_count 3.0" in out
    from prometheus_client.parser import text_string_to_metric_families

    fams = {f.name: f for f in text_string_to_metric_families(out)}
    assert set(fams) >= {"x", "h"}
    # gauges are levels, not counts: the same label set from two processes keeps the larger
    g1 = "# HELP last_ts T.\n# TYPE last_ts gauge\nlast_ts{name=\"nb\"} 1.7e9\nlast_ts{name=\"a\"} 5.0\n"
    g2 = "# HELP last_ts T.\n# TYPE last_ts gauge\nlast_ts{name=\"nb\"} 1.6e9\n"
    out = wk.merge_metrics([g1, g2])
    assert 'last_ts{name="nb"} 1700000000.0' in out and 'last_ts{name="a"} 5.0' in out
    # ... except a worker's share of the capacity: those add up
    c = ('# HELP controller_runtime_max_concurrent_reconciles M.\n# TYPE controller_runtime_max_concurrent_reconciles '
         'gauge\ncontroller_runtime_max_concurrent_reconciles{controller="x"} 8.0\n')
    assert 'controller_runtime_max_concurrent_reconciles{controller="x"} 16.0' in wk.merge_metrics([c, c])


def test_worker_command_lines_drop_what_only_the_supervisor_does():
    from odh_kubeflow_amd.cmd import kf_manager, odh_manager

    a = kf_manager.parse(["--master", "http://x", "--workers", "3", "--enable-leader-election", "--metrics-addr",
                          ":8080", "--probe-addr=:8081", "--max-concurrent-reconciles", "4"])
    argv = kf_manager.worker_argv(a, 2, "127.0.0.1:9999")
    assert "--enable-leader-election" not in argv and ":8080" not in argv and "--probe-addr=:8081" not in argv
    assert argv[argv.index("--worker") + 1] == "2/3" and argv[argv.index("--metrics-addr") + 1] == "127.0.0.1:9999"
    assert argv[argv.index("--max-concurrent-reconciles") + 1] == "4" and "--workers" not in argv
    o = odh_manager.parse(["--kube-rbac-proxy-image", "img", "--workers=2", "--leader-elect", "--webhook-port", "9443"])
    argv = odh_manager.worker_argv(o, 0, "127.0.0.1:1")
    assert "--leader-elect" not in argv and "--workers=2" not in argv and argv[argv.index("--worker") + 1] == "0/2"
    o = odh_manager.parse(["--kube-rbac-proxy-image", "img", "--workers=2", "--webhook-replicas", "3",
                           "--leader-elect", "--webhook-port", "9443"])
    argv = odh_manager.replica_argv(o, 1, "127.0.0.1:2")
    assert argv[argv.index("--webhook-replica") + 1] == "1/2" and "--webhook-replicas" not in argv
    assert "--leader-elect" not in argv and "--worker" not in argv and argv[argv.index("--webhook-port") + 1] == "9443"
    with pytest.raises(SystemExit):
        wk.parse_worker("3/3")
    assert wk.parse_worker("1/4") == (1, 4) and wk.parse_worker(None) is None


@pytest.mark.parametrize("flag", ["false", "true"])
def test_odh_manager_configmap_secret_caching_flag(tmp_path, flag):
    """``--cache-configmaps-secrets``: false keeps the reference's uncached, data-stripped
    ConfigMap/Secret reads (``odh/main.go:165-185``); true caches their data, in the workers
    and webhook replicas too (the flag travels on their command lines)."""
    from odh_kubeflow_amd.cmd import odh_manager
    from odh_kubeflow_amd.models.scheme import SCHEME

    for f in ("tls.crt", "tls.key"):
        (tmp_path / f).write_text("x")
    o = odh_manager.parse(["--kube-rbac-proxy-image", "img", "--master", "http://127.0.0.1:1", "--webhook-cert-dir",
                           str(tmp_path), "--cache-configmaps-secrets", flag, "--workers=2", "--webhook-replicas=2"])
    mgr = odh_manager.build(o, env={})
    cm, sec = SCHEME.resolve(kinds.CONFIG_MAP).key, SCHEME.resolve(kinds.SECRET).key
    if flag == "true":
        assert not mgr.client.uncached and not (mgr.cache.transforms or {}).get(cm)
    else:
        assert mgr.client.uncached == {cm, sec} and mgr.cache.transforms.get(cm) is not None
    for argv in (odh_manager.worker_argv(o, 0, "127.0.0.1:1"), odh_manager.replica_argv(o, 0, "127.0.0.1:2")):
        assert argv[argv.index("--cache-configmaps-secrets") + 1] == flag


@pytest.mark.slow
def test_managers_with_workers_serve_partitioned_namespaces(run):
    async def go():
        import aiohttp

        from odh_kubeflow_amd.parallel.platform import NodePlatform
        from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig
        from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
        from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS

        native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
        env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
        drivers = []
        platform = None
        try:
            platform = await NodePlatform(native.url, process=False).start()
            drivers.append(await ControlPlaneShard(ShardConfig(
                native.url, "team-0", arch="unsharded", bootstrap=True, env=env, process=True, workers=2,
                webhook_replicas=2)).start())
            for i in (1, 2):
                drivers.append(await ControlPlaneShard(ShardConfig(native.url, f"team-{i}", arch="unsharded",
                                                                   launch=False, env=env)).start())
            pids = drivers[0].control_plane_pids()
            assert sorted(k for k in pids if "worker" in k) == [
                "kf_manager_worker_0", "kf_manager_worker_1", "odh_manager_worker_0", "odh_manager_worker_1"]
            assert "odh_manager_webhook_replica_0" in pids  # --webhook-replicas 2: one webhook-only child
            ann = {"notebooks.opendatahub.io/inject-auth": "true"}
            for i, d in enumerate(drivers):
                await d.admin.create(notebook("nb", f"team-{i}", image="img", gpus=1, annotations=ann))
            for d in drivers:
                assert await d.wait_for(lambda: d.notebook_ready("nb"), 60)
            base = {p.name: p.base for p in drivers[0].procs}
            async with aiohttp.ClientSession() as http:
                async with http.get(base["kf_manager"] + "/debug/reconciles") as r:
                    doc = await r.json()
                assert doc["workers"] == 2
                assert sum(doc["reconciles"]["notebook-controller"].values()) >= 3 * 3
                # one worker wrote every object of a notebook: 3 namespaces over 2 workers, 2 + 1
                async with http.get(base["odh_manager"] + "/metrics") as r:
                    text = await r.text()
                assert text.count("# TYPE controller_runtime_reconcile_total counter") == 1
                assert 'controller_runtime_max_concurrent_reconciles{controller="odh-notebook-controller"} 16.0' \
                    in text
            # the supervisor and its webhook replica, one port: between them every admission
            # (the create and the odh unlock update) of the three notebooks was served
            wt = await drivers[0].webhook_timings()
            assert set(wt) <= {"odh_manager", "odh_manager_webhook_replica_0"}
            assert sum(d["served"] for d in wt.values()) >= 3 * 2
            # a worker dies: it is restarted and given its namespaces again
            victim = pids["kf_manager_worker_1"]
            os.kill(victim, signal.SIGKILL)
            await asyncio.sleep(1.0)
            await drivers[1].admin.create(notebook("nb2", "team-1", image="img", gpus=1, annotations=ann))
            await drivers[2].admin.create(notebook("nb2", "team-2", image="img", gpus=1, annotations=ann))
            for d in drivers[1:]:
                assert await d.wait_for(lambda: d.notebook_ready("nb2"), 60)
            for i, d in enumerate(drivers):
                for nm in ("nb", "nb2") if i else ("nb",):
                    await d.admin.delete(kinds.NOTEBOOK, nm, f"team-{i}")
            for i, d in enumerate(drivers):
                for nm in ("nb", "nb2") if i else ("nb",):
                    assert await d.wait_for(lambda: d.gone(nm), 60)
            assert await drivers[0].quiesce(0.002, 20)
            routes = await drivers[0].rest.list(kinds.HTTP_ROUTE, "opendatahub")
            assert routes == []  # every route cleaned up by the worker that owns its notebook
        finally:
            for d in reversed(drivers):
                await d.stop()
            if platform is not None:
                await platform.stop()
            await native.stop()
    run(go(), timeout=240)


def test_concurrent_live_reads_of_one_object_are_coalesced_but_fresh(run):
    """``CachedClient._live_get``: reads of one ConfigMap that arrive while a GET of it is in
    flight share the NEXT GET (sent when the current one answers), never one sent before
    they began — so a burst of admissions makes at most one GET in flight + one queued per
    object, and each still sees every write that completed before it started."""
    from odh_kubeflow_amd.models.errors import NotFound
    from odh_kubeflow_amd.runtime.client import CachedClient

    class Writer:
        def __init__(self):
            self.gets = 0
            self.version = 0
            self.gate = None

        async def get(self, kind, name, namespace=None):
            self.gets += 1
            seen = self.version  # the state as of the GET's start
            await self.gate.wait()
            if seen == 0:
                raise NotFound("configmaps", name)
            return {"metadata": {"name": name, "namespace": namespace, "resourceVersion": str(seen)},
                    "data": {"v": str(seen)}}

    class Reader:
        def watching(self, kind, ns):
            return False

    async def go():
        w = Writer()
        w.gate = asyncio.Event()
        c = CachedClient(Reader(), w, uncached=(kinds.CONFIG_MAP,))

        async def read():
            try:
                return (await c.get(kinds.CONFIG_MAP, "cm", "ns"))["data"]["v"]
            except NotFound:
                return None

        first = asyncio.ensure_future(read())
        await asyncio.sleep(0)  # its GET is in flight (sees version 0)
        w.version = 1  # a write completes: every read that begins from now on must see it
        later = [asyncio.ensure_future(read()) for _ in range(20)]
        await asyncio.sleep(0)
        assert w.gets == 1
        w.gate.set()
        assert await first is None  # began before the write: may miss it
        assert await asyncio.gather(*later) == ["1"] * 20  # all fresh, from ONE more GET
        assert w.gets == 2 and c.coalesced_reads == 19
    run(go())


def test_cancelled_queued_live_reader_is_cancelled_and_the_others_still_read(run):
    """A reader queued behind an in-flight GET that is cancelled (its admission timed out, the
    manager stops) raises CancelledError instead of going on to send a GET of its own; the
    readers queued with it still get one fresh GET between them."""
    from odh_kubeflow_amd.runtime.client import CachedClient

    class Writer:
        def __init__(self):
            self.gets = 0
            self.gate = asyncio.Event()

        async def get(self, kind, name, namespace=None):
            self.gets += 1
            await self.gate.wait()
            return {"metadata": {"name": name, "namespace": namespace, "resourceVersion": str(self.gets)}}

    class Reader:
        def watching(self, kind, ns):
            return False

    async def go():
        w = Writer()
        c = CachedClient(Reader(), w, uncached=(kinds.CONFIG_MAP,))
        first = asyncio.ensure_future(c.get(kinds.CONFIG_MAP, "cm", "ns"))
        await asyncio.sleep(0)
        queued = [asyncio.ensure_future(c.get(kinds.CONFIG_MAP, "cm", "ns")) for _ in range(3)]
        await asyncio.sleep(0)
        queued[0].cancel()
        await asyncio.sleep(0)
        w.gate.set()
        await first
        with pytest.raises(asyncio.CancelledError):
            await queued[0]
        rvs = [o["metadata"]["resourceVersion"] for o in await asyncio.gather(*queued[1:])]
        assert rvs == ["2", "2"] and w.gets == 2  # one more GET for the two left, none for the cancelled one
    run(go())


@pytest.mark.slow
def test_split_kf_workers_serve_each_namespace_set_in_two_processes(run):
    """``kf_manager --workers 2 --split-workers``: each namespace set is served by a notebook
    reconciler process and a culler + event re-emitter process, both assigned the set; the
    notebooks become Ready, and the pod/StatefulSet events are re-emitted by the aux worker."""
    async def go():
        import aiohttp

        from odh_kubeflow_amd.parallel.platform import NodePlatform
        from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig
        from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
        from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS

        native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
        env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
        drivers = []
        platform = None
        try:
            platform = await NodePlatform(native.url, process=False).start()
            drivers.append(await ControlPlaneShard(ShardConfig(
                native.url, "team-0", arch="unsharded", bootstrap=True, env=env, process=True, workers=2,
                kf_split_workers=True)).start())
            drivers.append(await ControlPlaneShard(ShardConfig(native.url, "team-1", arch="unsharded",
                                                               launch=False, env=env)).start())
            pids = drivers[0].control_plane_pids()
            assert sorted(k for k in pids if k.startswith("kf_manager_worker")) == [
                "kf_manager_worker_0_aux", "kf_manager_worker_0_notebook",
                "kf_manager_worker_1_aux", "kf_manager_worker_1_notebook"]
            for i, d in enumerate(drivers):
                await d.admin.create(notebook("nb", f"team-{i}", image="img", gpus=1))
            for d in drivers:
                assert await d.wait_for(lambda: d.notebook_ready("nb"), 60)
            base = {p.name: p.base for p in drivers[0].procs}
            async with aiohttp.ClientSession() as http:
                for _ in range(400):
                    async with http.get(base["kf_manager"] + "/debug/reconciles") as r:
                        doc = await r.json()
                    if sum((doc["reconciles"].get("notebook-events") or {}).values()) >= 2:
                        break
                    await asyncio.sleep(0.1)
            assert doc["workers"] == 4 and doc["assignments"]["0"] and doc["assignments"]["1"]
            assert sum(doc["reconciles"]["notebook-controller"].values()) >= 2
            assert sum(doc["reconciles"]["notebook-events"].values()) >= 2
        finally:
            for d in drivers:
                await d.stop()
            if platform is not None:
                await platform.stop()
            await native.stop()
    run(go(), timeout=120)
