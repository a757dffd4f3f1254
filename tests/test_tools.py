"""Operator tooling: the notebook load generator (kf/loadtest/start_notebooks.py counterpart)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_loadtest_local_cluster_measures_every_notebook():
    out = subprocess.run([sys.executable, "tools/loadtest.py", "-l", "4", "-n", "lt", "--local", "--inject-auth"],
                         cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["count"] == 4 and d["ready"] == 4 and d["p50_ready_ms"] > 0


def test_bench_culling_cpu_rehearsal():
    """BASELINE config #5 on a synthetic sysfs: idle notebooks reclaimed on their attributed GPU
    sample, busy ones kept (although Jupyter says idle), reclaimed again once the load ends."""
    import json
    import subprocess
    import sys

    # idle 2 s: last-activity has whole-second resolution, so 1 s could leave a resumed
    # notebook cullable before its GPU's first attributed sample
    out = subprocess.run([sys.executable, "tools/bench_culling.py", "--cpu", "--idle-s", "2", "--period-s", "0.1",
                          "--load-s", "2.5"], capture_output=True, text=True, timeout=120,
                         cwd=__import__("os").path.dirname(__import__("os").path.dirname(__file__)))
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["false_culls_under_load"] == 0 and d["culled"] == 16, d.get("false_cull_signals")
    assert d["gpu_busy_mean_under_load"] >= 90
    assert 0 <= d["idle_reclaim_ms_p50"] < 1500
    assert d["culls_on_attributed_gpu_idle_sample"] == 16
    for nb in d["per_notebook"].values():
        assert nb["idle_phase"]["amdgpu"].startswith("idle") and nb["after_unload"]["amdgpu"].startswith("idle")


def test_coverage_tool_units(tmp_path):
    import importlib.util
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("cov_tool", os.path.join(root, "tools", "coverage.py"))
    cov = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cov)
    src = tmp_path / "m.py"
    src.write_text("x = 1\n\ndef f(a):\n    if a:\n        return 2\n    return 3\n")
    assert cov.executable_lines(str(src)) >= {1, 3, 4, 5, 6}
    assert cov.flag_of("controllers/odh/route.py") == "odh" and cov.flag_of("controllers/notebook.py") == "kf"
    assert cov.flag_of("runtime/informer.py") == "runtime" and cov.flag_of("something_new.py") == "other"


def test_critical_path_from_audit_log(run, tmp_path):
    """tools/critical_path.py over a real audit log of the REST apiserver: every notebook's
    Ready path is found hop by hop, and every write is attributed per notebook."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import critical_path
    finally:
        sys.path.pop(0)
    from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.models.notebook import notebook

    from odh_kubeflow_amd.testing.apiserver import native

    if not native.available():
        pytest.skip("native apiserver not built")
    log = str(tmp_path / "audit.jsonl")

    async def go():
        from odh_kubeflow_amd.testing.apiserver.audit import AuditPolicy

        cfg = ClusterConfig(transport="native", odh=True, webhook=True, audit_log_path=log,
                            audit_policy=AuditPolicy([{"level": "Metadata"}]),
                            env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("bench-0")
            for i in range(3):
                await cl.admin.create(notebook(f"nb{i}", "bench-0", gpus=1))
            for i in range(3):
                assert await cl.wait_for(lambda i=i: cl.notebook_ready(f"nb{i}", "bench-0"), 20)
            assert await cl.settle(10)
            for i in range(3):
                await cl.admin.delete(kinds.NOTEBOOK, f"nb{i}", "bench-0")
            assert await cl.wait_for(lambda: all(cl.store.peek(kinds.NOTEBOOK, f"nb{i}", "bench-0") is None
                                                 for i in range(3)), 20)
    run(go(), timeout=90)
    with open(log) as f:
        out = critical_path.analyse(f, "bench-")
    assert out["notebooks"] == 3
    td = out["teardown"]  # delete → the odh finalizer removed
    assert td["notebooks"] == 3 and td["delete_to_finalizer_removed_ms"]["p50"] >= td["finalizer_write_serve_ms"]["p50"] > 0
    assert {"notebook_create", "sts_create", "pod_create", "pod_ready", "notebook_status"} <= set(out["hops"])
    assert out["create_to_notebook_status_ms"]["p50"] > 0
    w = out["writes_per_notebook"]
    by = w["by_client"]
    assert any(k.endswith(" create statefulsets") and v == 1.0 for k, v in by.items()), by
    assert any(k.endswith(" create notebooks") and v == 1.0 for k, v in by.items()), by
    assert w["total"] == pytest.approx(sum(by.values()), abs=0.1)


def test_critical_path_skips_an_optional_hop_that_is_not_on_the_path():
    """A notebook whose image-pull lock was gone before kf created its StatefulSet (replicas 1
    at once) has no lock-release hop; a later Notebook patch (finalizers) must not be taken
    for one, or the rest of its path is lost."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import critical_path
    finally:
        sys.path.pop(0)
    import json

    def ev(t, verb, res, name, sub=""):
        ts = f"2026-01-01T00:00:00.{t:03d}000Z"
        ts_done = f"2026-01-01T00:00:00.{t:03d}500Z"
        ref = {"resource": res, "namespace": "bench-0", "name": name, **({"subresource": sub} if sub else {})}
        return json.dumps({"stage": "ResponseComplete", "verb": verb, "objectRef": ref, "userAgent": "x/1",
                           "responseStatus": {"code": 200}, "requestReceivedTimestamp": ts,
                           "stageTimestamp": ts_done})

    lines = [ev(1, "create", "notebooks", "nb"), ev(2, "patch", "notebooks", "nb"),  # lock gone early
             ev(3, "create", "statefulsets", "nb"), ev(4, "create", "pods", "nb-0"),
             ev(5, "patch", "notebooks", "nb"),  # finalizer patch, after the pod exists
             ev(6, "create", "pods", "nb-0", "binding"), ev(7, "patch", "pods", "nb-0", "status"),
             ev(8, "update", "statefulsets", "nb", "status"), ev(9, "patch", "notebooks", "nb", "status")]
    out = critical_path.analyse(lines, "bench-")
    assert out["notebooks"] == 1
    assert "lock_release" not in out["hops"] and out["hops"]["pod_create"]
