"""controller-runtime metric families (names, labels, histogram buckets) as scraped."""

from prometheus_client import CollectorRegistry, generate_latest

from odh_kubeflow_amd.runtime.metrics import RuntimeMetrics


def test_runtime_metrics_exposition():
    reg = CollectorRegistry()
    m = RuntimeMetrics(reg)
    m.child(m.reconcile_total, "notebook", "success").inc()
    m.child(m.reconcile_total, "notebook", "success").inc()
    m.child(m.reconcile_total, "notebook", "requeue").inc()
    m.child(m.reconcile_errors, "notebook").inc()
    for dt in (0.0004, 0.0005, 0.003, 100.0):
        m.child(m.reconcile_time, "notebook").observe(dt)
    m.max_concurrent.labels("notebook").set(8)
    m.on_add("notebook", 3)
    m.on_add("notebook", 4)
    m.on_get("notebook", 2, 0.02)
    m.on_retry("notebook")

    g = reg.get_sample_value
    assert g("controller_runtime_reconcile_total", {"controller": "notebook", "result": "success"}) == 2
    assert g("controller_runtime_reconcile_total", {"controller": "notebook", "result": "requeue"}) == 1
    assert g("controller_runtime_reconcile_errors_total", {"controller": "notebook"}) == 1
    # le is inclusive: 0.0004 and 0.0005 in the 0.0005 bucket, 100 s only in +Inf
    b = {"controller": "notebook"}
    assert g("controller_runtime_reconcile_time_seconds_bucket", {**b, "le": "0.0005"}) == 2
    assert g("controller_runtime_reconcile_time_seconds_bucket", {**b, "le": "0.005"}) == 3
    assert g("controller_runtime_reconcile_time_seconds_bucket", {**b, "le": "60.0"}) == 3
    assert g("controller_runtime_reconcile_time_seconds_bucket", {**b, "le": "+Inf"}) == 4
    assert g("controller_runtime_reconcile_time_seconds_count", b) == 4
    assert abs(g("controller_runtime_reconcile_time_seconds_sum", b) - 100.0039) < 1e-9
    assert g("controller_runtime_max_concurrent_reconciles", b) == 8
    assert g("workqueue_adds_total", {"name": "notebook"}) == 2
    assert g("workqueue_depth", {"name": "notebook"}) == 2
    assert g("workqueue_retries_total", {"name": "notebook"}) == 1
    assert g("workqueue_queue_duration_seconds_count", {"name": "notebook"}) == 1
    text = generate_latest(reg).decode()
    assert "# TYPE controller_runtime_reconcile_total counter" in text
    assert "# TYPE workqueue_queue_duration_seconds histogram" in text


def test_gc_pause_recorder_histogram_and_since():
    """Every cyclic-GC collection is timed (``gc.callbacks``): ``odh_gc_pause_seconds`` per
    generation on the managers' /metrics, and ``since(seq)`` lists only newer pauses."""
    import gc

    from odh_kubeflow_amd.utils.gctune import PauseRecorder

    rec = PauseRecorder(keep=8)
    gc.callbacks.append(rec)
    try:
        gc.collect()
        first = rec.since(0)
        assert first["seq"] >= 1 and first["pauses"][-1][1] == 2 and first["pauses"][-1][2] >= 0
        gc.collect(0)
        newer = rec.since(first["seq"])
        assert [p[1] for p in newer["pauses"]] == [0] and newer["seq"] == first["seq"] + 1
    finally:
        gc.callbacks.remove(rec)
    reg = CollectorRegistry()
    reg.register(rec)
    text = generate_latest(reg).decode()
    assert 'odh_gc_pause_seconds_count{generation="2"} 1.0' in text
    assert 'odh_gc_pause_seconds_bucket{generation="0",le="+Inf"} 1.0' in text
