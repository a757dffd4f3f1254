"""Native amdgpu telemetry sampler against a synthetic sysfs tree (CPU only)."""

import time

from odh_kubeflow_amd.ops.telemetry import Telemetry, set_fake_counter, write_fake_sysfs


def test_discovers_gpu_nodes_and_skips_cpu(tmp_path):
    minors = write_fake_sysfs(str(tmp_path), gpus=8)
    t = Telemetry(str(tmp_path))
    devs = t.devices()
    assert len(devs) == 8
    assert [d.render_minor for d in devs] == minors
    assert all(d.vram_total == 288 * 10 ** 9 for d in devs)
    assert [d.physical for d in devs] == list(range(8))
    t.close()


def test_partition_mode_shares_physical(tmp_path):
    write_fake_sysfs(str(tmp_path), gpus=2, partitions=4)
    t = Telemetry(str(tmp_path))
    assert [d.physical for d in t.devices()] == [0, 0, 0, 0, 4, 4, 4, 4]
    t.close()


def test_read_and_window(tmp_path):
    minors = write_fake_sysfs(str(tmp_path), gpus=2)
    set_fake_counter(str(tmp_path), minors[1], busy=87, vram_used=5 << 30)
    t = Telemetry(str(tmp_path))
    assert t.read(1)["busy"] == 87 and t.read(1)["vram_used"] == 5 << 30
    assert t.read(0)["busy"] == 0
    t.start(interval_ms=5, capacity=1000)
    time.sleep(0.15)
    set_fake_counter(str(tmp_path), minors[0], busy=100)
    time.sleep(0.1)
    w1 = t.window(1, 10.0)
    assert w1.n > 5 and w1.busy_mean == 87 and w1.busy_max == 87
    w0 = t.window(0, 0.05)
    assert w0.busy_max == 100
    w0all = t.window(0, 10.0)
    assert 0 < w0all.busy_mean < 100
    assert t.sweeps() > 5
    t.close()


def test_missing_counter_is_unavailable_not_idle(tmp_path):
    import os

    minors = write_fake_sysfs(str(tmp_path), gpus=1)
    os.remove(os.path.join(str(tmp_path), "class", "drm", f"renderD{minors[0]}", "device", "gpu_busy_percent"))
    t = Telemetry(str(tmp_path))
    assert t.read(0)["busy"] == -1
    t.start(interval_ms=5, capacity=100)
    time.sleep(0.05)
    w = t.window(0, 5.0)
    assert w.n > 0 and w.unavailable == w.n and w.busy_mean == -1
    t.close()


def test_push_injects_samples(tmp_path):
    write_fake_sysfs(str(tmp_path), gpus=1)
    t = Telemetry(str(tmp_path))
    for b in (10, 20, 30):
        t.push(0, b)
    w = t.window(0, 5.0)
    assert w.n == 3 and abs(w.busy_mean - 20) < 1e-9 and w.busy_max == 30
    t.close()


def test_empty_root(tmp_path):
    t = Telemetry(str(tmp_path / "nothing"))
    assert len(t) == 0 and t.read(0) is None
    t.close()
