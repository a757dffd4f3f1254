"""bench.py under torch.distributed.run (world_size 2, gloo, CPU): the driver's multi-GPU
launch contract end to end — one JSON line from rank 0 with the contract fields."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-gpu-probe"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0 and d["p50_ready_ms"] > 0
    assert len(d["rank_ms_per_step"]) == 2
    cpu = d["cpu_ms_per_step"]
    assert len(cpu["ranks"]) == 2 and all(x > 0 for x in cpu["ranks"])
    assert cpu["apiserver"] >= 0 and cpu["scheduler"] >= 0  # rank 0's child processes
    # each rank's shard pod, as deployed: a kf, an odh and a webhook process
    assert {f"control_plane_{p}_{r}" for p in ("kf", "odh", "webhook") for r in (0, 1)} <= set(cpu), cpu
    if "apiserver_profile_per_step" in d:  # native apiserver built: write calls per notebook, by verb
        w = d["writes_per_notebook"]
        assert w["total"] == pytest.approx(w["create"] + w["update"] + w["patch"] + w["delete"], abs=0.05)
        assert w["create"] >= 3 and w["delete"] >= 1


def test_bench_single_process_contract():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-gpu-probe"], cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["odh_webhook_path"] is True


def test_bench_reference_emulation_serialises():
    """--reference-emulation restores the reference's blocking lock removal (1 s + 5 s
    backoff, ``odh/controllers/notebook_controller.go:143-174``): ≈6 s per notebook."""
    out = subprocess.run([sys.executable, "bench.py", "--arch", "inprocess", "--reference-emulation", "--steps", "1",
                          "--warmup", "0", "--no-gpu-probe"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d["config"]["reference_emulation"] is True
    assert 5500 < d["p50_ready_ms"] < 9000


def test_numa_bind_pins_to_the_gpus_physical_cores(tmp_path, monkeypatch):
    """``numa_bind``: the GPU's NUMA node (from its PCI address), one SMT thread per core,
    intersected with the allowed CPUs; any missing piece leaves placement alone."""
    import os

    from odh_kubeflow_amd.ops import telemetry
    from odh_kubeflow_amd.parallel import bench_dist

    root = tmp_path / "sys"
    telemetry.write_fake_sysfs(str(root), gpus=2)
    bdf = telemetry.Telemetry(str(root)).devices()[1].pci_bdf
    (root / "bus" / "pci" / "devices" / bdf).mkdir(parents=True)
    (root / "bus" / "pci" / "devices" / bdf / "numa_node").write_text("1\n")
    (root / "devices" / "system" / "node" / "node1").mkdir(parents=True)
    (root / "devices" / "system" / "node" / "node1" / "cpulist").write_text("4-7,12-15\n")
    for c in range(16):
        d = root / "devices" / "system" / "cpu" / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        d.joinpath("thread_siblings_list").write_text(f"{c % 8},{c % 8 + 8}\n")
    calls = []
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append(set(cpus)))
    out = bench_dist.numa_bind(1, str(root))
    assert out == {"gpu": bdf, "numa_node": 1, "cores": 4} and calls == [{4, 5, 6, 7}]
    monkeypatch.setenv("ODH_BENCH_NUMA_BIND", "0")
    assert bench_dist.numa_bind(1, str(root)) is None
    monkeypatch.delenv("ODH_BENCH_NUMA_BIND")
    assert bench_dist.numa_bind(0, str(root)) is None  # GPU 0 has no PCI numa_node file: untouched
    assert len(calls) == 1


def test_bench_namespaces_per_rank_assigned_by_the_shard_hash():
    """``--namespaces-per-rank M`` (sharded): each rank's M namespaces are created unlabelled and
    labelled by the shipped NamespaceShardAssigner, so a shard serves the namespaces that hash
    to it — whichever rank drives them; the per-shard load is reported."""
    import zlib

    from odh_kubeflow_amd.parallel.bench_dist import bench_namespaces

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "8", "--warmup", "1",
           "--no-gpu-probe", "--namespaces-per-rank", "4", "--burst", "4", "--burst-rounds", "1",
           "--resident", "16", "--resident-window", "1", "--resident-steps", "2"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d["config"]["namespaces_per_rank"] == 4 and d["burst"]["all_ok"]
    res = d["resident"]  # 16 resident notebooks over both ranks' namespaces, the culler checking them
    assert res["all_ok"] and res["notebooks"] == 16 and res["at_rest"]["notebook_triggered_reconciles_kf_odh"] == 0
    load = d["shard_load"]
    assert load["assigned_by"].startswith("NamespaceShardAssigner")
    want: dict = {}
    for r in range(2):
        for ns in bench_namespaces(r, 4):
            k = str(zlib.crc32(ns.encode()) % 2)
            want[k] = want.get(k, 0) + 1
    assert {k: v["namespaces"] for k, v in load["shards"].items()} == want
    assert sum(v["notebooks"] for v in load["shards"].values()) == 16
    for k, v in load["shards"].items():
        if v["notebooks"]:
            assert set(v["cpu_ms_per_notebook"]) == {f"control_plane_kf_{k}", f"control_plane_culler_{k}",
                                                     f"control_plane_odh_{k}", f"control_plane_webhook_{k}"}


def test_shard_load_report():
    from odh_kubeflow_amd.parallel.bench_dist import bench_namespaces, shard_load

    assert bench_namespaces(3) == ["bench-3"]
    nss = bench_namespaces(1, 3)
    assert len(set(nss)) == 3 and all(n.startswith("bench-1-") for n in nss) and nss == bench_namespaces(1, 3)
    out = shard_load({"a": 6, "b": 2, "c": 4}, {"a": "0", "b": "1", "c": "1"},
                     {"control_plane_kf_0": 0.06, "control_plane_kf_1": 0.03, "kubelet_1": 9.0, "rank": 1.0},
                     2.0, "hash")
    assert out["shards"]["0"] == {"namespaces": 1, "notebooks": 6, "notebooks_per_s": 3.0,
                                  "cpu_ms_per_notebook": {"control_plane_kf_0": 10.0}}
    assert out["shards"]["1"]["notebooks"] == 6 and out["shards"]["1"]["cpu_ms_per_notebook"] == {
        "control_plane_kf_1": 5.0}  # the platform's kubelet_1 is not shard 1's
    assert out["max_over_mean_notebooks"] == 1.0


def test_io_per_notebook_divides_traffic_and_counts_relists():
    """Watch events and requests are per notebook of the window; lists in the window (a watch
    answered 410 Gone, then relisted) are counted, not divided, and only reported when any."""
    from odh_kubeflow_amd.parallel.bench_dist import io_delta, io_per_notebook

    a = {"kf": {"watch_events": {"Pod": 2}, "requests": {"POST": 1}, "lists": {"Pod": 1, "Notebook": 1}}}
    b = {"kf": {"watch_events": {"Pod": 42}, "requests": {"POST": 21}, "lists": {"Pod": 2, "Notebook": 1}}}
    quiet = {"odh": {"watch_events": {"Service": 20}, "requests": {}, "lists": {"Service": 1}}}
    out = io_per_notebook([io_delta(a, b), io_delta(quiet, quiet)], 10)
    assert out["kf"]["watch_events"] == {"Pod": 4.0, "total": 4.0}
    assert out["kf"]["requests"] == {"POST": 2.0, "total": 2.0}
    assert out["kf"]["relists_in_window"] == {"Pod": 1, "total": 1} and "lists" not in out["kf"]
    assert "relists_in_window" not in out["odh"]


def test_on_top_io_net_of_the_populations_rest_traffic():
    """The on-top counts include the population's heartbeats of the same span: the at-rest rate
    times that span comes off, never below zero, and a kind the rest window lacks is kept."""
    from odh_kubeflow_amd.parallel.bench_dist import io_minus, io_per_notebook

    top = {"culler": {"watch_events": {"Notebook": 130, "Pod": 40}, "requests": {"PATCH": 110, "POST": 30}}}
    rest = {"culler": {"watch_events": {"Notebook": 300}, "requests": {"PATCH": 300, "GET": 5}}}
    out = io_per_notebook([io_minus(top, rest, 1 / 3)], 10)  # the on-top span: a third of the rest window
    assert out["culler"]["watch_events"] == {"Pod": 4.0, "Notebook": 3.0, "total": 7.0}
    assert out["culler"]["requests"] == {"POST": 3.0, "PATCH": 1.0, "total": 4.0}
    assert io_minus(top, {}, 1.0) == top
