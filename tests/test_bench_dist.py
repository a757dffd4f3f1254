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
