"""Operator tooling: the notebook load generator (kf/loadtest/start_notebooks.py counterpart)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_loadtest_local_cluster_measures_every_notebook():
    out = subprocess.run([sys.executable, "tools/loadtest.py", "-l", "4", "-n", "lt", "--local", "--inject-auth"],
                         cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["count"] == 4 and d["ready"] == 4 and d["p50_ready_ms"] > 0
