"""Takeover and cold start with 1000 resident notebooks (reference
``kf/main.go:91-93``, ``odh/main.go:159-160``: a new leader relists and resyncs before it
serves).

``tools/bench_failover.py`` runs one shard's kf, odh and webhook processes with
``--leader-elect`` plus a standby kf and odh replica against the native apiserver, fills the
cluster with 1000 Ready notebooks (every odh auth-path child), SIGKILLs the leaders, then
restarts the new leaders gracefully.  Asserted: the standbys lead and have reconciled every
notebook within 10 s of the kill (a 4 s lease here; the default is 15 s), reading nothing in
lists at takeover (warm standby caches); a fresh process after a graceful restart is serving
within 10 s; new notebooks become Ready after each.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.slow


def test_takeover_and_cold_start_with_1000_resident_notebooks():
    cmd = [sys.executable, "tools/bench_failover.py", "--resident", "1000", "--lease", "4", "--renew", "3",
           "--retry", "0.5"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["objects"]["Notebook"] == 1000 and d["objects"]["Pod"] == 1000
    for role in ("kf", "odh"):
        t = d["takeover_sigkill"][role]
        assert t["drained_s"] is not None and t["drained_s"] < 10.0, t
        assert t["lead_s"] >= 3.0  # a killed leader's lease must expire first (no release)
        assert t["relist_bytes_at_takeover"] < 1 << 20, t  # warm standby: no relist of the population
        c = d["cold_start_graceful"][role]
        assert c["drained_s"] is not None and c["drained_s"] < 10.0, c
        assert c["relist_bytes"] > 1 << 20  # a fresh process lists everything
    for k in ("after_takeover_ready_ms", "after_cold_start_ready_ms"):
        assert d[k]["p50"] is not None
