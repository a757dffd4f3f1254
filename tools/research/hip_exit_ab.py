#!/usr/bin/env python3
"""Where a GPU process's exit time goes — the tail of the odh-gpu-probe init container.

The kubelet sees an init container finish when its process is reaped, so a probe pays its
own exit: the kernel tearing down the process's GPU state (KFD queues and VM, the render
node's BOs) after ``_Exit``.  Each run spawns the program directly (no shell), stamps
``ODH_T0_NS``/``ODH_PROBE_T0_NS`` just before the spawn and times the reap; the program prints
its own CLOCK_REALTIME ``end_ns`` (``tools/research/native/hip_init_bench``) or its ``timings_ms``
(``odh-gpu-probe``), so exec, in-process work and exit are separated:

    exit_ms = reaped - end of the program's own work

Settings vary what the process holds when it leaves (no GPU, ROCr only, 16/256 MiB of VRAM,
buffers freed or not, runtime teardown or ``_Exit``) and run the probe itself at its
default and at a 16 MiB HBM sweep.

    python tools/hip_exit_ab.py [--repeats 5] > gpurun_out/<tag>/hip_exit_ab.jsonl
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BENCH = os.path.join(ROOT, "tools", "research", "native", "hip_init_bench")
PROBE = os.path.join(ROOT, "odh_kubeflow_amd", "ops", "_lib", "odh-gpu-probe")

SETTINGS = [
    ("no_gpu", BENCH, [], {"ODH_NO_GPU": "1"}),
    ("hsa_only", BENCH, [], {"ODH_HSA_ONLY": "1", "ODH_FAST_EXIT": "1"}),
    ("malloc256_free_return", BENCH, [], {}),
    ("malloc256_free_fastexit", BENCH, [], {"ODH_FAST_EXIT": "1"}),
    ("malloc256_keep_fastexit", BENCH, [], {"ODH_FAST_EXIT": "1", "ODH_NO_FREE": "1"}),
    ("malloc16_free_fastexit", BENCH, [], {"ODH_FAST_EXIT": "1", "ODH_MALLOC_MIB": "16"}),
    ("probe_default", PROBE, ["--json", "-"], {}),
    ("probe_hbm16", PROBE, ["--json", "-", "--hbm-mib", "16"], {}),
]


def run_once(exe, args, env_extra, timeout):
    env = dict(os.environ, **env_extra)
    t0 = time.time_ns()
    env["ODH_T0_NS"] = env["ODH_PROBE_T0_NS"] = str(t0)
    p = subprocess.Popen([exe, *args], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    out, err = p.communicate(timeout=timeout)
    reaped = time.time_ns()
    if p.returncode != 0:
        raise SystemExit(f"{exe} {args} rc={p.returncode}: {err.decode()[-400:]}")
    line = [ln for ln in out.decode().splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    wall = (reaped - t0) / 1e6
    if "end_ns" in r:
        work_end = r["end_ns"]
    else:  # the probe: exec + total (its own clock from main, release included)
        tm = r["timings_ms"]
        work_end = t0 + (tm["exec"] + tm["total"]) * 1e6
    return {"wall_ms": round(wall, 2), "exec_ms": r.get("exec_ms", r.get("timings_ms", {}).get("exec")),
            "exit_ms": round((reaped - work_end) / 1e6, 2), "r": r}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--timeout", type=float, default=60)
    ap.add_argument("--only", default="", help="comma-separated setting names")
    a = ap.parse_args(argv)
    only = set(filter(None, a.only.split(",")))
    summary = {}
    for name, exe, args, env in SETTINGS:
        if only and name not in only:
            continue
        if not os.access(exe, os.X_OK):
            raise SystemExit(f"build {exe} first")
        runs = []
        for i in range(a.repeats):
            r = run_once(exe, args, env, a.timeout)
            runs.append(r)
            print(json.dumps({"setting": name, "run": i, **r}), flush=True)
        summary[name] = {k: round(statistics.median(x[k] for x in runs), 2) for k in ("wall_ms", "exit_ms")}
    print(json.dumps({"summary_p50": summary}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
