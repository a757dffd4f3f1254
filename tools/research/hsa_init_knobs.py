#!/usr/bin/env python3
"""Does any ROCr runtime setting shorten ``hsa_init`` — the ~180 ms floor of the
odh-gpu-probe init container (pass r3_p8)?

Runs ``tools/research/native/hip_init_bench`` in its ``ODH_HSA_ONLY`` mode (hsa_init, then exit)
under each setting, interleaved round by round so box drift hits every setting alike, and
prints per-setting medians of hsa_init and of the whole process (spawn → reaped).

    python tools/hsa_init_knobs.py [--rounds 5] > gpurun_out/<tag>/hsa_init_knobs.jsonl
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

SETTINGS = {
    "default": {},
    "no_interrupt": {"HSA_ENABLE_INTERRUPT": "0"},
    "no_sdma": {"HSA_ENABLE_SDMA": "0"},
    "no_fragment_alloc": {"HSA_DISABLE_FRAGMENT_ALLOCATOR": "1"},
    "no_scratch_reclaim": {"HSA_NO_SCRATCH_RECLAIM": "1"},
    "rocr_visible_0": {"ROCR_VISIBLE_DEVICES": "0"},
    "no_peer_sdma": {"HSA_ENABLE_PEER_SDMA": "0"},
    "no_image_support": {"HSA_IMAGE_SUPPORT": "0"},
    "rocr_visible_0+no_scratch_reclaim": {"ROCR_VISIBLE_DEVICES": "0", "HSA_NO_SCRATCH_RECLAIM": "1"},
}


def once(env_extra):
    env = dict(os.environ, ODH_HSA_ONLY="1", ODH_FAST_EXIT="1", **env_extra)
    t0 = time.time_ns()
    env["ODH_T0_NS"] = str(t0)
    p = subprocess.run([BENCH], env=env, capture_output=True, text=True, timeout=60)
    wall = (time.time_ns() - t0) / 1e6
    if p.returncode != 0:
        return {"error": p.stdout[-300:] + p.stderr[-300:]}
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    return {"hsa_init_ms": r.get("hsa_init_ms"), "wall_ms": round(wall, 1)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="", help="comma list of settings")
    a = ap.parse_args(argv)
    settings = {k: v for k, v in SETTINGS.items() if not a.only or k in a.only.split(",")}
    if not os.access(BENCH, os.X_OK):
        raise SystemExit(f"build {BENCH} first")
    res = {k: [] for k in settings}
    for rnd in range(a.rounds):
        for name, env in settings.items():
            r = once(env)
            res[name].append(r)
            print(json.dumps({"round": rnd, "setting": name, **r}), flush=True)
    summary = {}
    for name, rs in res.items():
        ok = [r for r in rs if "error" not in r]
        if ok:
            summary[name] = {"hsa_init_ms_p50": round(statistics.median(r["hsa_init_ms"] for r in ok), 1),
                             "wall_ms_p50": round(statistics.median(r["wall_ms"] for r in ok), 1), "runs": len(ok)}
        else:
            summary[name] = {"error": rs[0]["error"] if rs else "no runs"}
    print(json.dumps({"summary": summary}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
