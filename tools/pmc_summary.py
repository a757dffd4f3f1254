"""Per-kernel summary of ``rocprofv3 --pmc`` passes (``tools/gpu_pass.sh <tag> pmc``).

    python tools/pmc_summary.py gpurun_out/r5_f1 > profiles/r5_f1/pmc_summary.json

Each pass directory holds ``run_counter_collection.csv`` (one row per dispatch and
counter).  Counters are averaged per kernel over its dispatches and joined across passes,
then turned into the quantities the probe kernels are judged by:

* ``mfma_busy_pct`` = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES × 256 CUs ÷ 8 SEs …)
  is not well defined across SQ aggregation, so the raw ratio
  ``SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES`` is reported next to the kernel's measured
  duration and its MFMA-implied rate: for 32×32×16 bf16 MFMA each instruction keeps a
  SIMD busy 32 cycles (MI355X_MICROARCH.md), so MFMA busy cycles ÷ 32 × 32768 FLOP
  gives the executed FLOP — compared with the GEMM's 2·M·N·K it checks that all the
  math ran on the matrix cores;
* ``lds_bank_conflict_pct`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``hbm_read_bytes`` = 2 × FETCH_SIZE × 1024 (gfx950 tallies a wide coalesced read at
  half its bytes, MI355X_MICROARCH.md) and ``hbm_write_bytes`` = WRITE_SIZE × 1024,
  with the achieved GB/s over the kernel's duration;
* ``l2_hit_pct`` = TCC_HIT / (TCC_HIT + TCC_MISS).
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


def load(root: str):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values
    dur = defaultdict(list)
    for path in sorted(glob.glob(os.path.join(root, "pmc*", "*counter_collection.csv"))):
        seen = set()
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                key = (path, row["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)  # us
    return per, dur


def summarize(root: str) -> dict:
    per, dur = load(root)
    out = {}
    for k, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        us = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else None
        s = {"dispatches_per_pass": max(len(v) for v in cs.values()), "median_us": round(us, 1) if us else None,
             "counters": {c: round(v, 1) for c, v in sorted(avg.items())}}
        if avg.get("SQ_BUSY_CYCLES"):
            s["mfma_busy_over_sq_busy"] = round(avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / avg["SQ_BUSY_CYCLES"], 3)
        if avg.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            s["mfma_flop_executed"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / 32 * 32768
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            s["lds_bank_conflict_pct"] = round(100 * avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"], 2)
        if "FETCH_SIZE" in avg:
            s["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in avg:
            s["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if us and ("hbm_read_bytes" in s or "hbm_write_bytes" in s):
            s["hbm_gbps"] = round((s.get("hbm_read_bytes", 0) + s.get("hbm_write_bytes", 0)) / (us * 1e3), 1)
        if avg.get("TCC_HIT_sum") is not None and avg.get("TCC_MISS_sum") is not None:
            tot = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
            s["l2_hit_pct"] = round(100 * avg["TCC_HIT_sum"] / tot, 1) if tot else None
        out[k] = s
    return out


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1]), indent=1))
