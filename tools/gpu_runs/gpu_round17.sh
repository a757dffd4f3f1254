#!/bin/bash
# GPU pass 17: HBM check (read path) variants: nontemporal vs plain loads, 4 vs 8 loads
# in flight per lane, 1k-8k slab blocks; torch read reference.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench17.json 2> gpurun_out/microbench17.err || { tail -30 gpurun_out/microbench17.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/microbench17.json"))
for k, v in d.items():
    if k.startswith("hbm_check") or k.startswith("torch_sum") or k.startswith("probe"):
        print(k, v)
PY
