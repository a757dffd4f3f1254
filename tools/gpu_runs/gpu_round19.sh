#!/bin/bash
# GPU pass 19: clock-warmed (0.25 s) microbenchmarks of every kernel variant;
# kernel numerics tests.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu19.log 2>&1 || { tail -60 gpurun_out/pytest_gpu19.log; exit 1; }
tail -1 gpurun_out/pytest_gpu19.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench19.json 2> gpurun_out/microbench19.err || { tail -30 gpurun_out/microbench19.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/microbench19.json"))
for k, v in d.items():
    if not k.startswith("hbm_write_v") and not k.startswith("hbm_check_v"):
        print(k, v)
PY
