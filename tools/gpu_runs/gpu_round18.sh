#!/bin/bash
# GPU pass 18: deep probe GEMM variants (cross-barrier prefetch x tile grouping GM 1/2/4/8),
# two passes each; kernel numerics tests.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu18.log 2>&1 || { tail -60 gpurun_out/pytest_gpu18.log; exit 1; }
tail -1 gpurun_out/pytest_gpu18.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench18.json 2> gpurun_out/microbench18.err || { tail -30 gpurun_out/microbench18.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/microbench18.json"))
for k, v in d.items():
    if k.startswith("probe") or k.startswith("gemm256") or k.startswith("torch_bf16"):
        print(k, v)
PY
