#!/bin/bash
# GPU pass 13: deep-pipelined 256² GEMM (BK=32, 4-buffer LDS ring, 3 stages in flight)
# numerics + A/B against the 2-buffer BK=64 kernel; full gpu test suite.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu14.log 2>&1 || { tail -60 gpurun_out/pytest_gpu14.log; exit 1; }
tail -2 gpurun_out/pytest_gpu14.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench14.json 2> gpurun_out/microbench14.err || { tail -30 gpurun_out/microbench14.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/microbench14.json"))
for k, v in d.items():
    if not k.startswith("hbm_write_v"):
        print(k, v)
PY
