#!/bin/bash
# GPU pass 10: GEMM fragment-pipelining A/B + gpu tests.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench10.json 2> gpurun_out/microbench10.err || { tail -30 gpurun_out/microbench10.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/microbench10.json"))
for k, v in d.items():
    if not k.startswith("hbm_write_v"):
        print(k, v)
PY
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
