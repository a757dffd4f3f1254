#!/bin/bash
# GPU pass 6: HBM write-path variants.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench6.json 2> gpurun_out/microbench6.err || { tail -30 gpurun_out/microbench6.err; exit 1; }
cat gpurun_out/microbench6.json
