#!/bin/bash
# First GPU pass: env probe, build, gpu tests, smoke, bench, rocprof stats.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 120 bash tools/gpu_env_probe.sh > /dev/null 2>&1
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1 || { tail -40 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof -o bench -- python3 /root/repo/bench.py --steps 10 --warmup 2 > /root/repo/gpurun_out/prof.log 2>&1 || { tail -30 /root/repo/gpurun_out/prof.log; exit 1; }
find /root/repo/gpurun_out/prof -name "*stats*" | head
