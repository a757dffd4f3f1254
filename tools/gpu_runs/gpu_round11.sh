#!/bin/bash
# GPU pass 11: re-validate the restored tree (prebuilt .so from the CPU container):
# gpu tests, smoke, default n=1 bench (in-process + sharded base point), rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 100 --warmup 5 > gpurun_out/b11_n1.log 2>&1 || { tail -40 gpurun_out/b11_n1.log; exit 1; }
grep '^{' gpurun_out/b11_n1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o run -- python3 bench.py --steps 40 --warmup 3 --no-inprocess-baseline > gpurun_out/b11_prof.log 2>&1 || { tail -40 gpurun_out/b11_prof.log; exit 1; }
find gpurun_out/prof11 -name '*stats*' | head
