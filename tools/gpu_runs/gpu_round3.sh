#!/bin/bash
# GPU pass 3: all gpu tests, smoke, bench (full odh path), torchrun nproc=1, rocprof kernel stats (csv).
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/bench_n1.log 2>&1 || { tail -40 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 > gpurun_out/bench_torchrun1.log 2>&1 || { tail -40 gpurun_out/bench_torchrun1.log; exit 1; }
grep '^{' gpurun_out/bench_torchrun1.log | tail -1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/prof3 -o bench -- python3 /root/repo/bench.py --steps 10 --warmup 2 > /root/repo/gpurun_out/prof3.log 2>&1 || { tail -30 /root/repo/gpurun_out/prof3.log; exit 1; }
find /root/repo/gpurun_out/prof3 -name "*stats*"
cd "${GRAFT_REPO_ROOT:-/root/repo}" && timeout -k 10 300 python bench.py --steps 20 --warmup 2 --transport native > gpurun_out/bench_native_n1.log 2>&1 || { tail -40 gpurun_out/bench_native_n1.log; exit 1; }
tail -1 gpurun_out/bench_native_n1.log
