#!/bin/bash
# GPU pass 4: gpu tests, in-process vs sharded bench at n=1, sharded rehearsal with 2/4 ranks sharing the box's GPU.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/bench_n1.log 2>&1 || { tail -40 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --arch sharded > gpurun_out/bench_sharded_n1.log 2>&1 || { tail -40 gpurun_out/bench_sharded_n1.log; exit 1; }
grep '^{' gpurun_out/bench_sharded_n1.log
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n bench.py --gpus $n --steps 30 --warmup 3 > gpurun_out/bench_sharded_n$n.log 2>&1 || { tail -40 gpurun_out/bench_sharded_n$n.log; exit 1; }
  grep '^{' gpurun_out/bench_sharded_n$n.log
done
