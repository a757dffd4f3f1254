#!/bin/bash
# GPU pass 5: gpu tests (new 256² LDS-DMA GEMM + fused verify), kernel A/B microbench, shard timeline, rocprof.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench.json 2> gpurun_out/microbench.err || { tail -30 gpurun_out/microbench.err; exit 1; }
cat gpurun_out/microbench.json
timeout -k 10 120 python tools/shard_timeline.py > gpurun_out/shard_timeline.txt 2>&1 || { tail -30 gpurun_out/shard_timeline.txt; exit 1; }
tail -75 gpurun_out/shard_timeline.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/bench_n1.log 2>&1 || { tail -40 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/prof5 -o bench -- python3 /root/repo/bench.py --steps 10 --warmup 2 > /root/repo/gpurun_out/prof5.log 2>&1 || { tail -30 /root/repo/gpurun_out/prof5.log; exit 1; }
find /root/repo/gpurun_out/prof5 -name "*kernel_stats*" | head -1 | xargs cat
