#!/bin/bash
# GPU pass 7: gpu tests, kernel microbench (slab HBM sweeps), in-process + sharded benches.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench7.json 2> gpurun_out/microbench7.err || { tail -30 gpurun_out/microbench7.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/microbench7.json"))
for k, v in d.items():
    if not k.startswith("hbm_write_v"):
        print(k, v)
PY
timeout -k 10 300 python bench.py --steps 40 --warmup 4 > gpurun_out/bench_n1.log 2>&1 || { tail -40 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log
timeout -k 10 300 python bench.py --steps 40 --warmup 4 --arch sharded > gpurun_out/bench_sharded_n1.log 2>&1 || { tail -40 gpurun_out/bench_sharded_n1.log; exit 1; }
grep '^{' gpurun_out/bench_sharded_n1.log
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2962$n bench.py --gpus $n --steps 40 --warmup 4 > gpurun_out/bench_sharded_n$n.log 2>&1 || { tail -40 gpurun_out/bench_sharded_n$n.log; exit 1; }
  grep '^{' gpurun_out/bench_sharded_n$n.log
done
