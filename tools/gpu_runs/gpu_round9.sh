#!/bin/bash
# GPU pass 9: after GC tuning + concurrent odh fan-out + overlapped probe.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d['max_ready_ms'], d.get('p50_teardown_ms'), d.get('gpu_probe', {}).get('gpu_ms_p50'))"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/b9_inproc_r$r.log 2>&1 || { tail -40 gpurun_out/b9_inproc_r$r.log; exit 1; }
  show gpurun_out/b9_inproc_r$r.log inproc
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --arch sharded > gpurun_out/b9_sh1.log 2>&1 || { tail -40 gpurun_out/b9_sh1.log; exit 1; }
show gpurun_out/b9_sh1.log sharded
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2963$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b9_sh$n.log 2>&1 || { tail -40 gpurun_out/b9_sh$n.log; exit 1; }
  show gpurun_out/b9_sh$n.log sharded
done
