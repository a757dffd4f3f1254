#!/bin/bash
# GPU pass 24: probe lock (concurrent probes of one GPU), per-process CPU ms/step of the
# sharded bench at 1/2/4/8 ranks, in-process 8-notebook run for the same-harness comparison.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('reconciles_per_notebook'), d.get('cpu_ms_per_step'))"; }
timeout -k 10 170 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu24.log 2>&1 || { tail -60 gpurun_out/pytest_gpu24.log; exit 1; }
tail -1 gpurun_out/pytest_gpu24.log
timeout -k 10 170 python bench.py --arch inprocess --gpus 8 --steps 40 --warmup 3 > gpurun_out/b24_inproc_n8.log 2>&1 || { tail -40 gpurun_out/b24_inproc_n8.log; exit 1; }
show gpurun_out/b24_inproc_n8.log inprocess
timeout -k 10 170 python bench.py --no-inprocess-baseline > gpurun_out/b24_n1.log 2>&1 || { tail -40 gpurun_out/b24_n1.log; exit 1; }
show gpurun_out/b24_n1.log sharded
for n in 2 4 8; do
  timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2979$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b24_sh$n.log 2>&1 || { tail -40 gpurun_out/b24_sh$n.log; exit 1; }
  show gpurun_out/b24_sh$n.log sharded
done
echo done
