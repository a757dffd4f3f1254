#!/bin/bash
# GPU pass 25: watcher wake-ups filtered by selector in the native apiserver, xGMI link probe (1-GPU: no links),
# gpu tests, in-process 8-notebook run, sharded 1/2/4/8 with per-process CPU.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('reconciles_per_notebook'), d.get('cpu_ms_per_step'))"; }
timeout -k 10 170 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu25.log 2>&1 || { tail -60 gpurun_out/pytest_gpu25.log; exit 1; }
tail -1 gpurun_out/pytest_gpu25.log
timeout -k 10 170 python bench.py --arch inprocess --gpus 8 --steps 40 --warmup 3 > gpurun_out/b25_inproc_n8.log 2>&1 || { tail -40 gpurun_out/b25_inproc_n8.log; exit 1; }
show gpurun_out/b25_inproc_n8.log inprocess
timeout -k 10 170 python bench.py --no-inprocess-baseline > gpurun_out/b25_n1.log 2>&1 || { tail -40 gpurun_out/b25_n1.log; exit 1; }
show gpurun_out/b25_n1.log sharded
for n in 2 4 8; do
  timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2980$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b25_sh$n.log 2>&1 || { tail -40 gpurun_out/b25_sh$n.log; exit 1; }
  show gpurun_out/b25_sh$n.log sharded
done
echo done
