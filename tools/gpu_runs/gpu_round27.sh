#!/bin/bash
# GPU pass 27: per-resource watch history lock in the native apiserver (watch threads off the store lock),
# same steps as pass 26: gpu tests, default bench (n=1 + in-process), sharded 2/4/8 with the apiserver profile.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('reconciles_per_notebook'), d.get('cpu_ms_per_step'), (d.get('inprocess_n1') or {}).get('value')); p=d.get('apiserver_profile_per_step') or {}; print('   apiserver', {k: v for k, v in p.items() if v})"; }
timeout -k 10 170 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu27.log 2>&1 || { tail -60 gpurun_out/pytest_gpu27.log; exit 1; }
tail -1 gpurun_out/pytest_gpu27.log
timeout -k 10 170 python bench.py > gpurun_out/b27_n1.log 2>&1 || { tail -40 gpurun_out/b27_n1.log; exit 1; }
show gpurun_out/b27_n1.log n1
for n in 2 4 8; do
  timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2982$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b27_sh$n.log 2>&1 || { tail -40 gpurun_out/b27_sh$n.log; exit 1; }
  show gpurun_out/b27_sh$n.log sharded
done
echo done
