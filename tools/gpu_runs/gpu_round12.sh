#!/bin/bash
# GPU pass 12: new bench default (sharded at N=1 + in-process secondary), 2/4-rank rehearsal
# on the one GPU (ranks share the device), rocprofv3 kernel stats of the default bench.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('gpu_probe', {}).get('gpu_ms_p50'), d.get('inprocess_n1'))"; }
timeout -k 10 400 python bench.py > gpurun_out/b12_default.log 2>&1 || { tail -40 gpurun_out/b12_default.log; exit 1; }
show gpurun_out/b12_default.log default
timeout -k 10 400 python bench.py --steps 100 --warmup 5 > gpurun_out/b12_n1.log 2>&1 || { tail -40 gpurun_out/b12_n1.log; exit 1; }
show gpurun_out/b12_n1.log n1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2973$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b12_sh$n.log 2>&1 || { tail -40 gpurun_out/b12_sh$n.log; exit 1; }
  show gpurun_out/b12_sh$n.log sharded
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o run -- python3 bench.py --steps 40 --warmup 3 --no-inprocess-baseline > gpurun_out/b12_prof.log 2>&1 || { tail -40 gpurun_out/b12_prof.log; exit 1; }
echo done
