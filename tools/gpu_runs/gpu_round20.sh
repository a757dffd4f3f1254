#!/bin/bash
# GPU pass 20: scheduler as its own process (rank 0 child) — n=1 x3, 2/4/8-rank rehearsal:
# gpu tests, smoke, default bench (n=1 sharded + in-process secondary), 2/4/8-rank rehearsal
# on the one GPU (ranks share the device; the 8-GPU node run is the driver's), rocprof stats.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('gpu_probe', {}).get('gpu_ms_p50'), d.get('rank_ms_per_step'), (d.get('inprocess_n1') or {}).get('value'))"; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu20.log 2>&1 || { tail -60 gpurun_out/pytest_gpu20.log; exit 1; }
tail -1 gpurun_out/pytest_gpu20.log
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke20.log 2>&1 || { tail -40 gpurun_out/smoke20.log; exit 1; }
tail -1 gpurun_out/smoke20.log
timeout -k 10 400 python bench.py > gpurun_out/b20_n1.log 2>&1 || { tail -40 gpurun_out/b20_n1.log; exit 1; }
show gpurun_out/b20_n1.log n1
for n in 2 4 8; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2976$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b20_sh$n.log 2>&1 || { tail -40 gpurun_out/b20_sh$n.log; exit 1; }
  show gpurun_out/b20_sh$n.log sharded
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20 -o run -- python3 bench.py --steps 40 --warmup 3 --no-inprocess-baseline > gpurun_out/b20_prof.log 2>&1 || { tail -40 gpurun_out/b20_prof.log; exit 1; }
echo done
