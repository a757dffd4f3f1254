#!/bin/bash
# GPU pass 28: end-of-round refresh of the current tree — gpu tests, smoke, headline bench
# (n=1 twice, 2/4/8-rank rehearsal), BASELINE configs #4 (webhook path) and #5 (culling),
# rocprofv3 kernel stats of the default bench.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('gpu_probe', {}).get('gpu_ms_p50'), d.get('cpu_ms_per_step'), (d.get('inprocess_n1') or {}).get('value'))"; }
timeout -k 10 170 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu28.log 2>&1 || { tail -60 gpurun_out/pytest_gpu28.log; exit 1; }
tail -1 gpurun_out/pytest_gpu28.log
timeout -k 10 170 python __graft_entry__.py smoke > gpurun_out/smoke28.log 2>&1 || { tail -40 gpurun_out/smoke28.log; exit 1; }
tail -1 gpurun_out/smoke28.log
for r in 1 2; do
  timeout -k 10 170 python bench.py > gpurun_out/b28_n1_r$r.log 2>&1 || { tail -40 gpurun_out/b28_n1_r$r.log; exit 1; }
  show gpurun_out/b28_n1_r$r.log n1
done
for n in 2 4 8; do
  timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2983$n bench.py --gpus $n --steps 100 --warmup 5 > gpurun_out/b28_sh$n.log 2>&1 || { tail -40 gpurun_out/b28_sh$n.log; exit 1; }
  show gpurun_out/b28_sh$n.log sharded
done
timeout -k 10 170 python tools/bench_webhook.py --rounds 20 > gpurun_out/webhook28.log 2>&1 || { tail -30 gpurun_out/webhook28.log; exit 1; }
tail -1 gpurun_out/webhook28.log
timeout -k 10 120 python tools/bench_culling.py > gpurun_out/cull28.log 2>&1 || { tail -30 gpurun_out/cull28.log; exit 1; }
tail -1 gpurun_out/cull28.log
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d gpurun_out/prof28 -o run -- python3 bench.py --steps 40 --warmup 3 --no-inprocess-baseline > gpurun_out/b28_prof.log 2>&1 || { tail -40 gpurun_out/b28_prof.log; exit 1; }
echo done
