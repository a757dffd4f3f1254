#!/bin/bash
# GPU pass 23: same-harness comparison against the reference's behaviour on MI355X —
# bench.py --reference-emulation (1 odh worker, blocking ≈6 s lock removal)
# vs the default path, 1 and 8 notebooks in one process; plus gpu tests, smoke, headline n=1.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['n_gpus'], d['value'], d['ms_per_step'], d['p50_ready_ms'], d['p95_ready_ms'], d.get('p50_teardown_ms'), d.get('gpu_probe', {}).get('gpu_ms_p50'), (d.get('inprocess_n1') or {}).get('value'))"; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu23.log 2>&1 || { tail -60 gpurun_out/pytest_gpu23.log; exit 1; }
tail -1 gpurun_out/pytest_gpu23.log
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke23.log 2>&1 || { tail -40 gpurun_out/smoke23.log; exit 1; }
tail -1 gpurun_out/smoke23.log
timeout -k 10 400 python bench.py > gpurun_out/b23_n1.log 2>&1 || { tail -40 gpurun_out/b23_n1.log; exit 1; }
show gpurun_out/b23_n1.log n1
timeout -k 10 200 python bench.py --arch inprocess --reference-emulation --steps 3 --warmup 1 > gpurun_out/b23_ref_n1.log 2>&1 || { tail -40 gpurun_out/b23_ref_n1.log; exit 1; }
show gpurun_out/b23_ref_n1.log ref_emulation
timeout -k 10 200 python bench.py --arch inprocess --reference-emulation --gpus 8 --steps 1 --warmup 0 > gpurun_out/b23_ref_n8.log 2>&1 || { tail -40 gpurun_out/b23_ref_n8.log; exit 1; }
show gpurun_out/b23_ref_n8.log ref_emulation
timeout -k 10 300 python bench.py --arch inprocess --gpus 8 --steps 40 --warmup 3 > gpurun_out/b23_inproc_n8.log 2>&1 || { tail -40 gpurun_out/b23_inproc_n8.log; exit 1; }
show gpurun_out/b23_inproc_n8.log inprocess
echo done
