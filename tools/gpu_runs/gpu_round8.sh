#!/bin/bash
# GPU pass 8: run-to-run variance of the in-process and sharded benches on one box.
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python -m odh_kubeflow_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/probe_microbench.py > gpurun_out/microbench8.json 2> gpurun_out/microbench8.err || { tail -30 gpurun_out/microbench8.err; exit 1; }
grep -A12 probe_run gpurun_out/microbench8.json
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 > gpurun_out/bench_n1_r$r.log 2>&1 || { tail -40 gpurun_out/bench_n1_r$r.log; exit 1; }
  tail -1 gpurun_out/bench_n1_r$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inproc', d['ms_per_step'], d['p50_ready_ms'], d.get('p50_teardown_ms'), d['gpu_probe']['probe_wall_ms_p50'])"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 --arch sharded > gpurun_out/bench_sh1_r$r.log 2>&1 || { tail -40 gpurun_out/bench_sh1_r$r.log; exit 1; }
  grep '^{' gpurun_out/bench_sh1_r$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded', d['ms_per_step'], d['p50_ready_ms'], d.get('p50_teardown_ms'), d['gpu_probe']['probe_wall_ms_p50'])"
done
timeout -k 10 300 python -m cProfile -o gpurun_out/inproc.prof bench.py --steps 60 --warmup 5 > gpurun_out/bench_prof.log 2>&1 || exit 1
python -c "
import pstats; p = pstats.Stats('gpurun_out/inproc.prof'); p.sort_stats('tottime').print_stats(25)" > gpurun_out/inproc_prof.txt
head -60 gpurun_out/inproc_prof.txt
