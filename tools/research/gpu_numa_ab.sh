#!/bin/bash
# A/B of the bench's NUMA binding (parallel/bench_dist.py::numa_bind) on one MI355X box:
# interleaved runs with and without it at 1, 2 and 4 ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-numa_ab}
mkdir -p "$out"
run() {  # tag nproc bind
  if [ "$2" = 1 ]; then
    ODH_BENCH_NUMA_BIND=$3 timeout -k 10 170 python bench.py > "$out/$1.log" 2>&1 || return 1
  else
    ODH_BENCH_NUMA_BIND=$3 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$2" \
      --master-addr 127.0.0.1 --master-port 2995$2 bench.py --gpus "$2" --steps 150 --warmup 5 > "$out/$1.log" 2>&1 || return 1
  fi
  python - "$out/$1.log" "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d["n_gpus"], d["notebooks_ready_per_s"], d["p50_ready_ms"], d["p95_ready_ms"], d.get("cpu_binding"))
PY
}
for r in 1 2; do
  run n1_bind_$r 1 1 && run n1_free_$r 1 0 || exit 1
done
for n in 2 4; do
  run n${n}_bind $n 1 && run n${n}_free $n 0 || exit 1
done
echo "numa ab done"
