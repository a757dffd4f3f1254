#!/bin/bash
# Interleaved A/B of two trees at N ranks on one box (the 2/4-rank rows swing more than N=1
# from box to box, so only an interleaved pair on the same box tells a code change from the
# machine):
#   git archive <rev> | tar -x -C ab_old && (cd ab_old && python -m odh_kubeflow_amd.ops.build)
#   gpurun --timeout 900 -- bash tools/research/tree_ab_ranks.sh <tag> [ranks] [rounds] [old_dir]
set -e -o pipefail
tag=${1:?usage: tree_ab_ranks.sh <tag> [ranks] [rounds] [old_dir]}
n=${2:-4}
rounds=${3:-2}
old=${4:-ab_old}
out=gpurun_out/$tag
mkdir -p "$out"
run() {  # <dir> <log> [extra bench flags: the new tree's post-window blocks off]
  local dir=$1 log=$2
  shift 2
  (cd "$dir" && timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port 2998$n bench.py --gpus "$n" --steps 100 --warmup 5 \
    --probe-sample 0 "$@") > "$log" 2>&1
}
for r in $(seq 1 "$rounds"); do
  run "$old" "$PWD/$out/old_n${n}_$r.log"
  run . "$out/new_n${n}_$r.log" --burst 0 --no-configs
  for f in "$out/old_n${n}_$r.log" "$out/new_n${n}_$r.log"; do
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['notebooks_ready_per_s'], d['p50_ready_ms'], d['cpu_ms_per_step'].get('apiserver'), {k: v for k, v in d['cpu_ms_per_step'].items() if k.startswith('control_plane')})" "$f"
  done
done
