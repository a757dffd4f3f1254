#!/bin/bash
# Interleaved A/B of two trees at N=1 on one box (box-to-box variance is ~10 %, so only an
# interleaved pair on the same box tells a code change from the machine):
#   git archive <rev> | tar -x -C ab_old && copy the built .so / binaries into ab_old
#   gpurun --timeout 900 -- bash tools/research/tree_ab.sh <tag> [ab_old] [rounds]
set -e
tag=${1:?usage: tree_ab.sh <tag> [old_dir] [rounds]}
old=${2:-ab_old}
rounds=${3:-3}
out=gpurun_out/$tag
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  (cd "$old" && timeout -k 10 150 python bench.py --steps 300 --warmup 10 > "$OLDPWD/$out/old_$r.log" 2>&1)
  timeout -k 10 150 python bench.py --steps 300 --warmup 10 > "$out/new_$r.log" 2>&1
  echo "round $r done"
done
