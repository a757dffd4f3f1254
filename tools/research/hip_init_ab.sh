#!/bin/bash
# A/B of a fresh process's HIP start-up (what the odh-gpu-probe init container pays per pod)
# under ROCm runtime settings.  One run per setting and repeat; each under its own timeout.
#   gpurun -- bash tools/hip_init_ab.sh <tag>
set -o pipefail
tag=${1:?tag}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/$tag
mkdir -p "$out"
bin=tools/research/native/hip_init_bench
[ -x "$bin" ] || { echo "build $bin first"; exit 2; }
run() {  # label env...
  label=$1; shift
  for r in 1 2 3; do
    s0=$(date +%s%N)
    line=$(env "$@" ODH_T0_NS=$s0 timeout -k 5 60 "$bin") || { echo "$label failed"; exit 1; }
    echo "{\"setting\":\"$label\",\"run\":$r,\"wall_ms\":$(( ($(date +%s%N) - s0) / 1000000 )),\"r\":$line}" >> "$out/hip_init_ab.jsonl"
  done
}
run default X=1
run hsa_first ODH_HSA_FIRST=1
run fast_exit ODH_FAST_EXIT=1
run rocr_visible ROCR_VISIBLE_DEVICES=0
run no_sdma HSA_ENABLE_SDMA=0
cat "$out/hip_init_ab.jsonl"
