#!/bin/bash
# Interleaved A/B of apiserver builds / settings under the current tree at N ranks on one box:
#   cur       the in-tree odh-apiserver (glibc's default malloc arenas: 8 x cores)
#   cap8      the same with malloc arenas capped at 8 (MALLOC_ARENA_MAX=8; the build's default until r4_apiab)
#   a32       capped at 32
#   h512      the watch history bounded at 512 events per resource (ODH_APISERVER_HISTORY; the default since r4_hist)
#   h1024     bounded at 1024 (the default until r4_hist)
#   r3        round 3's odh-apiserver (testing/native/bin/odh-apiserver-r3, built from c6e2b35)
#   gpurun --timeout 900 -- bash tools/research/apiserver_ab.sh <tag> [ranks] [rounds] [variants]
set -e -o pipefail
tag=${1:?usage: apiserver_ab.sh <tag> [ranks] [rounds] [variants]}
n=${2:-4}
rounds=${3:-2}
variants=${4:-"cur cap8 r3"}
steps=${STEPS:-100}
out=gpurun_out/$tag
mkdir -p "$out"
bin=$PWD/odh_kubeflow_amd/testing/native/bin
for r in $(seq 1 "$rounds"); do
  for v in $variants; do
    case $v in
      cur) envs=() ;;
      cap8) envs=(MALLOC_ARENA_MAX=8) ;;
      a32) envs=(MALLOC_ARENA_MAX=32) ;;
      h512) envs=(ODH_APISERVER_HISTORY=512) ;;
      h1024) envs=(ODH_APISERVER_HISTORY=1024) ;;
      r3) envs=(ODH_APISERVER_BINARY=$bin/odh-apiserver-r3) ;;
      *) echo "unknown variant $v"; exit 2 ;;
    esac
    env "${envs[@]}" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port 2999$n bench.py --gpus "$n" --steps "$steps" --warmup 5 \
      --probe-sample 0 --burst 0 --no-configs > "$out/${v}_n${n}_$r.log" 2>&1
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['notebooks_ready_per_s'], d['p50_ready_ms'], d['cpu_ms_per_step'].get('apiserver'), (d.get('apiserver_profile_per_step') or {}).get('lock_wait_ms'), d['child_rss_mib'].get('apiserver'), 'gone/step', (d.get('apiserver_profile_per_step') or {}).get('watch_gone'), 'relists', sum((p.get('relists_in_window') or {}).get('total', 0) for p in (d.get('io_per_notebook') or {}).values()))" "$out/${v}_n${n}_$r.log"
  done
done
