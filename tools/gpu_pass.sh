#!/bin/bash
# One parametrized MI355X pass (replaces the per-call scripts of round 1).
#
#   gpurun --timeout 900 -- bash tools/gpu_pass.sh <tag> [step ...]
#
# Steps (default: tests smoke bench probeexe prof):
#   tests    pytest -m gpu (one process, per-test timeout)
#   smoke    __graft_entry__.smoke()
#   bench    bench.py at N=1: the driver's invocation (--steps 20 --warmup 5) twice, then 300 steps
#   ranks    2/4-rank rehearsal of the N>1 launch on the one GPU (never 8: the driver owns N=8)
#   b20x4    the driver's invocation four times in a row (first-run effects on a fresh box)
#   s20v300  interleaved A/B on one box: the driver's 20-step invocation vs the 300-step run, 3 rounds
#   pyc      precompile the package's bytecode (compileall) before the steps that follow
#   unsharded  the default topology (one kf + one odh manager process) at 1, 2 and 4 ranks
#   workers  the same topology with --workers 4: 1, 2 and 4 ranks
#   wr2      --workers 4 --webhook-replicas 2: 1, 2 and 4 ranks
#   wcm      --workers 4 with the odh manager caching ConfigMap/Secret data, interleaved with without: 1 and 4 ranks
#   wpab     sharded: the webhook in the odh process vs a process of its own (deployed), interleaved, 1 and 4 ranks
#   burst64  64 notebooks at once into one unsharded control plane (--workers 1 and 4) and the sharded one
#   fair     ours vs --reference-emulation: vanilla / OpenShift-like (pull secret after 200 ms), 0 / 2 ms writes
#   pw4      4 ranks, --workers 4, one platform worker process per rank
#   nsr      --namespaces-per-rank 16: sharded at 2 and 4 ranks (NamespaceShardAssigner hash / balanced), unsharded
#            --workers 4 at 4 ranks (supervisor assignment) — per-shard notebooks, notebooks/s, CPU
#   rss300   4 ranks x 300 steps (sharded): the apiserver's resident set after a long window
#   archab   interleaved A/B at N=1: shard as kf/odh process pair vs one process vs unsharded
#   probeexe the odh-gpu-probe init-container program: 10 process runs (wall time, verdict)
#   hipinit  where a fresh process's HIP start-up goes, under ROCm runtime settings (tools/research/hip_init_ab.sh)
#   hsaknobs hsa_init under ROCr runtime settings, interleaved (tools/research/hsa_init_knobs.py)
#   hipexit  where a GPU process's exit goes: what it holds when it leaves (tools/research/hip_exit_ab.py)
#   webhook  BASELINE config #4 (tools/bench_webhook.py)
#   culling  BASELINE config #5 (tools/bench_culling.py)
#   realpods BASELINE configs #2/#3: 1 and 8 notebooks whose container is a real PyTorch-ROCm process
#   realbr   configs #2/#3 with the workbench's first GPU cell before Ready (--gpu-init before-ready)
#   realref  the same with the reference's serialising odh path (--reference-emulation)
#   refemu   bench.py --reference-emulation (control-plane lifecycle, reference behaviour)
#   cpprof   cProfile of the control-plane and node-platform processes over a 300-step bench (pstats top 40)
#   critpath hop-by-hop create→Ready from the apiserver audit log at 1 and 4 ranks (tools/gpu_critical_path.sh)
#   prof     rocprofv3 --kernel-trace --stats of the odh-gpu-probe program
#   pmc      rocprofv3 --pmc passes (MFMA busy, LDS bank conflicts, HBM bytes) of the probe kernels
#   probe    start-up probe: eager launches vs hipGraph replay (tools/probe_microbench.py --startup)
#   env      tools/gpu_env_probe.sh inventory
#
# Every GPU step runs under its own `timeout -k`; the first failure ends the pass (no retries).
set -o pipefail
tag=${1:?usage: gpu_pass.sh <tag> [step ...]}
shift
steps=${*:-tests smoke bench probeexe prof}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p "$out"

show() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
keys = ("n_gpus", "value", "ms_per_step", "rank_ms_per_step", "notebooks_ready_per_s", "p50_ready_ms",
        "p95_ready_ms", "reconciles_per_notebook", "writes_per_notebook", "cpu_ms_per_step", "gpu_probe_init_container")
print(sys.argv[2], {k: d.get(k) for k in keys})
b = d.get("burst")
if b:
    print(sys.argv[2], "burst", {k: b.get(k) for k in ("notebooks", "all_ready_s", "notebooks_per_s", "ready_ms",
                                                      "admission_ms", "webhook_handle_ms", "webhook_get_ms",
                                                      "cpu_ms_per_notebook", "rounds")})
rs = d.get("resident")
if rs:
    print(sys.argv[2], "resident", json.dumps({k: rs.get(k) for k in ("notebooks", "all_ok", "fill_s",
                                                                      "new_notebooks_on_top", "teardown_s", "errors")}))
    print(sys.argv[2], "resident at_rest", json.dumps(rs.get("at_rest"))[:2500])
sl = d.get("shard_load")
if sl:
    print(sys.argv[2], "shard_load", json.dumps(sl))
print(sys.argv[2], "child_rss_mib", d.get("child_rss_mib"))
c = d.get("configs")
if c:
    print(sys.argv[2], "configs", json.dumps(c)[:3000])
PY
}
fail() { echo "step $1 failed (rc=$2)"; tail -40 "$3"; exit 1; }

for s in $steps; do
  case $s in
    tests)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$out/pytest_gpu.log" 2>&1 || fail tests $? "$out/pytest_gpu.log"
      tail -1 "$out/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 170 python __graft_entry__.py smoke > "$out/smoke.log" 2>&1 || fail smoke $? "$out/smoke.log"
      tail -1 "$out/smoke.log" ;;
    bench)
      for r in 1 2; do
        timeout -k 10 170 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_n1_s20_r$r.log" 2>&1 \
          || fail bench $? "$out/bench_n1_s20_r$r.log"
        show "$out/bench_n1_s20_r$r.log" "n1 steps20 r$r"
      done
      timeout -k 10 200 python bench.py --gpus 1 --no-inprocess-baseline > "$out/bench_n1_s300.log" 2>&1 \
        || fail bench $? "$out/bench_n1_s300.log"
      show "$out/bench_n1_s300.log" "n1 steps300" ;;
    resident)  # R resident notebooks with the culler on: at rest, and new notebooks on top; heartbeat filter A/B
      # variants: split (culler in its own process, the default), inkf (culler in the kf process),
      # nofilter (ODH_HEARTBEAT_FILTER=false: every heartbeat reconciles kf + odh and runs the pipeline)
      for r in $(seq 1 "${ROUNDS:-1}"); do
        for v in ${VARIANTS:-split inkf nofilter}; do
          case $v in inkf) f="--culler-in-kf"; hb=true ;; nofilter) f=""; hb=false ;; *) f=""; hb=true ;; esac
          ODH_HEARTBEAT_FILTER=$hb timeout -k 10 400 python bench.py --gpus 1 --steps 100 --warmup 10 --no-configs \
            --no-inprocess-baseline --burst 0 --probe-sample 0 --resident "${RESIDENT:-1000}" --resident-window 5 $f \
            > "$out/bench_resident_${v}_r$r.log" 2>&1 || fail resident $? "$out/bench_resident_${v}_r$r.log"
          show "$out/bench_resident_${v}_r$r.log" "resident $v r$r"
        done
      done ;;
    nsscale)  # 4 ranks x M namespaces per rank (sharded, balanced): per-namespace watches vs one cluster-wide
      # watch per kind, interleaved; M=1 is the reference point for the apiserver's CPU per write
      for r in $(seq 1 "${ROUNDS:-1}"); do
        for v in ${NSVARIANTS:-m1 m64 m64cw}; do
          case $v in m1) f="" ;; m64) f="--namespaces-per-rank 64 --assign-policy balanced" ;;
                     m64cw) f="--namespaces-per-rank 64 --assign-policy balanced --cluster-wide-watches" ;;
                     m16) f="--namespaces-per-rank 16 --assign-policy balanced" ;;
                     m16cw) f="--namespaces-per-rank 16 --assign-policy balanced --cluster-wide-watches" ;; esac
          timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
            --master-port 29971 bench.py --gpus 4 --steps 100 --warmup 5 --no-configs --probe-sample 0 --burst 0 \
            --resident 0 $f > "$out/bench_ns_${v}_r$r.log" 2>&1 || fail nsscale $? "$out/bench_ns_${v}_r$r.log"
          python tools/summarize_bench.py "$out/bench_ns_${v}_r$r.log"
        done
      done ;;
    failover)  # takeover (SIGKILL, standby with warm caches) and graceful cold start with R resident notebooks
      timeout -k 10 600 python tools/bench_failover.py --resident "${RESIDENT:-1000}" > "$out/failover.log" 2>&1 \
        || fail failover $? "$out/failover.log"
      tail -1 "$out/failover.log" | cut -c1-3000 ;;
    rescp)  # hop by hop: the timed window's notebooks (empty cluster) vs those created on top of R resident
      DEBUG_WRITE_AUDITLOG=$PWD/$out/ares.jsonl timeout -k 10 400 python bench.py --gpus 1 --steps 100 --warmup 10 \
        --no-configs --no-inprocess-baseline --burst 0 --probe-sample 0 --resident "${RESIDENT:-1000}" \
        --resident-window 3 --resident-steps 50 > "$out/bench_rescp.log" 2>&1 || fail rescp $? "$out/bench_rescp.log"
      show "$out/bench_rescp.log" "rescp"
      python tools/critical_path.py $out/ares.jsonl --name-prefix nb-s > $out/critical_path_timed.json || exit 1
      python tools/critical_path.py $out/ares.jsonl --name-prefix nb-res- > $out/critical_path_on_top.json || exit 1
      rm -f $out/ares.jsonl
      echo "critical paths written" ;;
    b20x4)
      for r in 1 2 3 4; do
        echo "run $r start $(date +%s.%N)"
        timeout -k 10 170 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_x4_r$r.log" 2>&1 \
          || fail b20x4 $? "$out/bench_x4_r$r.log"
        show "$out/bench_x4_r$r.log" "x4 r$r"
      done ;;
    s20v300)
      for r in 1 2 3; do
        timeout -k 10 170 python bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_ab_s20_r$r.log" 2>&1 \
          || fail s20v300 $? "$out/bench_ab_s20_r$r.log"
        show "$out/bench_ab_s20_r$r.log" "s20 r$r"
        timeout -k 10 200 python bench.py --gpus 1 --steps 300 --warmup 5 --no-inprocess-baseline \
          > "$out/bench_ab_s300_r$r.log" 2>&1 || fail s20v300 $? "$out/bench_ab_s300_r$r.log"
        show "$out/bench_ab_s300_r$r.log" "s300 r$r"
      done ;;
    pyc)
      timeout -k 10 120 python -m compileall -q odh_kubeflow_amd bench.py __graft_entry__.py > "$out/pyc.log" 2>&1 \
        || fail pyc $? "$out/pyc.log"
      echo "bytecode compiled" ;;
    unsharded)
      timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --steps 100 --warmup 5 --probe-sample 0 \
        > "$out/bench_unsharded_n1.log" 2>&1 || fail unsharded $? "$out/bench_unsharded_n1.log"
      show "$out/bench_unsharded_n1.log" "unsharded n1"
      for n in 2 4; do
        timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port 2994$n bench.py --gpus $n --arch unsharded --steps 100 --warmup 5 \
          --probe-sample 0 > "$out/bench_unsharded_n$n.log" 2>&1 || fail unsharded $? "$out/bench_unsharded_n$n.log"
        show "$out/bench_unsharded_n$n.log" "unsharded n$n"
      done ;;
    workers)  # overlay mi355x: --workers 4 (kf split), 3 webhook processes, the odh manager's cached ConfigMaps/Secrets
      timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --cache-configmaps --kf-split-workers \
        --webhook-replicas 3 --steps 100 --warmup 5 --probe-sample 0 \
        --resident 0 --no-configs > "$out/bench_workers_n1.log" 2>&1 || fail workers $? "$out/bench_workers_n1.log"
      show "$out/bench_workers_n1.log" "workers4 n1"
      for n in 2 4; do
        timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port 2995$n bench.py --gpus $n --arch unsharded --workers 4 --cache-configmaps \
          --kf-split-workers --webhook-replicas 3 --steps 100 \
          --warmup 5 --probe-sample 0 --resident 0 > "$out/bench_workers_n$n.log" 2>&1 || fail workers $? "$out/bench_workers_n$n.log"
        show "$out/bench_workers_n$n.log" "workers4 n$n"
      done ;;
    wrab)  # overlay mi355x (split kf workers) at 4 streams: 2 / 3 / 4 odh webhook processes, interleaved x2, plus N=1
      timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --kf-split-workers --cache-configmaps \
        --webhook-replicas 2 --steps 100 --warmup 5 --probe-sample 0 --resident 0 --no-configs --burst 0 \
        > "$out/bench_wrab_n1.log" 2>&1 || fail wrab $? "$out/bench_wrab_n1.log"
      show "$out/bench_wrab_n1.log" "wrab n1"
      for r in 1 2; do
        for w in ${WRAB:-2 3 4}; do
          timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 2996$w bench.py --gpus 4 --arch unsharded --workers 4 \
            --kf-split-workers --cache-configmaps --webhook-replicas $w --steps 100 --warmup 5 --probe-sample 0 \
            --resident 0 --burst 0 > "$out/bench_wrab_wr${w}_r$r.log" 2>&1 || fail wrab $? "$out/bench_wrab_wr${w}_r$r.log"
          show "$out/bench_wrab_wr${w}_r$r.log" "wrab wr$w r$r"
        done
      done ;;
    splitab)  # overlay mi355x: the kf manager's workers whole vs split (notebook | culler,events), interleaved x2
      for r in 1 2; do
        for v in "base" "split --kf-split-workers"; do
          set -- $v
          tag=$1; shift
          timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --cache-configmaps "$@" --steps 100 \
            --warmup 5 --probe-sample 0 --resident 0 --no-configs --burst 0 > "$out/bench_splitab_${tag}_n1_r$r.log" 2>&1 \
            || fail splitab $? "$out/bench_splitab_${tag}_n1_r$r.log"
          show "$out/bench_splitab_${tag}_n1_r$r.log" "splitab $tag n1 r$r"
          timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29958 bench.py --gpus 4 --arch unsharded --workers 4 --cache-configmaps \
            "$@" --steps 100 --warmup 5 --probe-sample 0 --resident 0 --burst 0 \
            > "$out/bench_splitab_${tag}_n4_r$r.log" 2>&1 || fail splitab $? "$out/bench_splitab_${tag}_n4_r$r.log"
          show "$out/bench_splitab_${tag}_n4_r$r.log" "splitab $tag n4 r$r"
        done
      done ;;
    ovlab)  # overlay mi355x candidates at 1 and 4 streams, interleaved x2: as shipped vs split kf workers + 2 webhook procs
      for r in 1 2; do
        for v in "cur" "cand --kf-split-workers --webhook-replicas 2"; do
          set -- $v
          tag=$1; shift
          timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --cache-configmaps "$@" --steps 100 \
            --warmup 5 --probe-sample 0 --resident 0 --no-configs --burst 0 > "$out/bench_ovl_${tag}_n1_r$r.log" 2>&1 \
            || fail ovlab $? "$out/bench_ovl_${tag}_n1_r$r.log"
          show "$out/bench_ovl_${tag}_n1_r$r.log" "ovl $tag n1 r$r"
          timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29957 bench.py --gpus 4 --arch unsharded --workers 4 --cache-configmaps \
            "$@" --steps 100 --warmup 5 --probe-sample 0 --resident 0 --burst 0 \
            > "$out/bench_ovl_${tag}_n4_r$r.log" 2>&1 || fail ovlab $? "$out/bench_ovl_${tag}_n4_r$r.log"
          show "$out/bench_ovl_${tag}_n4_r$r.log" "ovl $tag n4 r$r"
        done
      done ;;
    wr2)
      timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --webhook-replicas 2 --steps 100 \
        --warmup 5 --probe-sample 0 > "$out/bench_wr2_n1.log" 2>&1 || fail wr2 $? "$out/bench_wr2_n1.log"
      show "$out/bench_wr2_n1.log" "workers4 wr2 n1"
      for n in 2 4; do
        timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port 2996$n bench.py --gpus $n --arch unsharded --workers 4 \
          --webhook-replicas 2 --steps 100 --warmup 5 --probe-sample 0 > "$out/bench_wr2_n$n.log" 2>&1 \
          || fail wr2 $? "$out/bench_wr2_n$n.log"
        show "$out/bench_wr2_n$n.log" "workers4 wr2 n$n"
      done ;;
    wcm)
      for r in 1 2; do
        for v in live cached; do
          case $v in cached) f="--cache-configmaps" ;; *) f="" ;; esac
          timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29985 bench.py --gpus 4 --arch unsharded --workers 4 $f \
            --steps 100 --warmup 5 --probe-sample 0 > "$out/bench_wcm_${v}_n4_r$r.log" 2>&1 \
            || fail wcm $? "$out/bench_wcm_${v}_n4_r$r.log"
          show "$out/bench_wcm_${v}_n4_r$r.log" "workers4 $v n4 r$r"
        done
      done
      timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --cache-configmaps --steps 100 \
        --warmup 5 --probe-sample 0 --no-configs > "$out/bench_wcm_cached_n1.log" 2>&1 \
        || fail wcm $? "$out/bench_wcm_cached_n1.log"
      show "$out/bench_wcm_cached_n1.log" "workers4 cached n1" ;;
    wcmr2)  # overlay mi355x (cached ConfigMaps) with 1 vs 2 odh webhook processes, 4 ranks, interleaved
      for r in $(seq 1 "${ROUNDS:-2}"); do
        for v in 1 2; do
          timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29983 bench.py --gpus 4 --arch unsharded --workers 4 \
            --cache-configmaps --webhook-replicas $v --steps 100 --warmup 5 --probe-sample 0 --no-configs \
            > "$out/bench_wcmr${v}_n4_r$r.log" 2>&1 || fail wcmr2 $? "$out/bench_wcmr${v}_n4_r$r.log"
          show "$out/bench_wcmr${v}_n4_r$r.log" "workers4 cached wr$v n4 r$r"
        done
      done ;;
    wcmr2n1)  # the same at 1 and 2 ranks (efficiency denominators), interleaved
      for r in 1 2; do
        for v in 1 2; do
          timeout -k 10 170 python bench.py --gpus 1 --arch unsharded --workers 4 --cache-configmaps \
            --webhook-replicas $v --steps 100 --warmup 5 --probe-sample 0 --no-configs \
            > "$out/bench_wcmr${v}_n1_r$r.log" 2>&1 || fail wcmr2n1 $? "$out/bench_wcmr${v}_n1_r$r.log"
          show "$out/bench_wcmr${v}_n1_r$r.log" "workers4 cached wr$v n1 r$r"
          timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29982 bench.py --gpus 2 --arch unsharded --workers 4 \
            --cache-configmaps --webhook-replicas $v --steps 100 --warmup 5 --probe-sample 0 --no-configs \
            > "$out/bench_wcmr${v}_n2_r$r.log" 2>&1 || fail wcmr2n1 $? "$out/bench_wcmr${v}_n2_r$r.log"
          show "$out/bench_wcmr${v}_n2_r$r.log" "workers4 cached wr$v n2 r$r"
        done
      done ;;
    wpab)
      for r in 1 2; do
        for v in shared own; do
          case $v in shared) f="--webhook-in-odh" ;; *) f="" ;; esac
          timeout -k 10 170 python bench.py --gpus 1 $f --steps 100 --warmup 5 --probe-sample 0 --no-configs \
            --no-inprocess-baseline > "$out/bench_wp_${v}_n1_r$r.log" 2>&1 || fail wpab $? "$out/bench_wp_${v}_n1_r$r.log"
          show "$out/bench_wp_${v}_n1_r$r.log" "webhook $v n1 r$r"
          timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
            --master-addr 127.0.0.1 --master-port 29984 bench.py --gpus 4 $f --steps 100 --warmup 5 --probe-sample 0 \
            > "$out/bench_wp_${v}_n4_r$r.log" 2>&1 || fail wpab $? "$out/bench_wp_${v}_n4_r$r.log"
          show "$out/bench_wp_${v}_n4_r$r.log" "webhook $v n4 r$r"
        done
      done ;;
    fair)
      # the reference's behaviour vs ours in two regimes — vanilla Kubernetes (nothing ever adds
      # the pull secret the reference's lock waits for: 1 s + 5 s) and OpenShift-like (every SA
      # gets its pull secret 200 ms after it appears) — with and without 2 ms of storage latency
      # per write; one notebook at a time and 8 at once
      for wl in 0 2; do
        for cl in vanilla openshift; do
          case $cl in openshift) cf="--openshift-pull-secret-ms 200" ;; *) cf="" ;; esac
          timeout -k 10 170 python bench.py --gpus 1 --steps 20 --warmup 3 --probe-sample 0 --no-configs \
            --no-inprocess-baseline --burst 8 --write-latency-ms $wl $cf > "$out/fair_ours_${cl}_wl$wl.log" 2>&1 \
            || fail fair $? "$out/fair_ours_${cl}_wl$wl.log"
          show "$out/fair_ours_${cl}_wl$wl.log" "ours $cl wl$wl"
          timeout -k 10 170 python bench.py --gpus 1 --reference-emulation --steps 2 --warmup 1 --probe-sample 0 \
            --no-configs --no-inprocess-baseline --burst 8 --burst-rounds 1 --write-latency-ms $wl $cf \
            > "$out/fair_ref_${cl}_wl$wl.log" 2>&1 || fail fair $? "$out/fair_ref_${cl}_wl$wl.log"
          show "$out/fair_ref_${cl}_wl$wl.log" "reference $cl wl$wl"
        done
      done ;;
    pw4)
      # 4 ranks, unsharded --workers 4, the node platform with one StatefulSet-controller and
      # kubelet process per rank (default: one per two ranks)
      timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
        --master-addr 127.0.0.1 --master-port 29964 bench.py --gpus 4 --arch unsharded --workers 4 --steps 100 \
        --warmup 5 --probe-sample 0 --platform-workers 4 > "$out/bench_workers_pw4_n4.log" 2>&1 \
        || fail pw4 $? "$out/bench_workers_pw4_n4.log"
      show "$out/bench_workers_pw4_n4.log" "workers4 pw4 n4" ;;
    nsr)
      for v in "sharded 2 1 hash" "sharded 2 1 balanced" "sharded 4 1 hash" "sharded 4 1 balanced" \
               "unsharded 4 4 hash"; do
        set -- $v
        timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 \
          --master-addr 127.0.0.1 --master-port 2997$2 bench.py --gpus $2 --arch $1 --workers $3 --steps 100 \
          --warmup 5 --probe-sample 0 --namespaces-per-rank 16 --assign-policy $4 \
          $([ "$1" = unsharded ] && echo --cache-configmaps) \
          > "$out/bench_nsr16_$1_n$2_$4.log" 2>&1 || fail nsr $? "$out/bench_nsr16_$1_n$2_$4.log"
        show "$out/bench_nsr16_$1_n$2_$4.log" "nsr16 $1 n$2 w$3 $4"
      done ;;
    rss300)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
        --master-addr 127.0.0.1 --master-port 29980 bench.py --gpus 4 --steps 300 --warmup 5 --probe-sample 0 \
        --burst 0 > "$out/bench_rss300_n4.log" 2>&1 || fail rss300 $? "$out/bench_rss300_n4.log"
      show "$out/bench_rss300_n4.log" "rss300 n4" ;;
    burst64)
      for v in "unsharded 1" "unsharded 4" "sharded 1"; do
        set -- $v
        timeout -k 10 170 python bench.py --gpus 1 --arch $1 --workers $2 --steps 20 --warmup 5 --probe-sample 0 \
          --burst 64 --no-inprocess-baseline > "$out/bench_burst64_$1_w$2.log" 2>&1 \
          || fail burst64 $? "$out/bench_burst64_$1_w$2.log"
        show "$out/bench_burst64_$1_w$2.log" "burst64 $1 w$2"
      done ;;
    archab)
      # interleaved A/B at N=1: the shard pod's kf / odh+webhook process pair (deployed), one
      # process per shard, and the reference's two-process layout (kf manager + odh manager)
      for r in 1 2 3; do
        for a in sharded single unsharded; do
          case $a in single) flags="--arch sharded --single-process-shard" ;; *) flags="--arch $a" ;; esac
          timeout -k 10 170 python bench.py --gpus 1 $flags --steps 300 --warmup 5 --probe-sample 0 \
            --no-inprocess-baseline > "$out/bench_ab_${a}_r$r.log" 2>&1 || fail archab $? "$out/bench_ab_${a}_r$r.log"
          show "$out/bench_ab_${a}_r$r.log" "$a r$r"
        done
      done ;;
    hipinit)
      timeout -k 10 300 bash tools/research/hip_init_ab.sh "$tag" > "$out/hip_init_ab.log" 2>&1 || fail hipinit $? "$out/hip_init_ab.log"
      cat "$out/hip_init_ab.log" ;;
    hsaknobs)
      timeout -k 10 300 python tools/research/hsa_init_knobs.py --rounds ${HSA_KNOB_ROUNDS:-5} ${HSA_KNOB_ONLY:+--only $HSA_KNOB_ONLY} \
        > "$out/hsa_init_knobs.jsonl" 2>&1 \
        || fail hsaknobs $? "$out/hsa_init_knobs.jsonl"
      tail -1 "$out/hsa_init_knobs.jsonl" ;;
    hipexit)
      timeout -k 10 300 python tools/research/hip_exit_ab.py --repeats 5 > "$out/hip_exit_ab.jsonl" 2>&1 \
        || fail hipexit $? "$out/hip_exit_ab.jsonl"
      tail -1 "$out/hip_exit_ab.jsonl" ;;
    cpprof)
      mkdir -p "$out/cprof"
      ODH_CONTROL_PLANE_PROFILE=$PWD/$out/cprof/cp ODH_PLATFORM_PROFILE=$PWD/$out/cprof/plat \
        timeout -k 10 200 python bench.py --gpus 1 --no-inprocess-baseline --probe-sample 0 --burst 0 --resident 0 \
        --no-configs > "$out/bench_cpprof.log" 2>&1 || fail cpprof $? "$out/bench_cpprof.log"
      show "$out/bench_cpprof.log" "n1 cprofiled (closed loop only)"
      for f in "$out"/cprof/*; do
        case $f in *control_plane*) cp "$f" "$f.pstats" ;; esac  # raw stats of the control plane, for offline reading
        python - "$f" > "$f.txt" <<'PY' || fail cpprof $? "$f.txt"
import pstats, sys
st = pstats.Stats(sys.argv[1])
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumulative").print_stats(40)
PY
        rm -f "$f"
      done
      ls "$out/cprof" ;;
    critpath)
      timeout -k 10 600 bash tools/gpu_critical_path.sh "$tag" > "$out/critpath.log" 2>&1 || fail critpath $? "$out/critpath.log"
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['create_to_notebook_status_ms'], {k: (v['gap_ms_p50'], v['serve_ms_p50']) for k, v in d['hops'].items()})" \
        "$out/critical_path_n1.json" ;;
    probeexe)
      for r in 1 2 3 4 5 6 7 8 9 10; do
        s0=$(date +%s%N)
        timeout -k 10 60 odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - > "$out/probeexe_$r.json" 2>&1 \
          || fail probeexe $? "$out/probeexe_$r.json"
        echo "run $r wall_ms $(( ($(date +%s%N) - s0) / 1000000 ))" >> "$out/probeexe_walls.txt"
      done
      for r in 1 2 3; do  # with the RCCL all-reduce step (amd.com/gpu-probe: "rccl")
        timeout -k 10 120 odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - --rccl-mib 64 \
          > "$out/probeexe_rccl_$r.json" 2>&1 || fail probeexe $? "$out/probeexe_rccl_$r.json"
      done
      cat "$out/probeexe_walls.txt"; tail -1 "$out/probeexe_10.json"; tail -1 "$out/probeexe_rccl_3.json" ;;
    ranks)
      for n in 2 4; do
        timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port 2993$n bench.py --gpus $n \
          > "$out/bench_n$n.log" 2>&1 || fail ranks $? "$out/bench_n$n.log"
        show "$out/bench_n$n.log" "n$n"
      done ;;
    webhook)
      timeout -k 10 170 python tools/bench_webhook.py --rounds 20 > "$out/webhook.log" 2>&1 || fail webhook $? "$out/webhook.log"
      tail -1 "$out/webhook.log" ;;
    culling)
      timeout -k 10 170 python tools/bench_culling.py > "$out/culling.log" 2>&1 || fail culling $? "$out/culling.log"
      tail -1 "$out/culling.log" ;;
    realpods)
      timeout -k 10 400 python tools/bench_real_pods.py --notebooks 1,8 --repeats 5 > "$out/realpods.log" 2>&1 \
        || fail realpods $? "$out/realpods.log"
      grep '^{' "$out/realpods.log" ;;
    realbr)
      timeout -k 10 400 python tools/bench_real_pods.py --notebooks 1,8 --repeats 5 --gpu-probe off \
        --gpu-init before-ready > "$out/realpods_before_ready.log" 2>&1 || fail realbr $? "$out/realpods_before_ready.log"
      grep '^{' "$out/realpods_before_ready.log" ;;
    realref)  # the reference behaviour stalls 6 s per notebook in silence: print a heartbeat meanwhile
      ( while sleep 30; do echo "realref running"; done ) & hb=$!
      timeout -k 10 240 python tools/bench_real_pods.py --notebooks 1,8 --repeats 1 --reference-emulation \
        > "$out/realpods_ref.log" 2>&1; rc=$?
      kill $hb
      [ $rc -eq 0 ] || fail realref $rc "$out/realpods_ref.log"
      grep '^{' "$out/realpods_ref.log" ;;
    refemu)
      timeout -k 10 200 python bench.py --reference-emulation --steps 3 --warmup 1 --no-inprocess-baseline \
        > "$out/bench_refemu.log" 2>&1 || fail refemu $? "$out/bench_refemu.log"
      show "$out/bench_refemu.log" "refemu" ;;
    prof)
      ODH_PROBE_EXIT_NORMALLY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- \
        odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - > "$out/probe_prof.log" 2>&1 || fail prof $? "$out/probe_prof.log"
      db=$(find "$out/prof" -name '*results.db' | head -1)
      if [ -n "$db" ]; then
        python3 tools/rocpd_stats.py "$db" > "$out/probe_kernel_stats.csv" && head -6 "$out/probe_kernel_stats.csv"
      fi ;;
    pmc)
      # one counter group per pass, each within the per-block limits
      i=0
      timeout -k 10 60 rocprofv3 --list-avail > "$out/pmc_avail.txt" 2>&1 || true
      for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
                   "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" \
                   "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        i=$((i + 1))
        ODH_PROBE_EXIT_NORMALLY=1 timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d "$out/pmc$i" -o run -- \
          python3 tools/probe_microbench.py --pmc-pass > "$out/pmc$i.log" 2>&1 || fail "pmc$i" $? "$out/pmc$i.log"
      done
      echo "pmc passes: $i" ;;
    probe)
      timeout -k 10 120 python tools/probe_microbench.py --startup > "$out/probe_startup.json" 2>&1 \
        || fail probe $? "$out/probe_startup.json"
      cat "$out/probe_startup.json" ;;
    env)
      timeout -k 10 200 bash tools/gpu_env_probe.sh > "$out/env.log" 2>&1 || fail env $? "$out/env.log" ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo "pass $tag done: $steps"
