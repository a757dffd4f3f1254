#!/bin/bash
# One measurement pass on a GPU box (run through gpurun from the repo root):
#   tools/gpu_pass.sh <tag> [tests] [driver N] [long STEPS] [resident R K] [streams K ARCH]
# Every GPU step has its own time limit and the steps are chained: the first failure ends
# the pass (no retries).  Results land in gpurun_out/<tag>/.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
ngpu=$(python -c 'import torch; print(torch.cuda.device_count())' 2>/dev/null)
echo "pass $tag: $(date -u +%FT%TZ) gpus=$ngpu cpus=$(nproc)" | tee "$out/SUMMARY.txt"
# a line a minute while a long step runs silently (gpurun takes 3 quiet minutes for a hang)
(while sleep 60; do date -u +%FT%TZ >> "$out/progress.txt"; done) &
beat=$!
trap 'kill $beat 2>/dev/null' EXIT
while [ $# -gt 0 ]; do
  what=$1; shift
  case $what in
    tests)
      timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$out/gpu_tests.log" 2>&1 || { echo "gpu tests failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      tail -1 "$out/gpu_tests.log" | tee -a "$out/SUMMARY.txt" ;;
    smoke)
      # the driver's round-end smoke: __graft_entry__.smoke() on cuda:0
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$out/smoke.log" 2>&1 || { echo "smoke failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      tail -1 "$out/smoke.log" | tee -a "$out/SUMMARY.txt" ;;
    driver)
      n=$1; shift
      for i in $(seq 1 "$n"); do
        timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$out/driver_$i.json" \
          > "$out/driver_$i.log" 2>&1 || { echo "driver run $i failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
        python tools/summarize_bench.py "$out/driver_$i.log" | tee -a "$out/SUMMARY.txt"
      done ;;
    long)
      steps=$1; shift
      timeout -k 10 600 python bench.py --gpus 1 --steps "$steps" --warmup 10 --no-configs --burst 0 --resident 0 \
        --json-out "$out/long_$steps.json" > "$out/long_$steps.log" 2>&1 \
        || { echo "long run failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python tools/summarize_bench.py "$out/long_$steps.log" | tee -a "$out/SUMMARY.txt" ;;
    resident)
      # resident R K: R notebooks at rest, the culler writing its check stamp every K-th check
      r=$1; k=$2; shift 2
      f="$out/resident_${r}_k${k}_p${CULLING_PERIOD:-1}_$(date +%s)"
      timeout -k 10 900 python bench.py --gpus 1 --steps 100 --warmup 10 --no-configs --burst 0 --storage-steps 0 \
        --no-gpu-probe --resident "$r" --culler-stamp-every "$k" --resident-window 5 --resident-steps 40 \
        --culling-period "${CULLING_PERIOD:-1}" \
        --json-out "$f.json" > "$f.log" 2>&1 || { echo "resident run failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python tools/summarize_bench.py "$f.log" | tee -a "$out/SUMMARY.txt" ;;
    rescp)
      # rescp R K: the resident run with the apiserver's audit log, then the create->Ready critical
      # path hop by hop of the timed (empty-cluster) notebooks and of those created on top
      r=$1; k=$2; shift 2
      f="$out/rescp_${r}_k${k}"
      DEBUG_WRITE_AUDITLOG=$PWD/$f.audit.jsonl timeout -k 10 900 python bench.py --gpus 1 --steps 100 --warmup 10 \
        --no-configs --burst 0 --storage-steps 0 --no-gpu-probe --resident "$r" --culler-stamp-every "$k" \
        --resident-window 5 --resident-steps 40 --json-out "$f.json" > "$f.log" 2>&1 \
        || { echo "rescp run failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python tools/summarize_bench.py "$f.log" | tee -a "$out/SUMMARY.txt"
      python tools/critical_path.py "$f.audit.jsonl" --name-prefix nb-s > "$f.cp_timed.json" || exit 1
      python tools/critical_path.py "$f.audit.jsonl" --name-prefix nb-res- > "$f.cp_on_top.json" || exit 1
      rm -f "$f.audit.jsonl" ;;
    streams)
      k=$1; shift
      arch=${1:-sharded}; shift
      extra=()
      # an optional number after the layout: the unsharded layout's webhook processes (default 3,
      # as overlay mi355x)
      wr=3; wrtag=""
      if [[ "${1:-}" =~ ^[0-9]+$ ]]; then wr=$1; wrtag="_wr$1"; shift; fi
      [ "$arch" = unsharded ] && extra=(--arch unsharded --workers 4 --kf-split-workers \
        --webhook-replicas "$wr" --cache-configmaps)
      f="streams_${k}_${arch}${wrtag}_$(date +%s)"
      cat /sys/fs/cgroup/cpu.stat > "$out/$f.cpustat0" 2>/dev/null || true
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$k" --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus "$k" --steps 100 --warmup 10 --no-gpu-probe --burst 0 --resident 0 \
        --storage-steps 0 "${extra[@]}" --json-out "$out/$f.json" > "$out/$f.log" 2>&1 \
        || { echo "streams $k $arch failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      cat /sys/fs/cgroup/cpu.stat > "$out/$f.cpustat1" 2>/dev/null || true
      python tools/summarize_bench.py "$out/$f.log" | tee -a "$out/SUMMARY.txt"
      # the box's CPU share over the run: cgroup v2 usage and CFS throttling
      python - "$out/$f.cpustat0" "$out/$f.cpustat1" <<'PY' | tee -a "$out/SUMMARY.txt"
import sys
def rd(p):
    try:
        return {l.split()[0]: int(l.split()[1]) for l in open(p) if len(l.split()) == 2}
    except OSError:
        return {}
a, b = rd(sys.argv[1]), rd(sys.argv[2])
print("  cgroup cpu.stat delta:", {k: b[k] - a.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec") if k in b})
PY
      ;;
    failover)
      # takeover and cold start with R resident notebooks (tools/bench_failover.py)
      r=$1; shift
      timeout -k 10 600 python tools/bench_failover.py --resident "$r" > "$out/failover_$r.log" 2>&1 \
        || { echo "failover failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      tail -1 "$out/failover_$r.log" | cut -c1-600 | tee -a "$out/SUMMARY.txt" ;;
    nsscale)
      # 4 ranks x M namespaces each (balanced assigner), per-namespace or cluster-wide watches
      m=$1; mode=$2; shift 2
      cw=(); [ "$mode" = cw ] && cw=(--cluster-wide-watches)
      f="$out/ns_m${m}_$mode"
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29523 bench.py --gpus 4 --steps 100 --warmup 10 --no-gpu-probe --burst 0 --resident 0 \
        --storage-steps 0 --namespaces-per-rank "$m" --assign-policy balanced "${cw[@]}" --json-out "$f.json" \
        > "$f.log" 2>&1 || { echo "nsscale $m $mode failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python tools/summarize_bench.py "$f.log" | tee -a "$out/SUMMARY.txt" ;;
    burst)
      # burst K ARCH: K notebooks at once into one control plane (sharded | unsharded | workers)
      k=$1; arch=$2; shift 2
      extra=(); [ "$arch" = unsharded ] && extra=(--arch unsharded)
      [ "$arch" = workers ] && extra=(--arch unsharded --workers 4 --kf-split-workers --webhook-replicas 3 --cache-configmaps)
      f="$out/burst${k}_$arch"
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-configs --no-gpu-probe --resident 0 \
        --storage-steps 0 --burst "$k" "${extra[@]}" --json-out "$f.json" > "$f.log" 2>&1 \
        || { echo "burst $k $arch failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python tools/summarize_bench.py "$f.log" | tee -a "$out/SUMMARY.txt" ;;
    critpath)
      # critpath ARCH: the closed loop's create->Ready critical path from the audit log, N=1 and
      # 4 ranks (ARCH sharded, or workers = overlay mi355x)
      arch=$1; shift
      extra=()
      [ "$arch" = workers ] && extra=(--arch unsharded --workers 4 --kf-split-workers --webhook-replicas 3 --cache-configmaps)
      DEBUG_WRITE_AUDITLOG=$PWD/$out/a1.jsonl timeout -k 10 300 python bench.py --steps 200 --burst 0 --probe-sample 0 \
        --no-configs --resident 0 --storage-steps 0 "${extra[@]}" > "$out/critpath_${arch}_n1.log" 2>&1 || exit 1
      python tools/critical_path.py "$out/a1.jsonl" --name-prefix nb-s > "$out/critical_path_${arch}_n1.json" || exit 1
      DEBUG_WRITE_AUDITLOG=$PWD/$out/a4.jsonl timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29934 bench.py --gpus 4 --steps 100 --warmup 5 \
        --burst 0 --probe-sample 0 --no-configs --resident 0 --storage-steps 0 "${extra[@]}" \
        > "$out/critpath_${arch}_n4.log" 2>&1 || exit 1
      python tools/critical_path.py "$out/a4.jsonl" --name-prefix nb-s > "$out/critical_path_${arch}_n4.json" || exit 1
      rm -f "$out/a1.jsonl" "$out/a4.jsonl"
      python -c "import json,sys; [print(f, json.load(open(f))['create_to_notebook_status_ms'], json.load(open(f)).get('teardown')) for f in sys.argv[1:]]" \
        "$out/critical_path_${arch}_n1.json" "$out/critical_path_${arch}_n4.json" | tee -a "$out/SUMMARY.txt" ;;
    probeprof)
      # rocprofv3 kernel trace + stats of one odh-gpu-probe run (no counters: a plain trace)
      ODH_PROBE_EXIT_NORMALLY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/probeprof" -o probe -- \
        ./odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - > "$out/probeprof.log" 2>&1 \
        || { echo "probeprof failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      for i in 1 2 3 4 5; do
        timeout -k 10 60 ./odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - --quiet >> "$out/probe_runs.jsonl" 2>&1 || exit 1
      done
      find "$out/probeprof" -name '*kernel_stats.csv' -exec cp {} "$out/probe_kernel_stats.csv" \;
      for db in "$out"/probeprof/*.db; do [ -f "$db" ] && python tools/rocpd_stats.py "$db" > "$out/probe_kernel_stats.csv"; done
      rm -f "$out"/probeprof/*.db
      echo "probe runs:" | tee -a "$out/SUMMARY.txt"
      python -c "import json,sys; [print(json.loads(l).get('timings_ms'), json.loads(l).get('setup_ms')) for l in open(sys.argv[1]) if l.startswith('{')]" \
        "$out/probe_runs.jsonl" | tee -a "$out/SUMMARY.txt" ;;
    probestreams)
      # the probe with 2, 1 and 0 created streams, interleaved, K rounds: the set-up time each costs
      k="$1"; shift
      for i in $(seq "$k"); do
        for ns in 2 1 0; do
          timeout -k 10 60 ./odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - --quiet --streams "$ns" \
            >> "$out/probe_streams.jsonl" 2>&1 || exit 1
        done
      done
      python tools/probe_streams.py "$out/probe_streams.jsonl" | tee -a "$out/SUMMARY.txt" ;;
    probegap)
      # K probe runs S seconds apart: hip_init with the previous GPU process long gone
      k="$1"; gap="$2"; shift 2
      for i in $(seq "$k"); do
        sleep "$gap"
        timeout -k 10 60 ./odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - --quiet >> "$out/probe_gap_$gap.jsonl" 2>&1 || exit 1
      done
      python tools/probe_streams.py "$out/probe_gap_$gap.jsonl" | sed "s/^/gap=${gap}s /" | tee -a "$out/SUMMARY.txt" ;;
    probebusy)
      # K probe runs S seconds apart while another process holds the GPU (a torch context, idle)
      k="$1"; gap="$2"; shift 2
      timeout -k 5 240 python -c "import torch, time; torch.zeros(1, device='cuda'); torch.cuda.synchronize(); print('held', flush=True); time.sleep(200)" \
        > "$out/holder.log" 2>&1 &
      hp=$!
      for i in $(seq 150); do grep -q held "$out/holder.log" && break; sleep 1; done
      grep -q held "$out/holder.log" || { kill "$hp"; wait "$hp"; echo "holder did not start" | tee -a "$out/SUMMARY.txt"; exit 1; }
      for i in $(seq "$k"); do
        sleep "$gap"
        timeout -k 10 60 ./odh_kubeflow_amd/ops/_lib/odh-gpu-probe --json - --quiet >> "$out/probe_busy_$gap.jsonl" 2>&1 \
          || { kill "$hp"; wait "$hp"; exit 1; }
      done
      kill "$hp"; wait "$hp"
      python tools/probe_streams.py "$out/probe_busy_$gap.jsonl" | sed "s/^/busy gap=${gap}s /" | tee -a "$out/SUMMARY.txt" ;;
    fair)
      # fair CLUSTER WL SIDE: the fair reference baseline (README "A fair reference baseline"):
      # CLUSTER vanilla | openshift (pull secrets 200 ms after each ServiceAccount), WL ms per
      # apiserver write, SIDE ours | ref (--reference-emulation); N=1, then 8 at once (the second of
      # two bursts: the first warms the apiserver's TLS connections to the webhook)
      cl="$1"; wl="$2"; side="$3"; shift 3
      extra=(); [ "$cl" = openshift ] && extra+=(--openshift-pull-secret-ms 200)
      if [ "$side" = ref ]; then extra+=(--reference-emulation --steps 2 --warmup 1); else extra+=(--steps 20 --warmup 3); fi
      timeout -k 10 400 python bench.py --burst 8 --burst-rounds 2 --resident 0 --storage-steps 0 --no-configs \
        --no-gpu-probe --write-latency-ms "$wl" "${extra[@]}" > "$out/fair_${side}_${cl}_wl$wl.log" 2>&1 \
        || { echo "fair $cl $wl $side failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python - "$out/fair_${side}_${cl}_wl$wl.log" <<'PY' | tee -a "$out/SUMMARY.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
b = d.get("burst") or {}
print(sys.argv[1].split("/")[-1], "p50", d.get("p50_ready_ms"), "8 at once: all Ready", b.get("all_ready_s"), "s, p50", (b.get("ready_ms") or {}).get("p50"))
PY
      ;;
    burstdebug)
      # burstdebug WL: burstcp with asyncio debug (callbacks over 100 ms logged) and every child's
      # stderr kept under $out/children
      wl="$1"; shift
      PYTHONASYNCIODEBUG=1 ODH_CHILD_STDERR_DIR=$PWD/$out/children timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
        --burst 8 --burst-rounds 2 --resident 0 --storage-steps 0 --no-configs --no-gpu-probe --write-latency-ms "$wl" \
        > "$out/burstdebug_wl$wl.log" 2>&1 || { echo "burstdebug failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric\"')][-1]); print(sys.argv[1], d['burst'].get('rounds'))" \
        "$out/burstdebug_wl$wl.log" | tee -a "$out/SUMMARY.txt"
      python tools/slow_callbacks.py "$out/children" | tee -a "$out/SUMMARY.txt" ;;
    burstcp)
      # burstcp WL: 8 at once (second of two bursts) at WL ms per apiserver write, with the audit
      # log: the burst notebooks' critical path, and the log itself (gzip) for the timeline
      wl="$1"; shift
      DEBUG_WRITE_AUDITLOG=$PWD/$out/burst_wl$wl.audit.jsonl timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
        --burst 8 --burst-rounds 2 --resident 0 --storage-steps 0 --no-configs --no-gpu-probe --write-latency-ms "$wl" \
        > "$out/burstcp_wl$wl.log" 2>&1 || { echo "burstcp failed rc=$?" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python tools/critical_path.py "$out/burst_wl$wl.audit.jsonl" --name-prefix burst-r1 > "$out/burstcp_wl$wl.json" || exit 1
      gzip -f "$out/burst_wl$wl.audit.jsonl"
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{\"metric\"')][-1]); print(sys.argv[1], d['burst'].get('rounds'), d['burst'].get('cgroup_cpu'))" \
        "$out/burstcp_wl$wl.log" | tee -a "$out/SUMMARY.txt"
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['create_to_notebook_status_ms'], {k: (v['gap_ms_p50'], v['serve_ms_p50']) for k, v in d['hops'].items()})" \
        "$out/burstcp_wl$wl.json" | tee -a "$out/SUMMARY.txt" ;;
    burststall)
      # burststall WL TRIM_S ROUNDS: ROUNDS bursts of 8 at WL ms per write with two stall
      # watchdogs — tools/stall_sampler.py (a process of its own: the box's stalls) and the
      # apiserver's ODH_STALL_WATCHDOG_MS thread (its process's) — and the apiserver's
      # malloc_trim every TRIM_S seconds (0: off)
      wl="$1"; trim="$2"; rounds="$3"; shift 3
      sfx="wl${wl}_t${trim}_$(date +%s)"; log="$out/burststall_$sfx.log"; smp="$out/stall_sampler_$sfx.txt"
      python tools/stall_sampler.py --ms ${STALL_MS:-20} --seconds 290 > "$smp" 2>&1 &
      spid=$!
      ODH_CHILD_STDERR_DIR=$PWD/$out/children_$sfx ODH_STALL_WATCHDOG_MS=${STALL_MS:-20} ODH_APISERVER_TRIM_S=$trim timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
        --burst 8 --burst-rounds "$rounds" --resident 0 --storage-steps 0 --no-configs --no-gpu-probe \
        --write-latency-ms "$wl" > "$log" 2>&1
      rc=$?
      kill $spid 2>/dev/null; wait $spid 2>/dev/null
      [ $rc = 0 ] || { echo "burststall failed rc=$rc" | tee -a "$out/SUMMARY.txt"; exit 1; }
      python - "$log" "$smp" "$out/children_$sfx" <<'PY' | tee -a "$out/SUMMARY.txt"
import glob, json, os, re, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
cl = []  # the control-plane processes' own reports (requests that took >= the threshold)
for f in sorted(glob.glob(os.path.join(sys.argv[3], "*.log"))):
    cl += [os.path.basename(f).split(".")[0] + ": " + l.strip() for l in open(f, errors="replace") if l.startswith("stall-watchdog")]
rounds = d["burst"].get("rounds") or []
print(sys.argv[1].split("/")[-1], "all_ready_s:", [r.get("all_ready_s") for r in rounds])
wd = [l.strip() for l in open(sys.argv[1]) if l.startswith("stall-watchdog")]
sm = [l.strip() for l in open(sys.argv[2]) if "ending at" in l]
print("  apiserver watchdog:", len(wd), wd[:12])
print("  sampler:", len(sm), sm[:12], [l.strip() for l in open(sys.argv[2]) if " end " in l])
for i, r in enumerate(rounds):
    t0, t1 = r.get("started_at") or 0, (r.get("started_at") or 0) + (r.get("all_ready_s") or 0) + 0.05
    hit = lambda ls: [l for l in ls if (m := re.search(r"ending at ([0-9.]+)", l)) and t0 <= float(m.group(1)) <= t1 + 0.3]
    print(f"  round {i}: {r.get('all_ready_s')} s, watchdog in window {hit(wd)}, sampler in window {hit(sm)}")
    for l in hit(cl)[:16]:
        print("     client:", l[:260])
print("  control-plane reports (not requeues):", [l[:220] for l in cl if "requeued" not in l][:24])
PY
      ;;
    cpuinfo)
      # the CPU share this box gives the command: quota, cpuset, SMT
      { echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "cpuset: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null)"
        echo "nproc: $(nproc)"; lscpu | grep -E "^(CPU\(s\)|Thread|Core|Socket|Model name)"; } | tee -a "$out/SUMMARY.txt" ;;
    probechain)
      # K runs GAP seconds apart, probe args after "--" up to the next step name "end"
      k="$1"; gap="$2"; shift 2
      pargs=(); while [ $# -gt 0 ] && [ "$1" != end ]; do pargs+=("$1"); shift; done; [ $# -gt 0 ] && shift
      timeout -k 10 300 python tools/probe_chain.py "$k" "$gap" "${pargs[@]}" | tee -a "$out/SUMMARY.txt" || exit 1 ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
done
echo "pass $tag done $(date -u +%FT%TZ)" | tee -a "$out/SUMMARY.txt"
