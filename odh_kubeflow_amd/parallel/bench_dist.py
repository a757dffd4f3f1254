"""Multi-GPU benchmark driver: one process per MI355X (``torch.distributed.run``).

Layout on an 8×MI355X node (see :mod:`.shard` and :mod:`.platform`):

* **rank 0** starts the native C++ apiserver (``odh-apiserver``: store, REST/watch,
  admission, GC) and the node's platform — ONE scheduler (first-free ``amd.com/gpu``
  allocation), ONE StatefulSet controller and ONE kubelet for all GPUs — as child
  processes, and broadcasts the URL;
* the control plane under test runs as the deployment runs it: ``--arch sharded`` (default,
  ``overlays/mi355x-sharded``): every rank starts its ``cmd/control_plane.py --shard r``;
  ``--arch unsharded`` (``overlays/mi355x``, the reference topology): rank 0 starts
  ``cmd/kf_manager.py`` + ``cmd/odh_manager.py`` and every rank's notebooks go through them;
* each rank drives its own namespace: one step = create one ``amd.com/gpu: 1`` Notebook →
  Ready → delete → Notebook and pod gone.  ``--namespaces-per-rank M``: the steps go round-robin
  over M namespaces per rank, created unlabelled; sharded, every shard's kf process runs the
  shipped ``NamespaceShardAssigner`` (``--assign-namespaces``), so a namespace lands on shard
  ``crc32(name) % N`` whichever rank drives it — the per-shard load is reported (``shard_load``).

**The timed region** is bracketed by barrier + ``torch.cuda.synchronize()`` on every rank;
the elapsed time is the max over ranks.  It contains exactly the K steps: the end barrier
follows the last step's "gone" with nothing in between.  ``value`` counts the reconciles the
notebook controllers completed inside it (read from their ``/debug/reconciles`` at the end
barrier): the trailing reconciles of the last deletion fall outside, as the warm-up's did
at the start — under continuous load they overlap the next step.  After the window the
control plane is quiesced (event-driven, :meth:`Manager.quiesce`) and the settled count
gives ``reconciles_per_notebook``.

**The start-up probe sample** (untimed, after the window, when a GPU is visible): a few
notebooks annotated ``amd.com/gpu-probe: "true"`` — the kf controller adds the
``odh-gpu-probe`` init container, the kubelet stand-in runs the native probe as a process on
the pod's GPU — report create→Ready with the probe against the timed (probe-off) p50, and the
probe's own verdict from the pod's ``initContainerStatuses`` termination message.

Coordination goes through ``torch.distributed`` (gloo carries the URL, the barriers and
the result gathers; when GPUs are present an RCCL all-reduce over xGMI checks the
collective path once at start-up).  Barriers run in an executor thread so every process
keeps serving its event loop while it waits.
"""

from __future__ import annotations

import asyncio
import json
import os
import statistics
import time
from typing import Optional

from .shard import driven

GPU_PROBE_ANNOTATION = "amd.com/gpu-probe"
NODE_GPUS = 8  # the node platform's MI355X count (NodePlatform gpus)
NOTEBOOK_IMAGE = "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_2.10"


def bench_namespace(rank: int) -> str:
    return f"bench-{rank}"


def bench_namespaces(rank: int, per_rank: int = 1) -> list:
    """The user namespaces rank ``rank`` drives: ``bench-r``, or M names that look like real
    users' (``bench-r-<10 hex digits>``, fixed per rank and index).  Sequential names
    (``bench-r-0``, ``bench-r-1`` …) differ in one character, and crc32 — linear over GF(2) —
    spreads such runs evenly over the shards, which real namespace names do not get."""
    if per_rank <= 1:
        return [bench_namespace(rank)]
    import hashlib

    return [f"{bench_namespace(rank)}-{hashlib.sha256(f'{rank}/{j}'.encode()).hexdigest()[:10]}"
            for j in range(per_rank)]


def shard_load(counts: dict, owner: dict, cpu_s: dict, elapsed: float, by: str,
               procs: tuple = ("control_plane", "kf_manager_", "odh_manager_")) -> dict:
    """Per shard (or worker): namespaces, notebooks driven through it in the timed window,
    its notebooks/s and its processes' CPU per notebook.  ``counts``: namespace → notebooks;
    ``owner``: namespace → shard key; ``cpu_s``: process name → CPU seconds in the window
    (a control-plane process — name starting with one of ``procs`` — is a shard's when its
    name ends in ``_<key>``)."""
    shards: dict = {}
    for ns, key in owner.items():
        d = shards.setdefault(str(key), {"namespaces": 0, "notebooks": 0})
        d["namespaces"] += 1
        d["notebooks"] += counts.get(ns, 0)
    for key, d in shards.items():
        n = d["notebooks"]
        d["notebooks_per_s"] = round(n / elapsed, 2) if elapsed > 0 else None
        mine = {p: v for p, v in cpu_s.items() if p.startswith(procs) and p.endswith(f"_{key}")}
        d["cpu_ms_per_notebook"] = {p: round(v * 1e3 / n, 3) for p, v in sorted(mine.items())} if n else {}
    loads = [d["notebooks"] for d in shards.values()]
    mean = statistics.fmean(loads) if loads else 0.0
    return {"assigned_by": by, "shards": dict(sorted(shards.items(), key=lambda kv: kv[0])),
            "max_over_mean_notebooks": round(max(loads) / mean, 3) if mean else None}


def culling_enabled(args) -> bool:
    """The MI355X overlays ship the culler on (``ENABLE_CULLING=true``,
    ``CULLING_ACTIVITY_SOURCE=combined``), so the benchmark runs it unless ``--no-culling``."""
    return not getattr(args, "no_culling", False)


def culler_env(args, proxy_url: Optional[str]) -> dict:
    """The overlays' culler settings with a scaled check period; its Jupyter requests go
    through the platform's kubectl-proxy stand-in (DEV mode, ``testing/cmd/jupyter_proxy.py``).
    No node-agent CA is configured, so the amdgpu half of ``combined`` has no samples and the
    Jupyter signal decides (the GPU signal is config #5's)."""
    env = {"ENABLE_CULLING": "true", "CULLING_ACTIVITY_SOURCE": "combined",
           "IDLENESS_CHECK_PERIOD_SECONDS": f"{getattr(args, 'culling_period', 1.0):g}",
           "CULL_CHECK_STAMP_EVERY": str(getattr(args, "culler_stamp_every", 10))}
    if proxy_url:
        env.update(DEV="true", CULLER_DEV_PROXY_URL=proxy_url)
    return env


def _dist_init():
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group(backend="gloo")
    return dist, torch


async def _in_thread(fn, *a):
    return await asyncio.get_running_loop().run_in_executor(None, fn, *a)


def _rccl_check(torch, dist, local_rank: int) -> Optional[float]:
    """One all-reduce over RCCL (xGMI) as a health check of the multi-GPU notebook path."""
    if torch.cuda.device_count() < dist.get_world_size():
        return None  # ranks share a GPU (rehearsal on a smaller box): RCCL needs one rank per device
    try:
        import datetime

        g = dist.new_group(backend="nccl", timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        x = torch.ones(1 << 20, device="cuda") * (dist.get_rank() + 1)
        t0 = time.perf_counter()
        dist.all_reduce(x, group=g)
        torch.cuda.synchronize()
        ws = dist.get_world_size()
        ok = float(x[0].item()) == ws * (ws + 1) / 2
        return (time.perf_counter() - t0) * 1e3 if ok else -1.0
    except Exception:
        return -1.0


def run_distributed(args) -> int:
    out = measure(args)
    if out is not None:
        print(json.dumps(out), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(out, f, indent=1)
    return 0


def measure(args) -> Optional[dict]:
    """Run the benchmark on this rank; rank 0 returns the report dict."""
    import torch as _t

    ndev = _t.cuda.device_count()  # does not initialise the GPU
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    binding = numa_bind(local % ndev) if ndev else None  # before any thread or child exists
    dist, torch = _dist_init()
    rank, world = dist.get_rank(), dist.get_world_size()
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    if ndev:
        torch.cuda.set_device(local_rank % ndev)
    rccl_ms = _rccl_check(torch, dist, local_rank) if ndev else None
    probe_sample = 0 if (args.no_gpu_probe or not ndev) else max(0, args.probe_sample)
    res = asyncio.run(_main(args, dist, torch, rank, world, ndev, probe_sample))
    out = None
    if rank == 0:
        from bench import report  # noqa: E402  (bench.py is the entry point on sys.path)

        out = report(args, world, res)
        arch = args.arch if args.arch in ("sharded", "unsharded") else "sharded"
        if arch == "sharded" and getattr(args, "single_process_shard", False):
            out["config"]["parallelism"] = (f"namespace-sharded control plane x{world}: one `cmd/control_plane.py "
                                            f"--shard r` process per MI355X rank (kf + odh reconcilers + odh webhook); "
                                            f"A/B variant of config/overlays/mi355x-sharded")
            out["config"]["architecture"] = "cmd/control_plane --shard, one process per shard (A/B variant)"
        elif arch == "sharded" and getattr(args, "webhook_in_odh", False):
            out["config"]["parallelism"] = (f"namespace-sharded control plane x{world}: per MI355X rank "
                                            f"`cmd/control_plane.py --shard r` as a kf process and an odh reconciler + "
                                            f"odh webhook process (A/B variant of config/overlays/mi355x-sharded)")
            out["config"]["architecture"] = "cmd/control_plane --shard r --controllers kf | odh,webhook (A/B variant)"
        elif arch == "sharded":
            sep = culling_enabled(args) and not getattr(args, "culler_in_kf", False)
            out["config"]["parallelism"] = (f"namespace-sharded control plane x{world}: per MI355X rank the shard pod "
                                            f"of config/overlays/mi355x-sharded, `cmd/control_plane.py --shard r` as a "
                                            f"kf process{', a culler + event re-emitter process' if sep else ''}, an odh reconciler "
                                            f"process and an odh webhook process")
            out["config"]["architecture"] = ("cmd/control_plane --shard r --controllers "
                                             + ("notebook | culler,events | odh | webhook (overlay mi355x-sharded)" if sep else
                                                "kf | odh | webhook" + (" (culler in the kf process: A/B variant)"
                                                                        if culling_enabled(args) else "")))
        else:
            w = max(1, getattr(args, "workers", 1))
            r = max(1, getattr(args, "webhook_replicas", 1))
            wk = (f" with --workers {w} (namespace-partitioned worker processes; the odh webhook on the supervisor"
                  + (f" and {r - 1} webhook-only replica{'s' if r > 2 else ''}, one port" if r > 1 else "") + ")") \
                if w > 1 else ""
            out["config"]["parallelism"] = (f"one kf manager + one odh manager Deployment for all {world} ranks' "
                                            f"notebooks{wk}")
            cm = getattr(args, "cache_configmaps", False)
            overlay = "overlay mi355x" if (w, r, cm) == (4, 1, True) else \
                "reference topology; overlay mi355x runs --workers 4, odh --cache-configmaps-secrets=true"
            if cm:
                overlay = "odh --cache-configmaps-secrets=true; " + overlay
            out["config"]["architecture"] = (f"cmd/kf_manager + cmd/odh_manager{f' --workers {w}' if w > 1 else ''}"
                                             f"{f' --webhook-replicas {r}' if w > 1 and r > 1 else ''} ({overlay})")
        w = getattr(args, "platform_workers", 0) or (world + 1) // 2
        out["config"]["platform_stand_ins"] = (f"native C++ apiserver (+GC); ONE scheduler (first-free amd.com/gpu "
                                               f"allocation); the node's StatefulSet controller and kubelet for its "
                                               f"8 GPUs, each as {w} worker process{'es' if w > 1 else ''} "
                                               f"(namespaces partitioned)")
        ps = getattr(args, "openshift_pull_secret_ms", -1.0)
        out["config"]["cluster"] = (f"OpenShift-like: OpenShift APIs served, every ServiceAccount's pull secret "
                                    f"added {ps:g} ms after it appears" if ps >= 0 else
                                    "vanilla Kubernetes + Gateway API (no OpenShift APIs, no pull secrets)")
        out["config"]["storage_write_latency_ms"] = getattr(args, "write_latency_ms", 0.0)
        out["rank_ms_per_step"] = res.get("rank_ms_per_step")
        out["recon_snapshot_lag_ms"] = res.get("recon_snapshot_lag_ms")
        out["io_per_notebook"] = res.get("io_per_notebook")
        out["lifecycle_ms_per_20_steps"] = res.get("lifecycle_ms_per_20_steps")
        out["cpu_ms_per_step"] = res.get("cpu_ms_per_step")
        out["child_rss_mib"] = res.get("child_rss_mib")
        out["cpu_binding"] = binding or "none (ODH_BENCH_NUMA_BIND=0, or no GPU NUMA information)"
        if res.get("apiserver_profile_per_step"):
            out["apiserver_profile_per_step"] = res["apiserver_profile_per_step"]
            out["writes_per_notebook"] = writes_per_notebook(res["apiserver_profile_per_step"], world)
        if rccl_ms is not None:
            out["rccl_allreduce_check_ms"] = round(rccl_ms, 3)
        if res.get("probe_sample"):
            out["gpu_probe_init_container"] = dict(probe_report(res["probe_sample"], out.get("p50_ready_ms")),
                                                   gap_before_each_s=getattr(args, "probe_gap_s", 0.5))
        if res.get("burst"):
            out["burst"] = res["burst"]
        if res.get("resident"):
            out["resident"] = res["resident"]
        if res.get("storage"):
            # the same closed loop on etcd-like storage, beside the zero-latency headline
            st = out["storage_" + f"{res['storage']['storage_write_latency_ms']:g}ms"] = res["storage"]
            if out.get("notebooks_ready_per_s") and st.get("notebooks_ready_per_s"):
                st["notebooks_per_s_vs_headline"] = round(st["notebooks_ready_per_s"] / out["notebooks_ready_per_s"], 3)
        out["config"]["culling"] = (f"on (overlay settings, check period {getattr(args, 'culling_period', 1.0):g} s)"
                                    if culling_enabled(args) else "off")
        if res.get("shard_load"):
            out["shard_load"] = res["shard_load"]
        out["config"]["namespaces_per_rank"] = max(1, getattr(args, "namespaces_per_rank", 1))
    dist.barrier()
    dist.destroy_process_group()
    return out


def probe_report(samples: list, p50_off: Optional[float]) -> dict:
    """create→Ready of the probe notebooks, and the probe's own verdict per notebook."""
    lat = [s["ready_ms"] for s in samples if s.get("ready_ms") is not None]
    res = [s.get("result") or {} for s in samples]
    tim = [r.get("timings_ms") or {} for r in res]
    dev = [(r.get("results") or [{}])[0] for r in res]

    def med(xs):
        xs = [x for x in xs if x is not None]
        return round(statistics.median(xs), 3) if xs else None

    p50 = med(lat)
    return {
        "notebooks": len(samples), "all_ok": all(r.get("ok") for r in res) and len(res) > 0,
        "p50_ready_ms": p50, "max_ready_ms": round(max(lat), 3) if lat else None,
        "added_ms_p50_vs_probe_off": round(p50 - p50_off, 3) if p50 is not None and p50_off is not None else None,
        "init_container_wall_ms_p50": med(s.get("wall_ms") for s in samples),
        "probe_timings_ms_p50": {k: med(t.get(k) for t in tim if (t.get(k) or 0) >= 0)
                                 for k in ("exec", "hip_init", "alloc_fill", "alloc", "code_load", "fill", "probe", "total")},
        "gemm_tflops_p50": med(d.get("gemm_tflops") for d in dev),
        "hbm_gbps_p50": med(d.get("hbm_gbps") for d in dev),
        "mechanism": "init container odh-gpu-probe (ops/csrc/probe_cli.cpp, no torch), injected by the kf "
                     "StatefulSet generator for amd.com/gpu-probe=\"true\"; run as a process by the kubelet stand-in",
    }


def writes_per_notebook(prof: dict, notebooks_per_step: int) -> dict:
    """Apiserver write calls per notebook lifecycle (create → Ready → delete), by verb.

    Counted at the apiserver, so every client is in it: the controllers, the platform stand-ins
    (scheduler binding, kubelet status, StatefulSet controller, GC) and the bench's own Notebook
    create and delete.  ``total`` is the figure the steady-state write gating and the
    single unlock patch of the odh create path are judged by."""
    n = max(1, notebooks_per_step)
    out = {v: round(prof.get(f"{v}_calls", 0.0) / n, 2) for v in ("create", "update", "patch", "delete")}
    out["total"] = round(sum(out.values()), 2)
    return out


def _pcts(xs, qs=(0.5, 0.95, 0.99)) -> dict:
    from bench import pct  # noqa: E402  (bench.py is the entry point)

    out = {f"p{int(q * 100)}": (round(pct(xs, q), 3) if xs else None) for q in qs}
    out["max"] = round(max(xs), 3) if xs else None
    return out


def _cgroup_cpu() -> Optional[dict]:
    """This container's cgroup-v2 CPU counters (``cpu.stat``): usage and CFS-quota throttling.
    On a box whose share is a CPU quota, a period whose quota is spent stops every process of
    the container until the next one — a stall no single process shows.  None when unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if len(line.split()) == 2)}
    except (OSError, ValueError):
        return None


def _cgroup_delta(a: Optional[dict], b: Optional[dict]) -> Optional[dict]:
    if not a or not b:
        return None
    d = {k: b.get(k, 0) - a.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec")}
    return {"usage_ms": round(d["usage_usec"] / 1e3, 1), "periods": d["nr_periods"],
            "throttled_periods": d["nr_throttled"], "throttled_ms": round(d["throttled_usec"] / 1e3, 1)}


async def _burst(args, shard, dist, native, children: dict, use_odh: bool, tag: str = "r0") -> Optional[dict]:
    """Open-loop capacity (the reference's load generator,
    ``kf/loadtest/start_notebooks.py:1-99``, applies N notebooks at once): ``--burst K``
    notebooks are created at once, split over the ranks, against the control plane that just
    ran the timed window.  Like the reference's ``jupyter_test.yaml`` they are CPU workbenches
    (500m / 1Gi; the node's eight MI355X could not hold K GPU pods); a burst of at most eight
    asks one ``amd.com/gpu`` each instead (config #3, one notebook per MI355X).  Reported: time from the
    first create to the last Ready, notebooks/s at saturation, create→Ready p50/p95/p99, the
    client's create latency (admission included), AdmissionReview latency at the apiserver
    (every admission in the burst: the creates and the controllers' UPDATEs), CPU per notebook
    per process, and teardown."""
    from ..models import kinds
    from ..models.notebook import notebook

    rank, world = dist.get_rank(), dist.get_world_size()
    total = int(args.burst)
    k = total // world + (1 if rank < total % world else 0)
    nss = shard.cfg.user_namespaces
    names = [f"burst-{tag}-{rank}-{i}" for i in range(k)]
    ns_of = {nm: nss[i % len(nss)] for i, nm in enumerate(names)}
    ann = {"notebooks.opendatahub.io/inject-auth": "true"} if use_odh else None
    res = {"cpu": "500m", "memory": "1Gi"}
    gpus = 1 if total <= NODE_GPUS else 0  # up to one per MI355X of the node: GPU notebooks (config #3)
    # untimed and after the headline: a failure here is reported in the block, never raised —
    # every rank still reaches every collective below, so no rank is left waiting at one
    errors: list = []

    async def safe(aw, default=None):
        try:
            return await aw
        except Exception as e:  # noqa: BLE001 — recorded in the burst block
            errors.append(f"rank {rank}: {e!r}"[:300])
            return default

    await safe(shard.quiesce())
    await _in_thread(dist.barrier)
    adm0 = (await safe(native.admissions(1 << 62), {})).get("seq") if native is not None else None
    wh0 = {k: {"served": d["served"], "gets": d.get("gets", 0)}
           for k, d in ((await safe(shard.webhook_timings(), {})) or {}).items()} if shard.cfg.launch else {}
    prof0 = await safe(_apiserver_prof(native))
    cpu0 = _cpu_snapshot(children, prof0)
    gc0 = {k: v["seq"] for k, v in ((await safe(shard.gc_pauses(), {})) or {}).items()} if shard.procs else {}
    await _in_thread(dist.barrier)
    cg0 = _cgroup_cpu()
    t0 = time.perf_counter()
    ready_at, create_ms = {}, []
    pending = set(names)

    def check() -> bool:
        for nm in list(pending):
            if shard.notebook_ready(nm, ns_of[nm]):
                ready_at[nm] = time.perf_counter()
                pending.discard(nm)
        return not pending

    async def create(nm):
        c0 = time.perf_counter()
        nb = driven(notebook(nm, ns_of[nm], image=NOTEBOOK_IMAGE, annotations=ann, gpus=gpus))
        c = nb["spec"]["template"]["spec"]["containers"][0]
        c.setdefault("resources", {}).setdefault("requests", {}).update(res)
        await shard.admin.create(nb)
        create_ms.append((time.perf_counter() - c0) * 1e3)

    await safe(asyncio.gather(*(create(nm) for nm in names)))
    ok = bool(await safe(shard.wait_until(check, 180), False))
    all_ready = max(ready_at.values()) - t0 if ready_at else None
    cgroup = _cgroup_delta(cg0, _cgroup_cpu())
    await _in_thread(dist.barrier)
    prof1 = await safe(_apiserver_prof(native))
    cpu1 = _cpu_snapshot(children, prof1)
    cpu = {kk: (cpu1.get(kk) or 0.0) - (cpu0.get(kk) or 0.0) for kk in children
           if cpu0.get(kk) is not None}
    adm = ((await safe(native.admissions(adm0), {})).get("us") or []) if native is not None and adm0 is not None else []
    # the apiserver over the burst: store-lock waits per resource, malloc_trim passes
    prof = _prof_per_step(prof0, prof1, 1) if native is not None else None
    # the control-plane processes' cyclic-GC pauses over the burst (their event loops stop)
    gcp = {k: [x[1:] for x in v["pauses"]] for k, v in ((await safe(shard.gc_pauses(gc0), {})) or {}).items()} \
        if shard.procs else {}
    whd = list(((await safe(shard.webhook_timings(wh0), {})) or {}).values()) if shard.cfg.launch else []
    wh = [x for d in whd for x in d["handle_ms"]]
    wh_get = [x for d in whd for x in d.get("get_ms") or []]
    t_del = time.perf_counter()
    await safe(asyncio.gather(*(shard.admin.delete(kinds.NOTEBOOK, nm, ns_of[nm]) for nm in names),
                              return_exceptions=True))
    gone = bool(await safe(shard.wait_until(lambda: all(shard.gone(nm, ns_of[nm]) for nm in names), 180), False))
    teardown = time.perf_counter() - t_del
    gathered = [None] * world
    await _in_thread(dist.all_gather_object, gathered, {
        "lat": [(ready_at[nm] - t0) * 1e3 for nm in names if nm in ready_at], "create": create_ms,
        "all_ready": all_ready, "ok": ok and gone, "cpu": cpu, "adm": adm, "teardown": teardown, "k": k,
        "wh": wh, "wh_get": wh_get, "prof": prof, "gc": gcp, "errors": errors, "cgroup": cgroup})
    if rank != 0:
        return None
    lat = [x for g in gathered for x in g["lat"]]
    span = max((g["all_ready"] or 0.0) for g in gathered)
    cpu_all: dict = {}
    for g in gathered:
        for kk, v in g["cpu"].items():
            cpu_all[kk] = cpu_all.get(kk, 0.0) + v
    adm_ms = [u / 1e3 for g in gathered for u in g["adm"]]
    return {
        "notebooks": total, "per_rank": [g["k"] for g in gathered], "all_ok": all(g["ok"] for g in gathered),
        "notebook": ("one amd.com/gpu each (one per MI355X of the node)" if gpus else
                     "CPU workbench, requests 500m / 1Gi (kf/loadtest/jupyter_test.yaml)")
                    + (", inject-auth" if use_odh else ""),
        "all_ready_s": round(span, 4), "notebooks_per_s": round(total / span, 2) if span else None,
        "ready_ms": _pcts(lat), "create_ms": _pcts([x for g in gathered for x in g["create"]]),
        "admission_ms": {**_pcts(adm_ms), "n": len(adm_ms)},
        # inside the webhook process: request decoded → response encoded (the rest of
        # admission_ms is the apiserver's call: connection, TLS, queueing for the event loop)
        "webhook_handle_ms": {**_pcts([x for g in gathered for x in g["wh"]]),
                              "n": sum(len(g["wh"]) for g in gathered)},
        # the webhook process's live reads (ConfigMaps it must confirm, as the reference reads them)
        "webhook_get_ms": {**_pcts([x for g in gathered for x in g["wh_get"]]),
                           "n": sum(len(g["wh_get"]) for g in gathered)},
        "cpu_ms_per_notebook": {kk: round(v * 1e3 / max(1, total), 3) for kk, v in sorted(cpu_all.items())},
        "teardown_s": round(max(g["teardown"] for g in gathered), 4),
        "gc_pause_ms": {proc: {"n": len(ps), "max": max(x[1] for x in ps),
                               "gen2": sum(1 for x in ps if x[0] == 2)}
                        for g in gathered for proc, ps in sorted(g["gc"].items()) if ps},
        **({"errors": [e for g in gathered for e in g["errors"]]} if any(g["errors"] for g in gathered) else {}),
        # the box's CPU share from the first create to this rank's last Ready (rank 0's view;
        # one container): a throttled period stalls every process at once
        "cgroup_cpu": gathered[0]["cgroup"],
        "apiserver": {k: v for k, v in (gathered[0]["prof"] or {}).items()
                      if k in ("lock_wait_ms", "lock_contended", "lock_wait_by_resource", "trim_ms", "trims",
                               "admit_wall_ms", "webhook_dials", "webhook_dial_ms", "watch_gone")},
    }


async def _resident(args, shard, dist, native, children: dict, use_odh: bool,
                    empty_p50_ms: Optional[float]) -> Optional[dict]:
    """A steady state with a population: the reference's load tool applies N
    notebooks and leaves them running (``kf/loadtest/start_notebooks.py:76-95``), and its culler
    rewrites every Notebook's ``last_activity_check_timestamp`` once per check period
    (``kf/controllers/culling_controller.go:171-196``).  ``--resident R`` notebooks (split over the
    ranks, CPU workbenches whose Jupyter servers report an idle kernel, the odh auth/route path
    like the timed ones) are created and left Ready with the culler checking each every
    ``--culling-period`` s; then

    * **at rest** (``--resident-window`` s, nothing else happening): each process's CPU per
      second, culler checks / heartbeat writes / admissions per second, reconciles per second
      by controller and trigger (the kf and odh reconciles triggered by Notebook events must be
      0: the heartbeat passes neither's predicate), watch events per second, RSS;
    * **on top** (``--resident-steps`` per rank): new notebooks' create→Ready, closed loop like
      the timed window, against the window's empty-cluster p50.

    Untimed; failures are reported in the block, never raised (every rank reaches every
    collective)."""
    from bench import breakdown_delta  # noqa: E402  (bench.py is the entry point)

    from ..models import kinds
    from ..models.notebook import LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, notebook

    rank, world = dist.get_rank(), dist.get_world_size()
    total = int(args.resident)
    k = total // world + (1 if rank < total % world else 0)
    nss = shard.cfg.user_namespaces
    names = [f"res-{rank}-{i}" for i in range(k)]
    ns_of = {nm: nss[i % len(nss)] for i, nm in enumerate(names)}
    ann = {"notebooks.opendatahub.io/inject-auth": "true"} if use_odh else None
    errors: list = []

    async def safe(aw, default=None):
        try:
            return await aw
        except Exception as e:  # noqa: BLE001 — recorded in the block
            errors.append(f"rank {rank}: {e!r}"[:300])
            return default

    sem = asyncio.Semaphore(32)

    async def create(nm):
        nb = notebook(nm, ns_of[nm], image=NOTEBOOK_IMAGE, annotations=ann)
        c = nb["spec"]["template"]["spec"]["containers"][0]
        # small requests: R of them must fit the one node (256 cores) next to the timed GPU pods
        c.setdefault("resources", {}).setdefault("requests", {}).update({"cpu": "50m", "memory": "256Mi"})
        async with sem:
            await shard.admin.create(nb)

    # the resident notebooks are not labelled driven: the driver's own cache never sees their
    # heartbeats; this cache follows them while they fill (and again while they go)
    from ..runtime.informer import InformerCache
    from .shard import notebook_is_ready

    async def watching():
        c = InformerCache(shard.rest, namespaces=nss)
        for kk in (kinds.NOTEBOOK, kinds.POD):
            await c.ensure_informer(kk)
        return c

    async def poll_until(pred, timeout: float) -> bool:
        deadline = time.monotonic() + timeout
        while not pred():
            if time.monotonic() > deadline:
                return False
            await asyncio.sleep(0.02)
        return True

    def all_ready(c) -> bool:
        return all(notebook_is_ready(c.get(kinds.NOTEBOOK, nm, ns_of[nm])) for nm in names)

    def all_checked(c) -> bool:  # the culler has initialised every resident notebook's annotations
        for nm in names:
            nb = c.get(kinds.NOTEBOOK, nm, ns_of[nm])
            if nb is None or LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION not in ((nb.get("metadata") or {})
                                                                             .get("annotations") or {}):
                return False
        return True

    await safe(shard.quiesce())
    fill = await safe(watching())
    await _in_thread(dist.barrier)
    t0 = time.perf_counter()
    await safe(asyncio.gather(*(create(nm) for nm in names)))
    ok = fill is not None and bool(await safe(poll_until(lambda: all_ready(fill), 300), False))
    fill_s = time.perf_counter() - t0
    ok = ok and bool(await safe(poll_until(lambda: all_checked(fill), 120), False))
    if fill is not None:
        await safe(fill.stop())
    await asyncio.sleep(2 * getattr(args, "culling_period", 1.0))  # every notebook's checks under way
    await _in_thread(dist.barrier)

    # ---- at rest
    prof0 = await safe(_apiserver_prof(native))
    cpu0 = _cpu_snapshot(children, prof0)
    b0 = await safe(shard.reconcile_breakdown(include_all=True), {})
    io0 = await safe(shard.io_counters(), {})
    adm0 = (await safe(native.admissions(1 << 62), {})).get("seq") if native is not None else None
    wh0 = await safe(shard.webhook_timings(), {}) if shard.cfg.launch else {}
    r0 = time.perf_counter()
    await asyncio.sleep(max(0.5, getattr(args, "resident_window", 3.0)))
    prof1 = await safe(_apiserver_prof(native))
    cpu1 = _cpu_snapshot(children, prof1)
    win = time.perf_counter() - r0
    b1 = await safe(shard.reconcile_breakdown(include_all=True), {})
    io1 = await safe(shard.io_counters(), {})
    adm1 = (await safe(native.admissions(1 << 62), {})).get("seq") if native is not None else None
    wh1 = await safe(shard.webhook_timings(), {}) if shard.cfg.launch else {}
    rss = {kk: _proc_rss_mib(pid) for kk, pid in children.items()}
    cpu = {kk: (cpu1.get(kk) or 0.0) - (cpu0.get(kk) or 0.0) for kk in children if cpu0.get(kk) is not None}
    rest_prof = _prof_per_step(prof0, prof1, 1) if prof0 and prof1 else None
    heartbeats = sum((d.get("heartbeats") or 0) - ((wh0.get(p) or {}).get("heartbeats") or 0)
                     for p, d in (wh1 or {}).items())
    heartbeats_full = sum((d.get("heartbeats_full") or 0) - ((wh0.get(p) or {}).get("heartbeats_full") or 0)
                          for p, d in (wh1 or {}).items())
    served = sum((d.get("served") or 0) - ((wh0.get(p) or {}).get("served") or 0) for p, d in (wh1 or {}).items())
    await _in_thread(dist.barrier)

    # ---- new notebooks on top of the population
    lat = []
    base = dict(ann or {})
    # untimed warm-up lifecycles first, as the empty-cluster window has (--warmup): after the
    # rest window every process has been idle (or only checking), and the first lifecycles of a
    # cold box run slower whatever the population
    for i in range(max(0, int(getattr(args, "resident_warmup", 10)))):
        if await safe(_lifecycle(shard, f"nb-rew-{i}", dict(base) or None, ns=nss[i % len(nss)])) is None:
            break
    await safe(shard.quiesce(timers=0.05))
    gc0 = {k: v["seq"] for k, v in ((await safe(shard.gc_pauses(), {})) or {}).items()} if shard.procs else {}
    top0 = await safe(shard.io_counters(), {})
    top_t0 = time.perf_counter()
    for i in range(max(0, int(getattr(args, "resident_steps", 20)))):
        r = await safe(_lifecycle(shard, f"nb-res-{i}", dict(base) or None, ns=nss[i % len(nss)]))
        if r is None:
            break
        lat.append(r[0] * 1e3)
    # the control-plane processes' cyclic-GC pauses meanwhile (their event loops stop): with R
    # notebooks in their caches a generation-2 pass walks all of them
    gcp = {k: [x[1:] for x in v["pauses"]] for k, v in ((await safe(shard.gc_pauses(gc0), {})) or {}).items()} \
        if shard.procs else {}
    await safe(shard.quiesce())
    top_io = io_delta(top0 or {}, await safe(shard.io_counters(), {}) or {})
    # the population's own traffic (heartbeats) goes on meanwhile: the at-rest rate times this
    # span is subtracted for the net per-notebook figure
    top_dt = time.perf_counter() - top_t0
    top_io_net = io_minus(top_io, io_delta(io0 or {}, io1 or {}), top_dt / max(win, 1e-9))
    await _in_thread(dist.barrier)

    # ---- teardown
    t_del = time.perf_counter()

    async def delete(nm):
        async with sem:
            await shard.admin.delete(kinds.NOTEBOOK, nm, ns_of[nm])
    gonec = await safe(watching())
    await safe(asyncio.gather(*(delete(nm) for nm in names), return_exceptions=True))
    gone = gonec is not None and bool(await safe(poll_until(lambda: all(
        gonec.get(kinds.NOTEBOOK, nm, ns_of[nm]) is None and gonec.get(kinds.POD, f"{nm}-0", ns_of[nm]) is None
        for nm in names), 300), False))
    teardown = time.perf_counter() - t_del
    if gonec is not None:
        await safe(gonec.stop())
    gathered = [None] * world
    await _in_thread(dist.all_gather_object, gathered, {
        "k": k, "ok": ok and gone, "fill_s": fill_s, "win": win, "cpu": cpu, "rss": rss, "lat": lat,
        "in_window": breakdown_delta(b0 or {}, b1 or {}), "io": io_delta(io0 or {}, io1 or {}), "prof": rest_prof,
        "adm": (adm1 - adm0) if adm0 is not None and adm1 is not None else None, "heartbeats": heartbeats,
        "heartbeats_full": heartbeats_full,
        "served": served, "teardown": teardown, "errors": errors, "gc": gcp, "top_io": top_io,
        "top_io_net": top_io_net})
    if rank != 0:
        return None
    win = max(g["win"] for g in gathered)
    per_s = 1.0 / win
    cpu_all: dict = {}
    for g in gathered:
        for kk, v in g["cpu"].items():
            cpu_all[kk] = cpu_all.get(kk, 0.0) + v
    recon: dict = {}
    for g in gathered:
        for ctrl, trig in g["in_window"].items():
            o = recon.setdefault(ctrl, {})
            for kk, v in trig.items():
                o[kk] = o.get(kk, 0) + v
    io = io_per_notebook([g["io"] for g in gathered], 1)
    for proc, d in io.items():  # per second of the window, not per notebook
        for sect in ("watch_events", "requests"):
            if sect in d:
                d[sect] = {kk: round(v * per_s, 1) for kk, v in d[sect].items()}
    prof = gathered[0]["prof"] or {}
    writes = {v: round(prof.get(f"{v}_calls", 0.0) * per_s, 1) for v in ("create", "update", "patch", "delete")}
    culler = recon.get("Culler", {})
    lat = [x for g in gathered for x in g["lat"]]
    p50 = _pcts(lat).get("p50")
    adm = gathered[0]["adm"]
    return {
        "notebooks": total, "per_rank": [g["k"] for g in gathered], "all_ok": all(g["ok"] for g in gathered),
        "notebook": "CPU workbench (50m / 256Mi) with an idle Jupyter kernel" + (", inject-auth" if use_odh else ""),
        "culling": {"period_s": getattr(args, "culling_period", 1.0), "source": "combined (Jupyter via the DEV "
                    "kubectl-proxy stand-in; no node-agent CA, so no GPU samples)"},
        "fill_s": round(max(g["fill_s"] for g in gathered), 3),
        "at_rest": {
            "window_s": round(win, 3),
            "cpu_ms_per_s": {kk: round(v * 1e3 * per_s, 2) for kk, v in sorted(cpu_all.items())},
            "culler_checks_per_s": round(sum(culler.values()) * per_s, 1),
            "apiserver_writes_per_s": writes,
            "admissions_per_s": round(adm * per_s, 1) if adm is not None else None,
            "webhook_heartbeat_fast_path_per_s": round(sum(g["heartbeats"] for g in gathered) * per_s, 1),
            # heartbeats that ran the pipeline: an input changed since the notebook's last full
            # admission (or this webhook had not admitted it yet) — 0 at rest
            "webhook_heartbeat_full_pipeline_per_s": round(sum(g["heartbeats_full"] for g in gathered) * per_s, 1),
            "webhook_admissions_per_s": round(sum(g["served"] for g in gathered) * per_s, 1),
            "reconciles_per_s": {ctrl: {"total": round(sum(t.values()) * per_s, 1),
                                        "by_trigger": {kk: round(v * per_s, 1) for kk, v in sorted(t.items())}}
                                 for ctrl, t in sorted(recon.items())},
            "notebook_triggered_reconciles_kf_odh": sum(
                t.get("Notebook", 0) for ctrl, t in recon.items()
                if ctrl in ("notebook-controller", "odh-notebook-controller")),
            "io_per_s": io,
            "rss_mib": {kk: v for g in gathered for kk, v in sorted(g["rss"].items()) if v is not None},
        },
        "new_notebooks_on_top": {"steps_per_rank": int(getattr(args, "resident_steps", 20)),
                                 "warmup_per_rank": int(getattr(args, "resident_warmup", 10)), "ready_ms": _pcts(lat),
                                 "empty_cluster_p50_ms": round(empty_p50_ms, 3) if empty_p50_ms else None,
                                 "p50_vs_empty": round(p50 / empty_p50_ms, 3) if p50 and empty_p50_ms else None,
                                 # per on-top notebook, to compare with the window's io_per_notebook:
                                 # what an R-sized cache costs each lifecycle (cache_scans: objects
                                 # list() examined that no index narrowed)
                                 "io_per_notebook": io_per_notebook([g["top_io"] for g in gathered],
                                                                    max(1, len(lat))),
                                 # the same, less the at-rest traffic of the span it was counted over
                                 "io_per_notebook_net_of_rest": io_per_notebook(
                                     [g["top_io_net"] for g in gathered], max(1, len(lat))),
                                 "gc_pause_ms": {proc: {"n": len(ps), "max": max(x[1] for x in ps),
                                                        "gen2": sum(1 for x in ps if x[0] == 2)}
                                                 for g in gathered for proc, ps in sorted(g["gc"].items()) if ps}},
        "teardown_s": round(max(g["teardown"] for g in gathered), 3),
        **({"errors": [e for g in gathered for e in g["errors"]]} if any(g["errors"] for g in gathered) else {}),
    }


def io_delta(a: dict, b: dict) -> dict:
    """Per process: watch events per kind, requests per verb and lists per kind (a list in the
    window is a relist: a watch answered 410 Gone) between two snapshots."""
    out = {}
    for proc, cur in b.items():
        prev = a.get(proc) or {}
        d = {}
        for sect in ("watch_events", "requests", "lists", "cache_scans"):
            p0 = prev.get(sect) or {}
            dd = {k: v - p0.get(k, 0) for k, v in (cur.get(sect) or {}).items()}
            d[sect] = {k: v for k, v in dd.items() if v}
        out[proc] = d
    return out


def io_minus(a: dict, rest: dict, f: float) -> dict:
    """``a`` less ``f`` times ``rest`` (both :func:`io_delta` results), never below 0."""
    out = {}
    for proc, d in a.items():
        r = rest.get(proc) or {}
        out[proc] = {sect: {k: v for k, v in ((k, max(0.0, v - f * (r.get(sect) or {}).get(k, 0)))
                                              for k, v in kv.items()) if v > 1e-9}
                     for sect, kv in d.items()}
    return out


def io_per_notebook(parts: list, notebooks: int) -> dict:
    """Merge the ranks' :func:`io_delta` and divide by the notebooks of the timed window (the
    deltas run to the settled point, so a lifecycle's trailing events are in)."""
    n = max(1, notebooks)
    out: dict = {}
    for part in parts:
        for proc, d in (part or {}).items():
            o = out.setdefault(proc, {})
            for sect, kv in d.items():
                s = o.setdefault(sect, {})
                for k, v in kv.items():
                    s[k] = s.get(k, 0) + v
    for proc, o in out.items():
        for sect, kv in list(o.items()):
            tot = sum(kv.values())
            if sect == "lists":  # rare: counted, not divided
                if tot:
                    o["relists_in_window"] = dict(kv, total=tot)
                del o[sect]
                continue
            o[sect] = {k: round(v / n, 2) for k, v in sorted(kv.items(), key=lambda x: -x[1])}
            o[sect]["total"] = round(tot / n, 2)
    return out


def _proc_cpu_s(pid: Optional[int]) -> Optional[float]:
    """CPU seconds of a child process, summed over its threads to the nanosecond
    (:func:`~odh_kubeflow_amd.utils.procutil.proc_cpu_ns`), None if unreadable."""
    from ..utils.procutil import proc_cpu_ns

    ns = proc_cpu_ns(pid)
    return None if ns is None else ns / 1e9


def _cpu_snapshot(children: dict, prof: Optional[dict]) -> dict:
    """CPU seconds of every child process; the native apiserver's from its own
    ``CLOCK_PROCESS_CPUTIME_ID`` (``process_cpu_ns`` of its profile), which keeps the time of
    connection threads that have exited (it runs one thread per connection)."""
    out = {k: _proc_cpu_s(pid) for k, pid in children.items()}
    if prof and prof.get("process_cpu_ns") is not None and "apiserver" in out:
        out["apiserver"] = prof["process_cpu_ns"] / 1e9
    return out


def _proc_rss_mib(pid: Optional[int]) -> Optional[float]:
    """Resident set size of a child process (``/proc/<pid>/status`` VmRSS), None if unreadable."""
    if pid is None:
        return None
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return round(int(line.split()[1]) / 1024.0, 1)
    except (OSError, IndexError, ValueError):
        return None
    return None


def _cpulist(text: str) -> set:
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def numa_bind(local_rank: int, sysfs: str = "/sys") -> Optional[dict]:
    """Pin this rank — and the processes it starts after this (its control plane, on rank 0
    the apiserver and the node platform) — to the physical cores of its MI355X's NUMA node.

    An 8×MI355X node is two sockets; left alone, the scheduler spreads a rank's processes
    over both, and every watch event, admission and REST call between them crosses the
    socket interconnect (measured on the one-GPU box: the slower of two ranks burnt 30–50 %
    more CPU per notebook than the other).  One SMT thread per core keeps siblings from
    competing.  ``ODH_BENCH_NUMA_BIND=0`` turns it off; any failure leaves placement alone."""
    if os.environ.get("ODH_BENCH_NUMA_BIND", "1") == "0":
        return None
    try:
        from ..ops.telemetry import Telemetry

        devs = Telemetry(sysfs).devices()
        bdf = devs[local_rank].pci_bdf
        with open(f"{sysfs}/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
        if node < 0:
            return None
        with open(f"{sysfs}/devices/system/node/node{node}/cpulist") as f:
            cpus = _cpulist(f.read())
        phys = set()
        for c in cpus:
            try:
                with open(f"{sysfs}/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                    if min(_cpulist(f.read())) == c:
                        phys.add(c)
            except OSError:
                phys.add(c)
        target = phys & os.sched_getaffinity(0)
        if len(target) < 4:
            return None
        os.sched_setaffinity(0, target)
        return {"gpu": bdf, "numa_node": node, "cores": len(target)}
    except Exception:  # noqa: BLE001 — no telemetry / sysfs: leave placement to the OS
        return None


async def _main(args, dist, torch, rank: int, world: int, ndev: int, probe_sample: int) -> dict:
    from .platform import NodePlatform
    from .shard import ControlPlaneShard, ShardConfig

    native = None
    platform = None
    url = [None, None]  # the apiserver; the culler's DEV-mode kubectl proxy (Jupyter stand-in)
    culling = culling_enabled(args)
    arch = args.arch if args.arch in ("sharded", "unsharded") else "sharded"
    if rank == 0:
        from ..testing.apiserver.native import NativeApiServer
        from ..testing.cluster import OPENSHIFT_CRDS

        audit = os.environ.get("DEBUG_WRITE_AUDITLOG")  # same debug aid as the test cluster
        pol = None
        if audit:
            from ..testing.apiserver.audit import AuditPolicy

            lv = os.environ.get("DEBUG_AUDIT_LEVEL", "Metadata")  # Request / RequestResponse: with bodies
            pol = AuditPolicy([{"level": lv}])  # every request: what each process sends
        openshift = getattr(args, "openshift_pull_secret_ms", -1.0) >= 0
        # vanilla Kubernetes (+ Gateway API): the OpenShift APIs are not served; OpenShift-like:
        # they are, and every ServiceAccount gets its dockercfg pull secret after D ms
        native = await NativeApiServer(() if openshift else OPENSHIFT_CRDS, gc=True, audit_log_path=audit,
                                       audit_policy=pol,
                                       write_latency_ms=getattr(args, "write_latency_ms", 0.0)).start()
        url[0] = native.url
        # the node's StatefulSet controller and kubelet: one worker process of each per two ranks
        platform = await NodePlatform(native.url, exec_init=probe_sample > 0, hip_devices=ndev,
                                      workers=getattr(args, "platform_workers", 0) or (world + 1) // 2,
                                      pull_secret_delay_ms=getattr(args, "openshift_pull_secret_ms", -1.0),
                                      jupyter_proxy=culling).start()
        url[1] = platform.jupyter_proxy_url
    await _in_thread(dist.broadcast_object_list, url, 0)
    env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
    if culling:
        env.update(culler_env(args, url[1]))
    per_rank = max(1, getattr(args, "namespaces_per_rank", 1))
    nss = bench_namespaces(rank, per_rank)
    shard = ControlPlaneShard(ShardConfig(
        apiserver_url=url[0], namespace=nss[0], namespaces=nss, assign=(arch == "sharded" and per_rank > 1),
        shard_count=world, assign_policy=getattr(args, "assign_policy", "hash"), shard=str(rank), arch=arch,
        launch=(arch == "sharded" or rank == 0), bootstrap=(rank == 0), odh=not args.no_odh,
        webhook=not args.no_odh, reference_emulation=args.reference_emulation, env=env, process=True,
        split=not getattr(args, "single_process_shard", False), workers=max(1, getattr(args, "workers", 1)),
        webhook_replicas=max(1, getattr(args, "webhook_replicas", 1)),
        kf_split_workers=bool(getattr(args, "kf_split_workers", False)),
        webhook_process=not getattr(args, "webhook_in_odh", False),
        cache_configmaps=getattr(args, "cache_configmaps", False), driven_only=True,
        culler_process=culling and not getattr(args, "culler_in_kf", False),
        cluster_watch=getattr(args, "cluster_wide_watches", False)))
    if rank == 0:
        await shard.start()  # cluster namespaces (and, unsharded, the managers + their webhook) first
        await _in_thread(dist.barrier)
    else:
        await _in_thread(dist.barrier)
        await shard.start()
    await _in_thread(dist.barrier)  # every control plane and webhook is registered before anyone creates
    if shard.cfg.assign:  # every shard's assigner is up: wait until it labelled this rank's namespaces
        labels = await shard.wait_assigned(60.0)
        if len(labels) != len(nss):
            raise RuntimeError(f"rank {rank}: namespaces not assigned to a shard: "
                               f"{sorted(set(nss) - set(labels))}")
        shard.labels = labels
        await _in_thread(dist.barrier)

    try:
        children = {"apiserver": native.proc.pid if native else None}
        if platform is not None:
            children.update(platform.pids())
        children.update(shard.control_plane_pids())
        result = await _drive(args, shard, dist, torch, children, native, probe_sample)
    finally:
        await _in_thread(dist.barrier)  # nobody tears down while others still serve
        await shard.stop()
        if platform is not None:
            await platform.stop()
        if native is not None:
            await native.stop()
    return result


async def _apiserver_prof(native) -> Optional[dict]:
    """The native apiserver's profile counters, with each resource's store-lock contention
    flattened in as ``lock_wait_ns@<resource>`` / ``lock_contended@<resource>``."""
    if native is None:
        return None
    try:
        st = await native.stats()
    except Exception:
        return None
    out = dict(st.get("prof") or {})
    out.pop("trim_max_ns", None)  # a running max, not a counter
    for k, v in (st.get("phases") or {}).items():  # write-path CPU by phase
        out[f"phase_{k}"] = v
    for res, v in (st.get("locks") or {}).items():
        out[f"lock_wait_ns@{res}"] = v.get("wait_ns", 0)
        out[f"lock_contended@{res}"] = v.get("contended", 0)
    return out


def _prof_per_step(p0: Optional[dict], p1: Optional[dict], steps: int) -> Optional[dict]:
    """Native apiserver profile delta over the timed region, per step (ms / counts)."""
    if not p0 or not p1:
        return None
    out, by_res = {}, {}
    for k, v in p1.items():
        d = (v - p0.get(k, 0)) / max(1, steps)
        if "@" in k:  # per resource: only the ones that waited in the window
            name, res = k.split("@", 1)
            if d:
                by_res.setdefault(res, {})["wait_ms" if name.startswith("lock_wait") else "contended"] = \
                    round(d / 1e6, 3) if name.endswith("_ns") else round(d, 2)
            continue
        out[k[:-3] + "_ms" if k.endswith("_ns") else k] = round(d / 1e6, 3) if k.endswith("_ns") else round(d, 2)
    if by_res:
        out["lock_wait_by_resource"] = dict(sorted(by_res.items(), key=lambda kv: -kv[1].get("wait_ms", 0)))
    return out


async def _lifecycle(shard, nm: str, ann: Optional[dict], timeout: float = 120.0,
                     ns: Optional[str] = None) -> tuple:
    """create → Ready → delete → gone in ``ns`` (default: the rank's first namespace);
    returns (create→Ready s, Ready→gone s, the pod)."""
    from ..models import kinds
    from ..models.notebook import notebook

    ns = ns or shard.cfg.namespace
    t0 = time.perf_counter()
    await shard.admin.create(driven(notebook(nm, ns, image=NOTEBOOK_IMAGE, gpus=1, annotations=ann)))
    if not await shard.wait_until(lambda: shard.notebook_ready(nm, ns), timeout):
        raise RuntimeError(f"notebook {ns}/{nm} not Ready")
    ready = time.perf_counter()
    pod = shard.peek(kinds.POD, f"{nm}-0", ns)
    await shard.admin.delete(kinds.NOTEBOOK, nm, ns)
    if not await shard.wait_until(lambda: shard.gone(nm, ns), 60):
        raise RuntimeError(f"teardown of {ns}/{nm} did not finish")
    return ready - t0, time.perf_counter() - ready, pod


async def _storage_block(args, shard, dist, native, base_ann: dict) -> Optional[dict]:
    """``--storage-steps`` closed-loop lifecycles per rank (create → Ready → delete → gone, as in
    the timed window) while the apiserver holds every write ``--storage-ms`` before it commits,
    as an etcd quorum write does (typically 1-5 ms on SSD-backed etcd; kube-apiserver adds
    its own).  Reported next to the headline, never in it: notebooks/s, create→Ready
    percentiles and reconciles/s of the window.  Rank 0 owns the apiserver and sets the
    latency; every rank reaches every collective (failures are reported)."""
    from bench import breakdown_delta, merge_breakdowns  # noqa: E402  (bench.py is the entry point)

    ms = float(args.storage_ms)
    errors: list = []
    lat: list = []
    if native is not None:
        try:
            await native.set_write_latency(ms)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e)[:300])
    await _in_thread(dist.barrier)
    nss = shard.cfg.user_namespaces
    el = 0.0
    in_window: dict = {}
    try:
        await shard.quiesce(timers=0.05)
        await _in_thread(dist.barrier)
        b0 = await shard.reconcile_breakdown()
        t0 = time.perf_counter()
        for i in range(int(args.storage_steps)):
            r, _gone, _pod = await _lifecycle(shard, f"nb-st{i}", dict(base_ann) or None, ns=nss[i % len(nss)])
            lat.append(r * 1e3)
        el = time.perf_counter() - t0
        b1 = await shard.reconcile_breakdown() if shard.cfg.arch == "sharded" else None
        await _in_thread(dist.barrier)
        if b1 is None:
            b1 = await shard.reconcile_breakdown() if shard.procs or shard.managers else {}
        in_window = breakdown_delta(b0, b1)
    except Exception as e:  # noqa: BLE001 — reported in the block
        errors.append(f"rank {dist.get_rank()}: {e!r}"[:300])
        await _in_thread(dist.barrier)
    finally:
        if native is not None:
            try:
                await native.set_write_latency(0.0)
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e)[:300])
    gathered = [None] * dist.get_world_size()
    await _in_thread(dist.all_gather_object, gathered, {"lat": lat, "el": el, "win": in_window, "errors": errors})
    if dist.get_rank() != 0:
        return None
    win = max(g["el"] for g in gathered) or None
    lat_all = [x for g in gathered for x in g["lat"]]
    recon = merge_breakdowns(g["win"] for g in gathered)
    n_recon = sum(sum(t.values()) for t in recon.values())
    out = {"storage_write_latency_ms": ms, "steps_per_rank": int(args.storage_steps),
           "notebooks_ready_per_s": round(len(lat_all) / win, 3) if win else None,
           "ready_ms": _pcts(lat_all), "reconciles_per_s": round(n_recon / win, 1) if win else None,
           "reconciles_per_notebook": round(n_recon / max(1, len(lat_all)), 2)}
    errs = [e for g in gathered for e in g["errors"]]
    if errs:
        out["errors"] = errs
    return out


async def _drive(args, shard, dist, torch, children: Optional[dict] = None, native=None,
                 probe_sample: int = 0) -> dict:
    from ..ops.probe_main import parse_result

    use_odh = not args.no_odh
    base_ann = {"notebooks.opendatahub.io/inject-auth": "true"} if use_odh else {}
    lat_ms, teardown_ms = [], []
    state = {"step": 0}
    nss = shard.cfg.user_namespaces
    ns_counts = {ns: 0 for ns in nss}  # timed notebooks per namespace

    async def one_step(timed: bool):
        state["step"] += 1
        ns = nss[state["step"] % len(nss)]
        ready_s, gone_s, _pod = await _lifecycle(shard, f"nb-s{state['step']}", dict(base_ann) or None, ns=ns)
        if timed:
            lat_ms.append(ready_s * 1e3)
            teardown_ms.append(gone_s * 1e3)
            ns_counts[ns] += 1

    from ..utils import gctune

    # the driver process's collector pause (a full collection walks torch's ~1M objects,
    # tens of ms) goes before the warm-up: between warm-up and timed steps it left every
    # control-plane process idle long enough to start the timed window cold
    gctune.tune()
    for _ in range(args.warmup):
        await one_step(False)
    await _in_thread(dist.barrier)  # every rank's warm-up done (unsharded: one control plane for all)
    # the warm-up's trailing work, not the culler's next check of each warm-up notebook: that
    # timer is a check period away (1 s), and waiting for it left every process idle for a
    # second before the window — long enough for the host to start the window cold
    await shard.quiesce(timers=0.05)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    await _in_thread(dist.barrier)
    b0 = await shard.reconcile_breakdown()
    io0 = await shard.io_counters()
    children = children or {}
    prof0 = await _apiserver_prof(native)
    child_cpu0 = _cpu_snapshot(children, prof0)
    cpu0 = time.process_time()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        await one_step(True)
    own = time.perf_counter() - t_start  # this rank's own steps
    from bench import breakdown_delta, merge_breakdowns  # noqa: E402  (bench.py is the entry point)

    # a sharded rank's control plane serves only its own steps, all done now: its in-window
    # count is read before the end barrier, so no reconcile that finishes after the window
    # is counted in it; the unsharded control plane serves every rank, so it is read after
    # the barrier, and the time that read takes is reported (``recon_snapshot_lag_ms``)
    own_cp = shard.cfg.arch == "sharded"
    b1 = await shard.reconcile_breakdown() if own_cp else None
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    await _in_thread(dist.barrier)
    elapsed = time.perf_counter() - t_start  # ---- end of the timed region
    if b1 is None:
        b1 = await shard.reconcile_breakdown() if shard.procs or shard.managers else {}
    snap_lag = time.perf_counter() - t_start - elapsed
    in_window = breakdown_delta(b0, b1)
    cpu = {"rank": time.process_time() - cpu0}
    prof1 = await _apiserver_prof(native)
    prof = _prof_per_step(prof0, prof1, args.steps)
    child_cpu1 = _cpu_snapshot(children, prof1)
    rss = {}
    for k, pid in children.items():
        c1 = child_cpu1.get(k)
        if c1 is not None and child_cpu0.get(k) is not None:
            cpu[k] = c1 - child_cpu0[k]
        r = _proc_rss_mib(pid)
        if r is not None:
            rss[k] = r
    # untimed: the trailing reconciles of the last deletion, for the per-lifecycle count
    await _in_thread(dist.barrier)
    idle = await shard.quiesce()
    settled = breakdown_delta(b0, await shard.reconcile_breakdown())
    io = io_delta(io0, await shard.io_counters())
    # who served which namespace: the shard labels (sharded, assigned) or the supervisors'
    # worker assignment (unsharded --workers; rank 0 launched the managers)
    owner = dict(shard.labels)
    if not owner and shard.cfg.arch != "sharded" and shard.cfg.launch and shard.cfg.workers > 1:
        for _proc, a in (await shard.worker_assignments()).items():
            for idx, names in a.items():
                for ns in names:
                    owner.setdefault(ns, f"worker_{idx}")
    samples = []
    for i in range(probe_sample):  # untimed: notebooks with the start-up probe init container
        # spaced: the previous probe's kernel-side GPU teardown (~0.1 s after its exit) would
        # hold this one's HIP init, which a notebook starting on an idle GPU never waits for
        await asyncio.sleep(max(0.0, getattr(args, "probe_gap_s", 0.5)))
        ann = {**base_ann, GPU_PROBE_ANNOTATION: "true"}
        try:
            ready_s, _gone, pod = await _lifecycle(shard, f"nb-probe-{i}", ann, timeout=180)
        except Exception as e:  # noqa: BLE001 — reported with the sample, the headline stands
            samples.append({"ready_ms": None, "result": {"ok": False, "error": repr(e)[:300]}})
            break
        st = ((pod or {}).get("status") or {}).get("initContainerStatuses") or [{}]
        term = (st[0].get("state") or {}).get("terminated") or {}
        result = parse_result(term.get("message", ""))
        samples.append({"ready_ms": ready_s * 1e3, "result": result, "exit_code": term.get("exitCode"),
                        "wall_ms": (result or {}).get("timings_ms", {}).get("total")})

    burst = None
    if getattr(args, "burst", 0) > 0:  # untimed: open-loop capacity of the same control plane
        rounds = []
        for r in range(max(1, getattr(args, "burst_rounds", 1))):
            t_wall = time.time()  # the audit log's and the stall watchdogs' clock
            b = await _burst(args, shard, dist, native, children, use_odh, tag=f"r{r}")
            if b is not None:
                b["started_at"] = round(t_wall, 6)
            rounds.append(b)
        burst = rounds[-1]
        if burst is not None and len(rounds) > 1:
            # the earlier rounds warm what a running cluster has warm (the apiserver's
            # connections to the webhook, the informers' namespaces); the last one is reported
            burst["rounds"] = [{k: b.get(k) for k in ("all_ready_s", "notebooks_per_s", "started_at")} |
                               {"admission_p99_ms": b["admission_ms"]["p99"],
                                "webhook_handle_p99_ms": b["webhook_handle_ms"]["p99"],
                                "webhook_dials": (b.get("apiserver") or {}).get("webhook_dials"),
                                "webhook_dial_ms": (b.get("apiserver") or {}).get("webhook_dial_ms"),
                                "cgroup_throttled_periods": (b.get("cgroup_cpu") or {}).get("throttled_periods")}
                               for b in rounds]

    resident = None
    if getattr(args, "resident", 0) > 0 and culling_enabled(args):
        # untimed: a resident population with the culler checking it
        resident = await _resident(args, shard, dist, native, children, use_odh,
                                   statistics.median(lat_ms) if lat_ms else None)

    storage = None
    if getattr(args, "storage_steps", 0) > 0 and getattr(args, "storage_ms", 0) > 0:
        # untimed: the same closed loop with every apiserver write paying an etcd-like storage
        # round trip — the headline's store answers writes in microseconds
        storage = await _storage_block(args, shard, dist, native, base_ann)

    el = torch.tensor([elapsed], dtype=torch.float64)
    await _in_thread(lambda: dist.all_reduce(el, op=dist.ReduceOp.MAX))
    gathered = [None] * dist.get_world_size()
    # this rank's lifecycle time (create → Ready → gone) per block of 20 timed steps: whether
    # the first steps of the window run slower than the rest (warm-up of the host, not the code)
    life = [a + b for a, b in zip(lat_ms, teardown_ms)]
    blocks = [round(statistics.fmean(life[i:i + 20]), 3) for i in range(0, len(life), 20)]
    trace = os.environ.get("ODH_BENCH_STEP_TRACE")  # debug aid: every timed step's two halves
    if trace:
        with open(f"{trace}.{dist.get_rank()}.json", "w") as f:
            json.dump({"create_to_ready_ms": lat_ms, "ready_to_gone_ms": teardown_ms}, f)
    await _in_thread(dist.all_gather_object, gathered, {"lat": lat_ms, "teardown": teardown_ms, "own_s": own,
                                                        "blocks": blocks,
                                                        "cpu": cpu, "rss": rss, "in_window": in_window,
                                                        "settled": settled, "idle": idle, "probe": samples,
                                                        "io": io, "snap_lag_ms": snap_lag * 1e3,
                                                        "ns_counts": ns_counts, "owner": owner})
    per_step = 1e3 / max(1, args.steps)
    cpu_ms = {"ranks": [round(g["cpu"]["rank"] * per_step, 3) for g in gathered]}
    for g in gathered:
        for k, v in g["cpu"].items():
            if k != "rank":
                cpu_ms[k] = round(v * per_step, 3)
    window = merge_breakdowns(g["in_window"] for g in gathered)
    load = None
    counts = {ns: n for g in gathered for ns, n in g["ns_counts"].items()}
    owners = {ns: o for g in gathered for ns, o in g["owner"].items() if ns in counts}
    if len(counts) > len(gathered) and owners:  # --namespaces-per-rank M > 1
        cpu_s = {k: v for g in gathered for k, v in g["cpu"].items() if k != "rank"}
        load = shard_load(counts, owners, cpu_s, float(el.item()),
                          ("NamespaceShardAssigner: crc32(name) % N" if shard.cfg.assign_policy == "hash" else
                           "NamespaceShardAssigner balanced: fewest namespaces, ties to crc32(name) % N")
                          if shard.cfg.arch == "sharded"
                          else "worker supervisor: least-loaded, sticky (runtime/workers.py)")
    return {"elapsed": float(el.item()), "reconciles": sum(sum(t.values()) for t in window.values()),
            "lat_ms": [x for g in gathered for x in g["lat"]], "odh": use_odh,
            "teardown_ms": [x for g in gathered for x in g["teardown"]],
            "rank_ms_per_step": [round(g["own_s"] * per_step, 3) for g in gathered], "cpu_ms_per_step": cpu_ms,
            "child_rss_mib": {k: v for g in gathered for k, v in g["rss"].items()},
            "apiserver_profile_per_step": prof, "breakdown": merge_breakdowns(g["settled"] for g in gathered),
            "quiesced": all(g["idle"] for g in gathered),
            "io_per_notebook": io_per_notebook([g["io"] for g in gathered], args.steps * len(gathered)),
            "burst": burst, "shard_load": load, "resident": resident, "storage": storage,
            "recon_snapshot_lag_ms": round(max(g["snap_lag_ms"] for g in gathered), 3),
            "probe_sample": [s for g in gathered for s in g["probe"]],
            "lifecycle_ms_per_20_steps": [round(statistics.fmean(b), 3) for b in zip(*(g["blocks"] for g in gathered))]}
