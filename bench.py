#!/usr/bin/env python3
"""Headline benchmark: Notebook-CR reconciles/sec + create→Ready latency at N GPU pods.

BASELINE.json metric: "Notebook-CR reconciles/sec + p50 pod-Ready latency at 1/2/4/8 GPU
pods"; configs 2/3 ("1 Notebook pod requesting amd.com/gpu=1 on one MI355X", "8
concurrent Notebook CRs, one per MI355X").

One *step* is one full notebook lifecycle wave on an 8×MI355X node:

  create N Notebook CRs at once (one ``amd.com/gpu: 1`` per GPU, PyTorch-ROCm image,
  odh auth/route path when available) → mutating webhook → kf + odh reconcilers →
  StatefulSet → scheduler + amd.com/gpu device allocation → node agent on the owning
  GPU runs the MI355X start-up probe (MFMA bf16 GEMM verified bit-exactly on the GPU +
  HBM3E pattern sweep) → pod Ready → Notebook status Ready → delete all N → finalizers
  and owned objects gone.

``value`` = reconciles completed by the notebook controllers during the K timed steps
÷ the timed wall time (whole job).  Weak scaling: N notebooks per step on N GPUs.
p50/p95 create→Ready latency over every timed notebook is reported alongside.

Launch (driver contract): ``python bench.py --gpus N --steps K --warmup W`` or under
``torch.distributed.run`` with one rank per GPU.  Data: synthetic Notebook CRs; no
images are pulled (the container runtime is the in-process node agent).
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "Notebook-CR reconciles/sec + p50 pod-Ready latency at 1/2/4/8 GPU pods"
MODEL = "kubeflow.org/v1 Notebook (amd.com/gpu=1, PyTorch-ROCm image) on 8xMI355X node"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--no-gpu-probe", action="store_true", help="skip the MI355X start-up probe (CPU dev runs)")
    p.add_argument("--no-odh", action="store_true", help="kf controller only (no webhook / odh reconciler)")
    p.add_argument("--reference-emulation", action="store_true",
                   help="reproduce the reference's serialising behaviour (1 worker, blocking lock removal)")
    p.add_argument("--transport", choices=("inprocess", "http", "native"), default="inprocess",
                   help="managers share the store (inprocess) or talk REST/watch to the apiserver (http)")
    p.add_argument("--arch", choices=("auto", "inprocess", "sharded"), default="auto",
                   help="sharded: namespace-sharded control plane, one rank per GPU, native apiserver (the headline "
                        "at every N); inprocess: one process, controllers share the store (envtest-style); auto: "
                        "sharded, plus the in-process figure as a secondary field at N=1")
    p.add_argument("--no-inprocess-baseline", action="store_true",
                   help="N=1 auto: skip the extra in-process (envtest-style) measurement")
    p.add_argument("--json-out", default=None)
    return p.parse_args(argv)


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    k = (len(xs) - 1) * q
    lo = int(k)
    hi = min(lo + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


async def run_local(args, n_gpus: int, probe) -> dict:
    from odh_kubeflow_amd.cluster import ClusterConfig, LocalCluster
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.models.notebook import notebook

    use_odh = not args.no_odh and _odh_available()
    cfg = ClusterConfig(gpus_per_node=8, odh=use_odh, webhook=use_odh, startup_probe=probe,
                        reference_emulation=args.reference_emulation, transport=args.transport,
                        env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
    lat_ms, teardown_ms = [], []
    recon = 0
    async with LocalCluster(cfg) as cl:
        await cl.ensure_namespace("bench")
        step_id = 0

        async def one_step(timed: bool):
            nonlocal step_id
            step_id += 1
            names = [f"nb-s{step_id}-g{i}" for i in range(n_gpus)]
            ann = {"notebooks.opendatahub.io/inject-auth": "true"} if use_odh else None
            t0 = {}
            ready_at = {}

            async def create(nm):
                t0[nm] = time.perf_counter()
                await cl.admin.create(notebook(nm, "bench", image="rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_2.10",
                                               gpus=1, annotations=ann))

            await asyncio.gather(*(create(nm) for nm in names))
            pending = set(names)
            deadline = time.monotonic() + 120
            while pending and time.monotonic() < deadline:
                for nm in list(pending):
                    if cl.notebook_ready(nm, "bench"):
                        ready_at[nm] = time.perf_counter()
                        pending.discard(nm)
                if pending:
                    await asyncio.sleep(0.0005)
            if pending:
                raise RuntimeError(f"notebooks not Ready: {sorted(pending)}")
            t_del = time.perf_counter()
            await asyncio.gather(*(cl.admin.delete(kinds.NOTEBOOK, nm, "bench") for nm in names))
            ok = await cl.wait_for(lambda: all(cl.store.peek(kinds.NOTEBOOK, nm, "bench") is None and
                                               cl.store.peek(kinds.POD, f"{nm}-0", "bench") is None
                                               for nm in names), 60, 0.0005)
            if not ok:
                left = [(k, o) for nm in names for k, o in ((kinds.NOTEBOOK, nm), (kinds.POD, f"{nm}-0"))
                        if cl.store.peek(k, o, "bench") is not None]
                raise RuntimeError(f"teardown did not finish: {[cl.store.peek(k, o, 'bench') for k, o in left]}")
            if timed:
                lat_ms.extend((ready_at[nm] - t0[nm]) * 1e3 for nm in names)
                teardown_ms.append((time.perf_counter() - t_del) * 1e3)

        for _ in range(args.warmup):
            await one_step(False)
        await cl.settle(5)
        from odh_kubeflow_amd.utils import gctune

        gctune.tune()  # start-up heap out of the cyclic collector's reach (see utils/gctune.py)
        r0 = cl.reconcile_count()
        b0 = cl.reconcile_breakdown()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            await one_step(True)
        # trailing reconciles of the last teardown finish inside the timed region; steps
        # themselves overlap the previous step's trailing work, as under continuous load
        await cl.settle(5)
        elapsed = time.perf_counter() - t_start
        recon = cl.reconcile_count() - r0
        breakdown = breakdown_delta(b0, cl.reconcile_breakdown())
        probes = [p for g in cl.gpu_runtimes for p in g.probe_results]
    return {"elapsed": elapsed, "reconciles": recon, "lat_ms": lat_ms, "odh": use_odh, "probes": probes,
            "teardown_ms": teardown_ms, "breakdown": breakdown}


def breakdown_delta(b0: dict, b1: dict) -> dict:
    """Reconciles per controller and triggering watch kind between two snapshots."""
    out = {}
    for ctrl, trig in b1.items():
        d = {k: v - b0.get(ctrl, {}).get(k, 0) for k, v in trig.items()}
        d = {k: v for k, v in d.items() if v}
        if d:
            out[ctrl] = d
    return out


def merge_breakdowns(parts) -> dict:
    out: dict = {}
    for b in parts:
        for ctrl, trig in (b or {}).items():
            o = out.setdefault(ctrl, {})
            for k, v in trig.items():
                o[k] = o.get(k, 0) + v
    return out


def _odh_available() -> bool:
    try:
        import odh_kubeflow_amd.controllers.odh.reconciler  # noqa: F401
        import odh_kubeflow_amd.webhook.notebook_webhook  # noqa: F401
        return True
    except ImportError:
        return False


def main(argv=None):
    args = parse(argv)
    rank = int(os.environ.get("RANK", "0"))
    n = args.gpus
    if args.arch in ("auto", "sharded"):
        # production architecture at every N (one control-plane shard per MI355X rank against
        # the native apiserver), so the 1/2/4/8 curve compares like with like
        inproc = None
        if n == 1 and args.arch == "auto" and not args.no_inprocess_baseline:
            # BASELINE config #1 (envtest-style: controllers share the in-process store)
            inproc = _run_inprocess(args, n)
        _single_rank_env()
        from odh_kubeflow_amd.parallel.bench_dist import measure

        out = measure(args)
        if out is not None and inproc is not None:
            out["inprocess_n1"] = {k: inproc.get(k) for k in (
                "value", "ms_per_step", "p50_ready_ms", "p95_ready_ms", "notebooks_ready_per_s",
                "reconciles_per_notebook", "p50_teardown_ms")}
    else:
        out = _run_inprocess(args, n)
    if rank == 0 and out is not None:
        print(json.dumps(out), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(out, f, indent=1)
    return 0


def _run_inprocess(args, n: int) -> dict:
    """One process: every controller, the webhook, the node agents share the object store."""
    import torch

    probe = None
    if not args.no_gpu_probe:
        if torch.cuda.device_count() == 0:
            raise SystemExit("no GPU visible; pass --no-gpu-probe for a CPU dev run")
        from odh_kubeflow_amd.ops import gpu

        ndev = torch.cuda.device_count()
        for d in range(min(n, ndev)):
            gpu.get_probe(d).run()  # node agent warm-up: allocate + fill resident probe buffers

        async def probe(devices):
            return await gpu.startup_probe(devices, local_index=lambda d: d % ndev)

    res = asyncio.run(run_local(args, n, probe))
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    out = report(args, n, res)
    out["config"]["architecture"] = "inprocess"
    return out


def _single_rank_env() -> None:
    if "MASTER_ADDR" not in os.environ:  # single rank without a launcher
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]),
                              RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")


def report(args, n, res) -> dict:
    el = res["elapsed"]
    lat = res["lat_ms"]
    probes = [p["results"][0] for p in res.get("probes", []) if p.get("results")]
    out = {
        "metric": METRIC,
        "value": round(res["reconciles"] / el, 2) if el > 0 else None,
        "unit": "reconciles/s",
        "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / max(1, args.steps) * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16", "data": "synthetic",
        "config": {"model": MODEL, "global_batch": n, "seq_len": 1,
                   "parallelism": f"node-agent per GPU x{n}; controllers max_concurrent=8",
                   "notebooks_per_step": n, "odh_webhook_path": res.get("odh", False)},
        "p50_ready_ms": round(pct(lat, 0.5), 3) if lat else None,
        "p95_ready_ms": round(pct(lat, 0.95), 3) if lat else None,
        "max_ready_ms": round(max(lat), 3) if lat else None,
        "notebooks_ready_per_s": round(len(lat) / el, 3) if el > 0 else None,
        "reconciles_per_notebook": round(res["reconciles"] / max(1, len(lat)), 2),
    }
    if res.get("breakdown"):
        # per controller: reconciles per notebook, split by the watch kind that queued them
        nbs = max(1, len(lat))
        out["reconciles_per_notebook_by_controller"] = {
            ctrl: {"total": round(sum(t.values()) / nbs, 2),
                   "by_trigger": {k: round(v / nbs, 2) for k, v in sorted(t.items(), key=lambda kv: -kv[1])}}
            for ctrl, t in sorted(res["breakdown"].items())}
    if getattr(args, "reference_emulation", False):
        # not the framework's numbers: the reference's serialising odh path, same harness
        out["config"]["reference_emulation"] = True
        out["config"]["parallelism"] = f"node-agent per GPU x{n}; reference emulation (1 odh worker, blocking lock removal)"
    if res.get("teardown_ms"):
        out["p50_teardown_ms"] = round(pct(res["teardown_ms"], 0.5), 3)
    if probes:
        out["gpu_probe"] = {"gpu_ms_p50": round(statistics.median(p.get("gpu_ms", 0) for p in probes), 3),
                            "gemm_tflops_p50": round(statistics.median(p.get("gemm_tflops", 0) for p in probes), 1),
                            "hbm_gbps_p50": round(statistics.median(p.get("hbm_gbps", 0) for p in probes), 1),
                            "probe_wall_ms_p50": round(statistics.median(p.get("wall_ms", 0) for p in probes), 3),
                            "all_ok": all(p.get("ok") for p in probes), "runs": len(probes)}
    return out


if __name__ == "__main__":
    sys.exit(main())
