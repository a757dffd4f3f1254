"""BASELINE configs #2 and #3 with real notebook processes on the MI355X.

    python tools/bench_real_pods.py [--notebooks 1,8] [--repeats 5] [--gpu-probe off,on] [--reference-emulation]

Config #2: one Notebook requesting ``amd.com/gpu: 1`` with a PyTorch-ROCm workbench;
config #3: eight at once, one per MI355X of the node.  The controllers, the webhook and
the (fake) scheduler/kubelet run as in the in-process test cluster; the notebook container
is a real process (``kubelet/process_runtime.py``): the Jupyter API served — Ready when its
readiness probe answers — and a first cell that imports PyTorch, initialises HIP on the
allocated GPU and runs a bf16 matmul.  ``--gpu-init first-cell`` (default, JupyterLab's
behaviour) runs that cell after Ready and reports create → first GPU cell done as well;
``before-ready`` holds Ready until the GPU is usable (round 2's workbench).  Image pull and container-runtime start are not included (no registry or
container runtime on the benchmark boxes); everything from ``kubectl apply`` to the
notebook server answering is.  On a one-GPU box the eight "node GPUs" all map to device 0.

Each N runs with the MI355X start-up probe off (the default deployment) and on
(``amd.com/gpu-probe: "true"``: the kf controller adds the ``odh-gpu-probe`` init container,
which the kubelet stand-in runs as its own process on the pod's GPU before the workbench).
Reported per N and probe setting: create→Ready p50/p95/max, split into control plane
(create → pod object exists: admission, odh lock, StatefulSet), pod start (pod exists →
Ready: scheduling, the init container, the workbench process), the workbench's own timings
and the probe's (process wall time, HIP init, allocation, GPU work); with both settings the
probe's added create→Ready latency (p50 on − p50 off).
``--reference-emulation`` restores the reference's serialising odh path (one worker, the
blocking 1 s + 5 s lock removal) for a same-harness comparison.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo = int(k)
    hi = min(lo + 1, len(xs) - 1)
    return round(xs[lo] + (xs[hi] - xs[lo]) * (k - lo), 1)


async def run_n(n: int, repeats: int, emu: bool, matmul: int, probe: bool, gpu_init: str = "first-cell") -> dict:
    from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
    from odh_kubeflow_amd.testing.kubelet.process_runtime import ProcessContainerRuntime
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.models.notebook import notebook

    ndev = 1
    try:
        import torch

        ndev = max(1, torch.cuda.device_count())
    except Exception:
        pass
    rts = []

    def factory(d):
        rt = ProcessContainerRuntime(matmul=matmul, visible_device=lambda g: g % ndev, gpu_init=gpu_init)
        rts.append(rt)
        return rt

    cfg = ClusterConfig(odh=True, webhook=True, runtime_factory=factory, reference_emulation=emu,
                        env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
    total, cp, start, cell = [], [], [], []
    reports = []
    async with LocalCluster(cfg) as cl:
        await cl.ensure_namespace("bench")
        for rep in range(repeats + 1):  # the first wave warms the page cache / torch import
            names = [f"nb-r{rep}-{i}" for i in range(n)]
            t0, pod_at, ready_at = {}, {}, {}
            for nm in names:
                t0[nm] = time.perf_counter()
                await cl.admin.create(notebook(nm, "bench", gpus=1,
                                               image="rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0",
                                               annotations={"amd.com/gpu-probe": "true" if probe else "false"}))
            deadline = time.monotonic() + 600
            while len(ready_at) < n and time.monotonic() < deadline:
                now = time.perf_counter()
                for nm in names:
                    if nm not in pod_at and cl.store.peek(kinds.POD, f"{nm}-0", "bench") is not None:
                        pod_at[nm] = now
                    if nm not in ready_at and cl.notebook_ready(nm, "bench"):
                        ready_at[nm] = now
                await asyncio.sleep(0.002)
            if len(ready_at) < n:
                raise RuntimeError(f"not Ready: {sorted(set(names) - set(ready_at))}")
            cell_at = {}

            async def cell_done(nm):
                rt = next((rt for rt in rts if f"bench/{nm}-0" in rt.reports), None)
                if rt is None:
                    raise RuntimeError(f"no workbench report for bench/{nm}-0")
                await rt.first_cell(f"bench/{nm}-0", 300)
                cell_at[nm] = time.perf_counter()

            await asyncio.gather(*(cell_done(nm) for nm in names))
            if rep > 0:
                for nm in names:
                    total.append((ready_at[nm] - t0[nm]) * 1e3)
                    cell.append((max(cell_at[nm], ready_at[nm]) - t0[nm]) * 1e3)
                    cp.append((pod_at.get(nm, ready_at[nm]) - t0[nm]) * 1e3)
                    start.append((ready_at[nm] - pod_at.get(nm, ready_at[nm])) * 1e3)
                for rt in rts:
                    for key, r in list(rt.reports.items()):
                        if any(key.endswith(f"/{nm}-0") for nm in names):
                            reports.append(r)
            for nm in names:
                await cl.admin.delete(kinds.NOTEBOOK, nm, "bench")
            await cl.wait_for(lambda: all(cl.store.peek(kinds.POD, f"{nm}-0", "bench") is None for nm in names), 120)
            await cl.wait_for(lambda: not any(rt.procs for rt in rts), 60)
        probes = [p for g in cl.gpu_runtimes for p in g.probe_results][n:]  # after the warm-up wave
    wb = {}
    for k in ("ready_ms", "spawn_to_ready_ms", "import_torch_ms", "first_matmul_ms", "first_cell_done_ms"):
        vals = [(r.get("first_cell") or r).get(k, r.get(k)) for r in reports]
        vals = [v for v in vals if v is not None]
        if vals:
            wb[k + "_p50"] = round(statistics.median(vals), 1)
    pr = None
    if probe:
        res = [p.get("result") or {} for p in probes]
        tim = [r.get("timings_ms") or {} for r in res]
        pr = {"runs": len(probes), "all_ok": bool(probes) and all(p["exitCode"] == 0 for p in probes),
              "process_wall_ms_p50": pct([p["wall_ms"] for p in probes], .5),
              **{f"{k}_ms_p50": pct([t[k] for t in tim if k in t], .5) for k in ("hip_init", "alloc_fill", "probe",
                                                                                 "total")},
              "gemm_tflops_p50": pct([(r.get("results") or [{}])[0].get("gemm_tflops", 0) for r in res], .5)}
    return {"notebooks": n, "repeats": repeats, "reference_emulation": emu, "gpu_probe": pr if probe else "off",
            "gpu_init": gpu_init,
            "create_to_ready_ms": {"p50": pct(total, .5), "p95": pct(total, .95), "max": pct(total, 1)},
            # Ready, then the user's first cell (torch import, HIP init, matmul) finished
            "create_to_first_gpu_cell_ms": {"p50": pct(cell, .5), "p95": pct(cell, .95), "max": pct(cell, 1)},
            "control_plane_ms_p50": pct(cp, .5), "pod_start_ms_p50": pct(start, .5), "workbench": wb,
            "gpu": ((reports[0].get("first_cell") or reports[0]).get("gpu") if reports else None)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--notebooks", default="1,8")
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--matmul", type=int, default=1024)
    ap.add_argument("--reference-emulation", action="store_true")
    ap.add_argument("--gpu-probe", default="off,on", help="start-up probe settings to run: off, on, or off,on")
    ap.add_argument("--gpu-init", default="first-cell", choices=("first-cell", "before-ready"),
                    help="workbench's first GPU cell after Ready (JupyterLab) or before it")
    a = ap.parse_args(argv)
    for n in [int(x) for x in a.notebooks.split(",")]:
        by = {}
        for setting in [x.strip() for x in a.gpu_probe.split(",") if x.strip()]:
            r = asyncio.run(run_n(n, a.repeats, a.reference_emulation, a.matmul, setting == "on", a.gpu_init))
            print(json.dumps(r), flush=True)
            by[setting] = r
        if "on" in by and "off" in by:
            on, off = by["on"]["create_to_ready_ms"]["p50"], by["off"]["create_to_ready_ms"]["p50"]
            print(json.dumps({"notebooks": n, "gpu_probe_added_ms_p50": round(on - off, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
