"""Multi-GPU benchmark driver: one process per MI355X (``torch.distributed.run``).

Layout on an 8×MI355X node (what a real deployment looks like):

* **rank 0** — the control plane: apiserver (store + REST/watch front end), the
  kube-controller-manager stand-ins (StatefulSet controller, scheduler with
  ``amd.com/gpu`` allocation, GC), the kf + odh managers and the admission webhook, plus
  the node agent of GPU 0;
* **rank r > 0** — the node agent of GPU r (``LOCAL_RANK``): a REST/watch client of
  rank 0's apiserver that starts the pods allocated to its GPU and gates their
  readiness on the MI355X start-up probe running on *its own* device.

Coordination goes through ``torch.distributed`` (the gloo group carries the apiserver
URL and the barriers; when GPUs are present an RCCL all-reduce over xGMI checks the
collective path once at start-up).  Barriers run in an executor thread so every
process keeps serving its event loop while it waits.  The timed region is bracketed
by barrier + ``torch.cuda.synchronize()`` on every rank and the elapsed time is the
max over ranks.
"""

from __future__ import annotations

import asyncio
import json
import os
import time
from typing import Optional

BENCH_NS = "bench"


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
    if torch.cuda.device_count() == 0:
        return None
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
    dist, torch = _dist_init()
    rank, world = dist.get_rank(), dist.get_world_size()
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    n = world
    probe = None
    if not args.no_gpu_probe:
        if torch.cuda.device_count() == 0:
            raise SystemExit("no GPU visible; pass --no-gpu-probe for a CPU dev run")
        from ..ops import gpu

        dev = local_rank % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        gpu.get_probe(dev).run()  # warm: allocate + fill the resident probe buffers

        async def probe(devices):
            return await gpu.startup_probe(devices, local_index=lambda d: dev)
    rccl_ms = _rccl_check(torch, dist, local_rank) if not args.no_gpu_probe else None
    res = asyncio.run(_main(args, dist, torch, rank, world, n, probe))
    if rank == 0:
        from bench import report  # noqa: E402  (bench.py is the entry point on sys.path)

        out = report(args, n, res)
        out["config"]["parallelism"] = f"node agent per GPU rank x{n}; control plane on rank 0; torch.distributed gloo"
        if rccl_ms is not None:
            out["rccl_allreduce_check_ms"] = round(rccl_ms, 3)
        print(json.dumps(out), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(out, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()
    return 0


async def _main(args, dist, torch, rank: int, world: int, n: int, probe) -> dict:
    from ..kubelet.agent import NodeAgent
    from ..runtime.manager import Manager
    from ..runtime.rest import RestConfig

    node = "mi355x-node-0"
    cl = None
    url = [None]
    if rank == 0:
        from ..cluster import ClusterConfig, LocalCluster

        use_odh = not args.no_odh
        cfg = ClusterConfig(gpus_per_node=8, odh=use_odh, webhook=use_odh, startup_probe=probe,
                            reference_emulation=args.reference_emulation, gpu_runtimes_in_process=False,
                            env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        cl = LocalCluster(cfg)
        await cl.start()
        from ..apiserver.http import ApiServer

        cl.apiserver = await ApiServer(cl.store).start("127.0.0.1", 0)
        url[0] = cl.apiserver.url
        await cl.ensure_namespace(BENCH_NS)
    await _in_thread(dist.broadcast_object_list, url, 0)
    # every rank runs the node agent of its own GPU
    if rank == 0:
        mgr = Manager.in_process(cl.store, name=f"kubelet-gpu{rank}")
    else:
        mgr = Manager.remote(RestConfig(host=url[0]), name=f"kubelet-gpu{rank}")
    agent = NodeAgent(mgr, node, [rank], node_gpus=8, startup_probe=probe, register_node=(rank == 0),
                      owns_cpu_pods=(rank == 0))
    await mgr.start()
    await _in_thread(dist.barrier)

    result = {}
    if rank == 0:
        result = await _drive(args, cl, n, agent)
    else:
        # serve until rank 0 has finished the timed region; the barriers mirror rank 0's
        await _in_thread(dist.barrier)  # before timed region
        t0 = time.perf_counter()
        await _in_thread(dist.barrier)  # after timed region
        result = {"elapsed": time.perf_counter() - t0}
    elapsed = torch.tensor([result.get("elapsed", 0.0)], dtype=torch.float64)
    await _in_thread(lambda: dist.all_reduce(elapsed, op=dist.ReduceOp.MAX))
    result["elapsed"] = float(elapsed.item())
    await _in_thread(dist.barrier)  # nobody tears down while others still serve
    await mgr.stop()
    if cl is not None:
        await cl.apiserver.stop()
        await cl.stop()
    return result


async def _drive(args, cl, n: int, agent) -> dict:
    import torch
    import torch.distributed as dist

    from ..models import kinds
    from ..models.notebook import notebook

    use_odh = not args.no_odh
    lat_ms = []
    state = {"recon": 0, "step": 0}

    async def one_step(timed: bool):
        state["step"] += 1
        names = [f"nb-s{state['step']}-g{i}" for i in range(n)]
        ann = {"notebooks.opendatahub.io/inject-auth": "true"} if use_odh else None
        r0 = cl.reconcile_count()
        t0, ready_at = {}, {}

        async def create(nm):
            t0[nm] = time.perf_counter()
            await cl.admin.create(notebook(nm, BENCH_NS, image="rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_2.10",
                                           gpus=1, annotations=ann))

        await asyncio.gather(*(create(nm) for nm in names))
        pending = set(names)
        deadline = time.monotonic() + 120
        while pending and time.monotonic() < deadline:
            for nm in list(pending):
                if cl.notebook_ready(nm, BENCH_NS):
                    ready_at[nm] = time.perf_counter()
                    pending.discard(nm)
            if pending:
                await asyncio.sleep(0.0005)
        if pending:
            raise RuntimeError(f"notebooks not Ready: {sorted(pending)}")
        await asyncio.gather(*(cl.admin.delete(kinds.NOTEBOOK, nm, BENCH_NS) for nm in names))
        ok = await cl.wait_for(lambda: all(cl.store.peek(kinds.NOTEBOOK, nm, BENCH_NS) is None and
                                           cl.store.peek(kinds.POD, f"{nm}-0", BENCH_NS) is None
                                           for nm in names), 60, 0.0005)
        if not ok:
            raise RuntimeError("teardown did not finish")
        await cl.settle(5)
        if timed:
            state["recon"] += cl.reconcile_count() - r0
            lat_ms.extend((ready_at[nm] - t0[nm]) * 1e3 for nm in names)

    for _ in range(args.warmup):
        await one_step(False)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    await _in_thread(dist.barrier)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        await one_step(True)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    await _in_thread(dist.barrier)
    elapsed = time.perf_counter() - t_start
    return {"elapsed": elapsed, "reconciles": state["recon"], "lat_ms": lat_ms, "odh": use_odh,
            "probes": agent.probe_results}
