"""Multi-GPU benchmark driver: one process per MI355X (``torch.distributed.run``).

Layout on an 8×MI355X node (see :mod:`.shard` for the design):

* **rank 0** starts the native C++ apiserver (``odh-apiserver``: store, REST/watch,
  admission, GC) and the scheduler (``cmd/scheduler.py``, the kube-scheduler stand-in
  with the ``amd.com/gpu`` allocator) as child processes and broadcasts the URL;
* **every rank r** runs a namespace shard of the control plane against it — kf + odh
  reconcilers, the odh webhook server, the StatefulSet controller and the node agent
  of GPU ``LOCAL_RANK`` — owning the notebooks of namespace ``bench-r``; rank 0's shard
  also registers the Node, and is otherwise identical to the others;
* each rank drives its own notebooks: one step = create one ``amd.com/gpu: 1`` Notebook
  in its namespace → Ready (pod started by whichever GPU's node agent the scheduler
  allocated, after the MI355X start-up probe on that GPU) → delete → gone.

Coordination goes through ``torch.distributed`` (gloo carries the URL, the barriers and
the result gathers; when GPUs are present an RCCL all-reduce over xGMI checks the
collective path once at start-up).  Barriers run in an executor thread so every process
keeps serving its event loop while it waits.  The timed region is bracketed by barrier +
``torch.cuda.synchronize()`` on every rank and the elapsed time is the max over ranks.
"""

from __future__ import annotations

import asyncio
import json
import os
import time
from typing import Optional


def bench_namespace(rank: int) -> str:
    return f"bench-{rank}"


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
    """Run the sharded benchmark on this rank; rank 0 returns the report dict."""
    binding = None
    if not args.no_gpu_probe:  # before any thread or child exists: they inherit the placement
        import torch as _t

        ndev = _t.cuda.device_count()  # does not initialise the GPU
        if ndev:
            binding = numa_bind(int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))) % ndev)
    dist, torch = _dist_init()
    rank, world = dist.get_rank(), dist.get_world_size()
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
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
    res = asyncio.run(_main(args, dist, torch, rank, world, local_rank, probe))
    out = None
    if rank == 0:
        from bench import report  # noqa: E402  (bench.py is the entry point on sys.path)

        out = report(args, world, res)
        out["config"]["parallelism"] = (f"namespace-sharded control plane x{world}: one `cmd/control_plane.py "
                                        f"--shard r` process per MI355X (kf + odh reconcilers + odh webhook), "
                                        f"as config/overlays/mi355x-sharded deploys it")
        out["config"]["architecture"] = "cmd/control_plane --shard (overlay mi355x-sharded)"
        out["config"]["platform_stand_ins"] = ("native C++ apiserver (+GC), cmd/scheduler.py, per-rank StatefulSet "
                                               "controller + fake kubelet of the rank's GPU")
        out["rank_ms_per_step"] = res.get("rank_ms_per_step")
        out["cpu_ms_per_step"] = res.get("cpu_ms_per_step")
        out["child_rss_mib"] = res.get("child_rss_mib")
        out["cpu_binding"] = binding or "none (ODH_BENCH_NUMA_BIND=0, or no GPU NUMA information)"
        if res.get("apiserver_profile_per_step"):
            out["apiserver_profile_per_step"] = res["apiserver_profile_per_step"]
            out["writes_per_notebook"] = writes_per_notebook(res["apiserver_profile_per_step"], world)
        if rccl_ms is not None:
            out["rccl_allreduce_check_ms"] = round(rccl_ms, 3)
    dist.barrier()
    dist.destroy_process_group()
    return out


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


def _proc_cpu_s(pid: Optional[int]) -> Optional[float]:
    """User + system CPU seconds of a child process (``/proc/<pid>/stat``), None if unreadable."""
    if pid is None:
        return None
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return None


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
    the apiserver and scheduler) — to the physical cores of its MI355X's NUMA node.

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


async def _main(args, dist, torch, rank: int, world: int, local_rank: int, probe) -> dict:
    from .shard import ControlPlaneShard, ShardConfig

    native = None
    sched = None
    url = [None]
    if rank == 0:
        from ..apiserver.native import NativeApiServer
        from ..cluster import OPENSHIFT_CRDS

        audit = os.environ.get("DEBUG_WRITE_AUDITLOG")  # same debug aid as the test cluster
        pol = None
        if audit:
            from ..apiserver.audit import AuditPolicy

            lv = os.environ.get("DEBUG_AUDIT_LEVEL", "Metadata")  # Request / RequestResponse: with bodies
            pol = AuditPolicy([{"level": lv}])  # every request: what each process sends
        native = await NativeApiServer(OPENSHIFT_CRDS, gc=True, audit_log_path=audit, audit_policy=pol).start()
        url[0] = native.url
        sched = await _start_scheduler(native.url)
    await _in_thread(dist.broadcast_object_list, url, 0)
    use_odh = not args.no_odh
    env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
    shard = ControlPlaneShard(ShardConfig(
        apiserver_url=url[0], namespace=bench_namespace(rank), gpu=local_rank % 8, shard=str(rank),
        bootstrap=(rank == 0), run_scheduler=False, odh=use_odh, webhook=use_odh, startup_probe=probe,
        reference_emulation=args.reference_emulation, env=env, process=True))
    if rank == 0:
        await shard.start()  # namespaces, Node, scheduler first
        await _in_thread(dist.barrier)
    else:
        await _in_thread(dist.barrier)
        await shard.start()
    await _in_thread(dist.barrier)  # every shard's webhook is registered before anyone creates

    try:
        children = {"apiserver": native.proc.pid if native else None, "scheduler": sched.pid if sched else None,
                    f"control_plane_{rank}": shard.control_plane_pid()}
        result = await _drive(args, shard, dist, torch, children, native)
    finally:
        await _in_thread(dist.barrier)  # nobody tears down while others still serve
        await shard.stop()
        if sched is not None:
            await _stop_child(sched)
        if native is not None:
            await native.stop()
    return result


async def _start_scheduler(url: str):
    """kube-scheduler stand-in as a child process of rank 0 (see ``cmd/scheduler.py``)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    proc = subprocess.Popen([sys.executable, "-m", "odh_kubeflow_amd.cmd.scheduler", "--master", url],
                            cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    line = await asyncio.wait_for(_in_thread(proc.stdout.readline), 120)
    if line.strip() != "ready":
        proc.kill()
        raise RuntimeError(f"scheduler process did not start (rc={proc.poll()})")
    return proc


async def _stop_child(proc) -> None:
    proc.terminate()
    try:
        await asyncio.wait_for(_in_thread(proc.wait), 10)
    except asyncio.TimeoutError:
        proc.kill()


async def _apiserver_prof(native) -> Optional[dict]:
    if native is None:
        return None
    try:
        return (await native.stats()).get("prof")
    except Exception:
        return None


def _prof_per_step(p0: Optional[dict], p1: Optional[dict], steps: int) -> Optional[dict]:
    """Native apiserver profile delta over the timed region, per step (ms / counts)."""
    if not p0 or not p1:
        return None
    out = {}
    for k, v in p1.items():
        d = (v - p0.get(k, 0)) / max(1, steps)
        out[k[:-3] + "_ms" if k.endswith("_ns") else k] = round(d / 1e6, 3) if k.endswith("_ns") else round(d, 2)
    return out


async def _drive(args, shard, dist, torch, children: Optional[dict] = None, native=None) -> dict:
    from ..models import kinds
    from ..models.notebook import notebook

    use_odh = not args.no_odh
    ns = shard.cfg.namespace
    lat_ms, teardown_ms = [], []
    state = {"recon": 0, "step": 0}

    async def one_step(timed: bool):
        state["step"] += 1
        nm = f"nb-s{state['step']}"
        ann = {"notebooks.opendatahub.io/inject-auth": "true"} if use_odh else None
        t0 = time.perf_counter()
        await shard.admin.create(notebook(nm, ns, image="rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_2.10",
                                          gpus=1, annotations=ann))
        if not await shard.wait_until(lambda: shard.notebook_ready(nm), 120):
            raise RuntimeError(f"notebook {ns}/{nm} not Ready")
        ready = time.perf_counter()
        await shard.admin.delete(kinds.NOTEBOOK, nm, ns)
        if not await shard.wait_until(lambda: shard.gone(nm), 60):
            raise RuntimeError(f"teardown of {ns}/{nm} did not finish")
        if timed:
            lat_ms.append((ready - t0) * 1e3)
            teardown_ms.append((time.perf_counter() - ready) * 1e3)

    for _ in range(args.warmup):
        await one_step(False)
    await shard.settle(5)
    from ..utils import gctune

    gctune.tune()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    await _in_thread(dist.barrier)
    b0 = await shard.reconcile_breakdown()
    children = children or {}
    child_cpu0 = {k: _proc_cpu_s(pid) for k, pid in children.items()}
    prof0 = await _apiserver_prof(native)
    cpu0 = time.process_time()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        await one_step(True)
    own = time.perf_counter() - t_start  # this rank's own steps (the barrier below equalises elapsed)
    await shard.settle(5)  # the last teardown's trailing reconciles stay inside the timed region
    from bench import breakdown_delta, merge_breakdowns  # noqa: E402  (bench.py is the entry point)

    breakdown = breakdown_delta(b0, await shard.reconcile_breakdown())
    state["recon"] = sum(sum(t.values()) for t in breakdown.values())
    # CPU time per step of every process on the path: where a step's work goes when ranks are added
    cpu = {"rank": time.process_time() - cpu0}
    prof = _prof_per_step(prof0, await _apiserver_prof(native), args.steps)
    rss = {}
    for k, pid in children.items():
        c1 = _proc_cpu_s(pid)
        if c1 is not None and child_cpu0.get(k) is not None:
            cpu[k] = c1 - child_cpu0[k]
        r = _proc_rss_mib(pid)
        if r is not None:
            rss[k] = r
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    await _in_thread(dist.barrier)
    elapsed = time.perf_counter() - t_start

    el = torch.tensor([elapsed], dtype=torch.float64)
    rc = torch.tensor([state["recon"]], dtype=torch.float64)
    await _in_thread(lambda: dist.all_reduce(el, op=dist.ReduceOp.MAX))
    await _in_thread(lambda: dist.all_reduce(rc, op=dist.ReduceOp.SUM))
    gathered = [None] * dist.get_world_size()
    await _in_thread(dist.all_gather_object, gathered, {"lat": lat_ms, "probes": shard.probe_results,
                                                        "teardown": teardown_ms, "own_s": own, "cpu": cpu,
                                                        "rss": rss, "breakdown": breakdown})
    per_step = 1e3 / max(1, args.steps)
    cpu_ms = {"ranks": [round(g["cpu"]["rank"] * per_step, 3) for g in gathered]}
    for g in gathered:
        for k, v in g["cpu"].items():
            if k != "rank":
                cpu_ms[k] = round(v * per_step, 3)
    return {"elapsed": float(el.item()), "reconciles": int(rc.item()),
            "lat_ms": [x for g in gathered for x in g["lat"]], "odh": use_odh,
            "probes": [p for g in gathered for p in g["probes"]],
            "teardown_ms": [x for g in gathered for x in g["teardown"]],
            "rank_ms_per_step": [round(g["own_s"] * per_step, 3) for g in gathered], "cpu_ms_per_step": cpu_ms,
            "child_rss_mib": {k: v for g in gathered for k, v in g["rss"].items()},
            "apiserver_profile_per_step": prof, "breakdown": merge_breakdowns(g["breakdown"] for g in gathered)}
