#!/usr/bin/env python3
"""BASELINE config #5: idle culling across 8 GPU notebooks on one MI355X node under load.

Eight ``amd.com/gpu: 1`` notebooks run on the 8 GPUs of one node; the culler uses the
``combined`` activity source (amdgpu busy counters, Jupyter kernel activity when there is
no GPU sample).  The notebook on GPU 0 runs a real MFMA load on the MI355X
(``odh_busy``, the node agent's load generator); the other seven are idle.  Measured:

* reclaim latency of each idle notebook: from the moment it became cullable
  (``last-activity`` + ``CULL_IDLE_TIME``) to its StatefulSet being scaled to 0 and its
  pod gone (the reference bounds this by ``IDLENESS_CHECK_PERIOD``, 1 min by default);
* false culls: the GPU-busy notebook must survive the whole load phase although its
  Jupyter kernels are idle (the reference, which only asks Jupyter, would cull it);
* after the load stops, the GPU-0 notebook's own reclaim latency.

The culler reaches the GPU signal the production way: the node's agent (``nodeagent/``)
attributes GPUs to pods from the (fake) kubelet's device-plugin checkpoint, which records
the PCI addresses of the allocated GPUs, and the culler asks it by pod UID.  On the GPU box
the amdgpu signal comes from ``/sys`` (the native sampler); node GPU 0 carries the PCI
address of this process's visible MI355X, the other seven node GPUs carry addresses no
local device has (they belong to other tenants of the host), so they resolve to "no
sample" and their notebooks fall back to Jupyter activity.  ``--cpu`` runs the same
scenario on a synthetic sysfs tree.

    python tools/bench_culling.py [--cpu] [--idle-s 2] [--period-s 0.25] [--load-s 6]
"""
import argparse
import asyncio
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster  # noqa: E402
from odh_kubeflow_amd.models import kinds  # noqa: E402
from odh_kubeflow_amd.models import meta as m  # noqa: E402
from odh_kubeflow_amd.models.notebook import STOP_ANNOTATION, notebook  # noqa: E402
from odh_kubeflow_amd.testing.notebook_server.jupyter import JupyterContainerRuntime  # noqa: E402

N = 8


def _telemetry(cpu: bool):
    """(telemetry, node GPU index -> device-plugin ID, sysfs root, render minors)."""
    from odh_kubeflow_amd.ops.telemetry import Telemetry, fake_bdf, write_fake_sysfs

    if cpu:
        root = tempfile.mkdtemp(prefix="odh-sysfs-")
        minors = write_fake_sysfs(root, gpus=N)
        tel = Telemetry(root).start(interval_ms=20, capacity=4000)
        return tel, fake_bdf, root, minors
    import torch

    from odh_kubeflow_amd.testing.kubelet.agent import pci_bus_index_map

    tel = Telemetry("/sys").start(interval_ms=20, capacity=4000)
    props = torch.cuda.get_device_properties(0)
    bus = getattr(props, "pci_bus_id", None)
    idx = pci_bus_index_map(tel, {0: bus}).get(0) if bus is not None else None
    real = tel.devices()[idx].pci_bdf if idx is not None else None

    def device_id_of(i):
        return real if i == 0 and real else f"0000:ee:{i:02x}.0"  # not a local device: "no sample"
    return tel, device_id_of, None, None


def _gpu_of(cl, ns, names):
    from odh_kubeflow_amd.nodeagent.checkpoint import read_checkpoint

    dm = cl.device_managers["mi355x-node-0"]
    cp = read_checkpoint(dm.checkpoint.path)
    ids = {dm.device_id_of(i): i for i in range(N)}
    return {nm: ids[cp[m.uid(cl.store.peek(kinds.POD, f"{nm}-0", ns))][0]] for nm in names}


async def run(args) -> dict:
    tel, device_id_of, root, minors = _telemetry(args.cpu)
    rt = JupyterContainerRuntime()
    env = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME_SECONDS": str(args.idle_s),
           "IDLENESS_CHECK_PERIOD_SECONDS": str(args.period_s), "CULLER_USE_POD_ENDPOINT": "true",
           "CULLING_ACTIVITY_SOURCE": "combined", "CULLING_GPU_BUSY_THRESHOLD": "5"}
    cfg = ClusterConfig(culler=True, env=env, runtime_factory=lambda d: rt, telemetry=tel, device_id_of=device_id_of)
    load = None
    out = {"metric": "culling reclaim latency across 8 GPU notebooks", "n_notebooks": N,
           "cull_idle_time_s": args.idle_s, "idleness_check_period_s": args.period_s, "load_s": args.load_s,
           "gpu_signal": "synthetic sysfs" if args.cpu else "amdgpu sysfs (gpu_busy_percent) of the visible MI355X",
           "gpu0_device_id": device_id_of(0), "attribution": "node agent (device-plugin checkpoint, by pod UID)"}
    try:
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("cull")
            names = [f"nb{i}" for i in range(N)]
            for nm in names:
                await cl.admin.create(notebook(nm, "cull", gpus=1))
            if not await cl.wait_for(lambda: all(cl.notebook_ready(nm, "cull") for nm in names), 60):
                raise RuntimeError("notebooks not Ready")
            gpu_of = _gpu_of(cl, "cull", names)
            busy_nb = next(nm for nm, g in gpu_of.items() if g == 0)
            t_kernels = time.time()
            for nm in names:  # every notebook has an idle kernel: Jupyter says "idle" for all of them
                rt.state("cull", nm).start_kernel(busy=False)
            # real MFMA load on the MI355X for the GPU-0 notebook (synthetic counter on --cpu)
            t_load = time.time()
            if args.cpu:
                from odh_kubeflow_amd.ops.telemetry import set_fake_counter

                set_fake_counter(root, minors[0], busy=97)
            else:
                from odh_kubeflow_amd.ops.gpu import LoadGenerator

                load = LoadGenerator(0, duty=1.0, chunk_ms=5.0).start()
            stopped_at = {}
            idle_names = [nm for nm in names if nm != busy_nb]

            def scaled_down(nm):
                sts = cl.store.peek(kinds.STATEFUL_SET, nm, "cull")
                return sts is not None and sts["spec"]["replicas"] == 0 and \
                    cl.store.peek(kinds.POD, f"{nm}-0", "cull") is None

            def poll():
                now = time.time()
                for nm in names:
                    if nm not in stopped_at and scaled_down(nm):
                        stopped_at[nm] = now
                return all(nm in stopped_at for nm in idle_names)

            ok = await cl.wait_for(poll, args.idle_s * 4 + 30, 0.005)
            if not ok:
                raise RuntimeError(f"idle notebooks not culled: {sorted(set(idle_names) - set(stopped_at))}")
            # keep the load on for the rest of the load phase: the busy notebook must survive
            while time.time() - t_load < args.load_s:
                poll()
                await asyncio.sleep(0.02)
            false_culls = int(busy_nb in stopped_at or STOP_ANNOTATION in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, busy_nb, "cull")))
            gpu_busy = await cl.reconcilers["culler"].gpu.busy(cl.store.peek(kinds.POD, f"{busy_nb}-0", "cull"), 1.0)
            if load is not None:
                load.stop()
                load = None
            else:
                from odh_kubeflow_amd.ops.telemetry import set_fake_counter

                set_fake_counter(root, minors[0], busy=0)
            t_unload = time.time()
            if not await cl.wait_for(lambda: poll() and busy_nb in stopped_at, args.idle_s * 4 + 30, 0.005):
                raise RuntimeError("GPU-0 notebook not culled after its load ended")

            # last-activity annotations carry whole seconds (RFC3339, as in the reference), so a
            # notebook is cullable from floor(kernel start) + CULL_IDLE_TIME on
            cullable = int(t_kernels) + args.idle_s
            lat = [(stopped_at[nm] - cullable) * 1e3 for nm in idle_names]
            out.update({
                "idle_reclaim_ms_p50": round(statistics.median(lat), 1),
                "idle_reclaim_ms_max": round(max(lat), 1),
                "busy_notebook": busy_nb, "false_culls_under_load": false_culls,
                "gpu0_busy_mean_under_load": None if gpu_busy is None else round(gpu_busy["busy_mean"], 1),
                # expected: CULL_IDLE_TIME + up to one check period (the busy window drains)
                # + up to 1 s of RFC3339 rounding
                "busy_notebook_culled_after_unload_ms": round((stopped_at[busy_nb] - t_unload) * 1e3, 1),
                "culler_checks": cl.reconcilers["culler"].checks, "culled": cl.reconcilers["culler"].culled,
                "agent_queries": cl.node_agents["mi355x-node-0"].queries,
                "agent_attributed_queries": cl.node_agents["mi355x-node-0"].attributed_queries,
            })
    finally:
        if load is not None:
            load.stop()
        tel.close()
    return out


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--cpu", action="store_true", help="synthetic sysfs + counters instead of the MI355X")
    p.add_argument("--idle-s", type=float, default=2.0)
    p.add_argument("--period-s", type=float, default=0.25)
    p.add_argument("--load-s", type=float, default=6.0)
    args = p.parse_args(argv)
    out = asyncio.run(run(args))
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
