#!/usr/bin/env python3
"""BASELINE config #5: idle culling across 8 GPU notebooks on one MI355X node, under load.

Eight ``amd.com/gpu: 1`` notebooks; the culler uses the ``combined`` activity source (amdgpu
busy counters through the node agent, Jupyter kernel activity alongside).  Every notebook has
an idle Jupyter kernel throughout, so the reference (Jupyter only,
``kf/controllers/culling_controller.go:161-196``) would cull all of them whatever the GPUs do.

* **idle phase** — the GPUs are idle: every notebook must be culled, and each cull is recorded
  with the signal it rested on (``amdgpu: idle <busy%>`` = an attributed GPU sample);
  reclaim latency = from the moment a notebook became cullable (``last-activity`` +
  ``CULL_IDLE_TIME``) to its StatefulSet at 0 replicas and its pod gone;
* **load phase** — a real MFMA load runs on the GPU and the notebooks are resumed (STOP
  annotation removed, as a user does): no notebook may be culled (false culls) although
  every Jupyter kernel is idle; after the load stops, each is culled on the idle GPU signal
  again.

Attribution is the production path: the node agent (``nodeagent/``) resolves each pod's GPUs
from the kubelet stand-in's device-plugin checkpoint (PCI addresses) and samples them from
``/sys`` (native sampler).  On a one-GPU box the eight node GPUs all carry the PCI address of
this process's visible MI355X (eight tenants of one GPU), so every notebook is attributed to
the real device.  ``--cpu`` runs the scenario on a synthetic sysfs tree (eight GPUs).

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

from odh_kubeflow_amd.models import kinds  # noqa: E402
from odh_kubeflow_amd.models import meta as m  # noqa: E402
from odh_kubeflow_amd.models.notebook import LAST_ACTIVITY_ANNOTATION, STOP_ANNOTATION, notebook  # noqa: E402
from odh_kubeflow_amd.utils.timeutil import parse_rfc3339  # noqa: E402
from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster  # noqa: E402
from odh_kubeflow_amd.testing.notebook_server.jupyter import JupyterContainerRuntime  # noqa: E402

N = 8


class _Load:
    """Busy GPU(s): a real MFMA load on the MI355X, or busy counters in the synthetic tree."""

    def __init__(self, cpu: bool, root, minors):
        self.cpu, self.root, self.minors, self.gen = cpu, root, minors, None

    def start(self, window_s: float):
        """Start the load and return once the GPU has been busy for a whole sampling window:
        the load thread's HIP start-up can take seconds on a fresh box, and a notebook resumed
        meanwhile would be sampled idle — a race of this tool, not a cull of a busy GPU."""
        if self.cpu:
            from odh_kubeflow_amd.ops.telemetry import set_fake_counter

            for mn in self.minors:
                set_fake_counter(self.root, mn, busy=97)
        else:
            from odh_kubeflow_amd.ops.gpu import LoadGenerator

            self.gen = LoadGenerator(0, duty=1.0, chunk_ms=5.0).start()
            if not self.gen.wait_running(60.0):
                raise RuntimeError("the MFMA load did not start on the GPU")
        time.sleep(window_s + 0.05)

    def stop(self):
        if self.cpu:
            from odh_kubeflow_amd.ops.telemetry import set_fake_counter

            for mn in self.minors:
                set_fake_counter(self.root, mn, busy=0)
        elif self.gen is not None:
            self.gen.stop()
            self.gen = None


def _telemetry(cpu: bool):
    """(telemetry, node GPU index -> device-plugin ID, sysfs root, render minors)."""
    from odh_kubeflow_amd.ops.telemetry import Telemetry, fake_bdf, write_fake_sysfs

    if cpu:
        root = tempfile.mkdtemp(prefix="odh-sysfs-")
        minors = write_fake_sysfs(root, gpus=N)
        tel = Telemetry(root).start(interval_ms=20, capacity=4000)
        for mn in minors:
            from odh_kubeflow_amd.ops.telemetry import set_fake_counter

            set_fake_counter(root, mn, busy=0)
        return tel, fake_bdf, root, minors
    import torch

    from odh_kubeflow_amd.testing.kubelet.agent import pci_bus_index_map

    tel = Telemetry("/sys").start(interval_ms=20, capacity=4000)
    props = torch.cuda.get_device_properties(0)
    bus = getattr(props, "pci_bus_id", None)
    idx = pci_bus_index_map(tel, {0: bus}).get(0) if bus is not None else None
    if idx is None:
        raise SystemExit("cannot find this process's MI355X in the KFD topology")
    real = tel.devices()[idx].pci_bdf
    return tel, (lambda i: real), None, None


async def run(args) -> dict:
    tel, device_id_of, root, minors = _telemetry(args.cpu)
    rt = JupyterContainerRuntime()
    env = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME_SECONDS": str(args.idle_s),
           "IDLENESS_CHECK_PERIOD_SECONDS": str(args.period_s), "CULLER_USE_POD_ENDPOINT": "true",
           "CULLING_ACTIVITY_SOURCE": "combined", "CULLING_GPU_BUSY_THRESHOLD": "5"}
    cfg = ClusterConfig(culler=True, env=env, runtime_factory=lambda d: rt, telemetry=tel, device_id_of=device_id_of)
    load = _Load(args.cpu, root, minors)
    out = {"metric": "culling reclaim latency across 8 GPU notebooks", "n_notebooks": N,
           "cull_idle_time_s": args.idle_s, "idleness_check_period_s": args.period_s, "load_s": args.load_s,
           "gpu_signal": "synthetic sysfs" if args.cpu else "amdgpu sysfs (gpu_busy_percent) of the visible MI355X",
           "attribution": "node agent: device-plugin checkpoint (PCI address) by pod UID, sampled from /sys",
           "device_ids": sorted({device_id_of(i) for i in range(N)})}
    names = [f"nb{i}" for i in range(N)]
    try:
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("cull")
            culler = cl.reconcilers["culler"]
            stopped_at = {}
            last_activity = {}  # the culler's last-activity stamp, as last seen before the cull

            def scaled_down(nm):
                sts = cl.store.peek(kinds.STATEFUL_SET, nm, "cull")
                return sts is not None and sts["spec"]["replicas"] == 0 and \
                    cl.store.peek(kinds.POD, f"{nm}-0", "cull") is None

            def poll():
                now = time.time()
                for nm in names:
                    if nm in stopped_at:
                        continue
                    nb = cl.store.peek(kinds.NOTEBOOK, nm, "cull") or {}
                    la = parse_rfc3339(m.annotations(nb).get(LAST_ACTIVITY_ANNOTATION))
                    if la is not None and STOP_ANNOTATION not in m.annotations(nb):
                        last_activity[nm] = la
                    if scaled_down(nm):
                        stopped_at[nm] = now
                return len(stopped_at) == N

            async def ready_with_idle_kernels():
                if not await cl.wait_for(lambda: all(cl.notebook_ready(nm, "cull") for nm in names), 60):
                    raise RuntimeError("notebooks not Ready: " + json.dumps({
                        nm: {"ready": cl.notebook_ready(nm, "cull"),
                             "stopped": STOP_ANNOTATION in m.annotations(cl.store.peek(kinds.NOTEBOOK, nm, "cull") or {}),
                             "sts_replicas": ((cl.store.peek(kinds.STATEFUL_SET, nm, "cull") or {}).get("spec") or {}).get("replicas"),
                             "pod": cl.store.peek(kinds.POD, f"{nm}-0", "cull") is not None} for nm in names}))
                t = time.time()
                for nm in names:  # an idle kernel: Jupyter says "idle" for every notebook
                    rt.state("cull", nm).start_kernel(busy=False)
                return t

            def signals_of(since):
                by = {}
                for c in list(culler.cull_log)[since:]:
                    by[c["notebook"].split("/")[-1]] = {k: v for k, v in c.items() if k not in ("notebook", "at")}
                return by

            # ---- idle phase: every notebook culled, on which signal
            for nm in names:
                await cl.admin.create(notebook(nm, "cull", gpus=1))
            t_kernels = await ready_with_idle_kernels()
            n_log = len(culler.cull_log)
            if not await cl.wait_for(poll, args.idle_s * 4 + 30, 0.005):
                raise RuntimeError(f"idle notebooks not culled: {sorted(set(names) - set(stopped_at))}")
            # a notebook is cullable from its last-activity stamp (whole seconds, RFC3339, as in
            # the reference) + CULL_IDLE_TIME on
            idle_lat = {nm: (stopped_at[nm] - (last_activity.get(nm, int(t_kernels)) + args.idle_s)) * 1e3
                        for nm in names}
            idle_sig = signals_of(n_log)

            # ---- load phase: the GPU(s) busy, the notebooks resumed: no culls; unload: culled
            # again.  The load starts first, as a user's job outlives a restart: otherwise the
            # first notebooks back could pass CULL_IDLE_TIME while the last ones still start.
            stopped_at.clear()
            await asyncio.get_running_loop().run_in_executor(None, load.start, args.period_s)
            for nm in names:
                await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {STOP_ANNOTATION: None}}},
                                     name=nm, namespace="cull")
            await ready_with_idle_kernels()
            t_load = time.time()
            while time.time() - t_load < args.load_s:
                poll()
                await asyncio.sleep(0.02)
            false_culls = sorted(nm for nm in names if nm in stopped_at or STOP_ANNOTATION in m.annotations(
                cl.store.peek(kinds.NOTEBOOK, nm, "cull")))
            busy_sample = await culler.gpu.busy(cl.store.peek(kinds.POD, "nb0-0", "cull"), 1.0)
            false_sig = {nm: sig for nm, sig in signals_of(n_log).items() if nm in false_culls}
            n_log = len(culler.cull_log)
            load.stop()
            t_unload = time.time()
            if not await cl.wait_for(poll, args.idle_s * 4 + 30, 0.005):
                raise RuntimeError(f"notebooks not culled after the load: {sorted(set(names) - set(stopped_at))}")
            unload_lat = {nm: (stopped_at[nm] - t_unload) * 1e3 for nm in names}
            unload_sig = signals_of(n_log)
            gpu_culls = sum(1 for s in list(idle_sig.values()) + list(unload_sig.values())
                            if str(s.get("amdgpu", "")).startswith("idle"))
            out.update({
                "idle_reclaim_ms_p50": round(statistics.median(idle_lat.values()), 1),
                "idle_reclaim_ms_max": round(max(idle_lat.values()), 1),
                "false_culls_under_load": len(false_culls), "falsely_culled": false_culls,
                "false_cull_signals": false_sig,
                "gpu_busy_mean_under_load": None if busy_sample is None else round(busy_sample["busy_mean"], 1),
                # expected: CULL_IDLE_TIME + up to one check period (the busy window drains)
                # + up to 1 s of RFC3339 rounding
                "culled_after_unload_ms_p50": round(statistics.median(unload_lat.values()), 1),
                "culls_on_attributed_gpu_idle_sample": gpu_culls,
                "per_notebook": {nm: {"gpu_device_id": device_id_of(i),
                                      "idle_phase": {"reclaim_ms": round(idle_lat[nm], 1), **idle_sig.get(nm, {})},
                                      "after_unload": {"culled_ms": round(unload_lat[nm], 1),
                                                       **unload_sig.get(nm, {})}}
                                 for i, nm in enumerate(names)},
                "culler_checks": culler.checks, "culled": culler.culled,
                "agent_queries": cl.node_agents["mi355x-node-0"].queries,
                "agent_attributed_queries": cl.node_agents["mi355x-node-0"].attributed_queries,
            })
    finally:
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
