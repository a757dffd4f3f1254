"""MI355X node agent process (``amd.com/gpu`` device plugin + kubelet stand-in + telemetry).

    python -m odh_kubeflow_amd.cmd.node_agent --master http://127.0.0.1:6443 \
        --node-name mi355x-node-0 --devices 0,1,2,3,4,5,6,7

``--probe`` gates pod readiness on the MI355X start-up probe (needs the GPUs and the
built ``libodh_gpu_probe.so``); ``--sysfs-root`` points the native telemetry sampler at
``/sys`` (default) or a synthetic tree.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys

log = logging.getLogger("setup")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-node-agent")
    p.add_argument("--master", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--node-name", default="mi355x-node-0")
    p.add_argument("--devices", default="0,1,2,3,4,5,6,7", help="node GPU indices this agent owns")
    p.add_argument("--node-gpus", type=int, default=8)
    p.add_argument("--probe", action="store_true", help="gate Ready on the MI355X start-up probe")
    p.add_argument("--sysfs-root", default="/sys")
    p.add_argument("--telemetry-interval-ms", type=int, default=200)
    p.add_argument("--activity-port", type=int, default=0)
    p.add_argument("--address", default="127.0.0.1")
    p.add_argument("--jupyter", action="store_true", help="serve the Jupyter API for started notebooks")
    p.add_argument("--debug-log", action="store_true")
    return p.parse_args(argv)


def build(args):
    from ..kubelet.agent import NodeAgent
    from ..runtime.manager import Manager
    from ..runtime.rest import RestConfig

    devices = [int(x) for x in args.devices.split(",") if x.strip()]
    mgr = Manager.remote(RestConfig.load(args.master, args.kubeconfig), name=f"kubelet-{args.node_name}")
    probe = None
    if args.probe:
        from ..ops import gpu

        import torch

        ndev = torch.cuda.device_count()
        for d in range(min(len(devices), ndev)):
            gpu.get_probe(d).run()

        async def probe(devs):
            return await gpu.startup_probe(devs, local_index=lambda d: devices.index(d) % ndev if d in devices
                                           else d % ndev)
    telemetry = None
    try:
        from ..ops.telemetry import Telemetry

        telemetry = Telemetry(args.sysfs_root).start(args.telemetry_interval_ms, 3000)
    except Exception as e:  # telemetry is optional; the culler falls back to Jupyter activity
        log.warning("amdgpu telemetry unavailable: %r", e)
    runtime = None
    if args.jupyter:
        from ..notebook_server.jupyter import JupyterContainerRuntime

        runtime = JupyterContainerRuntime(host=args.address)
    agent = NodeAgent(mgr, args.node_name, devices, args.node_gpus, runtime=runtime, startup_probe=probe,
                      telemetry=telemetry, address=args.address, activity_port=args.activity_port)
    return mgr, agent


async def amain(argv=None) -> int:
    from .common import setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log)
    mgr, _agent = build(args)
    await mgr.run_until(signal_event())
    return 0


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
