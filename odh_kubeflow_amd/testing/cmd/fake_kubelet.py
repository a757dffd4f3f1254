"""Development kubelet stand-in as a process (TEST / DEV ONLY — never deployed).

    python -m odh_kubeflow_amd.testing.cmd.fake_kubelet --master http://127.0.0.1:6443 \
        --node-name mi355x-node-0 --devices 0,1,2,3,4,5,6,7 --checkpoint-path /tmp/dp/kubelet_internal_checkpoint

The companion of ``cmd/apiserver.py --controllers`` (the envtest substitute plus the
StatefulSet controller / scheduler a real cluster has): it registers the Node, "runs" the
pods scheduled to its GPUs and writes their status, and records GPU allocations in a
kubelet device-plugin checkpoint — where the production node agent
(``cmd/node_agent.py``) reads them.  The MI355X start-up
init container (``odh-gpu-probe``) runs as a real process on the pod's GPUs with
``--exec-init`` (needs the GPUs and the built probe).  ``--jupyter`` serves the Jupyter API
for started notebooks (culling e2e).
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys

log = logging.getLogger("setup")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-fake-kubelet")
    p.add_argument("--master", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--node-name", default="mi355x-node-0")
    p.add_argument("--devices", default="0,1,2,3,4,5,6,7", help="node GPU indices this kubelet runs pods on")
    p.add_argument("--node-gpus", type=int, default=8)
    p.add_argument("--checkpoint-path", default=None, help="device-plugin checkpoint to write (default: a temp dir)")
    p.add_argument("--sysfs-root", default=None, help="take device-plugin IDs (PCI addresses) from this KFD tree")
    p.add_argument("--exec-init", action="store_true",
                   help="run the MI355X start-up probe init container (odh-gpu-probe) as a process on the pod's GPUs")
    p.add_argument("--hip-devices", type=int, default=0,
                   help="HIP devices on this box: node GPU i runs on device i %% N (a 1-GPU box hosts all 8)")
    p.add_argument("--ready-line", action="store_true", help="print 'ready' once the informers have synced")
    p.add_argument("--address", default="127.0.0.1")
    p.add_argument("--jupyter", action="store_true", help="serve the Jupyter API for started notebooks")
    p.add_argument("--partition", default="0/1",
                   help="i/W: kubelet worker i of W, running the pods of the namespaces platform worker i "
                        "claimed (testing/kubelet/statefulset.py NamespaceClaimer); worker 0 registers the Node")
    p.add_argument("--debug-log", action="store_true")
    return p.parse_args(argv)


def build(args):
    from ..kubelet.agent import FakeKubeletAgent
    from ...runtime.manager import Manager
    from ...runtime.rest import RestConfig

    devices = [int(x) for x in args.devices.split(",") if x.strip()]
    part, _, nparts = args.partition.partition("/")
    part, nparts = int(part), int(nparts or 1)
    cache_options = None
    if nparts > 1:
        from ..kubelet.statefulset import worker_owns

        cache_options = {"namespace_filter": lambda ns: worker_owns(ns, part)}
    mgr = Manager.remote(RestConfig.load(args.master, args.kubeconfig), name=f"kubelet-{args.node_name}",
                         cache_options=cache_options)
    device_id_of = None
    if args.sysfs_root:
        from ..kubelet.agent import default_device_id_of
        from ...ops.telemetry import Telemetry

        device_id_of = default_device_id_of(Telemetry(args.sysfs_root))
    runtime = None
    visible = (lambda d: d % args.hip_devices) if args.hip_devices else None
    if args.jupyter:
        from ..notebook_server.jupyter import JupyterContainerRuntime

        runtime = JupyterContainerRuntime(host=args.address)
        runtime.exec_init, runtime.visible_device = args.exec_init, visible
    elif args.exec_init:
        from ..kubelet.node import FakeContainerRuntime

        runtime = FakeContainerRuntime(exec_init=True, visible_device=visible)
    agent = FakeKubeletAgent(mgr, args.node_name, devices, args.node_gpus, runtime=runtime,
                             address=args.address, checkpoint_path=args.checkpoint_path, device_id_of=device_id_of,
                             one_runtime=True, register_node=part == 0)
    return mgr, agent


async def amain(argv=None) -> int:
    from ...cmd.common import setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log)
    mgr, _agent = build(args)
    if not args.ready_line:
        return await mgr.run_until(signal_event())
    stop = signal_event()

    async def announce():
        from ...models import kinds

        await mgr.elected.wait()
        await mgr.cache.wait_synced([kinds.POD])
        print("ready", flush=True)

    mgr_task = asyncio.ensure_future(mgr.run_until(stop))
    while mgr.elected is None:
        await asyncio.sleep(0.01)
    await announce()
    return await mgr_task


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
