"""kube-scheduler stand-in as its own process: binds pods and allocates ``amd.com/gpu``.

    python -m odh_kubeflow_amd.testing.cmd.scheduler --master http://127.0.0.1:6443

In a real cluster kube-scheduler (plus the AMD device plugin) is a separate process from
the notebook controllers; the multi-GPU benchmark runs this one as a child of rank 0 so
that no control-plane shard pays for the whole node's scheduling on its own event loop
(every shard then reaches the scheduler through the apiserver alike).  With
``--controllers statefulset`` it plays kube-controller-manager's StatefulSet controller
instead (its own process, as on a real cluster).  kube-controller-manager syncs
StatefulSets concurrently (``--concurrent-statefulset-syncs``, goroutines in one process);
this Python stand-in gets that concurrency from worker processes instead:
``--partition i/W`` makes this worker own the namespaces labelled
``testing.odh-kubeflow-amd/kcm-worker=i`` (claimed least-loaded first,
:class:`~odh_kubeflow_amd.testing.kubelet.statefulset.NamespaceClaimer`) and watch only those
(``InformerCache(namespace_filter=…)``), so W workers share the node's StatefulSets without
any one of them decoding every event.
Prints ``ready`` on stdout once its informers have synced.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys

log = logging.getLogger("scheduler")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-scheduler")
    p.add_argument("--master", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--max-concurrent", type=int, default=8,
                   help="scheduler workers: decisions are serialised by the allocator lock, the binds "
                        "(apiserver round trips) run concurrently")
    p.add_argument("--controllers", default="scheduler",
                   help="comma list of scheduler (kube-scheduler + device allocation), statefulset "
                        "(kube-controller-manager's StatefulSet controller) and pull-secrets (OpenShift's "
                        "ServiceAccount dockercfg controller, testing/kubelet/openshift.py)")
    p.add_argument("--pull-secret-delay-ms", type=float, default=200.0,
                   help="pull-secrets: how long after a ServiceAccount appears its pull secret is added")
    p.add_argument("--partition", default="0/1",
                   help="i/W: this is StatefulSet worker i of W (each owns the namespaces it claimed)")
    p.add_argument("--debug-log", action="store_true")
    return p.parse_args(argv)


async def amain(argv=None) -> int:
    from ..kubelet.node import SchedulerController
    from ...models import kinds
    from ...runtime.manager import Manager
    from ...runtime.rest import RestConfig
    from ...cmd.common import setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log)
    cfg = RestConfig.load(args.master, args.kubeconfig)
    ctrls = {c.strip() for c in args.controllers.split(",") if c.strip()}
    if "scheduler" not in ctrls:  # audit logs / critical path: name the component, not the program
        cfg.user_agent = cfg.user_agent.replace("scheduler", "controller_manager", 1)
    part, _, nparts = args.partition.partition("/")
    part, nparts = int(part), int(nparts or 1)
    cache_options = None
    if nparts > 1:
        from ..kubelet.statefulset import worker_owns

        cache_options = {"namespace_filter": lambda ns: worker_owns(ns, part)}
    mgr = Manager.remote(cfg, name="kube-scheduler" if "scheduler" in ctrls else "kube-controller-manager",
                         cache_options=cache_options)
    synced = []
    if "scheduler" in ctrls:
        SchedulerController(mgr.client, mgr.reader, mgr.get_event_recorder_for("default-scheduler")) \
            .setup_with_manager(mgr, max_concurrent=args.max_concurrent)
        synced += [kinds.POD, kinds.NODE]
    if "statefulset" in ctrls:
        from ..kubelet.statefulset import StatefulSetController

        StatefulSetController(mgr.client, mgr.reader, mgr.get_event_recorder_for("statefulset-controller")) \
            .setup_with_manager(mgr)
        synced += [kinds.STATEFUL_SET, kinds.POD]
        if nparts > 1:
            from ..kubelet.statefulset import NamespaceClaimer

            NamespaceClaimer(mgr.client, mgr.reader, part, nparts).setup_with_manager(mgr)
            synced += [kinds.NAMESPACE]
    if "pull-secrets" in ctrls:
        from ..kubelet.openshift import PullSecretController

        PullSecretController(mgr.client, mgr.reader, args.pull_secret_delay_ms / 1e3).setup_with_manager(mgr)
        synced += [kinds.SERVICE_ACCOUNT]
    await mgr.start()
    await mgr.cache.wait_synced(synced)
    from ...utils import gctune

    gctune.tune()  # as every long-running manager (Manager.run_until): no gen-2 pause mid-burst
    print("ready", flush=True)
    await signal_event().wait()
    await mgr.stop()
    await mgr.cache.stop()
    await mgr.rest.close()
    return 0


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
