"""Kubeflow notebook controller manager (reference ``components/notebook-controller/main.go``).

Flags keep the reference names (``--metrics-addr``, ``--probe-addr``,
``--enable-leader-election``, ``--leader-election-namespace``, ``--qps``, ``--burst``,
``--zap-devel``); additions: ``--kubeconfig`` / ``--master``,
``--max-concurrent-reconciles`` (default 8; the reference runs 1 worker), ``--workers W``
(the controllers in W namespace-partitioned child processes of this one, which leads,
aggregates their ``/metrics`` and restarts them: :mod:`~odh_kubeflow_amd.runtime.workers`),
``--split-workers`` (each of the W namespace sets served by two processes: the notebook
reconciler, and the culler + event re-emitter — the shard pod's split, so a notebook's
create → Ready reconciles never queue behind culling checks and Event re-emission).
Culling is wired only when ``ENABLE_CULLING=true`` (:111-123).  Leader-election ID
``kubeflow-notebook-controller``.

    python -m odh_kubeflow_amd.cmd.kf_manager --master http://127.0.0.1:6443
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import sys
from typing import List, Optional

log = logging.getLogger("setup")


def parse(argv: Optional[List[str]] = None) -> argparse.Namespace:
    p = argparse.ArgumentParser(prog="kf-notebook-controller")
    p.add_argument("--metrics-addr", default=":8080")
    p.add_argument("--probe-addr", default=":8081")
    p.add_argument("--leader-election-namespace", default="")
    p.add_argument("--enable-leader-election", action="store_true")
    p.add_argument("--burst", type=int, default=0)
    p.add_argument("--qps", type=int, default=0)
    p.add_argument("--zap-devel", dest="devel", action="store_true", default=True)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--master", default=None)
    p.add_argument("--max-concurrent-reconciles", type=int, default=8)
    # controller-runtime's LeaseDuration / RenewDeadline / RetryPeriod (defaults 15 s / 10 s / 2 s)
    p.add_argument("--leader-election-lease-duration", type=float, default=15.0)
    p.add_argument("--leader-election-renew-deadline", type=float, default=10.0)
    p.add_argument("--leader-election-retry-period", type=float, default=2.0)
    from .common import add_debug_flags, add_shard_flags, add_worker_flags

    add_shard_flags(p)
    add_debug_flags(p)
    add_worker_flags(p)
    p.add_argument("--split-workers", action="store_true",
                   help="with --workers: each namespace set served by a notebook-reconciler process and a "
                        "culler + event re-emitter process")
    p.add_argument("--worker-role", default="", choices=("", "notebook", "aux"), help=argparse.SUPPRESS)
    args = p.parse_args(argv)
    args.argv = list(sys.argv[1:] if argv is None else argv)
    return args


WORKER_STRIP_VALUE = ("--workers", "--worker", "--worker-role", "--metrics-addr", "--probe-addr",
                      "--leader-election-namespace")
WORKER_STRIP_BOOL = ("--enable-leader-election", "--enable-debug-endpoints", "--split-workers")


def worker_argv(args, index: int, metrics_addr: str, role: str = "") -> List[str]:
    """A worker's command line: the supervisor's, minus what the supervisor alone does
    (leader election, the public metrics and probe addresses)."""
    from ..runtime.workers import strip_flags

    base = strip_flags(args.argv, WORKER_STRIP_VALUE, WORKER_STRIP_BOOL)
    return [*base, "--worker", f"{index}/{args.workers}", "--metrics-addr", metrics_addr, "--probe-addr", "0",
            "--enable-debug-endpoints", *(["--worker-role", role] if role else [])]


def build(args, env=os.environ):
    from ..controllers.setup import setup_kf, shard_cache_options, with_own_services
    from ..runtime.leaderelection import LeaderElector, namespace_from_env
    from ..runtime.manager import Manager
    from ..runtime.rest import RestClient, RestConfig
    from .common import resolve_shard

    from ..runtime.workers import WorkerAssignments, WorkerSupervisor, parse_worker

    shard = resolve_shard(getattr(args, "shard", None), env)
    worker = parse_worker(getattr(args, "worker", None))
    cfg = RestConfig.load(args.master, args.kubeconfig)
    if args.qps:
        cfg.qps = float(args.qps)
    if args.burst:
        cfg.burst = args.burst
    elector = None
    if args.enable_leader_election and worker is None:
        elector = LeaderElector(RestClient(cfg), "kubeflow-notebook-controller" + (
                                    f"-shard-{shard}" if shard is not None else ""),
                                args.leader_election_namespace or namespace_from_env(),
                                lease_duration=args.leader_election_lease_duration,
                                renew_deadline=args.leader_election_renew_deadline,
                                retry_period=args.leader_election_retry_period)
    cache_options = shard_cache_options(shard, namespace_from_env(), args.cluster_wide_watches)
    assign = WorkerAssignments(*worker) if worker is not None else None
    if assign is not None:
        cache_options = assign.cache_options(cluster_watch=args.cluster_wide_watches)
    if args.worker_role != "aux":  # the notebook reconciler reads its own Services only
        cache_options = with_own_services(cache_options, "notebook")
    mgr = Manager.remote(cfg, name="notebook-controller", default_max_concurrent=args.max_concurrent_reconciles,
                         leader_elector=elector, metrics_addr=args.metrics_addr, probe_addr=args.probe_addr,
                         debug_endpoints=args.enable_debug_endpoints, cache_options=cache_options)
    if assign is not None:
        assign.cache = mgr.cache
        assign.on_lost = lambda: mgr.fail("supervisor gone")
        mgr.request_filter = assign.request_filter
        mgr.add(assign, needs_leader=False)  # its start returns once the initial namespaces arrived
    if args.workers > 1 and worker is None:
        # supervisor: the controllers run in the workers (runtime/workers.py)
        mgr.set_supervisor(WorkerSupervisor("odh_kubeflow_amd.cmd.kf_manager", args.workers,
                                            lambda i, addr, role="": worker_argv(args, i, addr, role), env=dict(env),
                                            cache=mgr.cache, system_namespaces=[namespace_from_env()],
                                            name="notebook-controller",
                                            roles=("notebook", "aux") if args.split_workers else ("",)))
        mgr.kf_reconcilers = {}
    elif args.worker_role == "notebook":
        mgr.kf_reconcilers = setup_kf(mgr, env, culling=False, event_reemit=False)
    elif args.worker_role == "aux":
        from ..controllers.setup import setup_culler, setup_event_reemitter

        mgr.kf_reconcilers = {"events": setup_event_reemitter(mgr)}
        culler = setup_culler(mgr, env)
        if culler is not None:
            mgr.kf_reconcilers["culler"] = culler
    else:
        mgr.kf_reconcilers = setup_kf(mgr, env)
    mgr.add_healthz_check("healthz")
    mgr.add_readyz_check("readyz")
    return mgr


async def amain(argv=None) -> int:
    from .common import run_announcing_ready, setup_logging, signal_event

    args = parse(argv)
    setup_logging(development=args.devel)
    mgr = build(args)
    log.info("starting manager")
    return await run_announcing_ready(mgr, signal_event())


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
