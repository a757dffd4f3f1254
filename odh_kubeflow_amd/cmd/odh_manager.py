"""OpenDataHub notebook controller manager + mutating webhook (reference
``components/odh-notebook-controller/main.go``).

Flags: ``--metrics-bind-address`` (:8080), ``--health-probe-bind-address`` (:8081),
``--kube-rbac-proxy-image`` (required), ``--webhook-cert-dir``
(``/tmp/k8s-webhook-server/serving-certs``), ``--webhook-port`` (8443),
``--leader-elect``, ``--debug-log``.  The cache strips ``managedFields`` from every
object and ``data`` from ConfigMaps/Secrets, whose reads go straight to the apiserver
(:165-185); ``--cache-configmaps-secrets=true`` caches their data instead (overlay
``mi355x``: an admission then waits for no live GET, ``docs/DEPLOY.md``).  The controller namespace comes from the service-account namespace file or
``K8S_NAMESPACE`` (:103-115).  Leader-election ID ``odh-notebook-controller``.

``--workers W`` runs the reconciler in W namespace-partitioned child processes
(:mod:`~odh_kubeflow_amd.runtime.workers`); this process then leads, serves the webhook on
its own event loop — admissions never queue behind a reconcile — and aggregates the
workers' ``/metrics``.  ``--webhook-replicas R`` (with ``--workers``) serves the webhook
from R processes: this one and R-1 webhook-only children, every one accepting on the same
port (``SO_REUSEPORT``: the kernel spreads the apiserver's connections over them).  One
event loop is one core, and at 4 concurrent notebook streams the supervisor's webhook ran at
≈60 % of one, so admissions — three per notebook, two of them on the create → Ready path —
queued behind each other.  A replica reads what an admission needs the way the supervisor
does: ConfigMaps and Secrets live (the reference's uncached reads) or, with
``--cache-configmaps-secrets=true``, from its cache; the controller namespace's objects from
its cache.
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
    p = argparse.ArgumentParser(prog="odh-notebook-controller")
    p.add_argument("--metrics-bind-address", default=":8080")
    p.add_argument("--health-probe-bind-address", default=":8081")
    p.add_argument("--kube-rbac-proxy-image", default="")
    p.add_argument("--webhook-cert-dir", default="/tmp/k8s-webhook-server/serving-certs")
    p.add_argument("--webhook-port", type=int, default=8443)
    p.add_argument("--webhook-host", default="0.0.0.0")
    p.add_argument("--webhook-cert-reload-seconds", type=float, default=10.0,
                   help="poll interval for rotated tls.crt/tls.key (certwatcher)")
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--debug-log", action="store_true")
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--master", default=None)
    p.add_argument("--max-concurrent-reconciles", type=int, default=8)
    from .common import add_debug_flags, add_shard_flags, add_worker_flags

    add_shard_flags(p)
    add_debug_flags(p)
    add_worker_flags(p)
    p.add_argument("--cache-configmaps-secrets", choices=("true", "false"), default="false",
                   help="cache ConfigMap/Secret data (false: the reference's uncached, data-stripped reads, "
                        "odh/main.go:165-185; true: reads — the webhook's included — served from the cache, "
                        "as a shard does)")
    p.add_argument("--webhook-replicas", type=int, default=1,
                   help="with --workers: processes serving the webhook on one port (SO_REUSEPORT), this one "
                        "and R-1 webhook-only children")
    p.add_argument("--webhook-replica", default=None, help=argparse.SUPPRESS)
    args = p.parse_args(argv)
    if not args.kube_rbac_proxy_image:
        p.print_usage(sys.stderr)
        raise SystemExit("missing required flag: --kube-rbac-proxy-image must be set")
    args.argv = list(sys.argv[1:] if argv is None else argv)
    return args


WORKER_STRIP_VALUE = ("--workers", "--worker", "--metrics-bind-address", "--health-probe-bind-address",
                      "--webhook-replicas", "--webhook-replica")
WORKER_STRIP_BOOL = ("--leader-elect", "--enable-debug-endpoints")


def worker_argv(args, index: int, metrics_addr: str) -> List[str]:
    """A reconciler worker's command line: the supervisor's, minus leader election and the
    public addresses (the webhook stays with the supervisor)."""
    from ..runtime.workers import strip_flags

    base = strip_flags(args.argv, WORKER_STRIP_VALUE, WORKER_STRIP_BOOL)
    return [*base, "--worker", f"{index}/{args.workers}", "--metrics-bind-address", metrics_addr,
            "--health-probe-bind-address", "0", "--enable-debug-endpoints"]


def replica_argv(args, index: int, metrics_addr: str) -> List[str]:
    """A webhook replica's command line: the supervisor's webhook flags (same port and
    certificates), no leader election, no reconciler."""
    from ..runtime.workers import strip_flags

    base = strip_flags(args.argv, WORKER_STRIP_VALUE, WORKER_STRIP_BOOL)
    return [*base, "--webhook-replica", f"{index}/{args.webhook_replicas - 1}", "--metrics-bind-address",
            metrics_addr, "--health-probe-bind-address", "0", "--enable-debug-endpoints"]


def build(args, env=os.environ):
    from ..controllers.setup import odh_namespace_labels, setup_odh, shard_cache_options, with_own_services
    from ..models import kinds
    from ..runtime.informer import strip_data
    from ..runtime.leaderelection import LeaderElector, namespace_from_env
    from ..runtime.manager import Manager
    from ..runtime.rest import RestClient, RestConfig
    from ..webhook.notebook_webhook import NotebookWebhook
    from ..webhook.server import WebhookServer
    from .common import ServerRunnable, resolve_shard

    from ..runtime.workers import WorkerAssignments, WorkerSupervisor, parse_worker

    shard = resolve_shard(getattr(args, "shard", None), env)
    worker = parse_worker(getattr(args, "worker", None))
    replica = parse_worker(getattr(args, "webhook_replica", None))  # a webhook-only child
    replicas = max(1, getattr(args, "webhook_replicas", 1))
    cfg = RestConfig.load(args.master, args.kubeconfig)
    namespace = namespace_from_env()
    log.info("Controller is running in namespace %s", namespace)
    lease = "odh-notebook-controller" + (f"-shard-{shard}" if shard is not None else "")
    elector = (LeaderElector(RestClient(cfg), lease, namespace)
               if args.leader_elect and worker is None and replica is None else None)
    cache_options = shard_cache_options(shard, namespace, args.cluster_wide_watches)
    assign = WorkerAssignments(*worker) if worker is not None else None
    if assign is not None:
        # the controller namespace holds the central HTTPRoutes and ImageStreams every worker reads
        cache_options = assign.cache_options(extra_namespaces=[namespace], cluster_watch=args.cluster_wide_watches)
        cache_options["namespace_labels"] = odh_namespace_labels()  # its notebooks' CRBs and HTTPRoutes only
    cache_options = with_own_services(cache_options, "odh")  # its <nb>-kube-rbac-proxy Services only
    cache_cm = getattr(args, "cache_configmaps_secrets", "false") == "true"
    mgr = Manager.remote(cfg, name="odh-notebook-controller",
                         uncached=() if cache_cm else (kinds.CONFIG_MAP, kinds.SECRET),
                         transforms=None if cache_cm else {kinds.CONFIG_MAP: strip_data, kinds.SECRET: strip_data},
                         default_max_concurrent=args.max_concurrent_reconciles, leader_elector=elector,
                         metrics_addr=args.metrics_bind_address, probe_addr=args.health_probe_bind_address,
                         debug_endpoints=args.enable_debug_endpoints, cache_options=cache_options)
    supervise = args.workers > 1 and worker is None and replica is None
    mgr.webhook_server = None
    if replica is not None:  # the supervisor's stdin protocol (its end of file ends this process)
        assign = WorkerAssignments(*replica)
        assign.on_lost = lambda: mgr.fail("supervisor gone")
    if assign is not None:
        assign.cache = mgr.cache
        assign.on_lost = lambda: mgr.fail("supervisor gone")
        mgr.request_filter = assign.request_filter
        mgr.add(assign, needs_leader=False)  # its start returns once the initial namespaces arrived
    if supervise:
        mgr.set_supervisor(WorkerSupervisor("odh_kubeflow_amd.cmd.odh_manager", args.workers,
                                            lambda i, addr: worker_argv(args, i, addr), env=dict(env), cache=mgr.cache,
                                            system_namespaces=[namespace],
                                            name="odh-notebook-controller"))
        mgr.odh_reconciler = None
        if replicas > 1:  # no namespaces to assign (no cache): the children only serve admissions
            mgr.add_webhook_replicas(WorkerSupervisor("odh_kubeflow_amd.cmd.odh_manager", replicas - 1,
                                                      lambda i, addr: replica_argv(args, i, addr), env=dict(env),
                                                      name="odh-webhook"))
    elif replica is not None:
        mgr.odh_reconciler = None
    else:
        mgr.odh_reconciler = setup_odh(mgr, namespace, env, shard=shard)
    if worker is None:
        wh = NotebookWebhook(mgr.client, namespace, kube_rbac_proxy_image=args.kube_rbac_proxy_image, env=env)
        # controller-runtime's webhook server refuses to start without its serving cert; admission
        # (failurePolicy: Fail) is never offered over plain HTTP
        missing = [f for f in ("tls.crt", "tls.key") if not os.path.exists(os.path.join(args.webhook_cert_dir, f))]
        if missing:
            raise SystemExit(f"webhook serving certificate missing in {args.webhook_cert_dir}: {', '.join(missing)} "
                             "(OpenShift: service-ca; elsewhere: the odh-webhook-certs Job, cmd/webhook_certs.py)")
        shared = replica is not None or (supervise and replicas > 1)
        server = WebhookServer(wh, args.webhook_cert_dir, args.webhook_host, args.webhook_port,
                               reload_interval=args.webhook_cert_reload_seconds, reuse_port=shared)
        mgr.add(ServerRunnable(server.start, server.stop), needs_leader=False)  # webhooks serve on every replica
        mgr.webhook_server = server
    mgr.add_healthz_check("healthz")
    mgr.add_readyz_check("readyz")
    return mgr


async def amain(argv=None) -> int:
    from .common import run_announcing_ready, setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log, development=args.debug_log)
    mgr = build(args)
    log.info("starting manager")
    return await run_announcing_ready(mgr, signal_event())


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
