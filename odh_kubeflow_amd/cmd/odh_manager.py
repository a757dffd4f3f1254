"""OpenDataHub notebook controller manager + mutating webhook (reference
``components/odh-notebook-controller/main.go``).

Flags: ``--metrics-bind-address`` (:8080), ``--health-probe-bind-address`` (:8081),
``--kube-rbac-proxy-image`` (required), ``--webhook-cert-dir``
(``/tmp/k8s-webhook-server/serving-certs``), ``--webhook-port`` (8443),
``--leader-elect``, ``--debug-log``.  The cache strips ``managedFields`` from every
object and ``data`` from ConfigMaps/Secrets, whose reads go straight to the apiserver
(:165-185).  The controller namespace comes from the service-account namespace file or
``K8S_NAMESPACE`` (:103-115).  Leader-election ID ``odh-notebook-controller``.
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
    from .common import add_debug_flags, add_shard_flags

    add_shard_flags(p)
    add_debug_flags(p)
    args = p.parse_args(argv)
    if not args.kube_rbac_proxy_image:
        p.print_usage(sys.stderr)
        raise SystemExit("missing required flag: --kube-rbac-proxy-image must be set")
    return args


def build(args, env=os.environ):
    from ..controllers.setup import setup_odh, shard_cache_options
    from ..models import kinds
    from ..runtime.informer import strip_data
    from ..runtime.leaderelection import LeaderElector, namespace_from_env
    from ..runtime.manager import Manager
    from ..runtime.rest import RestClient, RestConfig
    from ..webhook.notebook_webhook import NotebookWebhook
    from ..webhook.server import WebhookServer
    from .common import ServerRunnable, resolve_shard

    shard = resolve_shard(getattr(args, "shard", None), env)
    cfg = RestConfig.load(args.master, args.kubeconfig)
    namespace = namespace_from_env()
    log.info("Controller is running in namespace %s", namespace)
    lease = "odh-notebook-controller" + (f"-shard-{shard}" if shard is not None else "")
    elector = LeaderElector(RestClient(cfg), lease, namespace) if args.leader_elect else None
    mgr = Manager.remote(cfg, name="odh-notebook-controller", uncached=(kinds.CONFIG_MAP, kinds.SECRET),
                         transforms={kinds.CONFIG_MAP: strip_data, kinds.SECRET: strip_data},
                         default_max_concurrent=args.max_concurrent_reconciles, leader_elector=elector,
                         metrics_addr=args.metrics_bind_address, probe_addr=args.health_probe_bind_address,
                         debug_endpoints=args.enable_debug_endpoints, cache_options=shard_cache_options(shard, namespace))
    mgr.odh_reconciler = setup_odh(mgr, namespace, env, shard=shard)
    wh = NotebookWebhook(mgr.client, namespace, kube_rbac_proxy_image=args.kube_rbac_proxy_image, env=env)
    # controller-runtime's webhook server refuses to start without its serving cert; admission
    # (failurePolicy: Fail) is never offered over plain HTTP
    missing = [f for f in ("tls.crt", "tls.key") if not os.path.exists(os.path.join(args.webhook_cert_dir, f))]
    if missing:
        raise SystemExit(f"webhook serving certificate missing in {args.webhook_cert_dir}: {', '.join(missing)} "
                         "(OpenShift: service-ca; elsewhere: the odh-webhook-certs Job, cmd/webhook_certs.py)")
    server = WebhookServer(wh, args.webhook_cert_dir, args.webhook_host, args.webhook_port,
                           reload_interval=args.webhook_cert_reload_seconds)
    mgr.add(ServerRunnable(server.start, server.stop), needs_leader=False)  # webhooks serve on every replica
    mgr.add_healthz_check("healthz")
    mgr.add_readyz_check("readyz")
    mgr.webhook_server = server
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
