"""One process running the whole notebook control plane, optionally as one namespace shard.

    python -m odh_kubeflow_amd.cmd.control_plane --shard 3 \\
        --kube-rbac-proxy-image quay.io/brancz/kube-rbac-proxy:v0.18.1

The reference deploys two managers for the whole cluster: the kf notebook-controller
(``kf/main.go``: NotebookReconciler + optional culler) and the odh-notebook-controller
(``odh/main.go``: OpenshiftNotebookReconciler + the mutating webhook).  Both are
available unchanged (``cmd/kf_manager.py``, ``cmd/odh_manager.py``).  This process runs
all of it in one manager — one informer cache, one REST connection pool, one set of
watches — and with ``--shard K`` it owns only the namespaces labelled
``notebooks.amd.com/shard=K`` (``controllers/sharding.py``), so N shards split the
cluster's notebooks with constant per-shard watch traffic.  The ``mi355x-sharded``
overlay runs it as a StatefulSet (``--shard=ordinal``: replica k is shard k, one per
MI355X of an 8-GPU node) with one MutatingWebhookConfiguration and Service per shard;
the headline benchmark (``bench.py`` → ``parallel/bench_dist.py``) launches exactly
these processes, per rank.  A shard's pod runs the command four times, split by
``--controllers``: ``notebook`` (the notebook reconciler and namespace assigner),
``culler,events`` (the culler and the Pod/StatefulSet event re-emitter — the kf manager's two
auxiliary controllers, whose work is per resident notebook and per platform Event, off the
create→Ready path), ``odh`` and ``webhook`` — four event loops, so the odh pipeline never
queues behind the kf reconciles, nor an admission behind either (measured on one box, interleaved:
two processes against one, 252/268/257 vs 240/253/241 notebooks/s at N=1,
``profiles/r3_p13``; the webhook in its own process against sharing the odh one, 64
notebooks at once at 4 ranks: 1706/1651 vs 1446/1396 notebooks/s, AdmissionReview p99
1.2–1.7 vs 3.4–5.4 ms, the closed loop unchanged, ``profiles/r4_p11``).  Each reconciling
set has its own leader-election lease; a webhook-only process leads nothing (every replica
admits).

Flags are the union of the two reference managers' (odh spellings:
``--metrics-bind-address``, ``--health-probe-bind-address``, ``--leader-elect``,
``--kube-rbac-proxy-image``, ``--webhook-cert-dir``, ``--webhook-port``), plus
``--controllers``, ``--shard``, ``--shard-count``/``--assign-namespaces``.  Once the
caches are synced, the controllers are running and the webhook serves, it prints
``ready`` on stdout (the readiness handshake the benchmark and the e2e tests use).
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import sys
from typing import List, Optional

log = logging.getLogger("setup")

ALL_CONTROLLERS = ("kf", "odh", "webhook")
# finer splits of "kf": the notebook reconciler, the event re-emitter and the culler
KF_PARTS = ("notebook", "events", "culler")


def parse(argv: Optional[List[str]] = None) -> argparse.Namespace:
    from .common import add_debug_flags, add_shard_flags

    p = argparse.ArgumentParser(prog="notebook-control-plane")
    p.add_argument("--controllers", default="kf,odh,webhook",
                   help="comma list of kf (notebook + event re-emitter + culler when ENABLE_CULLING=true), "
                        "odh (OpenshiftNotebookReconciler), webhook (odh mutating webhook); or kf split in parts: "
                        "notebook (the notebook reconciler), events (the Pod/StatefulSet event re-emitter), "
                        "culler (the culler)")
    add_shard_flags(p)
    add_debug_flags(p)
    p.add_argument("--shard-count", type=int, default=0, help="number of shards (for --assign-namespaces)")
    p.add_argument("--assign-namespaces", action="store_true",
                   help="label unlabelled namespaces crc32(name) %% --shard-count (with --shard K: only those "
                        "that hash to K, so every shard claims its own)")
    p.add_argument("--assign-policy", choices=("hash", "balanced"), default="hash",
                   help="--assign-namespaces: hash (crc32 %% N) or balanced (the shard owning the fewest "
                        "namespaces, ties to the hash's; preconditioned claims)")
    p.add_argument("--assign-grace-seconds", type=float, default=5.0,
                   help="balanced: after this long an unclaimed namespace goes to its hash's shard")
    p.add_argument("--metrics-bind-address", default=":8080")
    p.add_argument("--health-probe-bind-address", default=":8081")
    p.add_argument("--kube-rbac-proxy-image", default="")
    p.add_argument("--webhook-cert-dir", default="/tmp/k8s-webhook-server/serving-certs")
    p.add_argument("--webhook-port", type=int, default=8443)
    p.add_argument("--webhook-host", default="0.0.0.0")
    p.add_argument("--webhook-cert-reload-seconds", type=float, default=10.0)
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--leader-election-namespace", default="")
    p.add_argument("--leader-election-lease-duration", type=float, default=15.0)
    p.add_argument("--leader-election-renew-deadline", type=float, default=10.0)
    p.add_argument("--leader-election-retry-period", type=float, default=2.0)
    p.add_argument("--debug-log", action="store_true")
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--master", default=None)
    p.add_argument("--qps", type=float, default=0.0)
    p.add_argument("--burst", type=int, default=0)
    p.add_argument("--max-concurrent-reconciles", type=int, default=8)
    p.add_argument("--cache-configmaps-secrets", choices=("auto", "true", "false"), default="auto",
                   help="cache ConfigMap/Secret data (auto: when sharded — a shard's cache spans few namespaces; "
                        "unsharded keeps the reference's uncached, data-stripped reads, odh/main.go:165-185)")
    p.add_argument("--reference-emulation", action="store_true", help=argparse.SUPPRESS)  # same-harness comparisons
    args = p.parse_args(argv)
    args.controller_set = [c.strip() for c in args.controllers.split(",") if c.strip()]
    bad = [c for c in args.controller_set if c not in ALL_CONTROLLERS + KF_PARTS]
    if bad:
        p.error(f"unknown --controllers entries: {bad}")
    if "kf" in args.controller_set and any(c in args.controller_set for c in KF_PARTS):
        p.error("--controllers: kf already runs notebook, events and culler")
    if ("odh" in args.controller_set or "webhook" in args.controller_set) and not args.kube_rbac_proxy_image:
        p.print_usage(sys.stderr)
        raise SystemExit("missing required flag: --kube-rbac-proxy-image must be set")
    if args.assign_namespaces and args.shard_count < 1:
        p.error("--assign-namespaces needs --shard-count")
    return args


def build(args, env=os.environ):
    from ..controllers.setup import setup_kf, setup_odh, shard_cache_options, with_own_services
    from ..models import kinds
    from ..runtime.informer import strip_data
    from ..runtime.leaderelection import LeaderElector, namespace_from_env
    from ..runtime.manager import Manager
    from ..runtime.rest import RestClient, RestConfig
    from .common import ServerRunnable, resolve_shard

    shard = resolve_shard(args.shard, env)
    cfg = RestConfig.load(args.master, args.kubeconfig)
    if set(args.controller_set) != set(ALL_CONTROLLERS):
        # a shard pod runs this program four times: the audit log tells its containers apart
        # (control_plane.notebook/…, control_plane.odh/…)
        prog, sep, rest = cfg.user_agent.partition("/")
        cfg.user_agent = f"{prog}.{'+'.join(args.controller_set)}{sep}{rest}"
    if args.qps:
        cfg.qps = float(args.qps)
    if args.burst:
        cfg.burst = args.burst
    namespace = namespace_from_env()
    cache_cm = args.cache_configmaps_secrets == "true" or (args.cache_configmaps_secrets == "auto" and shard is not None)
    uncached, transforms = (), None
    if not cache_cm:
        uncached = (kinds.CONFIG_MAP, kinds.SECRET)
        transforms = {kinds.CONFIG_MAP: strip_data, kinds.SECRET: strip_data}
    elector = None
    # a subset of the controllers (a shard pod's kf / odh containers) leads on its own lease
    subset = "" if set(args.controller_set) == set(ALL_CONTROLLERS) else "-" + "-".join(sorted(args.controller_set))
    # a webhook-only process leads nothing: admissions are served by every replica
    if args.leader_elect and set(args.controller_set) != {"webhook"}:
        lease = "notebook-control-plane" + (f"-shard-{shard}" if shard is not None else "") + subset
        elector = LeaderElector(RestClient(cfg), lease, args.leader_election_namespace or namespace,
                                lease_duration=args.leader_election_lease_duration,
                                renew_deadline=args.leader_election_renew_deadline,
                                retry_period=args.leader_election_retry_period)
    name = "notebook-control-plane" + (f"-shard-{shard}" if shard is not None else "") + subset
    # a process running one of the two Notebook-owning reconcilers watches only its own Services
    cache_options = with_own_services(shard_cache_options(shard, namespace, args.cluster_wide_watches),
                                      args.controller_set[0] if len(args.controller_set) == 1 else "")
    mgr = Manager.remote(cfg, name=name, uncached=uncached, transforms=transforms,
                         cache_options=cache_options,
                         default_max_concurrent=args.max_concurrent_reconciles, leader_elector=elector,
                         metrics_addr=args.metrics_bind_address, probe_addr=args.health_probe_bind_address,
                         debug_endpoints=args.enable_debug_endpoints)
    mgr.shard = shard
    emu = args.reference_emulation
    if "kf" in args.controller_set:
        mgr.kf_reconcilers = setup_kf(mgr, env, reference_emulation=emu)
    elif "notebook" in args.controller_set:
        mgr.kf_reconcilers = setup_kf(mgr, env, culling=False, event_reemit=False, reference_emulation=emu)
    if "events" in args.controller_set:
        from ..controllers.setup import setup_event_reemitter

        mgr.reemitter = setup_event_reemitter(mgr, reference_emulation=emu)
    if "culler" in args.controller_set:
        from ..controllers.setup import setup_culler

        mgr.culler = setup_culler(mgr, env, reference_emulation=emu)
    if "odh" in args.controller_set:
        mgr.odh_reconciler = setup_odh(mgr, namespace, env, shard=shard, reference_emulation=emu)
    if args.assign_namespaces:
        from ..controllers.sharding import NamespaceShardAssigner

        mgr.assigner = NamespaceShardAssigner(mgr.client, mgr.reader, args.shard_count, exclude=[namespace],
                                              only_shard=shard, policy=args.assign_policy,
                                              grace_s=args.assign_grace_seconds)
        mgr.assigner.setup_with_manager(mgr)
    mgr.webhook_server = None
    if "webhook" in args.controller_set:
        from ..webhook.notebook_webhook import NotebookWebhook
        from ..webhook.server import WebhookServer

        missing = [f for f in ("tls.crt", "tls.key") if not os.path.exists(os.path.join(args.webhook_cert_dir, f))]
        if missing:
            raise SystemExit(f"webhook serving certificate missing in {args.webhook_cert_dir}: {', '.join(missing)} "
                             "(OpenShift: service-ca; elsewhere: the odh-webhook-certs Job, cmd/webhook_certs.py)")
        wh = NotebookWebhook(mgr.client, namespace, kube_rbac_proxy_image=args.kube_rbac_proxy_image, env=env)
        server = WebhookServer(wh, args.webhook_cert_dir, args.webhook_host, args.webhook_port,
                               reload_interval=args.webhook_cert_reload_seconds)
        mgr.add(ServerRunnable(server.start, server.stop), needs_leader=False)
        mgr.webhook_server = server
    mgr.add_healthz_check("healthz")
    mgr.add_readyz_check("readyz")
    return mgr


async def amain(argv=None) -> int:
    from .common import run_announcing_ready, setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log, development=args.debug_log)
    mgr = build(args)
    log.info("starting control plane %s (controllers: %s)", mgr.name, ",".join(args.controller_set))
    return await run_announcing_ready(mgr, signal_event())


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
