"""MI355X node agent process (DaemonSet): amdgpu telemetry + pod→GPU attribution, read-only.

    python -m odh_kubeflow_amd.cmd.node_agent --port 9464 --sysfs-root /host/sys --proc-root /host/proc \
        --pod-resources-socket /var/lib/kubelet/pod-resources/kubelet.sock \
        --device-plugin-checkpoint /var/lib/kubelet/device-plugins/kubelet_internal_checkpoint

The agent has no apiserver client at all (no ``--master``/``--kubeconfig``): it cannot
write Nodes or pod status, and its ServiceAccount needs no RBAC.  Every attribution source
is optional; a missing one is reported on ``/gpu/pods`` and the others are used.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import sys

log = logging.getLogger("setup")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-node-agent")
    p.add_argument("--bind", default="0.0.0.0")
    p.add_argument("--port", type=int, default=9464)
    p.add_argument("--sysfs-root", default="/sys")
    p.add_argument("--proc-root", default="/proc", help="host /proc (pod UID from each GPU process's cgroup); "
                   "'' disables KFD per-process attribution")
    p.add_argument("--pod-resources-socket", default="/var/lib/kubelet/pod-resources/kubelet.sock")
    p.add_argument("--device-plugin-checkpoint",
                   default="/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint")
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.add_argument("--telemetry-interval-ms", type=int, default=200)
    p.add_argument("--telemetry-capacity", type=int, default=3000, help="samples kept per GPU (window length)")
    p.add_argument("--attribution-ttl-s", type=float, default=1.0)
    p.add_argument("--token-file", default="",
                   help="bearer token the /gpu/* and /metrics endpoints require (nodeagent/auth.py); "
                        "'' serves them unauthenticated")
    p.add_argument("--tls-cert-dir", default="",
                   help="serve HTTPS with tls.crt / tls.key from this directory (reloaded when rotated)")
    p.add_argument("--cert-reload-seconds", type=float, default=10.0)
    p.add_argument("--insecure", action="store_true",
                   help="serve plain HTTP (no --tls-cert-dir): tests and development only")
    p.add_argument("--debug-log", action="store_true")
    args = p.parse_args(argv)
    if not args.tls_cert_dir and not args.insecure:
        p.error("--tls-cert-dir is required (the token and the busy/idle answers must not cross the node "
                "network in cleartext); --insecure serves plain HTTP")
    return args


def build(args):
    from ..nodeagent.attribution import Attributor
    from ..nodeagent.podresources import PodResourcesClient
    from ..nodeagent.server import NodeTelemetryAgent
    from ..ops.telemetry import Telemetry

    telemetry = Telemetry(args.sysfs_root).start(args.telemetry_interval_ms, args.telemetry_capacity)
    log.info("amdgpu telemetry: %d KFD GPU node(s) under %s", len(telemetry), args.sysfs_root)
    pr = PodResourcesClient(args.pod_resources_socket) if args.pod_resources_socket else None
    if pr is not None and not pr.available():
        log.warning("pod-resources socket %s not there yet; using the device-plugin checkpoint and KFD until it "
                    "appears (checked on every attribution refresh)", args.pod_resources_socket)
    attributor = Attributor(telemetry, pod_resources=pr,
                            checkpoint_path=args.device_plugin_checkpoint or None,
                            proc_root=args.proc_root or None, resource=args.resource_name,
                            ttl_s=args.attribution_ttl_s)
    token = None
    if args.token_file:
        from ..nodeagent.auth import TokenFile

        token = TokenFile(args.token_file)
        if token.current() is None:
            log.warning("token file %s missing or empty: data endpoints refuse every request until it appears",
                        args.token_file)
    else:
        log.warning("no --token-file: /gpu/* and /metrics are served unauthenticated on the hostPort")
    if args.tls_cert_dir:
        missing = [f for f in ("tls.crt", "tls.key") if not os.path.exists(os.path.join(args.tls_cert_dir, f))]
        if missing:
            raise SystemExit(f"node agent serving certificate missing in {args.tls_cert_dir}: {', '.join(missing)} "
                             "(the enroll init container writes it: cmd/node_agent_enroll.py)")
    else:
        log.warning("--insecure: serving plain HTTP")
    return NodeTelemetryAgent(telemetry, attributor, host=args.bind, port=args.port, token=token,
                              tls_cert_dir=args.tls_cert_dir or None, cert_reload_s=args.cert_reload_seconds)


async def amain(argv=None) -> int:
    from .common import setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log)
    agent = build(args)
    await agent.start()
    log.info("node agent serving %s on %s:%d (pid %d)", agent.scheme, args.bind, agent.port, os.getpid())
    try:
        await signal_event().wait()
    finally:
        await agent.stop()
        agent.telemetry.close()
    return 0


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
