"""The MI355X node agent's identity enrollment (init container + renewal sidecar of the DaemonSet).

    python -m odh_kubeflow_amd.cmd.node_agent_enroll --node-name "$NODE_NAME" --host-ip "$HOST_IP" \\
        --cert-dir /var/run/odh/node-agent-tls [--once]

Keeps ``--cert-dir/tls.key`` + ``tls.crt`` a certificate for this node alone
(``nodeagent/identity.py``): a key generated here, a CertificateSigningRequest under signer
``amd.com/mi355x-node-agent``, the certificate the signer issues once it has checked that the
requester's token is bound to an agent pod on ``--node-name``.  The agent container serves the
pair from the shared memory-backed volume and reloads it on renewal; the agent itself keeps
no apiserver client (``cmd/node_agent.py``): only these containers mount a service account
token (projected, bound to the pod — the binding is what the signer verifies).

``--once``: enroll if needed, then exit (the init container: the agent starts with a
certificate).  Otherwise check every ``--check-seconds`` and renew within ``--renew-before``
of expiry.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys

log = logging.getLogger("node-agent-enroll")


def parse(argv=None):
    from ..nodeagent.identity import IDENTITY_DOMAIN, LEAF_VALIDITY_S

    p = argparse.ArgumentParser(prog="odh-node-agent-enroll")
    p.add_argument("--master", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--node-name", required=True, help="spec.nodeName (downward API)")
    p.add_argument("--host-ip", default="", help="status.hostIP (downward API): also in the certificate")
    p.add_argument("--cert-dir", required=True)
    p.add_argument("--identity-domain", default=IDENTITY_DOMAIN)
    p.add_argument("--expiration-seconds", type=int, default=LEAF_VALIDITY_S)
    p.add_argument("--renew-before", type=float, default=LEAF_VALIDITY_S / 3,
                   help="seconds before expiry at which a new key and certificate are requested")
    p.add_argument("--check-seconds", type=float, default=600.0)
    p.add_argument("--timeout-seconds", type=float, default=600.0, help="how long to wait for the signer")
    p.add_argument("--once", action="store_true")
    return p.parse_args(argv)


async def amain(argv=None) -> int:
    from ..nodeagent.identity import Enroller, EnrollmentDenied
    from ..runtime.rest import RestClient, RestConfig
    from .common import setup_logging, signal_event

    args = parse(argv)
    setup_logging()
    stop = None if args.once else signal_event()
    while True:
        # a fresh client per round: the projected token it reads is rotated by the kubelet
        client = RestClient(RestConfig.load(args.master, args.kubeconfig))
        try:
            e = Enroller(client, args.cert_dir, args.node_name, args.host_ip, args.identity_domain,
                         renew_before_s=args.renew_before, expiration_s=args.expiration_seconds)
            out = await e.ensure(args.timeout_seconds)
            log.info("node %s: certificate %s", args.node_name, out)
        except EnrollmentDenied as d:
            log.error("enrollment denied: %s", d)
            if args.once:
                return 1
        except Exception:  # noqa: BLE001 — apiserver unreachable, signer down: retried
            log.exception("enrollment failed")
            if args.once:
                return 1
        finally:
            await client.close()
        if args.once:
            return 0
        try:
            await asyncio.wait_for(stop.wait(), args.check_seconds)
            return 0
        except asyncio.TimeoutError:
            pass


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
