"""Signer of the MI355X node agents' per-node certificates (a Deployment, leader-elected).

    python -m odh_kubeflow_amd.cmd.node_agent_signer --leader-elect

Watches the CertificateSigningRequests of signer ``amd.com/mi355x-node-agent`` and issues a
certificate for ``<node>.<identity domain>`` only to a requester whose service account token
is bound to a live pod of the agents' DaemonSet on that node (``nodeagent/identity.py``
:class:`NodeAgentSigner`); every other request is Denied with the reason.  The CA lives in a
Secret only this Deployment reads (created on first start, rotated before it would outlive a
leaf); its certificate — with the previous one during a rotation — is published in the
ConfigMap the culler verifies the agents against.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys

log = logging.getLogger("node-agent-signer")


def parse(argv=None):
    from ..nodeagent.identity import IDENTITY_DOMAIN, LEAF_VALIDITY_S

    p = argparse.ArgumentParser(prog="odh-node-agent-signer")
    p.add_argument("--master", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--namespace", default=None, help="the agents' namespace (default: this pod's)")
    p.add_argument("--service-account", default="mi355x-node-agent")
    p.add_argument("--daemonset", default="mi355x-node-agent")
    p.add_argument("--identity-domain", default=IDENTITY_DOMAIN)
    p.add_argument("--validity-seconds", type=int, default=LEAF_VALIDITY_S)
    p.add_argument("--ca-secret", default="mi355x-node-agent-ca")
    p.add_argument("--ca-configmap", default="mi355x-node-agent-ca")
    p.add_argument("--ca-check-seconds", type=float, default=3600.0)
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--metrics-bind-address", default=":8080")
    p.add_argument("--health-probe-bind-address", default=":8081")
    return p.parse_args(argv)


class CaKeeper:
    """Leader runnable: loads (or creates / rotates) the CA into the signer, then re-checks it."""

    def __init__(self, client, signer, namespace: str, secret: str, configmap: str, period_s: float):
        self.client, self.signer = client, signer
        self.namespace, self.secret, self.configmap, self.period_s = namespace, secret, configmap, period_s
        self._task = None

    async def _once(self) -> None:
        from ..nodeagent.identity import ensure_ca

        crt, key = await ensure_ca(self.client, self.namespace, self.secret, self.configmap,
                                   leaf_validity_s=self.signer.policy.validity_s)
        self.signer.ca_crt, self.signer.ca_key = crt, key

    async def start(self) -> None:
        await self._once()

        async def loop():
            while True:
                await asyncio.sleep(self.period_s)
                try:
                    await self._once()
                except Exception:  # noqa: BLE001 — the current CA keeps signing; retried next period
                    log.exception("CA check failed")
        self._task = asyncio.ensure_future(loop())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()


def build(args):
    from ..models import kinds
    from ..nodeagent.identity import SIGNER_NAME, NodeAgentSigner, SignerPolicy
    from ..runtime.leaderelection import LeaderElector, namespace_from_env
    from ..runtime.manager import Manager
    from ..runtime.rest import RestClient, RestConfig

    cfg = RestConfig.load(args.master, args.kubeconfig)
    ns = args.namespace or namespace_from_env()
    elector = LeaderElector(RestClient(cfg), "mi355x-node-agent-signer", ns) if args.leader_elect else None
    # Pods are read live (one GET per request: the binding must be checked against the pod as
    # it is now); only this signer's CSRs are watched
    mgr = Manager.remote(cfg, name="node-agent-signer", uncached=(kinds.POD, kinds.DAEMON_SET),
                         cache_options={"field_selectors": {kinds.CSR: f"spec.signerName={SIGNER_NAME}"}},
                         leader_elector=elector, metrics_addr=args.metrics_bind_address,
                         probe_addr=args.health_probe_bind_address)
    policy = SignerPolicy(namespace=ns, service_account=args.service_account, daemonset=args.daemonset,
                          domain=args.identity_domain, validity_s=args.validity_seconds)
    signer = NodeAgentSigner(mgr.client, policy, "", "")
    signer.setup_with_manager(mgr)
    mgr.add(CaKeeper(mgr.client, signer, ns, args.ca_secret, args.ca_configmap, args.ca_check_seconds))
    mgr.add_healthz_check("healthz")
    mgr.add_readyz_check("readyz")
    mgr.signer = signer
    return mgr


async def amain(argv=None) -> int:
    from .common import run_announcing_ready, setup_logging, signal_event

    args = parse(argv)
    setup_logging()
    mgr = build(args)
    return await run_announcing_ready(mgr, signal_event())


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
