"""Webhook serving-cert provisioner (one-shot Job + renewal CronJob outside OpenShift).

    python -m odh_kubeflow_amd.cmd.webhook_certs --namespace opendatahub \
        --service-name odh-notebook-controller-webhook-service \
        --mwc-name odh-notebook-controller-mutating-webhook-configuration

OpenShift's service-ca operator writes the serving Secret and injects the ``caBundle``
(``odh/config/webhook/service.yaml:6-7``); the reference's kind CI does it by hand with
``openssl`` + ``kubectl patch`` (``.github/workflows/odh_notebook_controller_integration_test.yaml:190-216``).
This is that step as an idempotent in-cluster program (:func:`odh_kubeflow_amd.webhook.certs.provision`):
the odh manager pod mounts the Secret (the kubelet retries the mount until it exists) and
reloads the files when a renewal rotates them.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import logging
import sys

log = logging.getLogger("webhook-certs")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-webhook-certs")
    p.add_argument("--master", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--namespace", default=None, help="default: the pod's namespace (SA file / K8S_NAMESPACE)")
    p.add_argument("--secret-name", default="odh-notebook-controller-webhook-cert")
    p.add_argument("--service-name", action="append", default=None,
                   help="webhook Service the cert must cover (repeatable: one per control-plane shard)")
    p.add_argument("--mwc-name", action="append", default=None,
                   help="MutatingWebhookConfiguration whose caBundle to keep in sync (repeatable)")
    p.add_argument("--extra-host", action="append", default=[], help="additional SAN (DNS name or IP)")
    p.add_argument("--validity-days", type=int, default=365)
    p.add_argument("--renew-before-days", type=int, default=90)
    p.add_argument("--cluster-domain", default="cluster.local")
    p.add_argument("--random-secret", action="append", default=[],
                   help="also ensure this Secret holds a random bearer token under key 'token' (repeatable; "
                        "kept once it exists): the node agent / culler shared token, nodeagent/auth.py")
    # the node agents' serving certificates are per node, from cmd/node_agent_signer.py
    return p.parse_args(argv)


async def amain(argv=None) -> int:
    from ..runtime.leaderelection import namespace_from_env
    from ..runtime.rest import RestClient, RestConfig
    from ..webhook.certs import provision
    from .common import setup_logging

    args = parse(argv)
    setup_logging()
    client = RestClient(RestConfig.load(args.master, args.kubeconfig))
    try:
        out = await provision(client, args.namespace or namespace_from_env(), args.secret_name,
                              args.service_name or ["odh-notebook-controller-webhook-service"],
                              args.mwc_name or ["odh-notebook-controller-mutating-webhook-configuration"],
                              args.extra_host, args.validity_days, args.renew_before_days, args.cluster_domain)
        if args.random_secret:
            from ..nodeagent.auth import ensure_token_secret

            ns = args.namespace or namespace_from_env()
            out["tokens"] = {n: await ensure_token_secret(client, ns, n) for n in args.random_secret}
    finally:
        await client.close()
    print(json.dumps(out), flush=True)
    missing = [n for n, v in out["mwc"].items() if v == "missing"]
    if missing:
        log.error("MutatingWebhookConfiguration(s) not found: %s", ", ".join(missing))
        return 1
    return 0


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
