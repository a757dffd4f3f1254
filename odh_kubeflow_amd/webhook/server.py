"""HTTPS admission webhook server (controller-runtime ``webhook.Server`` analogue).

Serves ``POST /mutate-notebook-v1`` (``odh/main.go:213-227``) with AdmissionReview v1
over TLS from ``--webhook-cert-dir`` (``tls.crt`` / ``tls.key``) on ``--webhook-port``
(default 8443), plus ``/healthz`` for the TLS readiness dial the reference's envtest
suite performs (``odh/controllers/suite_test.go:237-246``).  Handlers run concurrently,
one task per request; the handler itself keeps no shared mutable state.
"""

from __future__ import annotations

import json
import logging
import os
import ssl
from typing import Optional

from aiohttp import web

from .notebook_webhook import WEBHOOK_PATH, NotebookWebhook

log = logging.getLogger("webhook.server")


class WebhookServer:
    def __init__(self, webhook: NotebookWebhook, cert_dir: Optional[str], host: str = "0.0.0.0", port: int = 8443,
                 path: str = WEBHOOK_PATH):
        self.webhook = webhook
        self.cert_dir = cert_dir
        self.host = host
        self.port = port
        self.path = path
        self._runner = None
        self.served = 0

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.cert_dir:
            return None
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_cert_chain(os.path.join(self.cert_dir, "tls.crt"), os.path.join(self.cert_dir, "tls.key"))
        return ctx

    async def _handle(self, req: web.Request) -> web.Response:
        self.served += 1
        try:
            review = json.loads(await req.read())
        except ValueError as e:
            return web.json_response({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                                      "response": {"uid": "", "allowed": False,
                                                   "status": {"code": 400, "message": str(e)}}})
        out = await self.webhook.handle(review)
        return web.Response(body=json.dumps(out, separators=(",", ":")).encode(), content_type="application/json")

    async def start(self) -> "WebhookServer":
        app = web.Application(client_max_size=16 * 1024 * 1024)
        app.router.add_post(self.path, self._handle)

        async def ok(_r):
            return web.Response(text="ok")

        app.router.add_get("/healthz", ok)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port, ssl_context=self.ssl_context())
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None


def mutating_webhook_configuration(ca_bundle_b64: str, url: Optional[str] = None, service_namespace: str = "opendatahub",
                                   service_name: str = "odh-notebook-controller-webhook-service",
                                   name: str = "mutating-webhook-configuration",
                                   namespace_selector: Optional[dict] = None) -> dict:
    """The object of ``odh/config/webhook/manifests.yaml`` (+ caBundle).

    ``name`` / ``namespace_selector`` give one configuration per namespace shard: a
    sharded control plane routes each shard's admission calls to that shard's own
    webhook server instead of load-balancing them across all of them.
    """
    cc = {"caBundle": ca_bundle_b64}
    if url:
        cc["url"] = url
    else:
        cc["service"] = {"name": service_name, "namespace": service_namespace, "path": WEBHOOK_PATH, "port": 443}
    return {
        "apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
        "metadata": {"name": name},
        "webhooks": [{
            "name": "notebooks.opendatahub.io", "admissionReviewVersions": ["v1"], "clientConfig": cc,
            "failurePolicy": "Fail", "sideEffects": "None",
            "rules": [{"apiGroups": ["kubeflow.org"], "apiVersions": ["v1"], "operations": ["CREATE", "UPDATE"],
                       "resources": ["notebooks"]}],
            **({"namespaceSelector": namespace_selector} if namespace_selector else {}),
        }],
    }
