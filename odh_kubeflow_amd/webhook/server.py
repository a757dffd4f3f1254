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

from ..runtime.http1 import Http1Server
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
        self._server = None
        self.served = 0

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.cert_dir:
            return None
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_cert_chain(os.path.join(self.cert_dir, "tls.crt"), os.path.join(self.cert_dir, "tls.key"))
        return ctx

    async def _handle(self, method: str, path: str, headers, data: bytes):
        if method == "GET" and path in ("/healthz", "/readyz"):
            return 200, "text/plain", b"ok"
        if path != self.path:
            return 404, "text/plain", b"not found"
        if method != "POST":
            return 405, "text/plain", b"method not allowed"
        self.served += 1
        try:
            review = json.loads(data)
        except ValueError as e:
            out = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                   "response": {"uid": "", "allowed": False, "status": {"code": 400, "message": str(e)}}}
        else:
            out = await self.webhook.handle(review)
        return 200, "application/json", json.dumps(out, separators=(",", ":")).encode()

    async def start(self) -> "WebhookServer":
        self._server = await Http1Server(self._handle, self.host, self.port, self.ssl_context()).start()
        self.port = self._server.port
        return self

    async def stop(self) -> None:
        if self._server is not None:
            await self._server.stop()
            self._server = None


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
            # the apiserver defaults, spelled out: the webhook's latency budget is explicit
            "timeoutSeconds": 10, "matchPolicy": "Equivalent", "reinvocationPolicy": "Never",
            "rules": [{"apiGroups": ["kubeflow.org"], "apiVersions": ["v1"], "operations": ["CREATE", "UPDATE"],
                       "resources": ["notebooks"]}],
            **({"namespaceSelector": namespace_selector} if namespace_selector else {}),
        }],
    }
