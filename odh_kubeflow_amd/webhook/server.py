"""HTTPS admission webhook server (controller-runtime ``webhook.Server`` analogue).

Serves ``POST /mutate-notebook-v1`` (``odh/main.go:213-227``) with AdmissionReview v1
over TLS from ``--webhook-cert-dir`` (``tls.crt`` / ``tls.key``) on ``--webhook-port``
(default 8443), plus ``/healthz`` for the TLS readiness dial the reference's envtest
suite performs (``odh/controllers/suite_test.go:237-246``).  Handlers run concurrently,
one task per request; the handler itself keeps no shared mutable state.

Certificate rotation (controller-runtime's ``certwatcher``): the cert files are polled every
``reload_interval`` seconds and, when ``tls.crt``/``tls.key`` changed (the kubelet swaps a
Secret volume atomically; service-ca / cert-manager / ``cmd/webhook_certs.py`` rotate the
Secret), loaded into the live TLS context, so new connections present the new certificate
without a restart.  A half-written or mismatched pair is ignored and retried; the old
certificate keeps serving.
"""

from __future__ import annotations

import asyncio
import logging
import os
import ssl
import time
from typing import Optional, Tuple

from ..runtime.http1 import Http1Server
from ..runtime.rest import dumps_json, loads_json  # native JSON, json's on what it declines
from .notebook_webhook import MATCH_CONDITIONS, WEBHOOK_PATH, NotebookWebhook

log = logging.getLogger("webhook.server")

# admissions per connection before a webhook replica sharing the port closes it (see start)
RECYCLE_AFTER = 100


class WebhookServer:
    def __init__(self, webhook: NotebookWebhook, cert_dir: Optional[str], host: str = "0.0.0.0", port: int = 8443,
                 path: str = WEBHOOK_PATH, reload_interval: float = 10.0, reuse_port: bool = False):
        self.webhook = webhook
        self.cert_dir = cert_dir
        self.host = host
        self.port = port
        self.path = path
        self.reload_interval = reload_interval
        self.reuse_port = reuse_port  # webhook replicas of one manager share the port (SO_REUSEPORT)
        self._server = None
        self._ctx: Optional[ssl.SSLContext] = None
        self._stamp: Optional[Tuple] = None
        self._watch: Optional[asyncio.Task] = None
        self.served = 0
        self.reloads = 0
        from collections import deque

        self.handle_s = deque(maxlen=4096)  # per admission: request decoded → response encoded (s)

    def _files(self) -> Tuple[str, str]:
        return os.path.join(self.cert_dir, "tls.crt"), os.path.join(self.cert_dir, "tls.key")

    def _file_stamp(self) -> Optional[Tuple]:
        try:
            return tuple((st.st_mtime_ns, st.st_size, st.st_ino) for st in map(os.stat, self._files()))
        except OSError:
            return None

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.cert_dir:
            return None
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        self._stamp = self._file_stamp()
        ctx.load_cert_chain(*self._files())
        return ctx

    def maybe_reload(self) -> bool:
        """Load rotated cert files into the live context; True when a new pair was loaded."""
        if self._ctx is None:
            return False
        stamp = self._file_stamp()
        if stamp is None or stamp == self._stamp:
            return False
        import shutil
        import tempfile

        # snapshot the pair, prove it on a scratch context, only then load it into the live one:
        # a failed load_cert_chain leaves an SSL_CTX with the new cert and the old key
        with tempfile.TemporaryDirectory(prefix="odh-webhook-reload-") as d:
            try:
                crt, key = (shutil.copy(f, os.path.join(d, os.path.basename(f))) for f in self._files())
                scratch = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
                scratch.load_cert_chain(crt, key)
                self._ctx.load_cert_chain(crt, key)
            except (ssl.SSLError, OSError) as e:  # mid-rotation: keep serving the old pair, retry next tick
                log.warning("webhook certificate reload failed (old certificate kept): %r", e)
                return False
        self._stamp = stamp
        self.reloads += 1
        log.info("webhook serving certificate reloaded from %s", self.cert_dir)
        return True

    async def _watch_certs(self) -> None:
        while True:
            await asyncio.sleep(self.reload_interval)
            self.maybe_reload()

    async def _handle(self, method: str, path: str, headers, data: bytes):
        if method == "GET" and path in ("/healthz", "/readyz"):
            return 200, "text/plain", b"ok"
        if path != self.path:
            return 404, "text/plain", b"not found"
        if method != "POST":
            return 405, "text/plain", b"method not allowed"
        self.served += 1
        t0 = time.perf_counter()
        try:
            review = loads_json(data)
        except ValueError as e:
            out = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                   "response": {"uid": "", "allowed": False, "status": {"code": 400, "message": str(e)}}}
        else:
            out = await self.webhook.handle(review)
        body = dumps_json(out)
        self.handle_s.append(time.perf_counter() - t0)
        return 200, "application/json", body

    async def start(self) -> "WebhookServer":
        self._ctx = self.ssl_context()
        # replicas sharing the port: the apiserver's pooled connections are re-made every 100
        # admissions, so each replica keeps getting its share (one TLS handshake per 100: ~10 µs
        # per admission).  At 1000 a 4-stream benchmark window never recycled, and one replica
        # in two of the runs sat idle (pass r5_f10)
        self._server = await Http1Server(self._handle, self.host, self.port, self._ctx,
                                         reuse_port=self.reuse_port,
                                         max_requests_per_conn=RECYCLE_AFTER if self.reuse_port else 0).start()
        self.port = self._server.port
        if self._ctx is not None and self.reload_interval > 0:
            self._watch = asyncio.ensure_future(self._watch_certs())
        return self

    async def stop(self) -> None:
        if self._watch is not None:
            self._watch.cancel()
            self._watch = None
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
            "matchConditions": [dict(c) for c in MATCH_CONDITIONS],
            **({"namespaceSelector": namespace_selector} if namespace_selector else {}),
        }],
    }
