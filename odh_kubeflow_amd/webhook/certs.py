"""Self-signed CA + serving certificate for the admission webhook.

On OpenShift the service-ca operator injects the serving Secret and the ``caBundle``
(``odh/config/webhook/service.yaml:6-7``, ``odh/config/webhook/kustomization.yaml:6-7``);
elsewhere the reference's kind CI creates them with the ``openssl`` CLI and patches the
``caBundle`` into the MutatingWebhookConfiguration
(``.github/workflows/odh_notebook_controller_integration_test.yaml:190-216``).  This
does the same programmatically (the ``cryptography`` package is not available).
"""

from __future__ import annotations

import base64
import os
import subprocess
import tempfile
from dataclasses import dataclass
from typing import Iterable, Optional


@dataclass
class WebhookCerts:
    cert_dir: str
    ca_pem: str

    @property
    def cert_file(self) -> str:
        return os.path.join(self.cert_dir, "tls.crt")

    @property
    def key_file(self) -> str:
        return os.path.join(self.cert_dir, "tls.key")

    @property
    def ca_bundle_b64(self) -> str:
        return base64.b64encode(self.ca_pem.encode()).decode()


def _run(args):
    subprocess.run(args, check=True, capture_output=True)


def generate(hosts: Iterable[str] = ("127.0.0.1", "localhost"), cert_dir: Optional[str] = None,
             days: int = 365) -> WebhookCerts:
    """CA (ECDSA P-256) + serving cert with SANs for ``hosts``, written as tls.crt/tls.key."""
    d = cert_dir or tempfile.mkdtemp(prefix="odh-webhook-certs-")
    os.makedirs(d, exist_ok=True)
    ca_key, ca_crt = os.path.join(d, "ca.key"), os.path.join(d, "ca.crt")
    key, csr, crt = os.path.join(d, "tls.key"), os.path.join(d, "tls.csr"), os.path.join(d, "tls.crt")
    ext = os.path.join(d, "san.ext")
    sans = []
    for h in hosts:
        sans.append(("IP:" if h.replace(".", "").isdigit() else "DNS:") + h)
    with open(ext, "w") as f:
        f.write("basicConstraints=CA:FALSE\nkeyUsage=digitalSignature,keyEncipherment\n"
                "extendedKeyUsage=serverAuth\nsubjectAltName=" + ",".join(sans) + "\n")
    _run(["openssl", "ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", ca_key])
    _run(["openssl", "req", "-x509", "-new", "-key", ca_key, "-sha256", "-days", str(days), "-subj",
          "/CN=odh-notebook-controller-webhook-ca", "-out", ca_crt])
    _run(["openssl", "ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", key])
    _run(["openssl", "req", "-new", "-key", key, "-subj", "/CN=odh-notebook-controller-webhook-service", "-out", csr])
    _run(["openssl", "x509", "-req", "-in", csr, "-CA", ca_crt, "-CAkey", ca_key, "-CAcreateserial", "-days",
          str(days), "-sha256", "-extfile", ext, "-out", crt])
    with open(ca_crt) as f:
        return WebhookCerts(d, f.read())
