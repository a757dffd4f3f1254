"""Self-signed CA + serving certificate for the admission webhook.

On OpenShift the service-ca operator injects the serving Secret and the ``caBundle``
(``odh/config/webhook/service.yaml:6-7``, ``odh/config/webhook/kustomization.yaml:6-7``);
elsewhere the reference's kind CI creates them with the ``openssl`` CLI and patches the
``caBundle`` into the MutatingWebhookConfiguration
(``.github/workflows/odh_notebook_controller_integration_test.yaml:190-216``).  This
does the same programmatically (the ``cryptography`` package is not available):

* :func:`generate` — CA + serving cert files;
* :func:`provision` — the in-cluster step the ``standalone``/``mi355x`` overlays run as a
  Job (and a CronJob for renewal, ``cmd/webhook_certs.py``): keep the serving Secret
  ``odh-notebook-controller-webhook-cert`` (``tls.crt``/``tls.key``/``ca.crt``) valid and
  the MutatingWebhookConfiguration's ``caBundle`` equal to its CA.  Idempotent: a valid
  cert with more than ``renew_before_days`` left and a matching ``caBundle`` is left alone.
"""

from __future__ import annotations

import base64
import os
import subprocess
import tempfile
from dataclasses import dataclass
from typing import Iterable, List, Optional


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


def service_hosts(service: str, namespace: str, cluster_domain: str = "cluster.local") -> List[str]:
    """The DNS names the apiserver may use for ``service`` (its TLS SANs)."""
    return [service, f"{service}.{namespace}", f"{service}.{namespace}.svc",
            f"{service}.{namespace}.svc.{cluster_domain}"]


def cert_not_after(pem: str) -> Optional[float]:
    """Expiry (epoch seconds) of a PEM certificate, via ``openssl x509 -enddate``."""
    import calendar
    import time

    try:
        out = subprocess.run(["openssl", "x509", "-noout", "-enddate"], input=pem.encode(), check=True,
                             capture_output=True).stdout.decode().strip()
    except (subprocess.CalledProcessError, OSError):
        return None
    raw = out.split("=", 1)[-1]  # e.g. "Oct 16 12:00:00 2027 GMT"
    try:
        return float(calendar.timegm(time.strptime(raw, "%b %d %H:%M:%S %Y %Z")))
    except ValueError:
        return None


def cert_sans(pem: str) -> Optional[set]:
    """DNS / IP subject alternative names of a PEM certificate (``openssl x509 -ext``)."""
    try:
        out = subprocess.run(["openssl", "x509", "-noout", "-ext", "subjectAltName"], input=pem.encode(),
                             check=True, capture_output=True).stdout.decode()
    except (subprocess.CalledProcessError, OSError):
        return None
    sans = set()
    for line in out.splitlines()[1:]:
        for part in line.split(","):
            kind, _, val = part.strip().partition(":")
            if kind in ("DNS", "IP Address") and val:
                sans.add(val.strip())
    return sans


def cert_matches_key(cert_pem: str, key_pem: str) -> bool:
    def pub(args, data):
        r = subprocess.run(args, input=data.encode(), capture_output=True)
        return r.stdout if r.returncode == 0 else None
    a = pub(["openssl", "x509", "-noout", "-pubkey"], cert_pem)
    b = pub(["openssl", "pkey", "-pubout"], key_pem)
    return a is not None and a == b


async def provision(client, namespace: str, secret_name: str = "odh-notebook-controller-webhook-cert",
                    service_name="odh-notebook-controller-webhook-service",
                    mwc_names: Iterable[str] = ("odh-notebook-controller-mutating-webhook-configuration",),
                    extra_hosts: Iterable[str] = (), validity_days: int = 365, renew_before_days: int = 90,
                    cluster_domain: str = "cluster.local") -> dict:
    """Ensure the serving Secret holds a valid cert and every named MWC trusts its CA.

    ``service_name``: one Service name or several (a sharded control plane serves admission
    behind one Service per shard plus one for unassigned namespaces; the cert covers all).
    A kept cert must still cover every wanted name, otherwise it is reissued.

    Returns ``{"secret": "created"|"rotated"|"kept", "mwc": {name: "patched"|"kept"|"missing"}}``.
    """
    import time

    from ..models import kinds
    from ..models.errors import ApiError, is_not_found

    def b64(s: str) -> str:
        return base64.b64encode(s.encode()).decode()

    def unb64(s: Optional[str]) -> str:
        return base64.b64decode(s or "").decode(errors="replace")

    secret = None
    try:
        secret = await client.get(kinds.SECRET, secret_name, namespace)
    except ApiError as e:
        if not is_not_found(e):
            raise
    services = [service_name] if isinstance(service_name, str) else list(service_name)
    hosts = [h for svc in services for h in service_hosts(svc, namespace, cluster_domain)] + list(extra_hosts)
    data = (secret or {}).get("data") or {}
    crt, key, ca = unb64(data.get("tls.crt")), unb64(data.get("tls.key")), unb64(data.get("ca.crt"))
    exp = cert_not_after(crt) if crt else None
    fresh = bool(crt and key and ca and exp and exp - time.time() > renew_before_days * 86400
                 and cert_matches_key(crt, key) and set(hosts) <= (cert_sans(crt) or set()))
    result = {"secret": "kept", "mwc": {}}
    if not fresh:
        with tempfile.TemporaryDirectory(prefix="odh-webhook-certs-") as d:
            g = generate(hosts, d, validity_days)
            with open(g.cert_file) as f:
                crt = f.read()
            with open(g.key_file) as f:
                key = f.read()
            ca = g.ca_pem
        body = {"apiVersion": "v1", "kind": "Secret", "type": "kubernetes.io/tls",
                "metadata": {"name": secret_name, "namespace": namespace,
                             "labels": {"app.kubernetes.io/managed-by": "odh-webhook-certs"}},
                "data": {"tls.crt": b64(crt), "tls.key": b64(key), "ca.crt": b64(ca)}}
        if secret is None:
            await client.create(body)
            result["secret"] = "created"
        else:
            body["metadata"]["resourceVersion"] = secret["metadata"]["resourceVersion"]
            await client.update(body)
            result["secret"] = "rotated"
    bundle = b64(ca)
    for name in mwc_names:
        try:
            mwc = await client.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, name)
        except ApiError as e:
            if is_not_found(e):
                result["mwc"][name] = "missing"
                continue
            raise
        hooks = mwc.get("webhooks") or []
        if all((h.get("clientConfig") or {}).get("caBundle") == bundle for h in hooks):
            result["mwc"][name] = "kept"
            continue
        for h in hooks:
            h.setdefault("clientConfig", {})["caBundle"] = bundle
        await client.update(mwc)
        result["mwc"][name] = "patched"
    return result
