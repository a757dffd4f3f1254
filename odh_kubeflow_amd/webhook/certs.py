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

CA_VALIDITY_DAYS = 3650
# after a CA rotation the old CA stays in every caBundle this long, so the serving pods keep
# being trusted with the old leaf until the kubelet has synced the Secret and they reloaded it
PREVIOUS_CA_GRACE_S = 3600.0
CA_ROTATED_AT_ANNOTATION = "odh-webhook-certs.opendatahub.io/ca-rotated-at"


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


def _ext_file(path: str, hosts: Iterable[str]) -> None:
    sans = [("IP:" if h.replace(".", "").isdigit() else "DNS:") + h for h in hosts]
    with open(path, "w") as f:
        f.write("basicConstraints=CA:FALSE\nkeyUsage=digitalSignature,keyEncipherment\n"
                "extendedKeyUsage=serverAuth\nsubjectAltName=" + ",".join(sans) + "\n")


def generate_ca(cert_dir: str, days: int = CA_VALIDITY_DAYS) -> None:
    """ECDSA P-256 CA as ``ca.crt`` / ``ca.key`` in ``cert_dir``."""
    ca_key, ca_crt = os.path.join(cert_dir, "ca.key"), os.path.join(cert_dir, "ca.crt")
    _run(["openssl", "ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", ca_key])
    _run(["openssl", "req", "-x509", "-new", "-key", ca_key, "-sha256", "-days", str(days), "-subj",
          "/CN=odh-notebook-controller-webhook-ca", "-out", ca_crt])


def issue_leaf(cert_dir: str, hosts: Iterable[str], days: int) -> None:
    """Serving cert ``tls.crt`` / ``tls.key`` for ``hosts``, signed by ``cert_dir``'s CA."""
    ca_key, ca_crt = os.path.join(cert_dir, "ca.key"), os.path.join(cert_dir, "ca.crt")
    key, csr, crt = (os.path.join(cert_dir, n) for n in ("tls.key", "tls.csr", "tls.crt"))
    ext = os.path.join(cert_dir, "san.ext")
    _ext_file(ext, hosts)
    _run(["openssl", "ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", key])
    _run(["openssl", "req", "-new", "-key", key, "-subj", "/CN=odh-notebook-controller-webhook-service", "-out", csr])
    _run(["openssl", "x509", "-req", "-in", csr, "-CA", ca_crt, "-CAkey", ca_key, "-CAcreateserial", "-days",
          str(days), "-sha256", "-extfile", ext, "-out", crt])


def generate(hosts: Iterable[str] = ("127.0.0.1", "localhost"), cert_dir: Optional[str] = None,
             days: int = 365) -> WebhookCerts:
    """CA (ECDSA P-256) + serving cert with SANs for ``hosts``, written as tls.crt/tls.key."""
    d = cert_dir or tempfile.mkdtemp(prefix="odh-webhook-certs-")
    os.makedirs(d, exist_ok=True)
    generate_ca(d, days)
    issue_leaf(d, hosts, days)
    with open(os.path.join(d, "ca.crt")) as f:
        return WebhookCerts(d, f.read())


def cert_signed_by(cert_pem: str, ca_pem: str) -> bool:
    """``openssl verify``: ``cert_pem`` chains to ``ca_pem``."""
    with tempfile.TemporaryDirectory(prefix="odh-verify-") as d:
        ca, crt = os.path.join(d, "ca.crt"), os.path.join(d, "tls.crt")
        for path, pem in ((ca, ca_pem), (crt, cert_pem)):
            with open(path, "w") as f:
                f.write(pem)
        r = subprocess.run(["openssl", "verify", "-CAfile", ca, crt], capture_output=True)
        return r.returncode == 0


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
                    cluster_domain: str = "cluster.local", ca_validity_days: int = CA_VALIDITY_DAYS,
                    previous_ca_grace_s: float = PREVIOUS_CA_GRACE_S) -> dict:
    """Ensure the serving Secret holds a valid cert and every named MWC trusts it — without a
    window in which admission (``failurePolicy: Fail``) is rejected.

    The CA is long-lived and kept in the Secret (``ca.key``): renewing the serving cert reissues
    only the leaf from the same CA, so the ``caBundle`` never changes and the pods' old and new
    leaves are both trusted while the kubelet syncs the Secret (~60–90 s) and the webhook server
    reloads it.  Only when the CA itself must go (missing ``ca.key`` from an older Secret, or a CA
    that would not outlive a new leaf) is a new CA made; then every ``caBundle`` first becomes
    new CA + old CA, the Secret is updated after that, and the old CA is dropped by the first run
    more than ``previous_ca_grace_s`` later.

    ``service_name``: one Service name or several (a sharded control plane serves admission
    behind one Service per shard plus one for unassigned namespaces; the cert covers all).

    Returns ``{"secret": "created"|"renewed"|"rotated"|"kept", "ca": "new"|"kept",
    "mwc": {name: "patched"|"kept"|"missing"}}`` ("renewed": new leaf, same CA; "rotated": new CA).
    """
    import time

    from ..models import kinds
    from ..models.errors import ApiError, is_not_found

    def b64(s: str) -> str:
        return base64.b64encode(s.encode()).decode()

    def unb64(s: Optional[str]) -> str:
        return base64.b64decode(s or "").decode(errors="replace")

    now = time.time()
    secret = None
    try:
        secret = await client.get(kinds.SECRET, secret_name, namespace)
    except ApiError as e:
        if not is_not_found(e):
            raise
    services = [service_name] if isinstance(service_name, str) else list(service_name)
    hosts = [h for svc in services for h in service_hosts(svc, namespace, cluster_domain)] + list(extra_hosts)
    data = (secret or {}).get("data") or {}
    ann = dict(((secret or {}).get("metadata") or {}).get("annotations") or {})
    crt, key, ca = unb64(data.get("tls.crt")), unb64(data.get("tls.key")), unb64(data.get("ca.crt"))
    ca_key, prev_ca = unb64(data.get("ca.key")), unb64(data.get("ca.previous.crt"))
    exp = cert_not_after(crt) if crt else None
    leaf_ok = bool(crt and key and ca and exp and exp - now > renew_before_days * 86400
                   and cert_matches_key(crt, key) and set(hosts) <= (cert_sans(crt) or set())
                   and cert_signed_by(crt, ca))
    ca_exp = cert_not_after(ca) if ca else None
    ca_ok = bool(ca and ca_key and ca_exp and ca_exp - now > validity_days * 86400 and cert_matches_key(ca, ca_key))
    result = {"secret": "kept", "ca": "kept", "mwc": {}}
    write = False
    if not leaf_ok:
        with tempfile.TemporaryDirectory(prefix="odh-webhook-certs-") as d:
            if ca_ok:
                for name, pem in (("ca.crt", ca), ("ca.key", ca_key)):
                    with open(os.path.join(d, name), "w") as f:
                        f.write(pem)
                result["secret"] = "renewed" if secret is not None else "created"
            else:
                generate_ca(d, max(ca_validity_days, validity_days + 1))
                if ca:
                    prev_ca = ca  # still trusted until the pods serve a leaf of the new CA
                    ann[CA_ROTATED_AT_ANNOTATION] = str(int(now))
                result["secret"] = "rotated" if secret is not None else "created"
                result["ca"] = "new"
            issue_leaf(d, hosts, validity_days)
            files = {}
            for name in ("tls.crt", "tls.key", "ca.crt", "ca.key"):
                with open(os.path.join(d, name)) as f:
                    files[name] = f.read()
        crt, key, ca, ca_key = files["tls.crt"], files["tls.key"], files["ca.crt"], files["ca.key"]
        write = True
    if prev_ca and now - float(ann.get(CA_ROTATED_AT_ANNOTATION, "0") or 0) >= previous_ca_grace_s:
        prev_ca = ""  # the grace period is over: the pods serve the new CA's leaf by now
        ann.pop(CA_ROTATED_AT_ANNOTATION, None)
        write = True
    # trust first: every caBundle holds the CA(s) the served leaves chain to BEFORE a new leaf
    # can reach a pod through the Secret
    bundle_pem = ca + (prev_ca if prev_ca and prev_ca.strip() != ca.strip() else "")
    bundle = b64(bundle_pem)
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
    if write or secret is None:
        body = {"apiVersion": "v1", "kind": "Secret", "type": "kubernetes.io/tls",
                "metadata": {"name": secret_name, "namespace": namespace, "annotations": ann,
                             "labels": {"app.kubernetes.io/managed-by": "odh-webhook-certs"}},
                "data": {"tls.crt": b64(crt), "tls.key": b64(key), "ca.crt": b64(ca)}}
        if ca_key:
            body["data"]["ca.key"] = b64(ca_key)
        if prev_ca:
            body["data"]["ca.previous.crt"] = b64(prev_ca)
        if secret is None:
            await client.create(body)
        else:
            body["metadata"]["resourceVersion"] = secret["metadata"]["resourceVersion"]
            await client.update(body)
    return result
