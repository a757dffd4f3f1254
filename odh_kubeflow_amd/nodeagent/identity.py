"""One identity per node for the MI355X node agents.

The culler decides GPU culls on the agents' answers (``controllers/culling.py``
``NodeAgentActivity``), so an answer must provably come from the agent of the pod's own
node.  A fleet-wide serving certificate does not do that: whoever roots one GPU node holds a
key that is valid for every other node's agent too.  Here each agent holds a key of its own
and a certificate that names its node, issued through the Kubernetes CertificateSigningRequest
API — the kubelet's own serving-certificate flow (``kubernetes.io/kubelet-serving``), with
the node bound by the agent pod's service account token rather than by the node's
credentials:

* **agent side** (:class:`Enroller`, ``cmd/node_agent_enroll.py`` as the DaemonSet's init
  container and renewal sidecar): generates a P-256 key on the node (it never leaves the
  pod's memory-backed volume) and submits a CSR for ``CN=system:node-agent:<node>``,
  ``DNS:<node>.<identity domain>``, ``IP:<hostIP>`` under signer :data:`SIGNER_NAME`, then
  writes the issued certificate next to the key; the agent's TLS context reloads it;
* **signer** (:class:`NodeAgentSigner`, ``cmd/node_agent_signer.py``): approves and signs only
  a request whose requester (set by the apiserver from the authenticated token, not by the
  client) is the agents' ServiceAccount with a token bound to a live pod of the agents'
  DaemonSet, and only for the node that pod runs on — the certificate's names come from the
  Pod object (``spec.nodeName``, ``status.hostIP``), never from the request.  Anything else is
  Denied with the reason;
* **culler**: verifies an agent's certificate against the agents' CA and the name
  ``<pod.spec.nodeName>.<identity domain>`` — node B's certificate answering for a pod on
  node A fails the TLS handshake, and the culler gets no data (never idleness).

CA: :func:`ensure_ca` keeps it in a Secret only the signer reads and publishes the trust
bundle (current + previous CA during a rotation) in a ConfigMap the culler mounts.
"""

from __future__ import annotations

import asyncio
import base64
import ipaddress
import logging
import os
import secrets
import subprocess
import tempfile
import time
from dataclasses import dataclass
from typing import Optional, Tuple

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_not_found
from ..runtime.controller import Request, Result
from ..webhook.certs import cert_matches_key, cert_not_after, cert_sans, generate_ca

log = logging.getLogger("nodeagent.identity")

SIGNER_NAME = "amd.com/mi355x-node-agent"
IDENTITY_DOMAIN = "mi355x-node-agent.nodes"
CN_PREFIX = "system:node-agent:"
# user-info extras kube-apiserver derives from a bound (projected) service account token
POD_NAME_EXTRA = "authentication.kubernetes.io/pod-name"
POD_UID_EXTRA = "authentication.kubernetes.io/pod-uid"
NODE_NAME_EXTRA = "authentication.kubernetes.io/node-name"
ALLOWED_USAGES = frozenset({"digital signature", "key encipherment", "server auth"})
LEAF_VALIDITY_S = 7 * 86400
CA_VALIDITY_DAYS = 3650
# the node key's mode: owner (the enrollment containers' uid) + the pod's fsGroup (the agent)
KEY_FILE_MODE = 0o640


def server_name(node: str, domain: str = IDENTITY_DOMAIN) -> str:
    """The DNS name an agent's certificate carries for ``node`` (the culler's TLS server name)."""
    return f"{node}.{domain}"


def _openssl(args, data: Optional[bytes] = None) -> bytes:
    return subprocess.run(["openssl", *args], input=data, check=True, capture_output=True).stdout


def _ip_norm(s: str) -> str:
    try:
        return ipaddress.ip_address(s.strip()).compressed
    except ValueError:
        return s.strip()


def _san_entry(host: str) -> str:
    try:
        ipaddress.ip_address(host)
        return f"IP:{host}"
    except ValueError:
        return f"DNS:{host}"


def new_key_and_csr(node: str, host_ip: str, domain: str = IDENTITY_DOMAIN) -> Tuple[str, str]:
    """A fresh P-256 key and a CSR for this node's agent identity (PEM strings)."""
    with tempfile.TemporaryDirectory(prefix="odh-agent-csr-") as d:
        key = os.path.join(d, "tls.key")
        _openssl(["ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", key])
        sans = ",".join([_san_entry(server_name(node, domain))] + ([_san_entry(host_ip)] if host_ip else []))
        csr = _openssl(["req", "-new", "-key", key, "-subj", f"/CN={CN_PREFIX}{node}",
                        "-addext", f"subjectAltName={sans}"])
        with open(key) as f:
            return f.read(), csr.decode()


@dataclass
class CsrFacts:
    self_signed_ok: bool
    cn: str
    dns: frozenset
    ips: frozenset
    curve: str


def csr_facts(csr_pem: str) -> CsrFacts:
    """What a PEM CSR asks for, and whether its self-signature verifies (``openssl req``)."""
    data = csr_pem.encode()
    try:
        text = _openssl(["req", "-noout", "-text", "-verify"], data).decode(errors="replace")
        ok = True
    except subprocess.CalledProcessError as e:
        text = (e.stdout or b"").decode(errors="replace")
        ok = False
    cn, dns, ips, curve = "", set(), set(), ""
    lines = text.splitlines()
    for i, line in enumerate(lines):
        s = line.strip()
        if s.startswith("Subject:"):
            for part in s[len("Subject:"):].split(","):
                k, _, v = part.strip().partition("=")
                if k.strip() == "CN":
                    cn = v.strip()
        elif s.startswith("ASN1 OID:"):
            curve = s.split(":", 1)[1].strip()
        elif s.startswith("X509v3 Subject Alternative Name") and i + 1 < len(lines):
            for part in lines[i + 1].split(","):
                kind, _, val = part.strip().partition(":")
                if kind == "DNS":
                    dns.add(val.strip())
                elif kind == "IP Address":
                    ips.add(_ip_norm(val))
    return CsrFacts(ok, cn, frozenset(dns), frozenset(ips), curve)


def sign_leaf(csr_pem: str, ca_crt: str, ca_key: str, node: str, host_ip: str, validity_s: int,
              domain: str = IDENTITY_DOMAIN) -> str:
    """The agent's serving certificate: the CSR's key and subject, names from the verified pod."""
    days = max(1, int(-(-validity_s // 86400)))
    with tempfile.TemporaryDirectory(prefix="odh-agent-sign-") as d:
        paths = {n: os.path.join(d, n) for n in ("req.csr", "ca.crt", "ca.key", "ext")}
        for n, pem in (("req.csr", csr_pem), ("ca.crt", ca_crt), ("ca.key", ca_key)):
            with open(paths[n], "w") as f:
                f.write(pem)
        sans = ",".join([_san_entry(server_name(node, domain))] + ([_san_entry(host_ip)] if host_ip else []))
        with open(paths["ext"], "w") as f:
            f.write("basicConstraints=critical,CA:FALSE\nkeyUsage=critical,digitalSignature\n"
                    f"extendedKeyUsage=serverAuth\nsubjectAltName={sans}\n")
        out = _openssl(["x509", "-req", "-in", paths["req.csr"], "-CA", paths["ca.crt"], "-CAkey", paths["ca.key"],
                        "-set_serial", "0x" + secrets.token_hex(16), "-days", str(days), "-sha256",
                        "-extfile", paths["ext"]])
    return out.decode()


def _b64(s: str) -> str:
    return base64.b64encode(s.encode()).decode()


def _unb64(s: Optional[str]) -> str:
    return base64.b64decode(s or "").decode(errors="replace")


def _now_rfc3339() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


# ------------------------------------------------------------------ CA


async def ensure_ca(client, namespace: str, secret_name: str, configmap_name: str,
                    validity_days: int = CA_VALIDITY_DAYS, leaf_validity_s: int = LEAF_VALIDITY_S) -> Tuple[str, str]:
    """The signing CA (cert, key PEM), kept in Secret ``secret_name`` (``ca.crt`` / ``ca.key``);
    ConfigMap ``configmap_name`` (``ca.crt``) holds the bundle the culler trusts.  A CA that
    would not outlive a new leaf is replaced; the old one stays in the bundle (Secret key
    ``ca.previous.crt``) until it expires, so leaves it issued keep verifying until renewed."""
    now = time.time()
    try:
        sec = await client.get(kinds.SECRET, secret_name, namespace)
    except ApiError as e:
        if not is_not_found(e):
            raise
        sec = None
    data = (sec or {}).get("data") or {}
    crt, key, prev = _unb64(data.get("ca.crt")), _unb64(data.get("ca.key")), _unb64(data.get("ca.previous.crt"))
    exp = cert_not_after(crt) if crt else None
    if not (crt and key and exp and exp - now > 2 * leaf_validity_s and cert_matches_key(crt, key)):
        with tempfile.TemporaryDirectory(prefix="odh-agent-ca-") as d:
            generate_ca(d, validity_days)
            with open(os.path.join(d, "ca.crt")) as f:
                new_crt = f.read()
            with open(os.path.join(d, "ca.key")) as f:
                new_key = f.read()
        prev = crt if crt and exp and exp > now else ""
        crt, key = new_crt, new_key
        body = {"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                "metadata": {"name": secret_name, "namespace": namespace,
                             "labels": {"app.kubernetes.io/managed-by": "odh-node-agent-signer"}},
                "data": {"ca.crt": _b64(crt), "ca.key": _b64(key), **({"ca.previous.crt": _b64(prev)} if prev else {})}}
        if sec is None:
            await client.create(body)
        else:
            body["metadata"]["resourceVersion"] = sec["metadata"]["resourceVersion"]
            await client.update(body)
        log.info("node-agent CA %s in Secret %s/%s", "rotated" if prev else "created", namespace, secret_name)
    elif prev and (cert_not_after(prev) or 0) <= now:
        prev = ""  # the previous CA expired: every leaf it issued has too
        sec["data"].pop("ca.previous.crt", None)
        await client.update(sec)
    bundle = crt + (prev if prev and prev.strip() != crt.strip() else "")
    try:
        cm = await client.get(kinds.CONFIG_MAP, configmap_name, namespace)
    except ApiError as e:
        if not is_not_found(e):
            raise
        cm = None
    if cm is None:
        await client.create({"apiVersion": "v1", "kind": "ConfigMap",
                             "metadata": {"name": configmap_name, "namespace": namespace,
                                          "labels": {"app.kubernetes.io/managed-by": "odh-node-agent-signer"}},
                             "data": {"ca.crt": bundle}})
    elif (cm.get("data") or {}).get("ca.crt") != bundle:
        cm["data"] = {"ca.crt": bundle}
        await client.update(cm)
    return crt, key


# ------------------------------------------------------------------ signer


@dataclass
class SignerPolicy:
    namespace: str  # the agents' namespace
    service_account: str = "mi355x-node-agent"
    daemonset: str = "mi355x-node-agent"
    domain: str = IDENTITY_DOMAIN
    validity_s: int = LEAF_VALIDITY_S


class Denied(Exception):
    def __init__(self, reason: str, message: str):
        super().__init__(message)
        self.reason = reason


def _extra(spec: dict, key: str) -> Optional[str]:
    v = (spec.get("extra") or {}).get(key)
    if isinstance(v, list) and len(v) == 1 and isinstance(v[0], str) and v[0]:
        return v[0]
    return None


def _condition(csr: dict, ctype: str) -> Optional[dict]:
    for c in (csr.get("status") or {}).get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


class NodeAgentSigner:
    """Approves, signs or denies the node agents' CSRs (signer :data:`SIGNER_NAME`)."""

    NAME = "node-agent-signer"

    def __init__(self, client, policy: SignerPolicy, ca_crt: str, ca_key: str):
        self.client = client
        self.policy = policy
        self.ca_crt = ca_crt
        self.ca_key = ca_key
        self.issued = 0
        self.denied = 0

    async def verify(self, csr: dict) -> Tuple[str, str]:
        """``(node, hostIP)`` the request may have a certificate for; raises :class:`Denied`."""
        p = self.policy
        spec = csr.get("spec") or {}
        want_user = f"system:serviceaccount:{p.namespace}:{p.service_account}"
        if spec.get("username") != want_user:
            raise Denied("NotNodeAgent", f"requested by {spec.get('username')!r}, not {want_user}")
        pod_name, pod_uid = _extra(spec, POD_NAME_EXTRA), _extra(spec, POD_UID_EXTRA)
        if not pod_name or not pod_uid:
            raise Denied("NoPodBinding", "the requester's token is not bound to a pod (use a projected "
                                         "service account token)")
        try:
            pod = await self.client.get(kinds.POD, pod_name, p.namespace)
        except ApiError as e:
            if is_not_found(e):
                raise Denied("PodGone", f"pod {p.namespace}/{pod_name} does not exist")
            raise
        if m.uid(pod) != pod_uid or m.is_deleting(pod):
            raise Denied("PodGone", f"pod {p.namespace}/{pod_name} ({pod_uid}) is gone or terminating")
        owner = next((r for r in (pod.get("metadata") or {}).get("ownerReferences") or [] if r.get("controller")), None)
        if not owner or owner.get("kind") != "DaemonSet" or owner.get("name") != p.daemonset:
            raise Denied("NotNodeAgent", f"pod {pod_name} is not a pod of DaemonSet {p.daemonset}")
        # the owner reference names THE DaemonSet (its uid), not just one of that name: anyone
        # who may create pods under the agents' ServiceAccount could otherwise forge the
        # reference and set spec.nodeName to any node; and the pod matches its selector
        try:
            ds = await self.client.get(kinds.DAEMON_SET, p.daemonset, p.namespace)
        except ApiError as e:
            if is_not_found(e):
                raise Denied("NotNodeAgent", f"DaemonSet {p.namespace}/{p.daemonset} does not exist")
            raise
        if not owner.get("uid") or owner.get("uid") != m.uid(ds):
            raise Denied("NotNodeAgent", f"pod {pod_name}'s owner reference is not DaemonSet "
                                         f"{p.daemonset} ({m.uid(ds)})")
        sel = ((ds.get("spec") or {}).get("selector") or {}).get("matchLabels") or {}
        labels = m.labels(pod)
        if not sel or any(labels.get(k) != v for k, v in sel.items()):
            raise Denied("NotNodeAgent", f"pod {pod_name} does not match DaemonSet {p.daemonset}'s selector")
        node = (pod.get("spec") or {}).get("nodeName") or ""
        host_ip = (pod.get("status") or {}).get("hostIP") or ""
        if not node:
            raise Denied("NotScheduled", f"pod {pod_name} has no node")
        token_node = _extra(spec, NODE_NAME_EXTRA)
        if token_node is not None and token_node != node:
            raise Denied("NodeMismatch", f"token bound to node {token_node}, pod runs on {node}")
        usages = set(spec.get("usages") or [])
        if "server auth" not in usages or not usages <= ALLOWED_USAGES:
            raise Denied("BadUsages", f"usages {sorted(usages)}: server auth only")
        facts = csr_facts(_unb64(spec.get("request")))
        if not facts.self_signed_ok:
            raise Denied("BadRequest", "the request's self-signature does not verify")
        if facts.curve != "prime256v1":
            raise Denied("BadRequest", f"key type {facts.curve or 'non-EC'}: P-256 only")
        if facts.cn != CN_PREFIX + node:
            raise Denied("NodeMismatch", f"CN {facts.cn!r} for a pod on node {node}")
        if facts.dns != {server_name(node, p.domain)} or not facts.ips <= ({_ip_norm(host_ip)} if host_ip else set()):
            raise Denied("NodeMismatch", f"names {sorted(facts.dns | facts.ips)} for a pod on node {node} "
                                         f"({host_ip or 'no hostIP'})")
        return node, host_ip

    async def reconcile(self, req: Request) -> Result:
        try:
            csr = await self.client.get(kinds.CSR, req.name)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            raise
        spec = csr.get("spec") or {}
        if spec.get("signerName") != SIGNER_NAME:
            return Result()
        status = csr.get("status") or {}
        if status.get("certificate") or _condition(csr, "Denied") or _condition(csr, "Failed"):
            return Result()
        if not self.ca_key:  # the CA is being loaded (the signer's first leader term)
            return Result(requeue_after=0.5)
        conditions = list(status.get("conditions") or [])
        try:
            node, host_ip = await self.verify(csr)
        except Denied as d:
            self.denied += 1
            log.warning("denied node-agent CSR %s: %s (%s)", req.name, d, d.reason)
            conditions.append({"type": "Denied", "status": "True", "reason": d.reason, "message": str(d),
                               "lastUpdateTime": _now_rfc3339()})
            await self.client.patch(kinds.CSR, {"metadata": {"resourceVersion": m.resource_version(csr)},
                                                "status": {"conditions": conditions}},
                                    name=req.name, subresource="approval")
            return Result()
        if not _condition(csr, "Approved"):
            conditions.append({"type": "Approved", "status": "True", "reason": "NodeAgentPodVerified",
                               "message": f"agent pod on node {node}", "lastUpdateTime": _now_rfc3339()})
            csr = await self.client.patch(kinds.CSR, {"metadata": {"resourceVersion": m.resource_version(csr)},
                                                      "status": {"conditions": conditions}},
                                          name=req.name, subresource="approval")
        validity = self.policy.validity_s
        if spec.get("expirationSeconds"):
            validity = min(validity, max(600, int(spec["expirationSeconds"])))
        pem = await asyncio.to_thread(sign_leaf, _unb64(spec.get("request")), self.ca_crt, self.ca_key, node,
                                      host_ip, validity, self.policy.domain)
        await self.client.patch(kinds.CSR, {"status": {"certificate": _b64(pem)}}, name=req.name,
                                subresource="status")
        self.issued += 1
        log.info("issued node-agent certificate for node %s (%s) from CSR %s", node, host_ip, req.name)
        return Result()

    def setup_with_manager(self, mgr):
        from ..runtime.controller import pred_funcs

        mine = pred_funcs(create=lambda o: (o.get("spec") or {}).get("signerName") == SIGNER_NAME,
                          update=lambda o, old: (o.get("spec") or {}).get("signerName") == SIGNER_NAME,
                          delete=lambda o: False)
        return mgr.builder().named(self.NAME).for_(kinds.CSR, [mine]).complete(self)


# ------------------------------------------------------------------ agent side


class EnrollmentDenied(Exception):
    pass


class Enroller:
    """Keeps ``cert_dir/tls.key`` + ``tls.crt`` a valid identity for this node: a new key and
    CSR whenever the certificate is missing, names another node / IP, or is within
    ``renew_before_s`` of expiry (the agent's :class:`~odh_kubeflow_amd.utils.tlsreload.ServingCert`
    reloads the pair)."""

    def __init__(self, client, cert_dir: str, node: str, host_ip: str, domain: str = IDENTITY_DOMAIN,
                 renew_before_s: float = LEAF_VALIDITY_S / 3, expiration_s: int = LEAF_VALIDITY_S,
                 poll_s: float = 0.5):
        self.client = client
        self.cert_dir = cert_dir
        self.node = node
        self.host_ip = host_ip
        self.domain = domain
        self.renew_before_s = renew_before_s
        self.expiration_s = expiration_s
        self.poll_s = poll_s
        self.requests = 0

    def _files(self) -> Tuple[str, str]:
        return os.path.join(self.cert_dir, "tls.crt"), os.path.join(self.cert_dir, "tls.key")

    def current_ok(self) -> bool:
        crt_path, key_path = self._files()
        try:
            with open(crt_path) as f:
                crt = f.read()
            with open(key_path) as f:
                key = f.read()
        except OSError:
            return False
        exp = cert_not_after(crt)
        want = {server_name(self.node, self.domain)} | ({_ip_norm(self.host_ip)} if self.host_ip else set())
        return bool(exp and exp - time.time() > self.renew_before_s and cert_matches_key(crt, key)
                    and {_ip_norm(x) for x in cert_sans(crt) or ()} == want)

    def _write(self, key: str, crt: str) -> None:
        os.makedirs(self.cert_dir, exist_ok=True)
        crt_path, key_path = self._files()
        # the key first, each file replaced atomically: a reader sees the old pair, a new key
        # with the old cert (refused by ServingCert's pair check, retried), or the new pair.
        # The key is group-readable for the pod's fsGroup: the agent container reads it as
        # another uid with every capability dropped (no CAP_DAC_OVERRIDE), as a member of
        # that group (deploy/manifests.py node_agent_daemonset)
        dir_gid = os.stat(self.cert_dir).st_gid
        for path, pem, mode in ((key_path, key, KEY_FILE_MODE), (crt_path, crt, 0o644)):
            fd, tmp = tempfile.mkstemp(dir=self.cert_dir, prefix=".tmp-")
            with os.fdopen(fd, "w") as f:
                f.write(pem)
            if os.stat(tmp).st_gid != dir_gid:  # no setgid directory: hand it to the volume's group
                try:
                    os.chown(tmp, -1, dir_gid)
                except OSError:
                    pass  # not a member: the mode still serves a same-uid reader
            os.chmod(tmp, mode)
            os.replace(tmp, path)

    async def ensure(self, timeout_s: float = 300.0) -> str:
        """``"kept"`` or ``"issued"``; raises :class:`EnrollmentDenied` / TimeoutError."""
        if await asyncio.to_thread(self.current_ok):
            return "kept"
        key, csr_pem = await asyncio.to_thread(new_key_and_csr, self.node, self.host_ip, self.domain)
        obj = {"apiVersion": "certificates.k8s.io/v1", "kind": "CertificateSigningRequest",
               "metadata": {"generateName": f"node-agent-{self.node}-"[:200]},
               "spec": {"request": _b64(csr_pem), "signerName": SIGNER_NAME, "expirationSeconds": self.expiration_s,
                        "usages": ["digital signature", "server auth"]}}
        self.requests += 1
        created = await self.client.create(obj)
        name = m.name(created)
        deadline = time.monotonic() + timeout_s
        while True:
            csr = await self.client.get(kinds.CSR, name)
            st = csr.get("status") or {}
            for c in st.get("conditions") or []:
                if c.get("type") in ("Denied", "Failed"):
                    raise EnrollmentDenied(f"CSR {name}: {c.get('reason')}: {c.get('message')}")
            if st.get("certificate"):
                crt = _unb64(st["certificate"])
                if not cert_matches_key(crt, key):
                    raise EnrollmentDenied(f"CSR {name}: the issued certificate is not for this key")
                self._write(key, crt)
                log.info("node-agent certificate for %s issued (CSR %s)", self.node, name)
                return "issued"
            if time.monotonic() > deadline:
                raise TimeoutError(f"CSR {name} not signed within {timeout_s:.0f} s")
            await asyncio.sleep(self.poll_s)
