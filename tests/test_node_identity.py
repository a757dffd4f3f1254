"""Per-node node-agent identity (``nodeagent/identity.py``): agents enroll through
the CertificateSigningRequest API; the signer issues a certificate only for the node the
requesting agent pod runs on; the culler refuses node B's certificate answering for a pod on
node A.  The apiserver stand-in authenticates each bearer token to a user whose extras carry
the bound pod, as kube-apiserver does for projected service account tokens."""

from __future__ import annotations

import asyncio
import os

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.nodeagent import identity as ident
from odh_kubeflow_amd.runtime.manager import Manager
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig
from odh_kubeflow_amd.testing.apiserver.http import ApiServer
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.webhook.certs import cert_sans, cert_signed_by

NS = "opendatahub"
AGENT_SA = f"system:serviceaccount:{NS}:mi355x-node-agent"


def _agent_user(pod: str, uid: str, node: str = None) -> dict:
    extra = {ident.POD_NAME_EXTRA: [pod], ident.POD_UID_EXTRA: [uid]}
    if node:
        extra[ident.NODE_NAME_EXTRA] = [node]
    return {"username": AGENT_SA, "groups": ["system:serviceaccounts", "system:authenticated"], "extra": extra}


USERS = {
    "admin": {"username": "system:admin", "groups": ["system:masters"]},
    "agent-a": _agent_user("agent-a", "uid-a", "gpu-a"),
    "agent-b": _agent_user("agent-b", "uid-b", "gpu-b"),
    "stale-a": _agent_user("agent-a", "uid-old"),  # a token of an earlier pod of that name
    "unbound": {"username": AGENT_SA, "groups": ["system:serviceaccounts"]},  # a legacy Secret token
    "someone": {"username": "system:serviceaccount:team:default",
                "extra": {ident.POD_NAME_EXTRA: ["agent-a"], ident.POD_UID_EXTRA: ["uid-a"]}},
    "rogue-pod": _agent_user("rogue", "uid-r"),  # the agents' SA, but a pod nobody's DaemonSet owns
    "forged-pod": _agent_user("forged", "uid-f"),
    "unselected-pod": _agent_user("unselected", "uid-u"),
}


def _agent_pod(name, node, ip, owner="mi355x-node-agent", kind="DaemonSet", owner_uid="ds",
               labels=(("app", "mi355x-node-agent"),)):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": NS, "labels": dict(labels),
                         "ownerReferences": [{"apiVersion": "apps/v1", "kind": kind, "name": owner, "uid": owner_uid,
                                              "controller": True}]},
            "spec": {"nodeName": node, "containers": [{"name": "agent", "image": "i"}]},
            "status": {"hostIP": ip, "phase": "Running"}}


class _Cluster:
    """Python apiserver with the users above, the two agent pods and a rogue one, and the
    signer running — entered inside the test's own event loop."""

    def __init__(self, signer: bool = True):
        self.with_signer = signer

    async def __aenter__(self):
        import copy

        self.users = copy.deepcopy(USERS)
        self.srv = await ApiServer(ObjectStore(), users=self.users).start("127.0.0.1", 0)
        self.admin = RestClient(RestConfig(host=self.srv.url, token="admin"))
        await self.admin.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NS}})
        ds = await self.admin.create({
            "apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "mi355x-node-agent", "namespace": NS},
            "spec": {"selector": {"matchLabels": {"app": "mi355x-node-agent"}},
                     "template": {"metadata": {"labels": {"app": "mi355x-node-agent"}},
                                  "spec": {"containers": [{"name": "agent", "image": "i"}]}}}})
        uids = {}
        ds_uid = ds["metadata"]["uid"]
        for pod in (_agent_pod("agent-a", "gpu-a", "10.0.0.1", owner_uid=ds_uid),
                    _agent_pod("agent-b", "gpu-b", "10.0.0.2", owner_uid=ds_uid),
                    _agent_pod("rogue", "gpu-a", "10.0.0.1", owner="debug", kind="ReplicaSet"),
                    # a pod of the agents' SA with a forged owner reference (right kind and name)
                    _agent_pod("forged", "gpu-a", "10.0.0.1", owner_uid="not-the-daemonset"),
                    # ... or with the right one but outside the DaemonSet's selector
                    _agent_pod("unselected", "gpu-a", "10.0.0.1", owner_uid=ds_uid, labels=())):
            uids[pod["metadata"]["name"]] = (await self.admin.create(pod))["metadata"]["uid"]
        # the tokens' bound-pod uids are the live pods' (the stand-in assigns uids on create)
        for tok, pod in (("agent-a", "agent-a"), ("agent-b", "agent-b"), ("rogue-pod", "rogue"),
                         ("someone", "agent-a"), ("forged-pod", "forged"), ("unselected-pod", "unselected")):
            self.users[tok]["extra"][ident.POD_UID_EXTRA] = [uids[pod]]
        self.mgr = None
        if self.with_signer:
            self.mgr = Manager.remote(RestConfig(host=self.srv.url, token="admin"), name="signer",
                                      uncached=(kinds.POD, kinds.DAEMON_SET))
            self.ca, key = await ident.ensure_ca(self.mgr.client, NS, "agent-ca", "agent-ca-bundle")
            self.signer = ident.NodeAgentSigner(self.mgr.client, ident.SignerPolicy(namespace=NS), self.ca, key)
            self.signer.setup_with_manager(self.mgr)
            await self.mgr.start()
        return self

    async def __aexit__(self, *exc):
        if self.mgr is not None:
            await self.mgr.stop()
        await self.admin.close()
        await self.srv.stop()


def _enroller(cl, token, node, ip, cert_dir):
    client = RestClient(RestConfig(host=cl.srv.url, token=token))
    return client, ident.Enroller(client, str(cert_dir), node, ip, poll_s=0.02)


async def _with_cluster(body, signer: bool = True):
    async with _Cluster(signer) as cl:
        return await body(cl)


def test_agent_enrolls_for_its_own_node(run, tmp_path):
    async def body(cl):
        client, e = _enroller(cl, "agent-a", "gpu-a", "10.0.0.1", tmp_path / "a")
        try:
            assert await e.ensure(10) == "issued"
            with open(tmp_path / "a" / "tls.crt") as f:
                crt = f.read()
            assert cert_sans(crt) == {"gpu-a.mi355x-node-agent.nodes", "10.0.0.1"}
            assert cert_signed_by(crt, cl.ca)
            # group-readable: the agent container reads it through the pod's fsGroup
            assert oct(os.stat(tmp_path / "a" / "tls.key").st_mode & 0o777) == "0o640"
            assert os.stat(tmp_path / "a" / "tls.key").st_gid == os.stat(tmp_path / "a").st_gid
            assert await e.ensure(10) == "kept" and e.requests == 1
            # the culler's trust bundle is published for it
            cm = await cl.admin.get(kinds.CONFIG_MAP, "agent-ca-bundle", NS)
            assert cm["data"]["ca.crt"].strip() == cl.ca.strip()
            csrs = await cl.admin.list(kinds.CSR)
            assert len(csrs) == 1 and csrs[0]["spec"]["username"] == AGENT_SA
            assert [c["type"] for c in csrs[0]["status"]["conditions"]] == ["Approved"]
        finally:
            await client.close()
    run(_with_cluster(body))


@pytest.mark.parametrize("token,node,ip,reason", [
    ("agent-b", "gpu-a", "10.0.0.1", "NodeMismatch"),  # node B's agent asking for node A's identity
    ("agent-a", "gpu-a", "10.0.0.9", "NodeMismatch"),  # the right node, another host's address
    ("someone", "gpu-a", "10.0.0.1", "NotNodeAgent"),  # not the agents' ServiceAccount
    ("unbound", "gpu-a", "10.0.0.1", "NoPodBinding"),  # a token not bound to a pod
    ("stale-a", "gpu-a", "10.0.0.1", "PodGone"),  # bound to a pod that no longer exists
    ("rogue-pod", "gpu-a", "10.0.0.1", "NotNodeAgent"),  # a pod of the agents' SA outside the DaemonSet
    ("forged-pod", "gpu-a", "10.0.0.1", "NotNodeAgent"),  # ownerReference names the DaemonSet, wrong uid
    ("unselected-pod", "gpu-a", "10.0.0.1", "NotNodeAgent"),  # not matched by the DaemonSet's selector
])
def test_signer_denies_what_the_requesting_pod_does_not_prove(run, tmp_path, token, node, ip, reason):
    async def body(cl):
        client, e = _enroller(cl, token, node, ip, tmp_path / "x")
        try:
            with pytest.raises(ident.EnrollmentDenied, match=reason):
                await e.ensure(10)
            assert not os.path.exists(tmp_path / "x" / "tls.crt")
            assert cl.signer.issued == 0 and cl.signer.denied == 1
        finally:
            await client.close()
    run(_with_cluster(body))


def test_requester_identity_comes_from_the_token_not_the_request(run):
    """A CSR that claims the agents' identity in its own spec is stamped with the real one."""
    async def body(cl):
        client = RestClient(RestConfig(host=cl.srv.url, token="someone"))
        try:
            _key, csr = ident.new_key_and_csr("gpu-a", "10.0.0.1")
            obj = await client.create({
                "apiVersion": "certificates.k8s.io/v1", "kind": "CertificateSigningRequest",
                "metadata": {"name": "forged"},
                "spec": {"request": ident._b64(csr), "signerName": ident.SIGNER_NAME,
                         "usages": ["digital signature", "server auth"], "username": AGENT_SA,
                         "extra": cl.users["agent-a"]["extra"]}})
            assert obj["spec"]["username"] == "system:serviceaccount:team:default"
            for _ in range(200):
                got = await client.get(kinds.CSR, "forged")
                if (got.get("status") or {}).get("conditions"):
                    break
                await asyncio.sleep(0.02)
            assert got["status"]["conditions"][0]["type"] == "Denied"
            assert not got["status"].get("certificate")
        finally:
            await client.close()
    run(_with_cluster(body))


def test_node_b_certificate_answering_for_node_a_is_refused(run, tmp_path):
    """VERDICT r4 #8 done-criterion, end to end: both agents enroll through the signer; node B's
    agent, with its valid certificate from the same CA, answers at the address the culler uses
    for a pod on node A — the culler gets no data; node A's agent is believed."""
    from odh_kubeflow_amd.controllers import culling as c
    from odh_kubeflow_amd.nodeagent.server import NodeTelemetryAgent

    class _NoGpus:  # telemetry of a node without GPUs: the handshake is what is tested
        def devices(self):
            return []

    async def body(cl):
        ca_file = tmp_path / "ca.crt"
        cm = await cl.admin.get(kinds.CONFIG_MAP, "agent-ca-bundle", NS)
        ca_file.write_text(cm["data"]["ca.crt"])
        agents, clients = [], []
        try:
            for tok, node, ip in (("agent-a", "gpu-a", "10.0.0.1"), ("agent-b", "gpu-b", "10.0.0.2")):
                client, e = _enroller(cl, tok, node, ip, tmp_path / node)
                clients.append(client)
                assert await e.ensure(10) == "issued"
                agents.append(await NodeTelemetryAgent(_NoGpus(), None, host="127.0.0.1", port=0,
                                                       tls_cert_dir=str(tmp_path / node)).start())
            a, b = agents
            pod_on_a = {"metadata": {"name": "nb-0", "namespace": "u", "uid": "p"}, "spec": {"nodeName": "gpu-a"},
                        "status": {"hostIP": "10.0.0.1"}}
            to_a = c.NodeAgentActivity(ca_file=str(ca_file), endpoint_for=lambda p: f"127.0.0.1:{a.port}")
            to_b = c.NodeAgentActivity(ca_file=str(ca_file), endpoint_for=lambda p: f"127.0.0.1:{b.port}")
            try:
                await to_a.busy(pod_on_a, 0.05)  # node A's own agent is asked, and answers
                assert a.queries == 1
                assert await to_b.busy(pod_on_a, 0.05) is None  # B's certificate: the handshake fails
                assert b.queries == 0  # nothing reached B's handler
            finally:
                await to_a.close()
                await to_b.close()
        finally:
            for x in agents:
                await x.stop()
            for client in clients:
                await client.close()
    run(_with_cluster(body))


def test_signer_and_enroll_commands(run, tmp_path, monkeypatch):
    """``cmd/node_agent_signer`` (CA created on start, only its signer's CSRs watched) and
    ``cmd/node_agent_enroll --once`` (the DaemonSet's init container) against the stand-in."""
    from odh_kubeflow_amd.cmd import node_agent_enroll, node_agent_signer

    async def body(cl):
        monkeypatch.setenv("KUBE_TOKEN", "admin")
        mgr = node_agent_signer.build(node_agent_signer.parse([
            "--master", cl.srv.url, "--namespace", NS, "--ca-secret", "cmd-ca", "--ca-configmap", "cmd-ca",
            "--metrics-bind-address", "0", "--health-probe-bind-address", "0"]))
        await mgr.start()
        try:
            # a CSR of another signer (a kubelet's) is not this signer's business
            _k, other = ident.new_key_and_csr("gpu-a", "10.0.0.1")
            await cl.admin.create({"apiVersion": "certificates.k8s.io/v1", "kind": "CertificateSigningRequest",
                                   "metadata": {"name": "kubelet-serving"},
                                   "spec": {"request": ident._b64(other), "usages": ["server auth"],
                                            "signerName": "kubernetes.io/kubelet-serving"}})
            monkeypatch.setenv("KUBE_TOKEN", "agent-b")
            rc = await node_agent_enroll.amain(["--master", cl.srv.url, "--node-name", "gpu-b", "--host-ip",
                                                "10.0.0.2", "--cert-dir", str(tmp_path / "b"), "--once",
                                                "--timeout-seconds", "20"])
            assert rc == 0 and mgr.signer.issued == 1
            with open(tmp_path / "b" / "tls.crt") as f:
                crt = f.read()
            assert cert_sans(crt) == {"gpu-b.mi355x-node-agent.nodes", "10.0.0.2"}
            cm = await cl.admin.get(kinds.CONFIG_MAP, "cmd-ca", NS)
            assert cert_signed_by(crt, cm["data"]["ca.crt"])
            kubelet = await cl.admin.get(kinds.CSR, "kubelet-serving")
            assert not (kubelet.get("status") or {}).get("conditions")
            # denied: --once exits non-zero and leaves no certificate
            rc = await node_agent_enroll.amain(["--master", cl.srv.url, "--node-name", "gpu-a", "--host-ip",
                                                "10.0.0.1", "--cert-dir", str(tmp_path / "x"), "--once",
                                                "--timeout-seconds", "20"])
            assert rc == 1 and not os.path.exists(tmp_path / "x" / "tls.crt")
        finally:
            await mgr.stop()
    run(_with_cluster(body, signer=False))
