"""Webhook TLS outside OpenShift: serving-cert provisioning (Secret + caBundle, the step the
reference's kind CI does by hand, ``.github/workflows/odh_notebook_controller_integration_test.yaml:190-216``),
cert rotation without restart (controller-runtime certwatcher), and the odh manager
refusing to serve admission without a certificate."""

import asyncio
import base64
import os
import shutil
import ssl
import subprocess
import sys

from odh_kubeflow_amd.testing.apiserver.inprocess import in_process_manager
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.webhook.certs import cert_not_after, generate, provision
from odh_kubeflow_amd.webhook.server import WebhookServer, mutating_webhook_configuration

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MWC = "odh-notebook-controller-mutating-webhook-configuration"


def _served_cert(port: int) -> str:
    return ssl.get_server_certificate(("127.0.0.1", port))


def test_cert_rotation_without_restart(run, tmp_path):
    live = tmp_path / "certs"
    generate(("127.0.0.1",), str(live))

    async def go():
        srv = await WebhookServer(None, str(live), "127.0.0.1", 0, reload_interval=0.05).start()
        try:
            first = await asyncio.to_thread(_served_cert, srv.port)
            assert first.strip() == (live / "tls.crt").read_text().strip()
            # a half-rotated pair (new cert, old key) is rejected; the old pair keeps serving
            new = generate(("127.0.0.1",), str(tmp_path / "new"))
            shutil.copy(new.cert_file, live / "tls.crt.tmp")
            os.replace(live / "tls.crt.tmp", live / "tls.crt")
            await asyncio.sleep(0.2)
            assert srv.reloads == 0
            assert (await asyncio.to_thread(_served_cert, srv.port)) == first
            shutil.copy(new.key_file, live / "tls.key.tmp")
            os.replace(live / "tls.key.tmp", live / "tls.key")
            for _ in range(100):
                if srv.reloads:
                    break
                await asyncio.sleep(0.05)
            assert srv.reloads == 1
            second = await asyncio.to_thread(_served_cert, srv.port)
            assert second != first and second.strip() == open(new.cert_file).read().strip()
        finally:
            await srv.stop()
    run(go())


def test_provision_secret_and_ca_bundle(run):
    async def go():
        store = ObjectStore()
        cli = in_process_manager(store, name="certs").client
        await cli.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "opendatahub"}})
        mwc = mutating_webhook_configuration("", service_namespace="opendatahub", name=MWC)
        mwc["webhooks"][0]["clientConfig"].pop("caBundle")
        await cli.create(mwc)
        out = await provision(cli, "opendatahub", mwc_names=[MWC, "absent"])
        assert out == {"secret": "created", "ca": "new", "mwc": {MWC: "patched", "absent": "missing"}}
        sec = await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
        assert sec["type"] == "kubernetes.io/tls" and set(sec["data"]) == {"tls.crt", "tls.key", "ca.crt", "ca.key"}
        bundle = (await cli.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, MWC))["webhooks"][0]["clientConfig"]["caBundle"]
        assert bundle == sec["data"]["ca.crt"]
        crt = base64.b64decode(sec["data"]["tls.crt"]).decode()
        sans = subprocess.run(["openssl", "x509", "-noout", "-ext", "subjectAltName"], input=crt.encode(),
                              capture_output=True).stdout.decode()
        assert "DNS:odh-notebook-controller-webhook-service.opendatahub.svc" in sans
        assert cert_not_after(crt) is not None
        # idempotent
        assert await provision(cli, "opendatahub", mwc_names=[MWC]) == {"secret": "kept", "ca": "kept",
                                                                         "mwc": {MWC: "kept"}}
        # a cert inside the renewal window is reissued from the SAME CA: the caBundle does not move,
        # so the old leaf (still served until the pods reload) and the new one are both trusted
        out = await provision(cli, "opendatahub", mwc_names=[MWC], validity_days=30, renew_before_days=400)
        assert out == {"secret": "renewed", "ca": "kept", "mwc": {MWC: "kept"}}
        sec2 = await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
        assert sec2["data"]["tls.crt"] != sec["data"]["tls.crt"] and sec2["data"]["ca.crt"] == sec["data"]["ca.crt"]
        # a CA that would not outlive a new leaf is replaced; every caBundle trusts old + new first
        out = await provision(cli, "opendatahub", mwc_names=[MWC], validity_days=5000)
        assert out == {"secret": "rotated", "ca": "new", "mwc": {MWC: "patched"}}
        sec3 = await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
        old_ca, new_ca = (base64.b64decode(x["data"]["ca.crt"]).decode() for x in (sec2, sec3))
        assert base64.b64decode(sec3["data"]["ca.previous.crt"]).decode() == old_ca
        bundle = base64.b64decode((await cli.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, MWC))
                                  ["webhooks"][0]["clientConfig"]["caBundle"]).decode()
        assert new_ca in bundle and old_ca in bundle
        # within the grace period nothing changes; after it the old CA is dropped everywhere
        assert (await provision(cli, "opendatahub", mwc_names=[MWC], validity_days=30))["mwc"] == {MWC: "kept"}
        out = await provision(cli, "opendatahub", mwc_names=[MWC], validity_days=30, previous_ca_grace_s=0)
        assert out == {"secret": "kept", "ca": "kept", "mwc": {MWC: "patched"}}
        sec4 = await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
        assert "ca.previous.crt" not in sec4["data"]
        bundle = (await cli.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, MWC))["webhooks"][0]["clientConfig"]["caBundle"]
        assert bundle == sec4["data"]["ca.crt"]
    run(go())


def test_legacy_secret_without_ca_key_is_kept_then_migrated(run):
    """A Secret written before the CA key was kept (tls.crt/tls.key/ca.crt only) is left alone
    while its leaf is valid; its renewal makes a new CA, trusted next to the old one."""
    async def go():
        store = ObjectStore()
        cli = in_process_manager(store, name="certs").client
        await cli.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "opendatahub"}})
        mwc = mutating_webhook_configuration("", service_namespace="opendatahub", name=MWC)
        await cli.create(mwc)
        await provision(cli, "opendatahub", mwc_names=[MWC])
        sec = await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
        sec["data"].pop("ca.key")
        await cli.update(sec)
        rv = (await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub"))["metadata"][
            "resourceVersion"]
        assert await provision(cli, "opendatahub", mwc_names=[MWC]) == {"secret": "kept", "ca": "kept",
                                                                         "mwc": {MWC: "kept"}}
        assert (await cli.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub"))["metadata"][
            "resourceVersion"] == rv
        out = await provision(cli, "opendatahub", mwc_names=[MWC], renew_before_days=400)
        assert out == {"secret": "rotated", "ca": "new", "mwc": {MWC: "patched"}}
        bundle = base64.b64decode((await cli.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, MWC))
                                  ["webhooks"][0]["clientConfig"]["caBundle"]).decode()
        assert bundle.count("BEGIN CERTIFICATE") == 2
    run(go())


def test_odh_manager_exits_without_serving_cert(tmp_path):
    p = subprocess.run([sys.executable, "-m", "odh_kubeflow_amd.cmd.odh_manager", "--master", "http://127.0.0.1:9",
                        "--kube-rbac-proxy-image", "x", "--webhook-cert-dir", str(tmp_path / "empty")],
                       cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT, K8S_NAMESPACE="opendatahub"),
                       capture_output=True, timeout=60)
    assert p.returncode != 0
    assert b"webhook serving certificate missing" in p.stderr


def test_e2e_admission_after_provisioning(tmp_path, run):
    """Start with a caBundle-less MutatingWebhookConfiguration: creates fail closed
    (failurePolicy: Fail, untrusted/unreachable webhook).  Run the provisioner Job's
    program, let the 'kubelet' project the Secret into the manager's cert dir, start the odh
    manager: admission works (the reconciliation lock is injected)."""
    from odh_kubeflow_amd.models import meta as m
    from odh_kubeflow_amd.models.errors import ApiError
    from odh_kubeflow_amd.models.notebook import notebook
    from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig
    from tests.test_processes_e2e import free_port, spawn, wait_http

    api_port, wh_port = free_port(), free_port()
    master = f"http://127.0.0.1:{api_port}"
    logf = open(tmp_path / "procs.log", "wb")
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--no-openshift-apis"], log=logf)]
    try:
        async def go():
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            for ns in ("opendatahub", "user"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            mwc = mutating_webhook_configuration("", url=f"https://127.0.0.1:{wh_port}/mutate-notebook-v1", name=MWC)
            mwc["webhooks"][0]["clientConfig"].pop("caBundle")
            await c.create(mwc)
            try:
                await c.create(notebook("early", "user"))
                raise AssertionError("admission must fail closed without a trusted webhook")
            except ApiError as e:
                assert "failed calling webhook" in str(e)
            job = await asyncio.to_thread(subprocess.run, [
                sys.executable, "-m", "odh_kubeflow_amd.cmd.webhook_certs", "--master", master,
                "--namespace", "opendatahub", "--mwc-name", MWC, "--extra-host", "127.0.0.1"],
                cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, timeout=60)
            assert job.returncode == 0, job.stderr.decode()[-2000:]
            assert b'"secret": "created"' in job.stdout
            # the kubelet's Secret volume projection
            sec = await c.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
            cert_dir = tmp_path / "serving-certs"
            cert_dir.mkdir()
            for k in ("tls.crt", "tls.key", "ca.crt"):
                (cert_dir / k).write_bytes(base64.b64decode(sec["data"][k]))
            procs.append(spawn(["odh_kubeflow_amd.cmd.odh_manager", "--master", master, "--metrics-bind-address", "0",
                                "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                                "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", str(cert_dir),
                                "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1"],
                               {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}, logf))
            await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
            nb = await c.create(notebook("nb", "user"))
            assert m.annotations(nb).get("kubeflow-resource-stopped") == "odh-notebook-controller-lock"
            await c.close()
        run(go(), timeout=120)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        logf.close()


def test_provision_node_agent_token_secret(run):
    """cmd/webhook_certs --random-secret: the node agent / culler token Secret is created once
    with a random token and never rotated by a re-run (the agents would lose each other)."""
    from odh_kubeflow_amd.nodeagent.auth import TOKEN_SECRET, ensure_token_secret

    async def go():
        store = ObjectStore()
        cli = in_process_manager(store, name="certs").client
        await cli.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "opendatahub"}})
        assert await ensure_token_secret(cli, "opendatahub") == "created"
        sec = await cli.get(kinds.SECRET, TOKEN_SECRET, "opendatahub")
        tok = base64.b64decode(sec["data"]["token"])
        assert len(tok) >= 32
        assert await ensure_token_secret(cli, "opendatahub") == "kept"
        assert (await cli.get(kinds.SECRET, TOKEN_SECRET, "opendatahub"))["data"]["token"] == sec["data"]["token"]
        sec = await cli.get(kinds.SECRET, TOKEN_SECRET, "opendatahub")
        sec["data"] = {}
        await cli.update(sec)
        assert await ensure_token_secret(cli, "opendatahub") == "filled"
    run(go())


def test_admission_survives_cert_renewal_and_ca_rotation(tmp_path, run):
    """failurePolicy: Fail admission keeps working at every moment of a renewal and of a CA
    rotation: right after the provisioner wrote the Secret (the pod still serves the old leaf,
    the kubelet has not synced yet), after the pod reloaded the new files, and after the old CA
    left the caBundle."""
    from odh_kubeflow_amd.models import meta as m
    from odh_kubeflow_amd.models.notebook import notebook
    from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig
    from tests.test_processes_e2e import free_port, spawn, wait_http

    api_port, wh_port = free_port(), free_port()
    master = f"http://127.0.0.1:{api_port}"
    logf = open(tmp_path / "procs.log", "wb")
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--no-openshift-apis"],
                   log=logf)]
    cert_dir = tmp_path / "serving-certs"
    cert_dir.mkdir()
    try:
        async def go():
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            for ns in ("opendatahub", "user"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            mwc = mutating_webhook_configuration("", url=f"https://127.0.0.1:{wh_port}/mutate-notebook-v1", name=MWC)
            mwc["webhooks"][0]["clientConfig"].pop("caBundle")
            await c.create(mwc)

            async def kubelet_sync():  # the Secret volume projection (tls.crt / tls.key items)
                sec = await c.get(kinds.SECRET, "odh-notebook-controller-webhook-cert", "opendatahub")
                for k in ("tls.crt", "tls.key"):
                    (cert_dir / (k + ".new")).write_bytes(base64.b64decode(sec["data"][k]))
                for k in ("tls.key", "tls.crt"):
                    os.replace(cert_dir / (k + ".new"), cert_dir / k)
                return base64.b64decode(sec["data"]["tls.crt"]).decode()

            n = [0]

            async def admitted():
                n[0] += 1
                nb = await c.create(notebook(f"nb{n[0]}", "user"))
                assert m.annotations(nb).get("kubeflow-resource-stopped") == "odh-notebook-controller-lock"

            async def serving(pem):
                for _ in range(200):
                    if (await asyncio.to_thread(_served_cert, wh_port)).strip() == pem.strip():
                        return
                    await asyncio.sleep(0.05)
                raise AssertionError("webhook server did not reload the new serving cert")

            prov = dict(mwc_names=[MWC], extra_hosts=["127.0.0.1"])
            await provision(c, "opendatahub", **prov)
            await kubelet_sync()
            procs.append(spawn(["odh_kubeflow_amd.cmd.odh_manager", "--master", master, "--metrics-bind-address", "0",
                                "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                                "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", str(cert_dir),
                                "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1",
                                "--webhook-cert-reload-seconds", "0.1"],
                               {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}, logf))
            await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
            await admitted()
            # renewal: new leaf, same CA
            assert (await provision(c, "opendatahub", renew_before_days=400, **prov))["secret"] == "renewed"
            await admitted()  # the pod still serves the old leaf
            await serving(await kubelet_sync())
            await admitted()
            # CA rotation: old + new CA trusted, then the Secret
            assert (await provision(c, "opendatahub", validity_days=5000, renew_before_days=400, **prov))["ca"] == "new"
            await admitted()  # old leaf, old CA still in the bundle
            await serving(await kubelet_sync())
            await admitted()  # new leaf, new CA
            assert (await provision(c, "opendatahub", previous_ca_grace_s=0, **prov))["mwc"] == {MWC: "patched"}
            await admitted()  # old CA gone from the bundle
            await c.close()
        run(go(), timeout=180)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        logf.close()

