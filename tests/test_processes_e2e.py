"""Multi-process e2e: the deployable processes wired like the reference's kind CI
(.github/workflows/odh_notebook_controller_integration_test.yaml:102-284): dev apiserver
(+ StatefulSet controller / scheduler / GC), kf manager, odh manager with its HTTPS
webhook registered through a MutatingWebhookConfiguration carrying a self-signed
caBundle, a dev kubelet stand-in (``cmd/fake_kubelet.py``, writing the device-plugin
checkpoint) and the production MI355X node agent (``cmd/node_agent.py``, read-only).
Create a notebook with inject-auth, wait for the pod to be Ready, check the agent
attributes the pod's GPU from the checkpoint, delete it and check the cluster-scoped
leftovers are gone."""

import asyncio
import os
import socket
import subprocess
import sys
import time

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(args, env_extra=None, log=None):
    env = dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {}))
    return subprocess.Popen([sys.executable, "-m", *args], cwd=ROOT, env=env, stdout=log or subprocess.DEVNULL,
                            stderr=subprocess.STDOUT)


async def wait_http(url: str, timeout: float = 30.0) -> None:
    import aiohttp

    deadline = time.monotonic() + timeout
    async with aiohttp.ClientSession() as s:
        while time.monotonic() < deadline:
            try:
                async with s.get(url, ssl=False) as r:
                    if r.status == 200:
                        return
            except Exception:
                pass
            await asyncio.sleep(0.1)
    raise TimeoutError(url)


async def eventually(fn, timeout=30.0, interval=0.1):
    deadline = time.monotonic() + timeout
    last = None
    while time.monotonic() < deadline:
        try:
            last = await fn()
            if last:
                return last
        except Exception as e:  # noqa: BLE001
            last = e
        await asyncio.sleep(interval)
    raise AssertionError(f"condition not met: {last!r}")


def test_processes_end_to_end(tmp_path, run):
    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    api_port, wh_port = free_port(), free_port()
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    try:
        async def go():
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            for ns in ("opendatahub", "user"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}
            procs.append(spawn(["odh_kubeflow_amd.cmd.kf_manager", "--master", master, "--metrics-addr", "0",
                                "--probe-addr", "0", "--enable-leader-election"], common, logf))
            procs.append(spawn(["odh_kubeflow_amd.cmd.odh_manager", "--master", master, "--metrics-bind-address", "0",
                                "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                                "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", certs.cert_dir,
                                "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1", "--leader-elect"],
                               common, logf))
            from odh_kubeflow_amd.ops.telemetry import write_fake_sysfs

            sysfs, cp = str(tmp_path / "sys"), str(tmp_path / "dp" / "kubelet_internal_checkpoint")
            write_fake_sysfs(sysfs, gpus=8)
            agent_port = free_port()
            procs.append(spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", master, "--devices",
                                "0,1,2,3,4,5,6,7", "--sysfs-root", sysfs, "--checkpoint-path", cp], common, logf))
            procs.append(spawn(["odh_kubeflow_amd.cmd.node_agent", "--insecure", "--bind", "127.0.0.1",
                                "--port", str(agent_port),
                                "--sysfs-root", sysfs, "--proc-root", "", "--pod-resources-socket", "",
                                "--device-plugin-checkpoint", cp], None, logf))
            await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
            await c.create(mutating_webhook_configuration(
                certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh_port}/mutate-notebook-v1"))
            await eventually(lambda: c.get(kinds.NODE, "mi355x-node-0"))
            t0 = time.monotonic()
            await c.create(notebook("nb", "user", gpus=1, annotations={"notebooks.opendatahub.io/inject-auth": "true"}))

            async def ready():
                nb = await c.get(kinds.NOTEBOOK, "nb", "user")
                st = nb.get("status") or {}
                return st.get("readyReplicas") == 1 and any(
                    x.get("type") == "Ready" and x.get("status") == "True" for x in st.get("conditions") or [])

            await eventually(ready, 60)
            dt = time.monotonic() - t0
            nb = await c.get(kinds.NOTEBOOK, "nb", "user")
            assert [x["name"] for x in nb["spec"]["template"]["spec"]["containers"]] == ["nb", "kube-rbac-proxy"]
            assert "kubeflow-resource-stopped" not in m.annotations(nb)
            pod = await c.get(kinds.POD, "nb-0", "user")
            assert m.annotations(pod)["amd.com/gpu-ids"] == "0"
            import json as _json
            import urllib.request

            from odh_kubeflow_amd.ops.telemetry import fake_bdf

            def activity():
                url = f"http://127.0.0.1:{agent_port}/gpu/activity?pod_uid={m.uid(pod)}&window=5"
                with urllib.request.urlopen(url, timeout=5) as r:
                    return _json.loads(r.read())
            act = await asyncio.to_thread(activity)
            assert act["attributed"] and act["devices"] == [fake_bdf(0)] and act["sources"] == ["checkpoint"]
            routes = await c.list(kinds.HTTP_ROUTE, "opendatahub")
            assert [m.name(r) for r in routes] == ["nb-user-nb"]
            leases = {m.name(x) for x in await c.list(kinds.LEASE, "opendatahub")}
            assert {"kubeflow-notebook-controller", "odh-notebook-controller"} <= leases
            await c.delete(kinds.NOTEBOOK, "nb", "user")

            async def gone():
                try:
                    await c.get(kinds.NOTEBOOK, "nb", "user")
                    return False
                except Exception:
                    return True

            await eventually(gone, 30)
            crbs = [m.name(x) for x in await c.list(kinds.CLUSTER_ROLE_BINDING)]
            assert "nb-rbac-user-auth-delegator" not in crbs
            await c.close()
            return dt

        dt = run(go(), timeout=120)
        assert dt < 30
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        logf.close()


def test_processes_notebook_lifecycle_like_reference_e2e(tmp_path, run):
    """The odh/e2e sequence (notebook_creation_test.go, notebook_update_test.go,
    notebook_deletion_test.go) against separate processes: create with inject-auth →
    HTTPRoute, NetworkPolicies, StatefulSet 1/1, sidecar with default resources → the
    notebook's Jupyter API answers → idle culling stops it (STS scaled to 0) → resume
    with a new image rolls the StatefulSet → delete removes every dependent."""
    import aiohttp

    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    api_port, wh_port = free_port(), free_port()
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    try:
        async def go():
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            for ns in ("opendatahub", "e2e"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}
            culling = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME_SECONDS": "2.5",
                       "IDLENESS_CHECK_PERIOD_SECONDS": "0.3", "CULLER_USE_POD_ENDPOINT": "true"}
            procs.append(spawn(["odh_kubeflow_amd.cmd.kf_manager", "--master", master, "--metrics-addr", "0",
                                "--probe-addr", "0"], {**common, **culling}, logf))
            procs.append(spawn(["odh_kubeflow_amd.cmd.odh_manager", "--master", master, "--metrics-bind-address", "0",
                                "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                                "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", certs.cert_dir,
                                "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1"], common, logf))
            procs.append(spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", master, "--jupyter",
                                "--checkpoint-path", str(tmp_path / "dp" / "cp")], common, logf))
            await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
            await c.create(mutating_webhook_configuration(
                certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh_port}/mutate-notebook-v1"))
            await eventually(lambda: c.get(kinds.NODE, "mi355x-node-0"))
            await c.create(notebook("e2e-nb", "e2e", gpus=1, image="rocm/pytorch:latest",
                                    annotations={"notebooks.opendatahub.io/inject-auth": "true"}))

            async def ready():
                nb = await c.get(kinds.NOTEBOOK, "e2e-nb", "e2e")
                st = nb.get("status") or {}
                return st.get("readyReplicas") == 1 and any(
                    x.get("type") == "Ready" and x.get("status") == "True" for x in st.get("conditions") or [])

            await eventually(ready, 60)
            # creation checks (notebook_creation_test.go)
            assert [m.name(r) for r in await c.list(kinds.HTTP_ROUTE, "opendatahub")] == ["nb-e2e-e2e-nb"]
            nps = {m.name(x) for x in await c.list(kinds.NETWORK_POLICY, "e2e")}
            assert nps == {"e2e-nb-ctrl-np", "e2e-nb-kube-rbac-proxy-np"}
            sts = await c.get(kinds.STATEFUL_SET, "e2e-nb", "e2e")
            assert sts["spec"]["replicas"] == 1 and (sts.get("status") or {}).get("readyReplicas") == 1
            proxy = [x for x in sts["spec"]["template"]["spec"]["containers"] if x["name"] == "kube-rbac-proxy"][0]
            assert proxy["resources"] == {"requests": {"cpu": "100m", "memory": "64Mi"},
                                          "limits": {"cpu": "100m", "memory": "64Mi"}}
            # the notebook server answers (service connectivity)
            pod = await c.get(kinds.POD, "e2e-nb-0", "e2e")
            ep = m.annotations(pod)["amd.com/notebook-endpoint"]
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://{ep}/notebook/e2e/e2e-nb/api/kernels") as r:
                    assert r.status == 200 and await r.json() == []

            # culling (notebook_creation_test.go :417-518): idle → STOP annotation → 0 replicas
            async def culled():
                nb = await c.get(kinds.NOTEBOOK, "e2e-nb", "e2e")
                stop = m.annotations(nb).get("kubeflow-resource-stopped")
                s = await c.get(kinds.STATEFUL_SET, "e2e-nb", "e2e")
                return stop and stop != "odh-notebook-controller-lock" and s["spec"]["replicas"] == 0
            await eventually(culled, 30)

            # a stopped notebook loses its activity annotations on the culler's next pass
            # (culling_controller.go:104-117) — that pass follows the STOP write, so wait for it
            async def stripped():
                nb = await c.get(kinds.NOTEBOOK, "e2e-nb", "e2e")
                return "notebooks.kubeflow.org/last-activity" not in m.annotations(nb)
            await eventually(stripped, 30)
            nb = await c.get(kinds.NOTEBOOK, "e2e-nb", "e2e")

            # update (notebook_update_test.go): resume with a new image → STS rolls
            nb["metadata"]["annotations"].pop("kubeflow-resource-stopped")
            nb["spec"]["template"]["spec"]["containers"][0]["image"] = "rocm/pytorch:updated"
            await c.update(nb)

            async def rolled():
                s = await c.get(kinds.STATEFUL_SET, "e2e-nb", "e2e")
                img = s["spec"]["template"]["spec"]["containers"][0]["image"]
                return s["spec"]["replicas"] == 1 and img == "rocm/pytorch:updated" and \
                    (s.get("status") or {}).get("readyReplicas") == 1
            await eventually(rolled, 30)

            # deletion (notebook_deletion_test.go): every dependent goes
            await c.delete(kinds.NOTEBOOK, "e2e-nb", "e2e")

            async def all_gone():
                left = []
                for k, n, ns in ((kinds.NOTEBOOK, "e2e-nb", "e2e"), (kinds.STATEFUL_SET, "e2e-nb", "e2e"),
                                 (kinds.SERVICE, "e2e-nb", "e2e"), (kinds.SERVICE, "e2e-nb-kube-rbac-proxy", "e2e"),
                                 (kinds.SERVICE_ACCOUNT, "e2e-nb", "e2e"),
                                 (kinds.CONFIG_MAP, "e2e-nb-kube-rbac-proxy-config", "e2e"),
                                 (kinds.NETWORK_POLICY, "e2e-nb-ctrl-np", "e2e"),
                                 (kinds.HTTP_ROUTE, "nb-e2e-e2e-nb", "opendatahub"),
                                 (kinds.CLUSTER_ROLE_BINDING, "e2e-nb-rbac-e2e-auth-delegator", None)):
                    try:
                        await c.get(k, n, ns)
                        left.append(n)
                    except Exception:
                        pass
                return not left
            await eventually(all_gone, 30)
            await c.close()

        run(go(), timeout=150)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        logf.close()


def test_kf_manager_leader_failover(tmp_path, run):
    """HA (kf/main.go:91-93 leader election): two kf managers, short leases; SIGKILL the leader
    (no graceful release) — the standby acquires the expired Lease and reconciles new work."""
    api_port = free_port()
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    managers = {}
    try:
        async def go():
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            for ns in ("opendatahub", "user"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            for name in ("kf-a", "kf-b"):
                managers[name] = spawn(["odh_kubeflow_amd.cmd.kf_manager", "--master", master, "--metrics-addr", "0",
                                        "--probe-addr", "0", "--enable-leader-election",
                                        "--leader-election-lease-duration", "2",
                                        "--leader-election-renew-deadline", "1.5",
                                        "--leader-election-retry-period", "0.2"],
                                       {"K8S_NAMESPACE": "opendatahub", "POD_NAME": name}, logf)
                procs.append(managers[name])

            async def holder():
                lease = await c.get(kinds.LEASE, "kubeflow-notebook-controller", "opendatahub")
                h = (lease.get("spec") or {}).get("holderIdentity") or ""
                return h.split("_")[0] if h else None

            first = await eventually(holder, 30)
            await c.create(notebook("nb1", "user"))
            await eventually(lambda: c.get(kinds.STATEFUL_SET, "nb1", "user"), 30)
            t_kill = time.monotonic()
            managers[first].kill()  # SIGKILL: the lease is not released, it has to expire
            managers[first].wait(10)
            await c.create(notebook("nb2", "user"))
            await eventually(lambda: c.get(kinds.STATEFUL_SET, "nb2", "user"), 30)
            takeover = time.monotonic() - t_kill
            second = await holder()
            lease = await c.get(kinds.LEASE, "kubeflow-notebook-controller", "opendatahub")
            await c.close()
            return first, second, lease["spec"].get("leaseTransitions", 0), takeover

        first, second, transitions, takeover = run(go(), timeout=90)
        assert second != first and {first, second} == {"kf-a", "kf-b"}
        assert transitions >= 1
        assert takeover < 15  # lease 2 s + retry 0.2 s + reconcile
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        logf.close()


def test_sharded_control_plane_processes(tmp_path, run):
    """The mi355x-sharded deployment as processes: two ``cmd/control_plane.py`` shards
    (each shard labels the unlabelled namespaces that hash to it), one MutatingWebhookConfiguration per shard plus
    the unassigned-namespace one, the dev apiserver and kubelet stand-in.  Notebooks in
    namespaces the assigner put on different shards both become Ready, each shard labels its
    own HTTPRoutes; with shard 1 down its namespace's admissions fail (failurePolicy Fail)
    while shard 0's keep working, and a restarted shard 1 picks its namespace up again."""
    from odh_kubeflow_amd.controllers.sharding import shard_for
    from odh_kubeflow_amd.models.errors import ApiError
    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    # two namespaces the assigner maps to different shards
    names = [f"team-{i}" for i in range(64)]
    ns0 = next(n for n in names if shard_for(n, 2) == "0")
    ns1 = next(n for n in names if shard_for(n, 2) == "1")
    api_port = free_port()
    wh = [free_port(), free_port()]
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}

    def shard(k):
        return spawn(["odh_kubeflow_amd.cmd.control_plane", "--master", master, "--shard", str(k), "--shard-count", "2",
                      "--assign-namespaces", "--metrics-bind-address", "0", "--health-probe-bind-address", "0",
                      "--kube-rbac-proxy-image", "quay.io/brancz/kube-rbac-proxy:v0.18.1",
                      "--webhook-cert-dir", certs.cert_dir, "--webhook-host", "127.0.0.1",
                      "--webhook-port", str(wh[k])], common, logf)

    try:
        async def go():
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "opendatahub"}})
            for k in (0, 1):
                sel = {"matchLabels": {"notebooks.amd.com/shard": str(k)}}
                await c.create(mutating_webhook_configuration(
                    certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh[k]}/mutate-notebook-v1",
                    name=f"notebook-webhook-shard-{k}", namespace_selector=sel))
            await c.create(mutating_webhook_configuration(
                certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh[0]}/mutate-notebook-v1",
                name="notebook-webhook-unassigned", namespace_selector={"matchExpressions": [
                    {"key": "notebooks.amd.com/shard", "operator": "DoesNotExist"}]}))
            procs.append(shard(0))
            procs.append(shard(1))
            procs.append(spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", master, "--devices",
                                "0,1,2,3,4,5,6,7"], common, logf))
            for k in (0, 1):
                await wait_http(f"https://127.0.0.1:{wh[k]}/healthz")
            for ns in (ns0, ns1):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})

            async def labelled():
                got = [m.labels(await c.get(kinds.NAMESPACE, ns)).get("notebooks.amd.com/shard") for ns in (ns0, ns1)]
                return got == ["0", "1"]
            await eventually(labelled, 30)  # the owning shard's assigner

            async def ready(ns, nm="nb"):
                st = (await c.get(kinds.NOTEBOOK, nm, ns)).get("status") or {}
                return st.get("readyReplicas") == 1 and any(
                    x.get("type") == "Ready" and x.get("status") == "True" for x in st.get("conditions") or [])

            for ns in (ns0, ns1):
                await c.create(notebook("nb", ns, gpus=1))
            for ns in (ns0, ns1):
                await eventually(lambda: ready(ns), 60)
            routes = {m.labels(r)["notebook-namespace"]: m.labels(r).get("notebooks.amd.com/shard")
                      for r in await c.list(kinds.HTTP_ROUTE, "opendatahub")}
            assert routes == {ns0: "0", ns1: "1"}

            # shard 1 down: its namespace is not admitted, shard 0's is
            procs[2].terminate()
            procs[2].wait(10)
            with pytest.raises(ApiError):
                await c.create(notebook("nb2", ns1))
            await c.create(notebook("nb2", ns0))
            await eventually(lambda: ready(ns0, "nb2"), 60)
            # back up: shard 1 serves its namespace again
            procs[2] = shard(1)
            await wait_http(f"https://127.0.0.1:{wh[1]}/healthz")
            await c.create(notebook("nb2", ns1))
            await eventually(lambda: ready(ns1, "nb2"), 60)
            await c.close()

        run(go(), timeout=240)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        logf.close()
