"""Fault injection: the managers talk to the apiserver through a proxy that cuts every
open connection (watch streams, pooled request connections) at random moments.

The reference has no fault injection; controller-runtime's informers survive
dropped watches by re-watching from the last resourceVersion (relisting on 410 Gone) and
its clients retry.  Here the kf and odh managers (separate processes, HTTPS webhook) and the
dev kubelet run against a proxy that resets all their connections every 50–150 ms while
notebooks are created, become Ready, and are deleted: every notebook must still converge
both ways, with its dependents cleaned up."""

import asyncio
import os
import random
import time

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig

from test_processes_e2e import eventually, free_port, spawn, wait_http

pytestmark = pytest.mark.slow


class ChaosProxy:
    """TCP proxy that can drop every connection it carries."""

    def __init__(self, target_port: int):
        self.target_port = target_port
        self.pairs = set()
        self.cuts = 0
        self.aborted = 0  # connections cut while in use (watches, pooled requests)
        self.server = None
        self.port = None

    async def _pipe(self, r, w):
        try:
            while True:
                data = await r.read(65536)
                if not data:
                    break
                w.write(data)
                await w.drain()
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            w.close()

    async def _handle(self, cr, cw):
        try:
            sr, sw = await asyncio.open_connection("127.0.0.1", self.target_port)
        except OSError:
            cw.close()
            return
        pair = (cw, sw)
        self.pairs.add(pair)
        try:
            await asyncio.gather(self._pipe(cr, sw), self._pipe(sr, cw))
        finally:
            self.pairs.discard(pair)

    async def start(self):
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    def cut_all(self):
        for cw, sw in list(self.pairs):
            self.aborted += 1
            for w in (cw, sw):
                try:
                    w.transport.abort()
                except Exception:  # noqa: BLE001 — already closed
                    pass
        self.cuts += 1

    async def close(self):
        self.cut_all()
        self.server.close()
        await self.server.wait_closed()


async def diagnostics(c, names, ns="chaos") -> str:
    """What each notebook's chain looks like (the reference e2e's logNotebookDiagnostics)."""
    out = []
    for n in names:
        row = [n]
        try:
            nb = await c.get(kinds.NOTEBOOK, n, ns)
            row.append(f"ann={sorted((nb['metadata'].get('annotations') or {}).items())}")
            row.append(f"fin={nb['metadata'].get('finalizers')} status={nb.get('status')}")
        except Exception as e:  # noqa: BLE001
            row.append(f"notebook: {e!r}")
        for kind, name in ((kinds.STATEFUL_SET, n), (kinds.POD, f"{n}-0")):
            try:
                o = await c.get(kind, name, ns)
                row.append(f"{kind.split('/')[-1]}: spec.replicas={(o.get('spec') or {}).get('replicas')} "
                           f"node={(o.get('spec') or {}).get('nodeName')} status={o.get('status')}")
            except Exception as e:  # noqa: BLE001
                row.append(f"{kind.split('/')[-1]}: {e!r}")
        out.append(" | ".join(row))
    return "\n".join(out)


def test_managers_converge_through_connection_resets(tmp_path, run):
    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    api_port, wh_port = free_port(), free_port()
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    rnd = random.Random(11)

    async def go():
        await wait_http(master + "/healthz")
        proxy = await ChaosProxy(api_port).start()
        via = f"http://127.0.0.1:{proxy.port}"
        c = RestClient(RestConfig(host=master))
        for ns in ("opendatahub", "chaos"):
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}
        procs.append(spawn(["odh_kubeflow_amd.cmd.kf_manager", "--master", via, "--metrics-addr", "0",
                            "--probe-addr", "0"], common, logf))
        procs.append(spawn(["odh_kubeflow_amd.cmd.odh_manager", "--master", via, "--metrics-bind-address", "0",
                            "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                            "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", certs.cert_dir,
                            "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1"], common, logf))
        procs.append(spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", via, "--checkpoint-path",
                            str(tmp_path / "dp" / "cp")], common, logf))
        await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
        await c.create(mutating_webhook_configuration(
            certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh_port}/mutate-notebook-v1"))
        await eventually(lambda: c.get(kinds.NODE, "mi355x-node-0"))

        stop = asyncio.Event()

        async def chaos():
            while not stop.is_set():
                await asyncio.sleep(rnd.uniform(0.05, 0.15))
                proxy.cut_all()
        chaos_task = asyncio.create_task(chaos())
        names = [f"nb{i}" for i in range(5)]
        try:
            for n in names:
                await c.create(notebook(n, "chaos", gpus=1,
                                        annotations={"notebooks.opendatahub.io/inject-auth": "true"}))

            async def all_ready():
                for n in names:
                    st = (await c.get(kinds.NOTEBOOK, n, "chaos")).get("status") or {}
                    if st.get("readyReplicas") != 1:
                        return False
                return True
            try:
                await eventually(all_ready, 90)
            except AssertionError:
                raise AssertionError("not all Ready:\n" + await diagnostics(c, names))
            for n in names:
                await c.delete(kinds.NOTEBOOK, n, "chaos")

            async def all_gone():
                left = [n for n in names if any(x["metadata"]["name"] == n
                                                for x in await c.list(kinds.NOTEBOOK, "chaos"))]
                crbs = [x["metadata"]["name"] for x in await c.list(kinds.CLUSTER_ROLE_BINDING)
                        if x["metadata"]["name"].endswith("-chaos-auth-delegator")]
                routes = await c.list(kinds.HTTP_ROUTE, "opendatahub")
                return not left and not crbs and not routes
            await eventually(all_gone, 90)
        finally:
            stop.set()
            await chaos_task
            await proxy.close()
            await c.close()
        return proxy.aborted

    try:
        t0 = time.monotonic()
        aborted = run(go(), timeout=240)
        # the faults hit live connections (every manager's watches at each cut) while the
        # notebooks converged
        assert aborted >= 10, aborted
        assert time.monotonic() - t0 < 230
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except Exception:  # noqa: BLE001
                p.kill()
        logf.close()
        if os.environ.get("ODH_KEEP_LOGS"):
            print(open(tmp_path / "procs.log", "rb").read().decode(errors="replace")[-5000:])


def test_odh_manager_crash_mid_burst_recovers(tmp_path, run):
    """SIGKILL the odh manager (reconciler + webhook) while a burst of auth notebooks is being
    reconciled, start a new one: every notebook still converges (idempotent reconcile: no
    duplicate children, the one-write unlock happens once per notebook), and deletion
    cleans every cluster-scoped and central-namespace dependent."""
    import signal

    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    api_port, wh_port = free_port(), free_port()
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = {"api": spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                           "--no-openshift-apis"], log=logf)}
    common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}
    odh_args = ["odh_kubeflow_amd.cmd.odh_manager", "--master", master, "--metrics-bind-address", "0",
                "--health-probe-bind-address", "0", "--kube-rbac-proxy-image", "quay.io/brancz/kube-rbac-proxy:v0.18.1",
                "--webhook-cert-dir", certs.cert_dir, "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1"]

    async def go():
        await wait_http(master + "/healthz")
        c = RestClient(RestConfig(host=master))
        for ns in ("opendatahub", "crash"):
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        procs["kf"] = spawn(["odh_kubeflow_amd.cmd.kf_manager", "--master", master, "--metrics-addr", "0",
                             "--probe-addr", "0"], common, logf)
        procs["odh"] = spawn(odh_args, common, logf)
        procs["kubelet"] = spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", master, "--checkpoint-path",
                                  str(tmp_path / "dp" / "cp")], common, logf)
        await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
        await c.create(mutating_webhook_configuration(
            certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh_port}/mutate-notebook-v1"))
        await eventually(lambda: c.get(kinds.NODE, "mi355x-node-0"))
        names = [f"nb{i}" for i in range(8)]
        for n in names:
            await c.create(notebook(n, "crash", gpus=1, annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
        await asyncio.sleep(0.05)  # mid-reconcile
        procs["odh"].send_signal(signal.SIGKILL)
        procs["odh"].wait(10)
        procs["odh"] = spawn(odh_args, common, logf)
        await wait_http(f"https://127.0.0.1:{wh_port}/healthz")

        async def all_ready():
            for n in names:
                st = (await c.get(kinds.NOTEBOOK, n, "crash")).get("status") or {}
                if st.get("readyReplicas") != 1:
                    return False
            return True
        try:
            await eventually(all_ready, 60)
        except AssertionError:
            raise AssertionError("not all Ready:\n" + await diagnostics(c, names, "crash"))
        # exactly one of each child per notebook (the exposure children — HTTPRoute — are
        # created after the unlock, so they may trail Ready by a moment: wait for them)
        async def children_complete():
            routes = await c.list(kinds.HTTP_ROUTE, "opendatahub")
            crbs = [x["metadata"]["name"] for x in await c.list(kinds.CLUSTER_ROLE_BINDING)
                    if x["metadata"]["name"].endswith("-crash-auth-delegator")]
            return sorted(r["metadata"]["name"] for r in routes) == sorted(f"nb-crash-{n}" for n in names) and \
                len(crbs) == len(names)
        await eventually(children_complete, 30)
        await asyncio.sleep(0.5)  # and no duplicate appears after the fact
        assert await children_complete()
        for n in names:
            nb = await c.get(kinds.NOTEBOOK, n, "crash")
            assert "kubeflow-resource-stopped" not in (nb["metadata"].get("annotations") or {})
            assert len(nb["metadata"]["finalizers"]) == len(set(nb["metadata"]["finalizers"])) == 3
        for n in names:
            await c.delete(kinds.NOTEBOOK, n, "crash")

        async def all_gone():
            left = await c.list(kinds.NOTEBOOK, "crash")
            crbs = [x for x in await c.list(kinds.CLUSTER_ROLE_BINDING)
                    if x["metadata"]["name"].endswith("-crash-auth-delegator")]
            return not left and not crbs and not await c.list(kinds.HTTP_ROUTE, "opendatahub")
        await eventually(all_gone, 60)
        await c.close()

    try:
        run(go(), timeout=180)
    finally:
        for p in procs.values():
            p.terminate()
        for p in procs.values():
            try:
                p.wait(10)
            except Exception:  # noqa: BLE001
                p.kill()
        logf.close()


def test_admission_path_resets_converge(tmp_path, run):
    """The apiserver → webhook HTTPS connections go through the resetting proxy too: an
    admission cut mid-request fails that write (``failurePolicy: Fail``, as the reference),
    the controllers' own admitted writes (the unlock patch) are retried by their requeue,
    and the users' writes are retried by the user (here: the test) — everything converges."""
    from odh_kubeflow_amd.models.errors import ApiError
    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    api_port, wh_port = free_port(), free_port()
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    rnd = random.Random(5)

    async def retry(fn):
        for _ in range(50):
            try:
                return await fn()
            except ApiError as e:
                if e.code not in (500, 503):
                    raise
                await asyncio.sleep(0.05)
        raise AssertionError("write never admitted")

    async def go():
        await wait_http(master + "/healthz")
        c = RestClient(RestConfig(host=master))
        for ns in ("opendatahub", "adm"):
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false"}
        procs.append(spawn(["odh_kubeflow_amd.cmd.kf_manager", "--master", master, "--metrics-addr", "0",
                            "--probe-addr", "0"], common, logf))
        procs.append(spawn(["odh_kubeflow_amd.cmd.odh_manager", "--master", master, "--metrics-bind-address", "0",
                            "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                            "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", certs.cert_dir,
                            "--webhook-port", str(wh_port), "--webhook-host", "127.0.0.1"], common, logf))
        procs.append(spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", master, "--checkpoint-path",
                            str(tmp_path / "dp" / "cp")], common, logf))
        await wait_http(f"https://127.0.0.1:{wh_port}/healthz")
        proxy = await ChaosProxy(wh_port).start()  # TCP-level: TLS passes through untouched
        await c.create(mutating_webhook_configuration(
            certs.ca_bundle_b64, url=f"https://127.0.0.1:{proxy.port}/mutate-notebook-v1"))
        await eventually(lambda: c.get(kinds.NODE, "mi355x-node-0"))
        stop = asyncio.Event()

        async def chaos():
            while not stop.is_set():
                await asyncio.sleep(rnd.uniform(0.01, 0.05))
                proxy.cut_all()
        task = asyncio.create_task(chaos())
        names = [f"nb{i}" for i in range(5)]
        try:
            for n in names:
                await retry(lambda n=n: c.create(notebook(n, "adm", gpus=1, annotations={
                    "notebooks.opendatahub.io/inject-auth": "true"})))

            async def all_ready():
                for n in names:
                    st = (await c.get(kinds.NOTEBOOK, n, "adm")).get("status") or {}
                    if st.get("readyReplicas") != 1:
                        return False
                return True
            try:
                await eventually(all_ready, 60)
            except AssertionError:
                raise AssertionError("not all Ready:\n" + await diagnostics(c, names, "adm"))
            for n in names:
                await retry(lambda n=n: c.delete(kinds.NOTEBOOK, n, "adm"))

            async def all_gone():
                return not await c.list(kinds.NOTEBOOK, "adm") and not await c.list(kinds.HTTP_ROUTE, "opendatahub")
            await eventually(all_gone, 60)
        finally:
            stop.set()
            await task
            await proxy.close()
            await c.close()
        return proxy.aborted

    try:
        aborted = run(go(), timeout=200)
        assert aborted >= 3, aborted
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except Exception:  # noqa: BLE001
                p.kill()
        logf.close()


def test_sharded_control_plane_follows_new_namespaces_through_resets(tmp_path, run):
    """Two ``cmd/control_plane`` shards reach the apiserver through the resetting proxy while
    new namespaces keep appearing: the owning shard's assigner labels each one, the owning shard's
    label-selected Namespace watch adds a per-namespace informer group for it — across
    dropped watches and relists — and every notebook in every namespace becomes Ready."""
    from odh_kubeflow_amd.models import meta as m
    from odh_kubeflow_amd.webhook.certs import generate
    from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

    api_port = free_port()
    wh = [free_port(), free_port()]
    certs = generate(("127.0.0.1", "localhost"), str(tmp_path / "certs"))
    logf = open(tmp_path / "procs.log", "wb")
    master = f"http://127.0.0.1:{api_port}"
    procs = [spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--controllers",
                    "--no-openshift-apis"], log=logf)]
    common = {"K8S_NAMESPACE": "opendatahub", "SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
    rnd = random.Random(3)

    async def go():
        await wait_http(master + "/healthz")
        proxy = await ChaosProxy(api_port).start()
        via = f"http://127.0.0.1:{proxy.port}"
        c = RestClient(RestConfig(host=master))
        await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "opendatahub"}})
        for k in (0, 1):
            await c.create(mutating_webhook_configuration(
                certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh[k]}/mutate-notebook-v1",
                name=f"notebook-webhook-shard-{k}",
                namespace_selector={"matchLabels": {"notebooks.amd.com/shard": str(k)}}))
        await c.create(mutating_webhook_configuration(
            certs.ca_bundle_b64, url=f"https://127.0.0.1:{wh[0]}/mutate-notebook-v1",
            name="notebook-webhook-unassigned", namespace_selector={"matchExpressions": [
                {"key": "notebooks.amd.com/shard", "operator": "DoesNotExist"}]}))
        for k in (0, 1):
            procs.append(spawn(["odh_kubeflow_amd.cmd.control_plane", "--master", via, "--shard", str(k),
                                "--shard-count", "2", "--assign-namespaces", "--metrics-bind-address", "0",
                                "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                                "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", certs.cert_dir,
                                "--webhook-host", "127.0.0.1", "--webhook-port", str(wh[k])], common, logf))
        procs.append(spawn(["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", master, "--devices",
                            "0,1,2,3,4,5,6,7"], common, logf))
        for k in (0, 1):
            await wait_http(f"https://127.0.0.1:{wh[k]}/healthz")
        await eventually(lambda: c.get(kinds.NODE, "mi355x-node-0"))
        stop = asyncio.Event()

        async def chaos():
            while not stop.is_set():
                await asyncio.sleep(rnd.uniform(0.05, 0.15))
                proxy.cut_all()
        task = asyncio.create_task(chaos())
        spaces = [f"team-{i}" for i in range(6)]
        try:
            for ns in spaces:
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})

            async def labelled():
                for ns in spaces:
                    if not m.labels(await c.get(kinds.NAMESPACE, ns)).get("notebooks.amd.com/shard"):
                        return False
                return True
            await eventually(labelled, 60)
            for ns in spaces:
                for _ in range(50):  # the owning shard's webhook may be mid-restart of a watch: retry
                    try:
                        await c.create(notebook("nb", ns, gpus=1))
                        break
                    except Exception:  # noqa: BLE001
                        await asyncio.sleep(0.05)

            async def all_ready():
                for ns in spaces:
                    st = (await c.get(kinds.NOTEBOOK, "nb", ns)).get("status") or {}
                    if st.get("readyReplicas") != 1:
                        return False
                return True

            async def state():  # what a failure report needs: where each notebook stopped
                out = {}
                for ns in spaces:
                    nb = await c.get(kinds.NOTEBOOK, "nb", ns)
                    sts = await c.get_or_none(kinds.STATEFUL_SET, "nb", ns)
                    pod = await c.get_or_none(kinds.POD, "nb-0", ns)
                    out[ns] = {"ready": (nb.get("status") or {}).get("readyReplicas"),
                               "annotations": sorted(m.annotations(nb)), "finalizers": m.finalizers(nb),
                               "sts_replicas": ((sts or {}).get("spec") or {}).get("replicas"),
                               "pod_phase": ((pod or {}).get("status") or {}).get("phase")}
                return out
            try:
                await eventually(all_ready, 90)
            except AssertionError:
                raise AssertionError(f"not all Ready: {await state()}")
            owners = {m.labels(r)["notebook-namespace"]: m.labels(r).get("notebooks.amd.com/shard")
                      for r in await c.list(kinds.HTTP_ROUTE, "opendatahub")}
            want = {ns: m.labels(await c.get(kinds.NAMESPACE, ns))["notebooks.amd.com/shard"] for ns in spaces}
            assert owners == want  # each notebook reconciled by the shard that owns its namespace
        finally:
            stop.set()
            await task
            await proxy.close()
            await c.close()
        return proxy.aborted

    try:
        aborted = run(go(), timeout=240)
        assert aborted >= 10, aborted
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except Exception:  # noqa: BLE001
                p.kill()
        logf.close()


@pytest.mark.parametrize("server_kind", ["python", "native"])
def test_informer_cache_matches_server_after_resets(run, server_kind):
    """An informer cache whose watches are reset every 20–80 ms while a writer creates,
    updates and deletes 120 ConfigMaps ends up exactly equal to the server's state (names
    and resourceVersions): watch resume from the last resourceVersion, 410 → relist, and the
    relist's ADDED / MODIFIED / DELETED reconciliation lose and invent nothing — over the
    Python and the C++ apiserver."""
    from odh_kubeflow_amd.testing.apiserver import native as native_mod
    from odh_kubeflow_amd.testing.apiserver.http import ApiServer
    from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
    from odh_kubeflow_amd.runtime.informer import InformerCache

    if server_kind == "native" and not native_mod.available():
        pytest.skip("native apiserver not built")
    rnd = random.Random(9)

    async def go():
        if server_kind == "python":
            srv = await ApiServer(ObjectStore()).start("127.0.0.1", 0)
            port, stop_srv = srv.port, srv.stop
        else:
            srv = await native_mod.NativeApiServer(history=64).start()
            port, stop_srv = srv.port, srv.stop
        writer = RestClient(RestConfig(host=f"http://127.0.0.1:{port}"))
        proxy = await ChaosProxy(port).start()
        reader = RestClient(RestConfig(host=f"http://127.0.0.1:{proxy.port}"))
        cache = InformerCache(reader)
        await cache.ensure_informer(kinds.CONFIG_MAP)
        stop = asyncio.Event()

        async def chaos():
            while not stop.is_set():
                await asyncio.sleep(rnd.uniform(0.02, 0.08))
                proxy.cut_all()
        task = asyncio.create_task(chaos())
        try:
            live = set()
            for i in range(120):
                op = rnd.random()
                if op < 0.5 or not live:
                    n = f"cm{i}"
                    await writer.create({"apiVersion": "v1", "kind": "ConfigMap",
                                         "metadata": {"name": n, "namespace": "default"}, "data": {"v": "0"}})
                    live.add(n)
                elif op < 0.8:
                    n = rnd.choice(sorted(live))
                    await writer.patch(kinds.CONFIG_MAP, {"data": {"v": str(i)}}, "merge", name=n, namespace="default")
                else:
                    n = rnd.choice(sorted(live))
                    await writer.delete(kinds.CONFIG_MAP, n, "default")
                    live.discard(n)
                if i % 10 == 0:
                    await asyncio.sleep(0.03)
        finally:
            stop.set()
            await task
        truth = {o["metadata"]["name"]: o["metadata"]["resourceVersion"]
                 for o in await writer.list(kinds.CONFIG_MAP, "default")}

        async def converged():
            got = {o["metadata"]["name"]: o["metadata"]["resourceVersion"]
                   for o in cache.list(kinds.CONFIG_MAP, "default")}
            return got == truth
        try:
            await eventually(converged, 30)
        finally:
            await cache.stop()
            await proxy.close()
            await reader.close()
            await writer.close()
            await stop_srv()
        return proxy.aborted

    aborted = run(go(), timeout=120)
    assert aborted >= 5, aborted
