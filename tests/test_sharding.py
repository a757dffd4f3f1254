"""Namespace-sharded control plane and the apiserver features it relies on.

* multi-namespace + label-selected informer caches (controller-runtime
  ``cache.Options{DefaultNamespaces, ByObject.Label}``);
* ``namespaceSelector`` on MutatingWebhookConfiguration (both apiservers);
* the GC "absent owner" rule (a dependent created after its owner is gone is collected);
* conflict retries that read through to the apiserver;
* two shards against one native apiserver, each owning one namespace.
"""

import asyncio

import pytest

from odh_kubeflow_amd.testing.apiserver.inprocess import in_process_manager
from odh_kubeflow_amd.testing.apiserver.http import ApiServer
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.errors import Conflict
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.client import CachedClient
from odh_kubeflow_amd.testing.apiserver.inprocess import InProcessClient, StoreReader
from odh_kubeflow_amd.runtime.informer import InformerCache
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig
from odh_kubeflow_amd.runtime.retry import retry_on_conflict


@pytest.fixture(params=["python", "native"])
def server_kind(request):
    return request.param


async def _server(kind: str, gc: bool = True):
    if kind == "native":
        from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer

        srv = await NativeApiServer(gc=gc).start()
        return srv, RestClient(RestConfig(host=srv.url))
    srv = await ApiServer(ObjectStore(gc=gc)).start("127.0.0.1", 0)
    return srv, RestClient(RestConfig(host=srv.url))


async def _wait(pred, timeout=10.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        if pred():
            return True
        await asyncio.sleep(0.005)
    return pred()


def _cm(name, ns, labels=None, owner=None):
    md = {"name": name, "namespace": ns}
    if labels:
        md["labels"] = labels
    if owner:
        md["ownerReferences"] = [owner]
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": md, "data": {"k": name}}


def test_informer_namespaces_and_label_selector(run, server_kind):
    async def go():
        srv, c = await _server(server_kind)
        try:
            for ns in ("a", "b", "c"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
                await c.create(_cm("x", ns))
            cache = InformerCache(c, namespaces=["a", "b"], selectors={kinds.POD: "gpu=1"})
            seen = []
            cache.subscribe(kinds.CONFIG_MAP, lambda et, o, old: seen.append((et, m.namespace(o))))
            await cache.wait_synced([kinds.CONFIG_MAP, kinds.POD])
            assert sorted(m.namespace(o) for o in cache.list(kinds.CONFIG_MAP)) == ["a", "b"]
            assert cache.get(kinds.CONFIG_MAP, "x", "c") is None and cache.get(kinds.CONFIG_MAP, "x", "a")
            assert [m.namespace(o) for o in cache.list(kinds.CONFIG_MAP, "b")] == ["b"]
            await c.create(_cm("y", "c"))
            await c.create(_cm("y", "a"))
            assert await _wait(lambda: cache.get(kinds.CONFIG_MAP, "y", "a") is not None)
            assert ("ADDED", "c") not in seen and seen.count(("ADDED", "a")) == 2

            # label-selected pods: enter on label add, leave (DELETED) on label change
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "a"},
                   "spec": {"containers": [{"name": "c", "image": "i"}]}}
            await c.create(pod)
            await asyncio.sleep(0.1)
            assert cache.get(kinds.POD, "p", "a") is None
            await c.patch(kinds.POD, {"metadata": {"labels": {"gpu": "1"}}}, name="p", namespace="a")
            assert await _wait(lambda: cache.get(kinds.POD, "p", "a") is not None)
            await c.patch(kinds.POD, {"metadata": {"labels": {"gpu": "2"}}}, name="p", namespace="a")
            assert await _wait(lambda: cache.get(kinds.POD, "p", "a") is None)
            await cache.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_mwc_namespace_selector(run, server_kind):
    async def go():
        from odh_kubeflow_amd.runtime.manager import Manager
        from odh_kubeflow_amd.webhook.certs import generate
        from odh_kubeflow_amd.webhook.notebook_webhook import NotebookWebhook
        from odh_kubeflow_amd.webhook.server import WebhookServer, mutating_webhook_configuration

        srv, c = await _server(server_kind)
        mgr = Manager.remote(RestConfig(host=srv.url), name="wh")
        wh = NotebookWebhook(mgr.client, "opendatahub", kube_rbac_proxy_image="quay.io/brancz/kube-rbac-proxy:v0.18.1")
        certs = generate(("127.0.0.1",))
        ws = await WebhookServer(wh, certs.cert_dir, "127.0.0.1", 0).start()
        try:
            for ns in ("opendatahub", "shard-a", "shard-b"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            await c.create(mutating_webhook_configuration(
                certs.ca_bundle_b64, url=f"https://127.0.0.1:{ws.port}/mutate-notebook-v1", name="wh-shard-a",
                namespace_selector={"matchLabels": {"kubernetes.io/metadata.name": "shard-a"}}))
            await asyncio.sleep(0.1)  # the python apiserver picks MWCs up from its watch
            await c.create(notebook("nb", "shard-b"))
            assert wh.requests == 0
            await c.create(notebook("nb", "shard-a"))
            assert wh.requests == 1
        finally:
            await ws.stop()
            await mgr.stop()
            await c.close()
            await srv.stop()
    run(go())


def test_gc_collects_dependent_of_absent_owner(run, server_kind):
    async def go():
        srv, c = await _server(server_kind)
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "g"}})
            owner = await c.create(_cm("owner", "g"))
            ref = {"apiVersion": "v1", "kind": "ConfigMap", "name": "owner", "uid": m.uid(owner), "controller": True}
            await c.delete(kinds.CONFIG_MAP, "owner", "g")
            await c.create(_cm("late", "g", owner=ref))  # e.g. a controller acting on a stale cache
            await asyncio.sleep(0.05)
            assert await c.get_or_none(kinds.CONFIG_MAP, "late", "g") is None
            # an owner of a kind the server does not serve cannot be verified: kept
            foreign = {"apiVersion": "example.com/v1", "kind": "Widget", "name": "w", "uid": "nope"}
            await c.create(_cm("kept", "g", owner=foreign))
            assert await c.get_or_none(kinds.CONFIG_MAP, "kept", "g") is not None
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_gc_cascade_is_done_when_the_owner_delete_answers(run, server_kind):
    """Background deletion of an owner collects its dependents and theirs (two levels)
    before the DELETE is answered — on the native server the cascade runs after the owner's
    commit has released the store lock, still inside the request."""
    async def go():
        srv, c = await _server(server_kind)
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "gc2"}})
            owner = await c.create(_cm("top", "gc2"))

            def ref(o):
                return {"apiVersion": "v1", "kind": "ConfigMap", "name": m.name(o), "uid": m.uid(o), "controller": True}
            mids = [await c.create(_cm(f"mid{i}", "gc2", owner=ref(owner))) for i in range(3)]
            for i, mid in enumerate(mids):
                await c.create(_cm(f"leaf{i}", "gc2", owner=ref(mid)))
            await c.delete(kinds.CONFIG_MAP, "top", "gc2")
            left = {m.name(o) for o in await c.list(kinds.CONFIG_MAP, "gc2")} - {"kube-root-ca.crt"}
            assert left == set(), left
        finally:
            await c.close()
            await srv.stop()
    run(go())


class _StaleReader(StoreReader):
    """Returns a frozen (stale) copy of every object."""

    def __init__(self, store):
        super().__init__(store)
        self.frozen = {}

    def get(self, kind, name, namespace=None):
        k = (kind, name, namespace)
        if k not in self.frozen:
            self.frozen[k] = super().get(kind, name, namespace)
        return self.frozen[k]


def test_retry_on_conflict_reads_live_without_sleeping(run):
    async def go():
        store = ObjectStore()
        live = InProcessClient(store)
        await live.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "r"}})
        await live.create(_cm("c", "r"))
        reader = _StaleReader(store)
        reader.get(kinds.CONFIG_MAP, "c", "r")  # freeze the current version
        await live.patch(kinds.CONFIG_MAP, {"data": {"k": "moved"}}, name="c", namespace="r")
        cached = CachedClient(reader, live)
        attempts = []

        async def fn():
            cur = await cached.get(kinds.CONFIG_MAP, "c", "r")
            attempts.append(cur["data"]["k"])
            cur["data"]["k2"] = "v"
            await cached.update(cur)

        loop = asyncio.get_running_loop()
        t0 = loop.time()
        await retry_on_conflict(fn)
        assert attempts == ["c", "moved"]  # stale cache, then a live read
        assert loop.time() - t0 < 0.009  # no backoff sleep before the live retry
        assert (await live.get(kinds.CONFIG_MAP, "c", "r"))["data"] == {"k": "moved", "k2": "v"}

        async def always():
            raise Conflict("configmaps", "c")

        with pytest.raises(Conflict):
            await retry_on_conflict(always)
    run(go())


def test_two_shards_one_native_apiserver(run):
    async def go():
        from odh_kubeflow_amd.parallel.platform import NodePlatform
        from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig
        from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
        from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS

        native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
        env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
        shards = []
        platform = None
        try:
            # one node: one scheduler + StatefulSet controller + kubelet for every shard
            platform = await NodePlatform(native.url, process=False).start()
            shards.append(await ControlPlaneShard(ShardConfig(native.url, "bench-0", shard="0", bootstrap=True,
                                                              env=env)).start())
            shards.append(await ControlPlaneShard(ShardConfig(native.url, "bench-1", shard="1", env=env)).start())
            ann = {"notebooks.opendatahub.io/inject-auth": "true"}
            for i, sh in enumerate(shards):
                await sh.admin.create(notebook("nb0", f"bench-{i}", image="img", gpus=1, annotations=ann))
            for sh in shards:
                assert await sh.wait_for(lambda: sh.notebook_ready("nb0"), 30)
            # isolation: a shard's control-plane cache (cmd/control_plane.py --shard i: the
            # namespaces labelled notebooks.amd.com/shard=i + the controller namespace) never
            # holds the other shard's objects; HTTPRoutes carry the shard label
            for i, sh in enumerate(shards):
                cp = sh.control_plane.cache
                assert {m.namespace(o) for o in cp.list(kinds.NOTEBOOK)} == {f"bench-{i}"}
                assert {m.namespace(o) for o in cp.list(kinds.POD)} == {f"bench-{i}"}
                routes = cp.list(kinds.HTTP_ROUTE)
                assert routes and {m.labels(r)["notebook-namespace"] for r in routes} == {f"bench-{i}"}
                assert {m.labels(r)["notebooks.amd.com/shard"] for r in routes} == {str(i)}
                assert sh.control_plane.webhook_server.webhook.requests >= 1
            # the device plugin's choice, not the shard's: two different GPUs, first free, and
            # the node's one kubelet started both pods
            gpus = sorted(m.annotations(p)["amd.com/gpu-ids"] for sh in shards for p in sh.cache.list(kinds.POD))
            assert gpus == ["0", "1"]
            assert sum(g.started for g in platform.agent.runtimes) == 2
            for i, sh in enumerate(shards):
                await sh.admin.delete(kinds.NOTEBOOK, "nb0", f"bench-{i}")
            for sh in shards:
                assert await sh.wait_for(lambda: sh.gone("nb0"), 30)
            for sh in shards:  # event-driven idle of each control plane
                assert await sh.quiesce(0.002, 10)
        finally:
            for sh in reversed(shards):
                await sh.stop()
            if platform is not None:
                await platform.stop()
            await native.stop()
    run(go())


def test_statefulset_workers_split_namespaces(run):
    """The node platform's StatefulSet controller and kubelet as two worker processes each:
    each new namespace is claimed by the least-loaded worker (4 namespaces → 2 + 2), each
    worker watches only its own, and every StatefulSet still gets its pod, scheduled (one
    scheduler: four different GPUs, first free) and Ready."""
    async def go():
        from odh_kubeflow_amd.parallel.platform import NodePlatform
        from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
        from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS
        from odh_kubeflow_amd.testing.kubelet.statefulset import WORKER_LABEL

        native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
        rest = RestClient(RestConfig(host=native.url))
        platform = None
        try:
            platform = await NodePlatform(native.url, process=True, workers=2).start()
            assert sorted(platform.pids()) == ["controller_manager_0", "controller_manager_1", "kubelet_0",
                                               "kubelet_1", "scheduler"]
            nss = [f"team-{i}" for i in range(4)]
            for ns in nss:
                await rest.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
                await rest.create({
                    "apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "s", "namespace": ns},
                    "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "s"}},
                             "template": {"metadata": {"labels": {"app": "s"}},
                                          "spec": {"containers": [{"name": "c", "image": "img",
                                                                   "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})
            loop = asyncio.get_running_loop()
            deadline = loop.time() + 30
            while loop.time() < deadline:
                ready = [((await rest.get(kinds.STATEFUL_SET, "s", ns)).get("status") or {}).get("readyReplicas")
                         for ns in nss]
                if ready == [1, 1, 1, 1]:
                    break
                await asyncio.sleep(0.05)
            assert ready == [1, 1, 1, 1]
            owners = [m.labels(await rest.get(kinds.NAMESPACE, ns)).get(WORKER_LABEL) for ns in nss]
            assert sorted(owners) == ["0", "0", "1", "1"], owners
            pods = [(await rest.get(kinds.POD, "s-0", ns)) for ns in nss]
            assert sorted(m.annotations(p)["amd.com/gpu-ids"] for p in pods) == ["0", "1", "2", "3"]
            assert len(await rest.list(kinds.NODE)) == 1
        finally:
            if platform is not None:
                await platform.stop()
            await rest.close()
            await native.stop()
    run(go())


def test_unsharded_topology_two_drivers(run):
    """``--arch unsharded``: one kf manager + one odh manager (the reference topology,
    overlay mi355x) serve two drivers' namespaces; the second driver launches nothing."""
    async def go():
        from odh_kubeflow_amd.parallel.platform import NodePlatform
        from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig
        from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
        from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS

        native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
        env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
        shards = []
        platform = None
        try:
            platform = await NodePlatform(native.url, process=False).start()
            shards.append(await ControlPlaneShard(ShardConfig(native.url, "bench-0", arch="unsharded", bootstrap=True,
                                                              env=env)).start())
            shards.append(await ControlPlaneShard(ShardConfig(native.url, "bench-1", arch="unsharded", launch=False,
                                                              env=env)).start())
            assert [len(sh.managers) for sh in shards] == [2, 0]
            for i, sh in enumerate(shards):
                await sh.admin.create(notebook("nb0", f"bench-{i}", image="img", gpus=1,
                                               annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
            for sh in shards:
                assert await sh.wait_for(lambda: sh.notebook_ready("nb0"), 30)
            wh = shards[0].managers[1].webhook_server.webhook
            assert wh.requests >= 2  # both namespaces admitted by the one odh webhook
            for i, sh in enumerate(shards):
                await sh.admin.delete(kinds.NOTEBOOK, "nb0", f"bench-{i}")
            for sh in shards:
                assert await sh.wait_for(lambda: sh.gone("nb0"), 30)
            assert await shards[0].quiesce(0.002, 10)
            b = await shards[0].reconcile_breakdown()
            assert sum(b["notebook-controller"].values()) >= 4  # kf reconciles of both notebooks
            assert b["odh-notebook-controller"].get("Notebook", 0) >= 2
            assert await shards[1].reconcile_breakdown() == {}
        finally:
            for sh in reversed(shards):
                await sh.stop()
            if platform is not None:
                await platform.stop()
            await native.stop()
    run(go())


@pytest.mark.parametrize("cluster_watch", [False, True])
def test_informer_namespace_selector_follows_labels(run, server_kind, cluster_watch):
    """``namespace_selector``: a namespace joins the cache when it gets the shard label
    (its objects arrive as ADDED), leaves it when relabelled (DELETED), and reads of a
    namespace outside the cache go live through CachedClient.  ``cluster_watch``: the same
    through ONE cluster-wide watch per kind that drops other namespaces' objects (a joining
    namespace is listed once), instead of a watch per namespace."""
    async def go():
        srv, c = await _server(server_kind)
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ctl"}})
            for ns, shard in (("a", "1"), ("b", "2"), ("c", None)):
                md = {"name": ns, **({"labels": {"notebooks.amd.com/shard": shard}} if shard else {})}
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": md})
                await c.create(_cm("x", ns))
            await c.create(_cm("x", "ctl"))
            cache = InformerCache(c, namespace_selector="notebooks.amd.com/shard=1", namespaces=["ctl"],
                                  cluster_watch=cluster_watch)
            seen = []
            cache.subscribe(kinds.CONFIG_MAP, lambda et, o, old: seen.append((et, m.namespace(o))))
            await cache.wait_synced([kinds.CONFIG_MAP])
            assert sorted(m.namespace(o) for o in cache.list(kinds.CONFIG_MAP)) == ["a", "ctl"]
            assert len(cache._group(kinds.CONFIG_MAP).all()) == (1 if cluster_watch else 2)
            assert cache.watching(kinds.CONFIG_MAP, "a") and not cache.watching(kinds.CONFIG_MAP, "c")
            assert cache.covers(kinds.CONFIG_MAP, "a") and not cache.covers(kinds.CONFIG_MAP, "c")
            assert cache.covers(kinds.NAMESPACE, "c")  # cluster-scoped kinds are never restricted

            # live read of an uncovered namespace (the webhook admits every namespace)
            client = CachedClient(cache, c)
            assert (await client.get(kinds.CONFIG_MAP, "x", "c"))["data"] == {"k": "x"}

            # c joins shard 1: its objects arrive, existing subscriptions see them
            await c.patch(kinds.NAMESPACE, {"metadata": {"labels": {"notebooks.amd.com/shard": "1"}}}, name="c")
            assert await _wait(lambda: cache.get(kinds.CONFIG_MAP, "x", "c") is not None)
            assert ("ADDED", "c") in seen
            # a moves to shard 2: gone from this cache, subscribers get DELETED
            await c.patch(kinds.NAMESPACE, {"metadata": {"labels": {"notebooks.amd.com/shard": "2"}}}, name="a")
            assert await _wait(lambda: cache.get(kinds.CONFIG_MAP, "x", "a") is None)
            assert ("DELETED", "a") in seen
            assert not cache.covers(kinds.CONFIG_MAP, "a")
            # a new object in a joined namespace streams in
            await c.create(_cm("y", "c"))
            assert await _wait(lambda: cache.get(kinds.CONFIG_MAP, "y", "c") is not None)
            await cache.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_namespace_claimer_takes_over_from_a_missing_worker(run):
    """Worker 0 of 2 never runs: worker 1 leaves it each new namespace, then claims the
    namespace itself once it stayed unclaimed for TAKEOVER_S."""
    from odh_kubeflow_amd.testing.kubelet.statefulset import WORKER_LABEL, NamespaceClaimer

    async def go():
        store = ObjectStore()
        mgr = in_process_manager(store, name="w1")
        c = NamespaceClaimer(mgr.client, mgr.reader, 1, 2)
        c.TAKEOVER_S = 0.3
        c.setup_with_manager(mgr)
        await mgr.start()
        try:
            await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            loop = asyncio.get_running_loop()
            t0 = loop.time()
            assert await _wait(lambda: m.labels(store.peek(kinds.NAMESPACE, "team")).get(WORKER_LABEL) == "1", 5)
            assert loop.time() - t0 >= 0.25  # it waited for worker 0 first
        finally:
            await mgr.stop()
    run(go())


def test_informer_namespace_filter_follows_objects(run, server_kind):
    """``namespace_filter`` without a selector: the cache follows every namespace the
    predicate admits (a platform worker's ``worker_owns``) — system namespaces for worker 0,
    labelled ones for their worker — and a relabelled namespace leaves it."""
    from odh_kubeflow_amd.testing.kubelet.statefulset import WORKER_LABEL, worker_owns

    async def go():
        srv, c = await _server(server_kind)
        try:
            for ns, w in (("kube-system", None), ("t0", "0"), ("t1", "1"), ("new", None)):
                md = {"name": ns, **({"labels": {WORKER_LABEL: w}} if w else {})}
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": md})
                await c.create(_cm("x", ns))
            caches = [InformerCache(c, namespace_filter=lambda o, i=i: worker_owns(o, i)) for i in (0, 1)]
            for cache in caches:
                await cache.wait_synced([kinds.CONFIG_MAP])
            assert await _wait(lambda: sorted(m.namespace(o) for o in caches[0].list(kinds.CONFIG_MAP))
                               == ["kube-system", "t0"])
            assert await _wait(lambda: [m.namespace(o) for o in caches[1].list(kinds.CONFIG_MAP)] == ["t1"])
            # "new" is claimed by worker 1; t0 moves to worker 1
            await c.patch(kinds.NAMESPACE, {"metadata": {"labels": {WORKER_LABEL: "1"}}}, name="new")
            await c.patch(kinds.NAMESPACE, {"metadata": {"labels": {WORKER_LABEL: "1"}}}, name="t0")
            assert await _wait(lambda: sorted(m.namespace(o) for o in caches[1].list(kinds.CONFIG_MAP))
                               == ["new", "t0", "t1"])
            assert await _wait(lambda: [m.namespace(o) for o in caches[0].list(kinds.CONFIG_MAP)] == ["kube-system"])
            for cache in caches:
                await cache.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_live_read_kinds_are_read_once_per_version(run, server_kind):
    """ConfigMaps read live (the odh manager's ``DisableFor``, cached stripped of their data):
    a second read of an unchanged object costs no request — the stripped informer vouches
    for its resourceVersion — a changed one is read again, an absent one is NotFound
    without a read, and this client's own write is read back through until the informer
    has it."""
    from odh_kubeflow_amd.models.errors import NotFound
    from odh_kubeflow_amd.runtime.informer import strip_data

    async def go():
        srv, c = await _server(server_kind)
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "a"}})
            await c.create(_cm("x", "a"))
            cache = InformerCache(c, transforms={kinds.CONFIG_MAP: strip_data})
            client = CachedClient(cache, c, uncached=[kinds.CONFIG_MAP])
            await cache.wait_synced([kinds.CONFIG_MAP])
            assert "data" not in cache.get(kinds.CONFIG_MAP, "x", "a")  # the cache holds no payloads
            n0 = c.requests
            assert (await client.get(kinds.CONFIG_MAP, "x", "a"))["data"] == {"k": "x"}
            assert c.requests == n0 + 1
            for _ in range(3):
                got = await client.get(kinds.CONFIG_MAP, "x", "a")
                assert got["data"] == {"k": "x"}
                got["data"]["k"] = "mutated by the caller"  # callers own their copy
            assert c.requests == n0 + 1 and client.validated_reads == 3
            # changed by someone else: once the informer shows the new version, read again
            cur = await c.get(kinds.CONFIG_MAP, "x", "a")
            cur["data"] = {"k": "new"}
            new_rv = (await c.update(cur))["metadata"]["resourceVersion"]
            assert await _wait(lambda: m.resource_version(cache.get(kinds.CONFIG_MAP, "x", "a")) == new_rv)
            n1 = c.requests
            assert (await client.get(kinds.CONFIG_MAP, "x", "a"))["data"] == {"k": "new"}
            assert c.requests == n1 + 1
            # absent from the synced informer: NotFound, no request
            with pytest.raises(NotFound):
                await client.get(kinds.CONFIG_MAP, "missing", "a")
            assert c.requests == n1 + 1
            # this client's own create: served from its response, never a stale NotFound
            await client.create(_cm("mine", "a"))
            assert (await client.get(kinds.CONFIG_MAP, "mine", "a"))["data"] == {"k": "mine"}
            # inside an admission absences are confirmed live, once, and prefetch makes those
            # reads concurrently: later reads of the same keys cost no request
            from odh_kubeflow_amd.runtime.client import CONFIRM_ABSENCE

            tok = CONFIRM_ABSENCE.set(set())
            try:
                n2 = c.requests
                await client.prefetch([(kinds.CONFIG_MAP, "gone1", "a"), (kinds.CONFIG_MAP, "gone2", "a")])
                assert c.requests == n2 + 2
                for nm in ("gone1", "gone2"):
                    with pytest.raises(NotFound):
                        await client.get(kinds.CONFIG_MAP, nm, "a")
                assert c.requests == n2 + 2
            finally:
                CONFIRM_ABSENCE.reset(tok)
            await cache.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_namespace_shard_assigner(run):
    from odh_kubeflow_amd.controllers.sharding import NamespaceShardAssigner, shard_for
    from odh_kubeflow_amd.runtime.manager import Manager

    async def go():
        store = ObjectStore()
        mgr = in_process_manager(store, name="cp")
        a = NamespaceShardAssigner(mgr.client, mgr.reader, 4, exclude=["opendatahub"])
        a.setup_with_manager(mgr)
        await mgr.start()
        try:
            for ns, labels in (("team-a", None), ("team-b", {"notebooks.amd.com/shard": "3"}),
                               ("kube-system", None), ("opendatahub", None)):
                await store.create({"apiVersion": "v1", "kind": "Namespace",
                                    "metadata": {"name": ns, **({"labels": labels} if labels else {})}})
            assert await mgr.wait_idle(5, settle=0.05)
            lab = {ns: m.labels(store.peek(kinds.NAMESPACE, ns)).get("notebooks.amd.com/shard")
                   for ns in ("team-a", "team-b", "kube-system", "opendatahub")}
            assert lab == {"team-a": shard_for("team-a", 4), "team-b": "3", "kube-system": None, "opendatahub": None}
            assert shard_for("team-a", 4) == shard_for("team-a", 4) and 0 <= int(shard_for("x", 8)) < 8
        finally:
            await mgr.stop()
    run(go())


def test_each_shard_assigns_only_its_own_namespaces(run):
    """--assign-namespaces on every shard: shard k labels exactly the unlabelled namespaces that
    hash to k, so no replica is needed for namespaces it will not own; with shard 1 absent its
    namespaces stay unlabelled (they wait for their owner), everyone else's are labelled."""
    from odh_kubeflow_amd.controllers.sharding import NamespaceShardAssigner, shard_for
    from odh_kubeflow_amd.runtime.manager import Manager

    names = [f"team-{i}" for i in range(24)]

    async def go():
        store = ObjectStore()
        mgrs, assigners = [], []
        for k in ("0", "2"):  # shards 0 and 2 of 3 up, shard 1 down
            mgr = in_process_manager(store, name=f"cp-{k}")
            a = NamespaceShardAssigner(mgr.client, mgr.reader, 3, exclude=["opendatahub"], only_shard=k)
            a.setup_with_manager(mgr)
            await mgr.start()
            mgrs.append(mgr)
            assigners.append(a)
        try:
            for ns in names:
                await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            for mgr in mgrs:
                assert await mgr.wait_idle(5, settle=0.05)
            for ns in names:
                got = m.labels(store.peek(kinds.NAMESPACE, ns)).get("notebooks.amd.com/shard")
                want = shard_for(ns, 3)
                assert got == (None if want == "1" else want), ns
            owned = {k: sum(1 for ns in names if shard_for(ns, 3) == k) for k in ("0", "2")}
            assert [a.assigned for a in assigners] == [owned["0"], owned["2"]] and all(owned.values())
        finally:
            for mgr in mgrs:
                await mgr.stop()
    run(go())


def test_balanced_assignment_evens_out_the_hash(run):
    """policy="balanced" (overlay mi355x-sharded): every shard's assigner gives a new namespace to
    the shard owning the fewest, ties to the hash's — 24 namespaces over 3 shards come out 8/8/8
    where crc32 alone is uneven; each namespace is labelled exactly once (preconditioned claims)."""
    from odh_kubeflow_amd.controllers.sharding import NamespaceShardAssigner, shard_for

    names = [f"user-{i:02d}-x" for i in range(24)]

    async def go():
        store = ObjectStore()
        mgrs, assigners = [], []
        for k in ("0", "1", "2"):
            mgr = in_process_manager(store, name=f"cp-{k}")
            a = NamespaceShardAssigner(mgr.client, mgr.reader, 3, exclude=["opendatahub"], only_shard=k,
                                       policy="balanced")
            a.setup_with_manager(mgr)
            await mgr.start()
            mgrs.append(mgr)
            assigners.append(a)
        try:
            for ns in names:
                await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
                for mgr in mgrs:
                    assert await mgr.wait_idle(5, settle=0.01)
            got = [m.labels(store.peek(kinds.NAMESPACE, ns)).get("notebooks.amd.com/shard") for ns in names]
            assert sorted(got.count(k) for k in "012") == [8, 8, 8], got
            assert sum(a.assigned for a in assigners) == 24
            by_hash = sorted(sum(1 for ns in names if shard_for(ns, 3) == k) for k in "012")
            assert by_hash != [8, 8, 8]  # the names chosen are ones the hash spreads unevenly
        finally:
            for mgr in mgrs:
                await mgr.stop()
    run(go())


def test_balanced_plan_is_reused_until_the_namespace_store_changes(run):
    """plan() scans every Namespace; it is kept while the cache's Namespace store is unchanged
    and recomputed (with the new namespace in it) after one is added or relabelled."""
    from odh_kubeflow_amd.controllers.sharding import NamespaceShardAssigner

    async def go():
        srv, c = await _server("python")
        cache = InformerCache(c)
        try:
            for ns in ("a-1", "a-2", "a-3"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            await cache.wait_synced([kinds.NAMESPACE])
            a = NamespaceShardAssigner(None, cache, 2, only_shard="0", policy="balanced")
            p1 = a.plan()
            assert sorted(p1) == ["a-1", "a-2", "a-3"] and a.plans == 1
            assert a.plan() is p1 and a.plan_hits == 1
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "a-4"}})
            assert await _wait(lambda: "a-4" in a.plan())
            plans = a.plans
            assert plans >= 2
            await c.patch(kinds.NAMESPACE, {"metadata": {"labels": {"notebooks.amd.com/shard": "1"}}}, name="a-1")
            assert await _wait(lambda: "a-1" not in a.plan())
            assert a.plans > plans
            hits = a.plan_hits
            a.plan()
            assert a.plan_hits == hits + 1
        finally:
            await cache.stop()
            await c.close()
            await srv.stop()
    run(go())


def test_balanced_assignment_falls_back_to_the_hash_shard(run):
    """The balanced target is down (shard 1 of 3): after the grace period the hash's shard claims
    the namespace, so at most the namespaces that hash to the dead shard wait (as with policy
    hash; those the plan gives a live shard are claimed by it), and none lands on the dead one."""
    from odh_kubeflow_amd.controllers.sharding import NamespaceShardAssigner, shard_for

    names = [f"team-{i}" for i in range(9)]

    async def go():
        store = ObjectStore()
        mgrs = []
        for k in ("0", "2"):
            mgr = in_process_manager(store, name=f"cp-{k}")
            NamespaceShardAssigner(mgr.client, mgr.reader, 3, only_shard=k, policy="balanced",
                                   grace_s=0.5).setup_with_manager(mgr)
            await mgr.start()
            mgrs.append(mgr)
        try:
            for ns in names:
                await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
            must = [ns for ns in names if shard_for(ns, 3) != "1"]
            assert must
            for _ in range(300):
                got = {ns: m.labels(store.peek(kinds.NAMESPACE, ns)).get("notebooks.amd.com/shard") for ns in names}
                if all(got[ns] is not None for ns in must):
                    break
                await asyncio.sleep(0.02)
            assert all(got[ns] in ("0", "2") for ns in must), got
            assert "1" not in got.values(), got
        finally:
            for mgr in mgrs:
                await mgr.stop()
    run(go(), timeout=30)


def test_control_plane_flags(tmp_path):
    from odh_kubeflow_amd.cmd import control_plane
    from odh_kubeflow_amd.cmd.common import resolve_shard

    with pytest.raises(SystemExit):
        control_plane.parse(["--controllers", "kf,odh"])  # odh needs --kube-rbac-proxy-image
    a = control_plane.parse(["--controllers", "kf", "--shard", "ordinal"])
    assert a.controller_set == ["kf"]
    assert resolve_shard("ordinal", {"POD_NAME": "odh-kubeflow-amd-control-plane-5"}) == "5"
    assert resolve_shard(None, {}) is None and resolve_shard("3", {}) == "3"
    with pytest.raises(SystemExit):
        resolve_shard("ordinal", {"HOSTNAME": "no-ordinal"})
    with pytest.raises(SystemExit):
        resolve_shard("not a label!", {})
    # the webhook never starts without its serving certificate (odh/main.go semantics)
    a = control_plane.parse(["--kube-rbac-proxy-image", "img", "--webhook-cert-dir", str(tmp_path),
                             "--master", "http://127.0.0.1:1"])
    with pytest.raises(SystemExit, match="serving certificate missing"):
        control_plane.build(a, {})


def test_terminating_namespace_stays_in_the_shard_cache(run):
    """Notebooks in a Terminating namespace still carry odh finalizers: the shard must keep
    watching the namespace until it is actually gone."""
    async def go():
        store = ObjectStore()
        srv = await ApiServer(store).start("127.0.0.1", 0)
        c = RestClient(RestConfig(host=srv.url))
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace",
                            "metadata": {"name": "a", "labels": {"notebooks.amd.com/shard": "1"}}})
            await c.create(_cm("x", "a"))
            cache = InformerCache(c, namespace_selector="notebooks.amd.com/shard=1")
            await cache.wait_synced([kinds.CONFIG_MAP])
            assert cache.get(kinds.CONFIG_MAP, "x", "a") is not None
            # Terminating: deletionTimestamp set, object still there
            await c.patch(kinds.NAMESPACE, {"metadata": {"finalizers": ["test/hold"]}}, name="a")
            await c.delete(kinds.NAMESPACE, "a")
            assert await _wait(lambda: m.is_deleting(store.peek(kinds.NAMESPACE, "a") or {}))
            await asyncio.sleep(0.1)
            assert cache.covers(kinds.CONFIG_MAP, "a") and cache.get(kinds.CONFIG_MAP, "x", "a") is not None
            await cache.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_webhook_only_control_plane_takes_no_lease(tmp_path):
    """The shard pod's webhook container (``--controllers=webhook --leader-elect``) admits on
    every replica: it builds no leader elector and no reconciler, while the kf and odh
    containers of the same pod each lead on a lease of their own."""
    from odh_kubeflow_amd.cmd import control_plane
    from odh_kubeflow_amd.webhook.certs import generate

    certs = generate(("127.0.0.1",), str(tmp_path / "tls"))
    env = {"K8S_NAMESPACE": "opendatahub"}
    common = ["--master", "http://127.0.0.1:1", "--shard", "0", "--leader-elect", "--kube-rbac-proxy-image", "img",
              "--webhook-cert-dir", certs.cert_dir, "--metrics-bind-address", "0", "--health-probe-bind-address", "0"]
    wh = control_plane.build(control_plane.parse(common + ["--controllers", "webhook"]), env)
    assert wh.leader_elector is None and wh.webhook_server is not None
    assert not getattr(wh, "odh_reconciler", None) and not getattr(wh, "kf_reconcilers", None)
    leases = set()
    for cs in ("kf", "odh"):
        mgr = control_plane.build(control_plane.parse(common + ["--controllers", cs]), env)
        assert mgr.leader_elector is not None and mgr.webhook_server is None
        leases.add(mgr.leader_elector.name)
    assert len(leases) == 2


def test_namespace_scoped_kinds_follow_the_namespace_set(run, server_kind):
    """``InformerCache(namespace_labels=…)``: a namespace-restricted cache lists and watches only
    the ClusterRoleBindings labelled with one of its namespaces, re-scoped when the set changes —
    a namespace joining brings its objects (ADDED) without re-announcing the ones already held."""
    mine = {"a"}

    async def go():
        srv, c = await _server(server_kind)
        try:
            for ns in ("a", "b"):
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
                await c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                                "metadata": {"name": f"crb-{ns}", "labels": {"opendatahub.io/namespace": ns}},
                                "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                            "name": "view"}, "subjects": []})
            cache = InformerCache(c, namespace_filter=lambda o: m.name(o) in mine,
                                  namespace_labels={kinds.CLUSTER_ROLE_BINDING: "opendatahub.io/namespace"})
            seen = []
            cache.subscribe(kinds.CLUSTER_ROLE_BINDING, lambda et, o, old: seen.append((et, m.name(o))))
            await cache.wait_synced([kinds.CLUSTER_ROLE_BINDING, kinds.NAMESPACE])
            assert await _wait(lambda: [m.name(o) for o in cache.list(kinds.CLUSTER_ROLE_BINDING)] == ["crb-a"])
            mine.add("b")
            cache.refresh_namespace("b")
            assert await _wait(lambda: len(cache.list(kinds.CLUSTER_ROLE_BINDING)) == 2)
            assert seen == [("ADDED", "crb-a"), ("ADDED", "crb-b")] and cache.rescopes >= 1
            mine.discard("a")
            cache.refresh_namespace("a")
            assert await _wait(lambda: [m.name(o) for o in cache.list(kinds.CLUSTER_ROLE_BINDING)] == ["crb-b"])
            assert seen[-1] == ("DELETED", "crb-a")
            await cache.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_fill_namespace_does_not_resurrect_an_object_deleted_during_the_list(run):
    """a namespace joins a cluster-wide informer's filter and is listed once.  A
    DELETED event of one of its objects that arrives while that list is in flight finds
    nothing stored; the list, taken before the deletion, must not put the object back."""
    from odh_kubeflow_amd.models.scheme import SCHEME
    from odh_kubeflow_amd.runtime.informer import _Informer

    def cm(name, rv):
        return {"apiVersion": "v1", "kind": "ConfigMap",
                "metadata": {"name": name, "namespace": "joined", "resourceVersion": str(rv)}}

    class Rest:
        def __init__(self):
            self.gate = None

        async def list_rv(self, *a, **kw):
            await self.gate  # the list's answer is held until the test releases it
            return [cm("deleted-meanwhile", 5), cm("kept", 7), cm("updated-meanwhile", 4)], "7"

    class Cache:
        label_index_keys = ()
        transforms = {}
        last_event = 0.0

        def __init__(self):
            self.rest = Rest()

    async def go():
        cache = Cache()
        inf = _Informer(cache, SCHEME.resolve(kinds.CONFIG_MAP), "v1")
        events = []
        inf.handlers[1] = (None, lambda et, o, old: events.append((et, m.name(o), m.resource_version(o))))
        cache.rest.gate = asyncio.get_running_loop().create_future()
        fill = asyncio.ensure_future(inf.fill_namespace("joined"))
        await asyncio.sleep(0)
        inf._apply("DELETED", cm("deleted-meanwhile", 6))  # nothing stored yet: only a tombstone
        inf._apply("MODIFIED", cm("updated-meanwhile", 8))
        cache.rest.gate.set_result(None)
        await fill
        assert ("joined", "deleted-meanwhile") not in inf.items
        assert m.resource_version(inf.items[("joined", "updated-meanwhile")]) == "8"  # the newer event wins
        assert ("joined", "kept") in inf.items
        assert not inf._fill_tombstones  # dropped with the fill
        assert ("ADDED", "deleted-meanwhile", "5") not in events
        # outside a fill, deletions leave no tombstone behind
        inf._apply("DELETED", cm("kept", 9))
        assert not inf._fill_tombstones and ("joined", "kept") not in inf.items
    run(go())
