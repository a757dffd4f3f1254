"""Differential test of the two test apiservers at the REST level.

The same seeded sequence of creates, updates (with and without a resourceVersion
precondition), status updates, merge / JSON patches, deletes (with finalizers pending),
gets and label-selected lists goes to the Python REST apiserver and to the C++ one; every
response must agree in status code and — after masking what each server assigns on its own
(uids, timestamps, resourceVersion values, Service IPs) — in body.  Scenarios are run over
both servers (``ODH_CLUSTER_TRANSPORT``), so a divergence here is a test that could pass
over one and fail over the other."""

import asyncio
import random

import pytest

from odh_kubeflow_amd.testing.apiserver import native
from odh_kubeflow_amd.testing.apiserver.http import ApiServer
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.errors import ApiError
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig

pytestmark = pytest.mark.skipif(not native.available(), reason="native apiserver not built")

MASK_META = ("uid", "resourceVersion", "creationTimestamp", "managedFields", "deletionTimestamp")


def mask(o):
    if isinstance(o, list):
        return [mask(x) for x in o]
    if not isinstance(o, dict):
        return o
    out = {}
    for k, v in o.items():
        if k == "metadata" and isinstance(v, dict):
            md = {kk: vv for kk, vv in v.items() if kk not in MASK_META}
            if "deletionTimestamp" in v:
                md["deletionTimestamp"] = "<set>"
            out[k] = mask(md)
        elif k in ("clusterIP", "clusterIPs"):
            continue
        else:
            out[k] = mask(v)
    return out


def ops(seed: int, n: int):
    """A seeded op sequence; each op is (verb, args) with objects built fresh per server."""
    rnd = random.Random(seed)
    names = [f"o{i}" for i in range(6)]
    out = []
    for _ in range(n):
        kind = rnd.choice(["cm", "nb", "svc"])
        name = rnd.choice(names)
        verb = rnd.choice(["create", "create", "get", "update", "update_stale", "status", "merge", "json", "delete",
                           "list", "finalize"])
        out.append((verb, kind, name, rnd.randint(0, 3), rnd.choice(["a", "b"])))
    return out


KIND = {"cm": kinds.CONFIG_MAP, "nb": kinds.NOTEBOOK, "svc": kinds.SERVICE}


def build(kind, name, i, lbl):
    if kind == "cm":
        return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": "d",
                                                                      "labels": {"t": lbl}}, "data": {"i": str(i)}}
    if kind == "svc":
        return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "namespace": "d", "labels": {"t": lbl}},
                "spec": {"selector": {"app": name}, "ports": [{"port": 80 + i, "targetPort": 8888}]}}
    nb = notebook(name, "d")
    nb["metadata"]["labels"] = {"t": lbl}
    return nb


async def play(c, seq):
    results = []

    async def call(fn):
        try:
            return (200, mask(await fn()))
        except ApiError as e:
            return (e.code, e.reason)
    await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "d"}})
    for verb, kind, name, i, lbl in seq:
        k = KIND[kind]
        if verb == "create":
            r = await call(lambda: c.create(build(kind, name, i, lbl)))
        elif verb == "get":
            r = await call(lambda: c.get(k, name, "d"))
        elif verb in ("update", "update_stale", "status"):
            async def upd():
                cur = await c.get(k, name, "d")
                if verb == "update_stale":
                    cur["metadata"]["resourceVersion"] = "1"
                if kind == "cm":
                    cur["data"] = {"i": str(i), "u": "1"}
                elif kind == "svc":
                    cur["spec"]["ports"][0]["port"] = 90 + i
                else:
                    cur["spec"]["template"]["spec"]["containers"][0]["image"] = f"img:{i}"
                if verb == "status":
                    cur["status"] = {"readyReplicas": i} if kind == "nb" else {"loadBalancer": {}}
                    return await c.update_status(cur)
                return await c.update(cur)
            r = await call(upd)
        elif verb == "merge":
            r = await call(lambda: c.patch(k, {"metadata": {"labels": {"t": lbl, "m": str(i)}}}, "merge",
                                           name=name, namespace="d"))
        elif verb == "json":
            r = await call(lambda: c.patch(k, [{"op": "add", "path": "/metadata/annotations",
                                                "value": {"x": str(i)}}], "json", name=name, namespace="d"))
        elif verb == "finalize":
            r = await call(lambda: c.patch(k, {"metadata": {"finalizers": ["example.com/f"] if i % 2 else None}},
                                           "merge", name=name, namespace="d"))
        elif verb == "delete":
            r = await call(lambda: c.delete(k, name, "d"))
        else:
            async def ls():
                items = await c.list(k, "d", labels={"t": lbl})
                return sorted(o["metadata"]["name"] for o in items)
            r = await call(ls)
        results.append((verb, kind, name, r))
    return results


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_python_and_native_apiservers_answer_alike(run, seed):
    seq = ops(seed, 150)

    async def go():
        py = await ApiServer(ObjectStore()).start("127.0.0.1", 0)
        nat = await native.NativeApiServer().start()
        cp = RestClient(RestConfig(host=f"http://127.0.0.1:{py.port}"))
        cn = RestClient(RestConfig(host=nat.url))
        try:
            a = await play(cp, seq)
            b = await play(cn, seq)
        finally:
            await cp.close()
            await cn.close()
            await py.stop()
            await nat.stop()
        for x, y in zip(a, b):
            assert x == y, (x, y)
    run(go(), timeout=120)


def test_event_field_selector_watch_on_both_apiservers(run):
    """The kf event re-emitter's cache lists/watches Events with ``involvedObject.kind!=Notebook``
    (``NotebookEventReemitter.EVENT_FIELD_SELECTOR``): the Notebook events it writes itself never
    come back to it, from either apiserver, while Pod events do."""
    from odh_kubeflow_amd.controllers.notebook import NotebookEventReemitter
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.runtime.informer import InformerCache

    def ev(name, kind):
        return {"apiVersion": "v1", "kind": "Event", "metadata": {"name": name, "namespace": "d"},
                "involvedObject": {"kind": kind, "name": "x", "namespace": "d"}, "reason": "R", "message": "m"}

    async def check(client):
        await client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "d"}})
        await client.create(ev("before-nb", "Notebook"))
        await client.create(ev("before-pod", "Pod"))
        cache = InformerCache(client, field_selectors={kinds.EVENT: NotebookEventReemitter.EVENT_FIELD_SELECTOR})
        seen = []
        cache.subscribe(kinds.EVENT, lambda et, o, old: seen.append((et, o["metadata"]["name"])))
        try:
            await cache.ensure_informer(kinds.EVENT)
            await cache.wait_synced([kinds.EVENT])
            await client.create(ev("after-nb", "Notebook"))
            await client.create(ev("after-pod", "Pod"))
            for _ in range(200):
                if ("ADDED", "after-pod") in seen:
                    break
                await asyncio.sleep(0.01)
            await asyncio.sleep(0.05)
            assert not cache.set_field_selector(kinds.EVENT, "reason=X")  # the informer already runs
        finally:
            await cache.stop()
        assert sorted(n for _, n in seen) == ["after-pod", "before-pod"], seen

    async def go():
        py = await ApiServer(ObjectStore()).start("127.0.0.1", 0)
        nat = await native.NativeApiServer().start()
        cp = RestClient(RestConfig(host=f"http://127.0.0.1:{py.port}"))
        cn = RestClient(RestConfig(host=nat.url))
        try:
            await check(cp)
            await check(cn)
        finally:
            await cp.close()
            await cn.close()
            await py.stop()
            await nat.stop()
    run(go(), timeout=60)


def test_selector_filtered_watch_survives_history_rollover(run):
    """A label-selected watch whose selector rejects every event it sees is still advanced
    (the apiserver's periodic wake-up of filtered watchers), so after many times the bounded
    history of unwanted writes it delivers the next wanted one — no 410 Gone, no relist."""
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.models import meta as m

    async def go():
        nat = await native.NativeApiServer(history=64).start()
        c = RestClient(RestConfig(host=nat.url))
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "u"}})
            first = await c.create({"apiVersion": "v1", "kind": "ConfigMap",
                                    "metadata": {"name": "seed", "namespace": "u"}})
            seen = []

            async def consume(ns):
                async for et, obj in c.watch(kinds.CONFIG_MAP, ns, m.resource_version(first),
                                             labels="want=yes", timeout_s=20):
                    seen.append((ns, et, m.name(obj)))
                    return

            tasks = [asyncio.ensure_future(consume("u")), asyncio.ensure_future(consume(None))]
            await asyncio.sleep(0.1)
            for i in range(600):  # > 9x the history, none of them wanted
                if i % 16 == 15:  # let a starved watcher thread run (the suite shares 8 CPUs)
                    await asyncio.sleep(0.002)
                await c.create({"apiVersion": "v1", "kind": "ConfigMap",
                                "metadata": {"name": f"x{i}", "namespace": "u", "labels": {"want": "no"}}})
            await c.create({"apiVersion": "v1", "kind": "ConfigMap",
                            "metadata": {"name": "hit", "namespace": "u", "labels": {"want": "yes"}}})
            await asyncio.wait_for(asyncio.gather(*tasks), 10)
            assert sorted(seen, key=str) == sorted([("u", "ADDED", "hit"), (None, "ADDED", "hit")], key=str)
        finally:
            await c.close()
            await nat.stop()
    run(go(), timeout=60)


def test_native_metrics_document_is_complete_json(run):
    """GET /metrics of the native apiserver: one JSON document with the request profile, the
    write path's CPU by phase and the per-resource store-lock contention (the benchmark's
    ``apiserver_profile_per_step``), whatever the counters' magnitudes."""
    async def go():
        nat = await native.NativeApiServer().start()
        c = RestClient(RestConfig(host=nat.url))
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "m"}})
            for i in range(5):
                await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"c{i}", "namespace": "m"}})
                await c.patch("v1/ConfigMap", {"data": {"k": str(i)}}, name=f"c{i}", namespace="m")
            st = await nat.stats()
        finally:
            await c.close()
            await nat.stop()
        assert st["writes"] >= 11 and st["prof"]["patch_calls"] == 5
        for k in ("webhook_dials", "webhook_dial_ns", "trims", "lock_wait_ns", "admit_wall_ns", "watch_gone"):
            assert k in st["prof"], k
        assert set(st["phases"]) == {f"{p}_cpu_ns" for p in ("parse", "admit", "validate", "defaults", "patch",
                                                             "prepare", "dump")}
        assert st["phases"]["parse_cpu_ns"] > 0 and st["phases"]["patch_cpu_ns"] > 0
        assert isinstance(st["locks"], dict)
    run(go(), timeout=60)


def test_native_counts_watches_answered_gone(run):
    """A watch from a resourceVersion that fell off the bounded history is answered 410 Gone
    and counted (``prof.watch_gone``: the benchmark's relist signal)."""
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.models import meta as m
    from odh_kubeflow_amd.models.errors import Gone

    async def go():
        nat = await native.NativeApiServer(history=8).start()
        c = RestClient(RestConfig(host=nat.url))
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "g"}})
            first = await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c0", "namespace": "g"}})
            for i in range(1, 40):
                await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"c{i}", "namespace": "g"}})
            assert (await nat.stats())["prof"]["watch_gone"] == 0
            with pytest.raises(Gone):
                async for _ in c.watch(kinds.CONFIG_MAP, "g", m.resource_version(first), timeout_s=5):
                    pass
            assert (await nat.stats())["prof"]["watch_gone"] == 1
        finally:
            await c.close()
            await nat.stop()
    run(go(), timeout=60)
