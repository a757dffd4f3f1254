"""Watch-event economy: own-write echoes, per-watch predicates, trigger attribution.

The reference's reconcilers register their watches without predicates
(``kf/controllers/notebook_controller.go:778-826``, ``odh/controllers/notebook_controller.go:707-855``),
so every status write, finalizer edit and garbage-collected child queues a reconcile that
finds nothing to do.  These tests pin the filtered behaviour: the wasted reconciles are
gone, while every change a reconcile actually reads (drift, deletion of a live child, pod
readiness, stop/restart annotations) still triggers one.
"""

from odh_kubeflow_amd.testing.apiserver.inprocess import in_process_manager
from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.controller import Request, Result
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore


def _cm(name, data=None):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": "ns"},
            "data": data or {"k": "v"}}


def test_own_write_echo_does_not_requeue_but_other_writers_do(run):
    async def go():
        store = ObjectStore()
        await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ns"}})
        mgr = in_process_manager(store, name="t")
        seen = []

        async def reconcile(req):
            seen.append(req)
            cm = await mgr.client.get_or_none(kinds.CONFIG_MAP, req.name, req.namespace)
            if cm is not None and cm["data"].get("k") == "v":
                cm["data"]["k"] = "written-by-reconcile"
                await mgr.client.update(cm)
            return Result()

        # a second controller watching the same kind still sees the first one's writes
        other = []

        async def observe(req):
            other.append(req)
            return Result()

        c = mgr.builder().named("writer").for_(kinds.CONFIG_MAP).complete(reconcile)
        oc = mgr.builder().named("observer").for_(kinds.CONFIG_MAP).complete(observe)
        await mgr.start()
        try:
            await store.create(_cm("a"))
            assert await mgr.wait_idle(5, settle=0.05)
            # ADDED → reconcile (writes) → the write's echo is skipped: one reconcile
            assert seen == [Request("ns", "a")]
            assert c.echoes_skipped == 1
            assert c.reconciles_by_trigger == {"ConfigMap": 1}
            assert other and oc.echoes_skipped == 0  # not the observer's write: never skipped
            # someone else's change does trigger
            cm = await store.get(kinds.CONFIG_MAP, "a", "ns")
            cm["data"]["k"] = "user"
            await store.update(cm)
            assert await mgr.wait_idle(5, settle=0.05)
            assert seen == [Request("ns", "a"), Request("ns", "a")]
        finally:
            await mgr.stop()
    run(go())


def test_echo_skip_can_be_disabled_like_controller_runtime(run):
    async def go():
        store = ObjectStore()
        await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ns"}})
        mgr = in_process_manager(store, name="t")
        mgr.skip_own_write_echoes = False
        seen = []

        async def reconcile(req):
            seen.append(req)
            cm = await mgr.client.get_or_none(kinds.CONFIG_MAP, req.name, req.namespace)
            if cm is not None and cm["data"].get("k") == "v":
                cm["data"]["k"] = "x"
                await mgr.client.update(cm)
            return Result()

        mgr.builder().named("writer").for_(kinds.CONFIG_MAP).complete(reconcile)
        await mgr.start()
        try:
            await store.create(_cm("a"))
            assert await mgr.wait_idle(5, settle=0.05)
            assert len(seen) == 2  # the echo of its own update reconciles again
        finally:
            await mgr.stop()
    run(go())


def _nb_counts(cl):
    return dict(cl.kf.controllers[0].reconciles_by_trigger)


def test_kf_ignores_status_and_finalizer_edits_but_not_annotations(run):
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
            assert await cl.settle()
            n0 = cl.kf.controllers[0].reconciles
            # a finalizer edit (what the odh controller does) and a foreign status write
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"finalizers": ["x.io/f"]}}, name="nb1", namespace="user")
            await cl.admin.patch(kinds.NOTEBOOK, {"status": {"readyReplicas": 1}}, name="nb1", namespace="user",
                                 subresource="status")
            assert await cl.settle()
            assert cl.kf.controllers[0].reconciles == n0
            # an annotation edit (stop) does
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {"kubeflow-resource-stopped": "t"}}},
                                 name="nb1", namespace="user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.STATEFUL_SET, "nb1", "user")["spec"]["replicas"] == 0)
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"finalizers": None}}, name="nb1", namespace="user")
    run(go())


def test_culler_heartbeat_reconciles_nothing_but_stop_and_restart_do(run):
    """The culler rewrites last-activity / last_activity_check_timestamp on every check of every
    running notebook: neither the kf nor the odh Notebook watch passes that change alone, so R
    resident notebooks cost no reconciles per check period.  The culler's STOP, the restart
    annotation and any other annotation edit still pass."""
    from odh_kubeflow_amd.models.notebook import LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION

    async def go():
        cfg = ClusterConfig(odh=True, webhook=True, env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user", annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
            assert await cl.settle()
            kf, odh = cl.kf.controllers[0], cl.odh.controllers[0]
            k0, o0 = kf.reconciles, odh.reconciles
            for i in range(3):
                await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                    LAST_ACTIVITY_ANNOTATION: "2026-01-01T00:00:00Z",
                    LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION: f"2026-01-01T00:0{i}:00Z"}}}, name="nb1", namespace="user")
            assert await cl.settle()
            assert (kf.reconciles - k0, odh.reconciles - o0) == (0, 0)
            # a heartbeat together with another annotation change passes both
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION: "2026-01-01T00:05:00Z", "x.io/other": "1"}}},
                name="nb1", namespace="user")
            assert await cl.settle()
            assert kf.reconciles - k0 >= 1 and odh.reconciles - o0 >= 1
            # restart: the pod is replaced; stop: the StatefulSet scales to 0
            uid = m.uid(cl.store.peek(kinds.POD, "nb1-0", "user"))
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                "notebooks.opendatahub.io/notebook-restart": "true"}}}, name="nb1", namespace="user")
            assert await cl.wait_for(lambda: m.uid(cl.store.peek(kinds.POD, "nb1-0", "user") or {}) not in ("", uid), 10)
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {
                "kubeflow-resource-stopped": "2026-01-01T00:06:00Z"}}}, name="nb1", namespace="user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.STATEFUL_SET, "nb1", "user")["spec"]["replicas"] == 0)
    run(go())


def test_deleted_children_of_live_notebook_are_recreated(run):
    """Drift repair still works with the owner-alive delete filter (STS and Service)."""
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb1", "user"))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
            uid = m.uid(cl.store.peek(kinds.SERVICE, "nb1", "user"))
            await cl.admin.delete(kinds.SERVICE, "nb1", "user")
            assert await cl.wait_for(lambda: (cl.store.peek(kinds.SERVICE, "nb1", "user") or {})
                                     .get("metadata", {}).get("uid", uid) != uid, 10)
            sts_uid = m.uid(cl.store.peek(kinds.STATEFUL_SET, "nb1", "user"))
            await cl.admin.delete(kinds.STATEFUL_SET, "nb1", "user", propagation="Orphan")
            assert await cl.wait_for(lambda: (cl.store.peek(kinds.STATEFUL_SET, "nb1", "user") or {})
                                     .get("metadata", {}).get("uid", sts_uid) != sts_uid, 10)
            assert await cl.wait_for(lambda: cl.notebook_ready("nb1", "user"), 10)
    run(go())


def test_lifecycle_reconciles_per_notebook_and_triggers(run):
    """create → Ready → delete through the full odh path: at most 12 reconciles per notebook
    (the reference-emulation path does ~18), none of them triggered by garbage collection."""
    async def go():
        cfg = ClusterConfig(odh=True, webhook=True, env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("bench")
            ann = {"notebooks.opendatahub.io/inject-auth": "true"}

            async def one(i):
                nm = f"nb{i}"
                await cl.admin.create(notebook(nm, "bench", gpus=1, annotations=ann))
                assert await cl.wait_for(lambda: cl.notebook_ready(nm, "bench"), 10)
                await cl.admin.delete(kinds.NOTEBOOK, nm, "bench")
                assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, nm, "bench") is None and
                                         cl.store.peek(kinds.POD, f"{nm}-0", "bench") is None, 10)
            await one(0)
            assert await cl.settle()
            r0, b0 = cl.reconcile_count(), cl.reconcile_breakdown()
            for i in range(1, 6):
                await one(i)
            assert await cl.settle()
            per_nb = (cl.reconcile_count() - r0) / 5
            assert per_nb <= 12, (per_nb, cl.reconcile_breakdown())
            b1 = cl.reconcile_breakdown()
            kf = {k: v - b0["notebook-controller"].get(k, 0) for k, v in b1["notebook-controller"].items()}
            # kf: creation + lock removal (Notebook), pod readiness (Pod), readyReplicas (STS)
            assert kf.get("Notebook", 0) <= 2 * 5 and kf.get("Service", 0) == 0, kf
    run(go())


def test_noop_patch_does_not_claim_another_writers_version(run):
    """A patch that changes nothing is answered with the live object — whatever version
    another client wrote last.  Claiming that version as an own write hid the other write's
    event from the patching controller (the odh lock removal never reached kf: the notebook
    stayed at 0 replicas).  Only writes that certainly produced a new version are claimed."""
    from odh_kubeflow_amd.runtime.client import CURRENT_RECONCILE

    async def go():
        store = ObjectStore()
        await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ns"}})
        mgr = in_process_manager(store, name="t")
        await store.create(_cm("a"))
        mine = await store.get(kinds.CONFIG_MAP, "a", "ns")
        theirs = dict(mine, data={"k": "v", "k2": "other"})
        theirs = await store.update(theirs)
        req = Request("ns", "a")
        tok = CURRENT_RECONCILE.set(("writer", req))
        try:
            out = await mgr.client.patch(mine, {"data": {"k": "v"}}, "merge")  # no-op
            assert m.resource_version(out) == m.resource_version(theirs)
            assert mgr.client.own_write(out, "writer") is None
            out = await mgr.client.patch(out, [{"op": "add", "path": "/status", "value": {}}], "json")
            assert mgr.client.own_write(out, "writer") is None
            # a tested removal certainly wrote a new version: its echo is the writer's own
            out = await mgr.client.patch(out, [{"op": "test", "path": "/data/k2", "value": "other"},
                                               {"op": "remove", "path": "/data/k2"}], "json")
            assert mgr.client.own_write(out, "writer") == req
            # an update with a precondition, answered with a new version, too
            out["data"]["k"] = "w"
            out = await mgr.client.update(out)
            assert mgr.client.own_write(out, "writer") == req
        finally:
            CURRENT_RECONCILE.reset(tok)
    run(go())


def test_inflight_echo_claim_is_settled_against_the_response(run):
    """An event that overtakes a preconditioned write's response is claimed provisionally;
    when the response shows another version, the request goes back to its controller."""
    import asyncio

    from odh_kubeflow_amd.runtime.client import CURRENT_RECONCILE

    async def go():
        store = ObjectStore()
        await store.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ns"}})
        mgr = in_process_manager(store, name="t")
        client = mgr.client
        requeued = []
        client.requeue = lambda name, r: requeued.append((name, r))
        await store.create(_cm("a"))
        cm = await store.get(kinds.CONFIG_MAP, "a", "ns")
        sent = int(m.resource_version(cm))
        gate = asyncio.Event()

        class SlowWriter:
            def __init__(self, inner, answer_rv):
                self.inner, self.answer_rv = inner, answer_rv

            async def update(self, obj):
                await gate.wait()
                return dict(obj, metadata=dict(obj["metadata"], resourceVersion=str(self.answer_rv)))

        req = Request("ns", "a")
        foreign = dict(cm, metadata=dict(cm["metadata"], resourceVersion=str(sent + 1)))
        for answer, expect_requeue in ((sent + 2, True), (sent + 1, False)):
            requeued.clear()
            client.writer = SlowWriter(client.writer, answer)
            tok = CURRENT_RECONCILE.set(("writer", req))
            try:
                t = asyncio.ensure_future(client.update(dict(cm)))
                await asyncio.sleep(0)
            finally:
                CURRENT_RECONCILE.reset(tok)
            assert client.own_write(foreign, "writer") == req  # provisional
            gate.set()
            await t
            gate.clear()
            client.writer = client.writer.inner
            assert requeued == ([("writer", req)] if expect_requeue else []), answer
    run(go())
