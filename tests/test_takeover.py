"""Controller takeover: a fresh kf + odh control plane started against a cluster whose
notebooks are already running adopts them without a single write to what they own.

This is the in-place switch of docs/DEPLOY.md (reference managers scaled to 0, these
started) and the crash/restart path of a leader (SURVEY §5 failure recovery): the new
managers list everything, reconcile every notebook once, and must find their generated
StatefulSets, Services, pods and odh children (NetworkPolicies, kube-rbac-proxy objects,
HTTPRoutes, finalizers) already as desired — the reference's steady-state contract
(``common/reconcilehelper/util.go:107-195``, ``odh/controllers/notebook_controller.go``
create-or-update helpers), now on objects the apiserver has defaulted."""

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import STOP_ANNOTATION, notebook

OWNED = (kinds.NOTEBOOK, kinds.STATEFUL_SET, kinds.SERVICE, kinds.POD, kinds.CONFIG_MAP, kinds.SECRET,
         kinds.SERVICE_ACCOUNT, kinds.NETWORK_POLICY, kinds.ROLE_BINDING, kinds.CLUSTER_ROLE_BINDING,
         kinds.HTTP_ROUTE, kinds.REFERENCE_GRANT)


async def snapshot(client) -> dict:
    out = {}
    for k in OWNED:
        for o in await client.list(k):
            md = o["metadata"]
            out[(o.get("kind"), md.get("namespace", ""), md["name"])] = (md["uid"], md["resourceVersion"])
    return out


@pytest.mark.parametrize("transport", ["inprocess", "http", "native"])
def test_fresh_control_plane_adopts_running_notebooks_without_writes(run, transport):
    if transport == "native":
        from odh_kubeflow_amd.testing.apiserver import native

        if not native.available():
            pytest.skip("native apiserver not built")

    async def go():
        cfg = ClusterConfig(transport=transport, odh=True, webhook=True, env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("team")
            auth = {"notebooks.opendatahub.io/inject-auth": "true"}
            await cl.admin.create(notebook("plain", "team"))
            await cl.admin.create(notebook("gpu", "team", gpus=1))
            await cl.admin.create(notebook("authed", "team", gpus=1, annotations=auth))
            await cl.admin.create(notebook("parked", "team"))
            for n in ("plain", "gpu", "authed", "parked"):
                assert await cl.wait_for(lambda n=n: cl.notebook_ready(n, "team"), 20), n
            # stopped after it ran, as the culler or the dashboard stops one (a stop annotation
            # given at create is overwritten by the odh webhook's lock, reference behaviour)
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"annotations": {STOP_ANNOTATION: "2026-01-01T00:00:00Z"}}},
                                 "merge", name="parked", namespace="team")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.POD, "parked-0", "team") is None, 10)
            assert await cl.settle(10)
            parked = cl.store.peek(kinds.STATEFUL_SET, "parked", "team")
            assert parked is not None and parked["spec"]["replicas"] == 0
            before = await snapshot(cl.admin)
            assert {"NetworkPolicy", "HTTPRoute", "ServiceAccount"} <= {k[0] for k in before}, before

            # the old control plane goes away; a new one (fresh caches, queues, reconcilers) takes over
            old = [cl.kf, cl.odh]
            for mgr in old:
                await mgr.stop()
                cl.managers.remove(mgr)
            cl._build_kf()
            cl._build_odh()
            assert cl.kf not in old and cl.odh not in old
            await cl.kf.start()
            await cl.odh.start()
            assert await cl.settle(15)
            # every notebook was reconciled by the new managers (initial list → one request each)
            assert cl.reconcile_breakdown()["notebook-controller"].get("Notebook", 0) >= 4
            assert cl.reconcile_breakdown()["odh-notebook-controller"].get("Notebook", 0) >= 4
            after = await snapshot(cl.admin)
            changed = sorted(k for k in before if after.get(k) != before[k])
            assert changed == [], changed
            assert sorted(set(after) - set(before)) == []
            for n in ("plain", "gpu", "authed"):
                assert cl.notebook_ready(n, "team")
    run(go(), timeout=120)
