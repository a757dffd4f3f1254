"""The e2e suite (``e2e/``, the reference's ``odh/e2e`` sequence) in both harnesses:

* local processes — the whole suite, as ``make e2e-test`` runs it without a cluster;
* the cluster harness — its deployment checks, culler-ConfigMap switch and rollouts against
  an apiserver reached through a kubeconfig, with a stand-in Deployment controller that
  reports rollouts the way kube-controller-manager does (observedGeneration, updated and
  ready replicas)."""

import asyncio
import os
import subprocess
import sys

import pytest
import yaml

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def test_e2e_suite_against_local_processes(tmp_path):
    r = subprocess.run([sys.executable, "-m", "pytest", "e2e", "-q", "-p", "no:cacheprovider", "--basetemp",
                        str(tmp_path / "bt")], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "13 passed" in r.stdout, r.stdout[-2000:]


def _deployment(name, ns):
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "namespace": ns},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}},
                                  "spec": {"containers": [{"name": "manager", "image": "img"}]}}}}


def test_cluster_harness_checks_and_rollouts(run, tmp_path):
    from e2e.harness import ClusterHarness

    kc = str(tmp_path / "kubeconfig")
    prefix, ns = "odh-kubeflow-amd-", "opendatahub"

    async def setup_and_serve(stop: asyncio.Event, cl):
        for name in ("deployment", "manager"):
            await cl.admin.create(_deployment(prefix + name, ns))
        await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                               "metadata": {"name": prefix + "config", "namespace": ns}, "data": {"USE_ISTIO": "false"}})
        await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                               "metadata": {"name": prefix + "notebook-controller-culler-config", "namespace": ns},
                               "data": {"ENABLE_CULLING": "false", "CULL_IDLE_TIME": "1440"}})
        with open(os.path.join(ROOT, "config", "crd", "bases", "kubeflow.org_notebooks.yaml")) as f:
            crd = yaml.safe_load(f)
        await cl.admin.create(crd)
        while not stop.is_set():  # kube-controller-manager's rollout bookkeeping
            for d in await cl.admin.list(kinds.DEPLOYMENT, ns):
                st = d.get("status") or {}
                gen = m.meta(d).get("generation", 1)
                if st.get("observedGeneration") != gen:
                    d["status"] = {"observedGeneration": gen, "replicas": 1, "updatedReplicas": 1,
                                   "readyReplicas": 1, "availableReplicas": 1}
                    await cl.admin.update_status(d)
            await asyncio.sleep(0.05)

    async def go():
        async with LocalCluster(ClusterConfig(transport="http", kubeconfig_path=kc, odh=False)) as cl:
            await cl.ensure_namespace(ns)
            stop = asyncio.Event()
            server = asyncio.create_task(setup_and_serve(stop, cl))
            h = None
            try:
                await asyncio.sleep(0.3)
                h = await asyncio.to_thread(ClusterHarness, "e2e", ns, kc, prefix)
                h.interval = 0.05
                res = await asyncio.to_thread(h.controllers)
                assert all(ok for _, ok, _ in res), res
                assert {n for n, _, _ in res} >= {"Deployment odh-kubeflow-amd-deployment",
                                                   "Deployment odh-kubeflow-amd-manager", "Notebook CRD"}
                await asyncio.to_thread(h.enable_culling)
                cm = await cl.admin.get(kinds.CONFIG_MAP, prefix + "notebook-controller-culler-config", ns)
                assert cm["data"] == {"ENABLE_CULLING": "true", "CULL_IDLE_TIME": "2", "IDLENESS_CHECK_PERIOD": "1"}
                dep = await cl.admin.get(kinds.DEPLOYMENT, prefix + "deployment", ns)
                assert "kubectl.kubernetes.io/restartedAt" in dep["spec"]["template"]["metadata"]["annotations"]
                assert m.meta(dep)["generation"] == 2  # the rollout bumped the template
                await asyncio.to_thread(h.restore_culling)
                cm = await cl.admin.get(kinds.CONFIG_MAP, prefix + "notebook-controller-culler-config", ns)
                assert cm["data"] == {"ENABLE_CULLING": "false", "CULL_IDLE_TIME": "1440"}
                # a missing workload is reported, not hidden
                await cl.admin.delete(kinds.DEPLOYMENT, prefix + "manager", ns)
                res = await asyncio.to_thread(h.controllers)
                assert [(n, ok) for n, ok, _ in res if not ok] == [("Deployment odh-kubeflow-amd-manager", False)]
            finally:
                stop.set()
                await server
                if h is not None:
                    await asyncio.to_thread(h.close)
    run(go(), timeout=120)
