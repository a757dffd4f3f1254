"""API version conversion, reconcilehelper field copies, kf metrics and the legacy OAuth cleanup.

Reference behaviour pinned here:
* ``kf/api/v1/notebook_conversion.go:25-69`` — hub conversion drops ``Condition.Status`` and
  ``Condition.LastTransitionTime``; the CRD itself uses ``conversion.strategy: None``;
* ``common/reconcilehelper/util.go:107-219`` — which fields trigger an update;
* ``kf/pkg/metrics/metrics.go:13-99`` — ``notebook_running`` per namespace from StatefulSets,
  creation counters;
* ``odh/controllers/notebook_oauth.go:35-96`` — legacy OAuthClient + finalizer cleanup.
"""

from prometheus_client import CollectorRegistry

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import convert, notebook
from odh_kubeflow_amd.utils.reconcilehelper import copy_service_fields, copy_statefulset_fields, copy_virtual_service


def _nb_with_status():
    nb = notebook("nb", "u")
    nb["status"] = {"readyReplicas": 1, "containerState": {"running": {"startedAt": "2026-01-01T00:00:00Z"}},
                    "conditions": [{"type": "Ready", "status": "True", "reason": "R", "message": "ok",
                                    "lastProbeTime": "2026-01-01T00:00:00Z",
                                    "lastTransitionTime": "2026-01-01T00:00:01Z"}]}
    return nb


def test_convert_strategy_none_only_changes_api_version():
    nb = _nb_with_status()
    out = convert(nb, "v1beta1")
    assert out["apiVersion"] == "kubeflow.org/v1beta1"
    assert out["status"] == nb["status"] and out["spec"] == nb["spec"]
    assert nb["apiVersion"] == "kubeflow.org/v1"  # input untouched


def test_convert_lossy_reproduces_hub_field_copy():
    out = convert(_nb_with_status(), "v1alpha1", lossy=True)
    c = out["status"]["conditions"][0]
    assert c["type"] == "Ready" and c["reason"] == "R" and c["message"] == "ok"
    assert c["lastProbeTime"] == "2026-01-01T00:00:00Z"
    assert "lastTransitionTime" not in c and c["status"] == ""
    assert out["status"]["readyReplicas"] == 1


def test_convert_rejects_unknown_version():
    import pytest

    with pytest.raises(ValueError):
        convert(notebook("nb", "u"), "v2")


def _sts(replicas=1, image="a", labels=None, ann=None):
    return {"apiVersion": "apps/v1", "kind": "StatefulSet",
            "metadata": {"name": "s", "namespace": "u", "labels": labels or {"x": "1"}, "annotations": ann or {}},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"statefulset": "s"}},
                     "template": {"metadata": {"labels": {"statefulset": "s"}},
                                  "spec": {"containers": [{"name": "c", "image": image}]}}}}


def test_copy_statefulset_fields_detects_and_applies_drift():
    want, have = _sts(), _sts()
    assert copy_statefulset_fields(want, have) is False
    for mutate in (lambda s: s["spec"].__setitem__("replicas", 0),
                   lambda s: s["spec"]["template"]["spec"]["containers"][0].__setitem__("image", "b"),
                   lambda s: s["metadata"]["labels"].__setitem__("x", "2")):
        want, have = _sts(), _sts()
        mutate(want)
        assert copy_statefulset_fields(want, have) is True
        assert copy_statefulset_fields(want, have) is False  # converged
        assert have["spec"] == want["spec"] and have["metadata"]["labels"] == want["metadata"]["labels"]


def test_copy_statefulset_fields_reference_quirk_new_keys_do_not_require_update():
    """util.go:107-121 only walks the EXISTING object's labels/annotations: a key that is
    new in the desired object is copied but does not by itself trigger an Update."""
    want, have = _sts(ann={"k": "v"}), _sts()
    want["metadata"]["labels"]["y"] = "2"
    assert copy_statefulset_fields(want, have) is False
    assert have["metadata"]["labels"] == {"x": "1", "y": "2"} and have["metadata"]["annotations"] == {"k": "v"}


def test_copy_service_fields_never_touches_cluster_ip():
    want = {"metadata": {"labels": {}, "annotations": {}},
            "spec": {"selector": {"statefulset": "s"}, "ports": [{"name": "http-notebook", "port": 80}]}}
    have = {"metadata": {"labels": {}, "annotations": {}},
            "spec": {"selector": {"statefulset": "s"}, "ports": [{"name": "http-notebook", "port": 80}],
                     "clusterIP": "10.0.0.7"}}
    assert copy_service_fields(want, have) is False
    want["spec"]["ports"][0]["port"] = 8080
    assert copy_service_fields(want, have) is True
    assert have["spec"]["ports"][0]["port"] == 8080 and have["spec"]["clusterIP"] == "10.0.0.7"


def test_copy_virtual_service_compares_whole_spec():
    want = {"metadata": {}, "spec": {"hosts": ["*"], "http": [{"match": [{"uri": {"prefix": "/a/"}}]}]}}
    have = {"metadata": {}, "spec": {"hosts": ["*"], "http": [{"match": [{"uri": {"prefix": "/b/"}}]}]}}
    assert copy_virtual_service(want, have) is True and have["spec"] == want["spec"]
    assert copy_virtual_service(want, have) is False


def test_kf_metrics_running_per_namespace_and_create_counter(run):
    async def go():
        async with LocalCluster(ClusterConfig()) as cl:
            for ns in ("a", "b"):
                await cl.ensure_namespace(ns)
            for ns, nm in (("a", "x"), ("a", "y"), ("b", "z")):
                await cl.admin.create(notebook(nm, ns))
            assert await cl.wait_for(lambda: all(cl.notebook_ready(n, ns) for ns, n in
                                                 (("a", "x"), ("a", "y"), ("b", "z"))))
            reg = cl.kf.registry
            assert reg.get_sample_value("notebook_running", {"namespace": "a"}) == 2
            assert reg.get_sample_value("notebook_running", {"namespace": "b"}) == 1
            assert reg.get_sample_value("notebook_create_total", {"namespace": "a"}) == 2
            assert isinstance(reg, CollectorRegistry)
    run(go())


def test_legacy_oauth_client_and_finalizer_removed_on_delete(run):
    async def go():
        from odh_kubeflow_amd.controllers.odh.constants import OAUTH_CLIENT_FINALIZER as OAUTH_FINALIZER
        from odh_kubeflow_amd.controllers.odh.oauth import oauth_client_name

        async with LocalCluster(ClusterConfig(odh=True, webhook=True, openshift=True,
                                              env={"SET_PIPELINE_RBAC": "false",
                                                   "SET_PIPELINE_SECRET": "false"})) as cl:
            await cl.ensure_namespace("u")
            nb = notebook("old", "u")
            nb["metadata"]["finalizers"] = [OAUTH_FINALIZER]
            nb = await cl.admin.create(nb)
            await cl.admin.create({"apiVersion": "oauth.openshift.io/v1", "kind": "OAuthClient",
                                   "metadata": {"name": oauth_client_name(nb)}, "grantMethod": "auto"})
            assert await cl.wait_for(lambda: cl.notebook_ready("old", "u"))
            await cl.admin.delete(kinds.NOTEBOOK, "old", "u")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "old", "u") is None)
            assert cl.store.peek(kinds.OAUTH_CLIENT, oauth_client_name(nb)) is None
            assert m.name(nb) == "old"
    run(go())
