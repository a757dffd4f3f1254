"""Feast config mount: unit cases + admission through the in-process apiserver.

Case list follows odh/controllers/notebook_feast_config_test.go: ``isFeastEnabled``
(:40-106), ``mountFeastConfig`` (:108-302), ``unmountFeastConfig`` (:304-397) and the
integration scenarios (:399-735).  The reference's "integration" cases replay the
webhook flow on an in-memory object; here the notebook goes through the real
mutating admission path of the in-process apiserver, so the stored object is checked.
"""

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.controllers.odh import feast
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook

LABEL = "opendatahub.io/feast-integration"
VOL = "odh-feast-config"
MOUNT = {"name": VOL, "readOnly": True, "mountPath": "/opt/app-root/src/feast-config"}


def spec(nb):
    return nb["spec"]["template"]["spec"]


def feast_volumes(nb):
    return [v for v in spec(nb).get("volumes") or [] if v["name"] == VOL]


def feast_mounts(nb, container=None):
    c = [c for c in spec(nb)["containers"] if c["name"] == (container or nb["metadata"]["name"])][0]
    return [vm for vm in c.get("volumeMounts") or [] if vm["name"] == VOL]


# ------------------------------------------------------------------ isFeastEnabled


@pytest.mark.parametrize("labels,want", [
    ({}, False),                       # label not present
    ({LABEL: "true"}, True),
    ({LABEL: "false"}, False),
    ({LABEL: "invalid-value"}, False),
    ({LABEL: "True"}, False),          # exact match, like the Go comparison
    (None, False),                     # nil labels
])
def test_is_feast_enabled(labels, want):
    nb = notebook("nb", "ns", labels=labels)
    if labels is None:
        nb["metadata"].pop("labels", None)
    assert feast.is_feast_enabled(nb) is want


# ------------------------------------------------------------------ mountFeastConfig


def test_mount_adds_volume_and_mount():
    nb = notebook("nb", "ns")
    feast.mount_feast_config(nb, "nb-feast-config")
    assert feast_volumes(nb) == [{"name": VOL, "configMap": {"name": "nb-feast-config"}}]
    assert feast_mounts(nb) == [MOUNT]
    assert feast.is_feast_mounted(nb)


def test_mount_updates_existing_volume_and_mount_in_place():
    nb = notebook("nb", "ns")
    spec(nb)["volumes"] = [{"name": "other", "emptyDir": {}},
                           {"name": VOL, "configMap": {"name": "old-config"}}]
    spec(nb)["containers"][0]["volumeMounts"] = [{"name": VOL, "mountPath": "/old/path"},
                                                 {"name": "other", "mountPath": "/other"}]
    feast.mount_feast_config(nb, "new-config")
    assert spec(nb)["volumes"] == [{"name": "other", "emptyDir": {}},
                                   {"name": VOL, "configMap": {"name": "new-config"}}]
    assert spec(nb)["containers"][0]["volumeMounts"] == [MOUNT, {"name": "other", "mountPath": "/other"}]


def test_mount_errors_when_notebook_container_missing():
    nb = notebook("nb", "ns", container_name="not-the-notebook")
    with pytest.raises(ValueError, match="notebook image container not found nb"):
        feast.mount_feast_config(nb, "nb-feast-config")
    with pytest.raises(ValueError, match="error mounting Feast config volume"):
        feast.new_feast_config(nb)


def test_mount_touches_only_the_notebook_container():
    nb = notebook("nb", "ns")
    spec(nb)["containers"] = [{"name": "sidecar", "image": "s"}, {"name": "nb", "image": "i"},
                              {"name": "another", "image": "a", "volumeMounts": [{"name": "x", "mountPath": "/x"}]}]
    feast.new_feast_config(nb)
    assert feast_mounts(nb, "nb") == [MOUNT]
    assert "volumeMounts" not in spec(nb)["containers"][0]
    assert spec(nb)["containers"][2]["volumeMounts"] == [{"name": "x", "mountPath": "/x"}]
    assert feast_volumes(nb) == [{"name": VOL, "configMap": {"name": "nb-feast-config"}}]


# ------------------------------------------------------------------ unmountFeastConfig


def test_unmount_removes_volume_and_mount_only():
    nb = notebook("nb", "ns")
    spec(nb)["volumes"] = [{"name": "keep", "emptyDir": {}}]
    spec(nb)["containers"][0]["volumeMounts"] = [{"name": "keep", "mountPath": "/keep"}]
    feast.new_feast_config(nb)
    feast.unmount_feast_config(nb)
    assert spec(nb)["volumes"] == [{"name": "keep", "emptyDir": {}}]
    assert spec(nb)["containers"][0]["volumeMounts"] == [{"name": "keep", "mountPath": "/keep"}]
    assert not feast.is_feast_mounted(nb)


def test_unmount_without_feast_config_is_a_no_op():
    nb = notebook("nb", "ns")
    before = repr(nb)
    feast.unmount_feast_config(nb)
    assert repr(nb) == before


# ------------------------------------------------------------------ through admission


async def live(cl, kind, name, namespace=None):
    """Read through to the apiserver (the cluster view is eventually consistent over REST)."""
    from odh_kubeflow_amd.models.errors import ApiError, is_not_found

    try:
        return await cl.admin.get(kind, name, namespace)
    except ApiError as e:
        if is_not_found(e):
            return None
        raise


def _cluster():
    return LocalCluster(ClusterConfig(odh=True, webhook=True, kf=False, gc=False,
                                      env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}))


def test_admission_label_enabled_with_configmap(run):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace("feast")
            await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": "nb-feast-config", "namespace": "feast"},
                                   "data": {"feature_store.yaml": "project: feast_project"}})
            await cl.admin.create(notebook("nb", "feast", labels={LABEL: "true"}))
            nb = await live(cl, kinds.NOTEBOOK, "nb", "feast")
            assert feast_volumes(nb) == [{"name": VOL, "configMap": {"name": "nb-feast-config"}}]
            assert feast_mounts(nb) == [MOUNT]
    run(go())


def test_admission_label_enabled_without_configmap_still_mounts_reference(run):
    """The pod, not admission, fails when the ConfigMap is missing (reference :508-558)."""
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace("feast")
            await cl.admin.create(notebook("nb", "feast", labels={LABEL: "true"}))
            nb = await live(cl, kinds.NOTEBOOK, "nb", "feast")
            assert feast_volumes(nb) == [{"name": VOL, "configMap": {"name": "nb-feast-config"}}]
    run(go())


@pytest.mark.parametrize("value", ["false", "", "yes"])
def test_admission_label_disabled_skips_mount(run, value):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace("feast")
            await cl.admin.create(notebook("nb", "feast", labels={LABEL: value}))
            assert feast_volumes(await live(cl, kinds.NOTEBOOK, "nb", "feast")) == []
    run(go())


def test_admission_label_removed_unmounts_on_update(run):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace("feast")
            await cl.admin.create(notebook("nb", "feast", labels={LABEL: "true"}))
            # stopped notebook: the restart guard lets webhook-only template changes through
            await cl.admin.patch(kinds.NOTEBOOK, {"metadata": {"labels": {LABEL: None}}}, name="nb",
                                 namespace="feast")
            nb = await live(cl, kinds.NOTEBOOK, "nb", "feast")
            assert "kubeflow-resource-stopped" in nb["metadata"]["annotations"]
            assert feast_volumes(nb) == [] and feast_mounts(nb) == []
    run(go())


def test_admission_premounted_volume_with_disabled_label_is_unmounted(run):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace("feast")
            nb = notebook("nb", "feast", labels={LABEL: "false"})
            spec(nb)["volumes"] = [{"name": VOL, "configMap": {"name": "some-config"}}]
            spec(nb)["containers"][0]["volumeMounts"] = [{"name": VOL, "mountPath": MOUNT["mountPath"]}]
            await cl.admin.create(nb)
            stored = await live(cl, kinds.NOTEBOOK, "nb", "feast")
            assert not feast.is_feast_mounted(stored) and feast_mounts(stored) == []
    run(go())
