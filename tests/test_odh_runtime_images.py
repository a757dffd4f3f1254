"""Pipeline runtime-images ConfigMap: ImageStream table through admission.

Mirrors odh/controllers/notebook_runtime_test.go (:28-530): a ConfigMap without data is
not mounted; ImageStreams labelled ``opendatahub.io/runtime-image=true`` in the
controller namespace become ``pipeline-runtime-images`` entries keyed by
``formatKeyName(display_name)``, serialised exactly like Go's ``json.Marshal``
(sorted keys, compact, UTF-8 kept); tags without the metadata annotation produce no
ConfigMap and no mount.  The expected payloads below are the reference test's own
fixtures, so byte-compatibility with the Go encoder is checked, not assumed.
"""

import copy

import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.controllers.odh import runtime_images
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook

CENTRAL = "opendatahub"
NS = "user"
CM = "pipeline-runtime-images"
MOUNT = {"name": "runtime-images", "mountPath": "/opt/app-root/pipeline-runtimes/"}
VOLUME = {"name": "runtime-images", "configMap": {"name": CM, "optional": True}}


def _meta_json(display, md_display, tags, schema="runtime-image"):
    import json

    return json.dumps([{"display_name": display, "metadata": {"tags": tags, "display_name": md_display,
                                                              "pull_policy": "IfNotPresent"},
                        "schema_name": schema}], indent=2)


def tag(name, image, display, md_display=None, annotation="opendatahub.io/runtime-image-metadata",
        schema="runtime-image"):
    return {"name": name, "from": {"kind": "DockerImage", "name": image},
            "annotations": {annotation: _meta_json(display, md_display or display, [name], schema)}}


def image_stream(name, tags, label="true"):
    return {"apiVersion": "image.openshift.io/v1", "kind": "ImageStream",
            "metadata": {"name": name, "namespace": CENTRAL, "labels": {"opendatahub.io/runtime-image": label}},
            "spec": {"lookupPolicy": {"local": True}, "tags": tags}}


SHA_IMAGE = ("quay.io/modh/odh-pipeline-runtime-datascience-cpu-py311-ubi9@sha256:"
             "5aa8868be00f304084ce6632586c757bc56b28300779495d14b08bcfbcd3357f")

CASES = [
    ("two tags",
     image_stream("some-image", [
         tag("some-tag", "quay.io/opendatahub/test", "Python 3.11 (UBI9)"),
         tag("some-tag2", "quay.io/opendatahub/test2", "Hohoho Python 3.12 (UBI9)", "Python 3.12 (UBI9)")]),
     {"python-3.11-ubi9.json": '{"display_name":"Python 3.11 (UBI9)","metadata":{"display_name":"Python 3.11 '
                               '(UBI9)","image_name":"quay.io/opendatahub/test","pull_policy":"IfNotPresent",'
                               '"tags":["some-tag"]},"schema_name":"runtime-image"}',
      "hohoho-python-3.12-ubi9.json": '{"display_name":"Hohoho Python 3.12 (UBI9)","metadata":{"display_name":'
                                      '"Python 3.12 (UBI9)","image_name":"quay.io/opendatahub/test2","pull_policy"'
                                      ':"IfNotPresent","tags":["some-tag2"]},"schema_name":"runtime-image"}'}),
    ("one tag",
     image_stream("some-image", [tag("some-tag", SHA_IMAGE, "Python 3.11 (UBI9)")]),
     {"python-3.11-ubi9.json": '{"display_name":"Python 3.11 (UBI9)","metadata":{"display_name":"Python 3.11 '
                               '(UBI9)","image_name":"' + SHA_IMAGE + '","pull_policy":"IfNotPresent",'
                               '"tags":["some-tag"]},"schema_name":"runtime-image"}'}),
    ("irrelevant data",
     image_stream("some-image", [tag("some-tag", "quay.io/opendatahub/test", "Python 3.11 (UBI9)",
                                     annotation="opendatahub.io/runtime-image-metadata-fake",
                                     schema="runtime-image-fake")]),
     None),
    ("formatKeyName edge cases",
     image_stream("format-key-test-image", [
         tag("tag1", "quay.io/opendatahub/test1", "foo  bar"),
         tag("tag2", "quay.io/opendatahub/test2", " !@#$|| invalid chars"),
         tag("tag3", "quay.io/opendatahub/test3", "CZ ěščřžýáíé")]),
     {"foo-bar.json": '{"display_name":"foo  bar","metadata":{"display_name":"foo  bar","image_name":'
                      '"quay.io/opendatahub/test1","pull_policy":"IfNotPresent","tags":["tag1"]},'
                      '"schema_name":"runtime-image"}',
      "invalid-chars.json": '{"display_name":" !@#$|| invalid chars","metadata":{"display_name":" !@#$|| invalid '
                            'chars","image_name":"quay.io/opendatahub/test2","pull_policy":"IfNotPresent","tags":'
                            '["tag2"]},"schema_name":"runtime-image"}',
      "cz.json": '{"display_name":"CZ ěščřžýáíé","metadata":{"display_name":"CZ ěščřžýáíé","image_name":'
                 '"quay.io/opendatahub/test3","pull_policy":"IfNotPresent","tags":["tag3"]},'
                 '"schema_name":"runtime-image"}'}),
]


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
    return LocalCluster(ClusterConfig(odh=False, webhook=True, kf=False, gc=False, openshift=True,
                                      env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}))


def _mounted(nb):
    spec = nb["spec"]["template"]["spec"]
    return (VOLUME in (spec.get("volumes") or []),
            all(MOUNT in (c.get("volumeMounts") or []) for c in spec["containers"]))


@pytest.mark.parametrize("name,ist,want", CASES, ids=[c[0] for c in CASES])
def test_runtime_images_configmap_and_mount(run, name, ist, want):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace(CENTRAL)
            await cl.ensure_namespace(NS)
            await cl.admin.create(copy.deepcopy(ist))
            nb = notebook("test-notebook-runtime", NS)
            nb["spec"]["template"]["spec"]["containers"].append({"name": "sidecar", "image": "s"})
            await cl.admin.create(nb)
            cm = await live(cl, kinds.CONFIG_MAP, CM, NS)
            stored = await live(cl, kinds.NOTEBOOK, "test-notebook-runtime", NS)
            if want is None:
                assert cm is None
                assert _mounted(stored) == (False, False)
            else:
                assert cm["data"] == want
                assert cm["metadata"]["labels"] == {"opendatahub.io/managed-by": "workbenches"}
                assert _mounted(stored) == (True, True)  # every container, not just the notebook's
    run(go())


def test_configmap_without_data_is_not_mounted(run):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace(CENTRAL)
            await cl.ensure_namespace(NS)
            await cl.admin.create({"apiVersion": "v1", "kind": "ConfigMap",
                                   "metadata": {"name": CM, "namespace": NS}, "data": {}})
            await cl.admin.create(notebook("test-notebook-runtime-empty-cf", NS))
            assert await live(cl, kinds.CONFIG_MAP, CM, NS) is not None
            stored = await live(cl, kinds.NOTEBOOK, "test-notebook-runtime-empty-cf", NS)
            assert _mounted(stored) == (False, False)
    run(go())


def test_configmap_follows_imagestream_changes_on_next_admission(run):
    async def go():
        async with _cluster() as cl:
            await cl.ensure_namespace(CENTRAL)
            await cl.ensure_namespace(NS)
            await cl.admin.create(copy.deepcopy(CASES[1][1]))
            await cl.admin.create(notebook("a", NS))
            assert set((await live(cl, kinds.CONFIG_MAP, CM, NS))["data"]) == {"python-3.11-ubi9.json"}
            ist = await cl.admin.get(kinds.IMAGE_STREAM, "some-image", CENTRAL)
            ist["spec"]["tags"].append(tag("t2", "quay.io/x/y", "R Studio"))
            await cl.admin.update(ist)
            await cl.admin.create(notebook("b", NS))
            assert set((await live(cl, kinds.CONFIG_MAP, CM, NS))["data"]) == {"python-3.11-ubi9.json", "r-studio.json"}
    run(go())


def test_unlabelled_or_tagless_imagestreams_ignored():
    ist = image_stream("x", [tag("t", "img", "Name")], label="false")
    assert runtime_images.runtime_images_data([ist]) == {}
    assert runtime_images.runtime_images_data([image_stream("y", [])]) == {}
    no_url = image_stream("z", [tag("t", "", "Name")])
    assert runtime_images.runtime_images_data([no_url]) == {}
    bad_json = image_stream("w", [{"name": "t", "from": {"name": "img"},
                                   "annotations": {"opendatahub.io/runtime-image-metadata": "not json"}}])
    assert runtime_images.runtime_images_data([bad_json]) == {}


def test_configmap_created_meanwhile_is_reconciled_not_left_as_found(run):
    """a ConfigMap another actor created inside the informer's lag reads as absent
    from the data-stripped cache; the create then answers AlreadyExists.  It is read live and
    its data brought up to date (the reference would have read it live in the first place)."""
    from odh_kubeflow_amd.models.errors import AlreadyExists, NotFound
    from odh_kubeflow_amd.runtime.client import LIVE_READS

    class Client:
        def __init__(self):
            self.live_reads = 0
            self.updated = []

        async def list(self, kind, namespace=None, **kw):
            return [copy.deepcopy(CASES[1][1])]

        async def get(self, kind, name, namespace=None):
            if not LIVE_READS.get():
                raise NotFound("configmaps", name)  # what the lagging cache says
            self.live_reads += 1
            return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": namespace,
                                                                          "resourceVersion": "7"},
                    "data": {"stale.json": "{}"}}

        async def create(self, obj):
            raise AlreadyExists("configmaps", obj["metadata"]["name"])

        async def update(self, obj):
            self.updated.append(obj)
            return obj

    async def go():
        c = Client()
        await runtime_images.sync_runtime_images_configmap(c, NS, CENTRAL)
        assert c.live_reads == 1 and len(c.updated) == 1
        assert set(c.updated[0]["data"]) == {"python-3.11-ubi9.json"}
        assert c.updated[0]["metadata"]["resourceVersion"] == "7"
    run(go())
