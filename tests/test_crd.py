"""``notebooks.kubeflow.org`` CRD: structurally equal to the reference per version
(``kf/config/crd/bases/kubeflow.org_notebooks.yaml`` + ``kf/config/crd/patches/validation_patches.yaml``),
and enforced like kube-apiserver enforces a structural schema — prune, default, validate —
by all three apiservers (in-process store, Python REST, native C++)."""

import copy
import os

import pytest
import yaml

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import crd, openapi
from odh_kubeflow_amd.models.errors import ApiError
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.utils import jsonpatch

REF = "/root/reference/components/notebook-controller/config/crd"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
def test_crd_structurally_equal_to_reference():
    with open(os.path.join(REF, "bases", "kubeflow.org_notebooks.yaml")) as f:
        ref = yaml.safe_load(f)
    with open(os.path.join(REF, "patches", "validation_patches.yaml")) as f:
        ops = yaml.safe_load(f)
    ref = jsonpatch.apply_patch(ref, ops)  # what `kustomize build config/crd` serves
    ours = crd.notebook_crd()
    for k in ("group", "names", "scope"):
        assert ours["spec"][k] == ref["spec"][k]
    assert [(v["name"], v["served"], v["storage"], v["subresources"]) for v in ours["spec"]["versions"]] == \
        [(v["name"], v["served"], v["storage"], v["subresources"]) for v in ref["spec"]["versions"]]
    for mine, theirs in zip(ours["spec"]["versions"], ref["spec"]["versions"]):
        assert mine["schema"]["openAPIV3Schema"] == theirs["schema"]["openAPIV3Schema"], mine["name"]
    assert ours["spec"]["conversion"] == {"strategy": "None"}  # trivial_conversion_patch.yaml
    # the generated manifest is that object
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "config", "crd", "bases", "kubeflow.org_notebooks.yaml")) as f:
        assert yaml.safe_load(f) == ours


def _nb(**container):
    nb = notebook("nb", "u", gpus=1)
    nb["spec"]["template"]["spec"]["containers"][0].update(container)
    return nb


INVALID = [
    ("containerPort string", dict(ports=[{"containerPort": "eight"}]),
     'spec.template.spec.containers[0].ports[0].containerPort: Invalid value: "eight": '
     'spec.template.spec.containers[0].ports[0].containerPort in body must be of type integer: "string"'),
    ("bad quantity", dict(resources={"limits": {"memory": "lots"}}),
     "spec.template.spec.containers[0].resources.limits.memory: Invalid value: \"lots\""),
    ("missing image", dict(image=None), "spec.template.spec.containers[0].image: Required value"),
    ("duplicate port", dict(ports=[{"containerPort": 8888}, {"containerPort": 8888}]),
     'spec.template.spec.containers[0].ports[1]: Duplicate value: {"containerPort":8888, "protocol":"TCP"}'),
    ("int32 overflow", dict(ports=[{"containerPort": 2 ** 40}]), "should be a valid int32"),
    ("env not a list", dict(env={"A": "1"}), "spec.template.spec.containers[0].env: Invalid value: \"object\""),
]


def test_schema_processing_unit():
    schema = crd.version_schema()
    nb = _nb(ports=[{"containerPort": 8888, "name": "notebook-port"}], bogusField=1)
    nb["spec"]["template"]["spec"]["nodeSelector"] = {"amd.com/gpu.product-name": "AMD_Instinct_MI355X"}
    nb["spec"]["unknownTopLevel"] = True
    nb["status"] = {"conditions": [], "readyReplicas": 0, "containerState": {}, "extra": 1}
    errs = openapi.process(schema, nb)
    assert errs == []
    c = nb["spec"]["template"]["spec"]["containers"][0]
    assert "bogusField" not in c and "unknownTopLevel" not in nb["spec"] and "extra" not in nb["status"]
    assert c["ports"][0]["protocol"] == "TCP"  # schema default
    assert nb["spec"]["template"]["spec"]["nodeSelector"]  # additionalProperties map kept
    for _, kw, want in INVALID:
        bad = _nb(**kw)
        if kw.get("image", 1) is None:
            del bad["spec"]["template"]["spec"]["containers"][0]["image"]
        errs = openapi.process(schema, bad)
        assert any(want in e for e in errs), (want, errs)
    no_containers = copy.deepcopy(nb)
    no_containers["spec"]["template"]["spec"]["containers"] = []
    assert openapi.process(schema, no_containers) == [
        "spec.template.spec.containers: Invalid value: 0: spec.template.spec.containers in body should have at "
        "least 1 items"]


@pytest.mark.parametrize("transport", ["inprocess", "http", "native"])
def test_invalid_podspec_rejected_at_create(run, transport):
    async def go():
        async with LocalCluster(ClusterConfig(kf=False, transport=transport)) as cl:
            await cl.ensure_namespace("u")
            for label, kw, want in INVALID:
                bad = _nb(**kw)
                if kw.get("image", 1) is None:
                    del bad["spec"]["template"]["spec"]["containers"][0]["image"]
                with pytest.raises(ApiError) as ei:
                    await cl.admin.create(bad)
                assert ei.value.code == 422 and want in str(ei.value), (label, str(ei.value))
                assert 'Notebook.kubeflow.org "nb" is invalid' in str(ei.value) or ei.value.reason == "Invalid"
            ok = await cl.admin.create(_nb(ports=[{"containerPort": 8888}], surprise="x"))
            c = ok["spec"]["template"]["spec"]["containers"][0]
            assert c["ports"] == [{"containerPort": 8888, "protocol": "TCP"}] and "surprise" not in c
            # an update that breaks the schema is refused too
            ok["spec"]["template"]["spec"]["containers"][0]["ports"][0]["containerPort"] = "x"
            with pytest.raises(ApiError) as ei:
                await cl.admin.update(ok)
            assert ei.value.code == 422
    run(go(), timeout=60)
