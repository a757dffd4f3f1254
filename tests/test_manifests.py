"""Generated deployment manifests: CRD shape + schema, kustomize tree integrity, RBAC
coverage of every kind the controllers touch, samples valid against the CRD."""

import os

import pytest
import yaml

from odh_kubeflow_amd.deploy import manifests
from odh_kubeflow_amd.models import openapi
from odh_kubeflow_amd.models.notebook import notebook

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_crd_names_versions_and_status():
    crd = manifests.notebook_crd()
    spec = crd["spec"]
    assert crd["metadata"]["name"] == "notebooks.kubeflow.org"
    assert spec["names"] == {"kind": "Notebook", "listKind": "NotebookList", "plural": "notebooks",
                             "singular": "notebook"}
    assert spec["scope"] == "Namespaced" and spec["conversion"] == {"strategy": "None"}
    assert [(v["name"], v["served"], v["storage"]) for v in spec["versions"]] == [
        ("v1", True, True), ("v1alpha1", True, False), ("v1beta1", True, False)]
    assert all(v["subresources"] == {"status": {}} for v in spec["versions"])
    st = openapi.crd_version_schema(crd, "v1")["properties"]["status"]
    assert set(st["properties"]) == {"conditions", "readyReplicas", "containerState"}
    assert set(st["properties"]["conditions"]["items"]["properties"]) == {
        "type", "status", "lastProbeTime", "lastTransitionTime", "reason", "message"}


@pytest.mark.parametrize("version", ["v1", "v1alpha1", "v1beta1"])
def test_crd_schema_validation(version):
    schema = openapi.crd_version_schema(manifests.notebook_crd(), version)
    assert openapi.validate(schema, notebook("nb", "ns", gpus=8, version=version)) == []
    bad = notebook("nb", "ns")
    bad["spec"]["template"]["spec"]["containers"] = []
    assert any("at least 1 items" in e for e in openapi.validate(schema, bad))
    bad["spec"]["template"]["spec"]["containers"] = [{"name": "x"}]
    assert openapi.validate(schema, bad) == ["spec.template.spec.containers[0].image: Required value"]
    st = {"status": {"readyReplicas": 1, "conditions": [{"type": "Ready", "status": "True"}], "containerState": {}}}
    assert openapi.validate(schema, {**notebook("nb", "ns"), **st}) == []
    assert openapi.validate(schema, {**notebook("nb", "ns"), "status": {"readyReplicas": "x", "conditions": [],
                                                                         "containerState": {}}})


def test_checked_in_config_matches_generator():
    for path, doc in manifests.tree().items():
        full = os.path.join(ROOT, "config", path)
        assert os.path.exists(full), f"run `python -m odh_kubeflow_amd.deploy.manifests`: missing {path}"
        with open(full) as f:
            text = f.read()
        if isinstance(doc, str):
            assert text.endswith(doc)
        elif isinstance(doc, list):
            assert list(yaml.safe_load_all(text)) == doc
        else:
            assert yaml.safe_load(text) == doc, path


def test_kustomizations_reference_existing_files():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "config")):
        if "kustomization.yaml" not in files:
            continue
        k = yaml.safe_load(open(os.path.join(dirpath, "kustomization.yaml")))
        for r in k.get("resources", []):
            assert os.path.exists(os.path.join(dirpath, r)), (dirpath, r)
        for g in k.get("configMapGenerator", []):
            for e in g.get("envs", []):
                assert os.path.exists(os.path.join(dirpath, e))


def _allowed(role, group, resource, verb):
    for r in role["rules"]:
        if group in r["apiGroups"] and resource in r["resources"] and (verb in r["verbs"] or "*" in r["verbs"]):
            return True
    return False


def test_rbac_covers_controller_access():
    kf, odh = manifests.kf_role(), manifests.odh_role()
    for res, verb in (("statefulsets", "create"), ("statefulsets", "update"), ("services", "create"),
                      ("notebooks/status", "update"), ("virtualservices", "create")):
        group = {"statefulsets": "apps", "services": "", "notebooks/status": "kubeflow.org",
                 "virtualservices": "networking.istio.io"}[res]
        assert _allowed(kf, group, res, verb), res
    assert _allowed(kf, "", "pods", "delete") and _allowed(kf, "", "events", "create")
    for group, res, verb in (("gateway.networking.k8s.io", "httproutes", "delete"),
                             ("gateway.networking.k8s.io", "referencegrants", "create"),
                             ("rbac.authorization.k8s.io", "clusterrolebindings", "delete"),
                             ("networking.k8s.io", "networkpolicies", "update"),
                             ("kubeflow.org", "notebooks", "patch"), ("", "configmaps", "create"),
                             ("", "serviceaccounts", "create"), ("oauth.openshift.io", "oauthclients", "delete"),
                             ("image.openshift.io", "imagestreams", "list")):
        assert _allowed(odh, group, res, verb), (group, res, verb)


def test_samples_request_mi355x_and_validate():
    crd = manifests.notebook_crd()
    for name in ("notebook_v1_1gpu.yaml", "notebook_v1_8gpu_auth.yaml", "notebook_v1alpha1.yaml",
                 "notebook_v1beta1.yaml"):
        doc = yaml.safe_load(open(os.path.join(ROOT, "config", "samples", name)))
        v = doc["apiVersion"].split("/")[1]
        assert openapi.validate(openapi.crd_version_schema(crd, v), doc) == []
        res = doc["spec"]["template"]["spec"]["containers"][0]["resources"]
        assert int(res["limits"]["amd.com/gpu"]) in (1, 8)
        assert "rocm" in doc["spec"]["template"]["spec"]["containers"][0]["image"]
