"""kube-rbac-proxy sidecar resource annotations: the full validation table.

Mirrors odh/controllers/auth_proxy_resources_test.go: ``TestParseAndValidateAuthSidecarResources``
(defaults 100m / 64Mi for requests and limits, whitespace trimming, invalid formats,
request > explicit or default limit, negative values) and
``TestInjectKubeRbacProxyWithResourceValidation`` (a failed validation injects nothing).
"""

import copy

import pytest

from odh_kubeflow_amd.controllers.odh import auth
from odh_kubeflow_amd.models.notebook import notebook

CPU_REQ = "notebooks.opendatahub.io/auth-sidecar-cpu-request"
MEM_REQ = "notebooks.opendatahub.io/auth-sidecar-memory-request"
CPU_LIM = "notebooks.opendatahub.io/auth-sidecar-cpu-limit"
MEM_LIM = "notebooks.opendatahub.io/auth-sidecar-memory-limit"
IMAGE = "test-rbac-image"


def nb(ann=None):
    return notebook("test-notebook", "default", image="test-image", annotations=ann)


VALID = [
    ("no annotations - all defaults", None, ("100m", "64Mi", "100m", "64Mi")),
    ("all custom values", {CPU_REQ: "200m", MEM_REQ: "128Mi", CPU_LIM: "400m", MEM_LIM: "256Mi"},
     ("200m", "128Mi", "400m", "256Mi")),
    ("partial annotations with defaults", {CPU_REQ: "50m", MEM_LIM: "128Mi"}, ("50m", "64Mi", "100m", "128Mi")),
    ("whitespace trimming", {CPU_REQ: " 150m ", MEM_REQ: "\t256Mi\n", CPU_LIM: " 300m ", MEM_LIM: " 512Mi "},
     ("150m", "256Mi", "300m", "512Mi")),
    ("equal requests and limits", {CPU_REQ: "200m", CPU_LIM: "200m", MEM_REQ: "128Mi", MEM_LIM: "128Mi"},
     ("200m", "128Mi", "200m", "128Mi")),
]

INVALID = [
    ("invalid CPU request format", {CPU_REQ: "invalid-cpu"}, "invalid value for annotation"),
    ("invalid memory request format", {MEM_REQ: "invalid-memory"}, "invalid value for annotation"),
    ("invalid CPU limit format", {CPU_LIM: "invalid-cpu"}, "invalid value for annotation"),
    ("invalid memory limit format", {MEM_LIM: "invalid-memory"}, "invalid value for annotation"),
    ("CPU request greater than explicit limit", {CPU_REQ: "500m", CPU_LIM: "200m"},
     "CPU request (500m) cannot be greater than CPU limit (200m)"),
    ("memory request greater than explicit limit", {MEM_REQ: "512Mi", MEM_LIM: "256Mi"},
     "memory request (512Mi) cannot be greater than memory limit (256Mi)"),
    ("CPU request higher than default limit", {CPU_REQ: "200m"},
     "CPU request (200m) cannot be greater than CPU limit (100m)"),
    ("memory request higher than default limit", {MEM_REQ: "128Mi"},
     "memory request (128Mi) cannot be greater than memory limit (64Mi)"),
    ("negative CPU request", {CPU_REQ: "-100m"}, "cannot be negative"),
    ("negative memory request", {MEM_REQ: "-64Mi"}, "cannot be negative"),
    ("negative CPU limit", {CPU_LIM: "-200m"}, "cannot be negative"),
    ("negative memory limit", {MEM_LIM: "-128Mi"}, "cannot be negative"),
]


@pytest.mark.parametrize("name,ann,want", VALID, ids=[v[0] for v in VALID])
def test_parse_valid(name, ann, want):
    res = auth.parse_and_validate_auth_sidecar_resources(nb(ann))
    assert (res["requests"]["cpu"], res["requests"]["memory"], res["limits"]["cpu"], res["limits"]["memory"]) == want


@pytest.mark.parametrize("name,ann,msg", INVALID, ids=[v[0] for v in INVALID])
def test_parse_invalid(name, ann, msg):
    with pytest.raises(auth.SidecarResourceError) as ei:
        auth.parse_and_validate_auth_sidecar_resources(nb(ann))
    assert msg in str(ei.value)


@pytest.mark.parametrize("name,ann,want", VALID, ids=[v[0] for v in VALID])
def test_inject_applies_validated_resources(name, ann, want):
    obj = nb(ann)
    auth.inject_kube_rbac_proxy(obj, IMAGE)
    sidecars = [c for c in obj["spec"]["template"]["spec"]["containers"] if c["name"] == "kube-rbac-proxy"]
    assert len(sidecars) == 1
    r = sidecars[0]["resources"]
    assert (r["requests"]["cpu"], r["requests"]["memory"], r["limits"]["cpu"], r["limits"]["memory"]) == want
    assert sidecars[0]["image"] == IMAGE


@pytest.mark.parametrize("name,ann,msg", INVALID, ids=[v[0] for v in INVALID])
def test_inject_failure_leaves_notebook_untouched(name, ann, msg):
    obj = nb(ann)
    before = copy.deepcopy(obj)
    with pytest.raises(auth.SidecarResourceError):
        auth.inject_kube_rbac_proxy(obj, IMAGE)
    assert obj == before
