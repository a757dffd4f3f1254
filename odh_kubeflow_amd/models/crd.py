"""The ``notebooks.kubeflow.org`` CustomResourceDefinition, byte-compatible with the reference.

``kf/config/crd/bases/kubeflow.org_notebooks.yaml`` is what controller-gen renders from
``kf/api/{v1,v1alpha1,v1beta1}/notebook_types.go`` with the full ``core/v1`` PodSpec
expanded under ``spec.template.spec``, then
``kf/config/crd/patches/validation_patches.yaml:1-29`` requires ``name`` and ``image`` on
every container and ``minItems: 1`` on ``containers``.  The PodSpec subtree is the
Kubernetes API's own published schema and cannot be regenerated without Go and the
``k8s.io/api`` module, so it is vendored as data (``schema/podspec.json``); everything
else — the three versions, storage/served flags, the status subresource, the Notebook
status schema and the validation constraints — is built here.

The same schema drives admission-time validation in both fake apiservers
(:mod:`odh_kubeflow_amd.models.openapi`; ``testing/native/apiserver``): a malformed PodSpec is
refused at create/update exactly as kube-apiserver refuses it, unknown fields are pruned
and schema ``default`` values are applied.
"""

from __future__ import annotations

import copy
import functools
import json
import os
from typing import Dict, List

VERSIONS = ("v1", "v1alpha1", "v1beta1")
STORAGE_VERSION = "v1"
_SCHEMA_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "schema", "podspec.json")


@functools.lru_cache(maxsize=1)
def _podspec() -> dict:
    with open(_SCHEMA_FILE) as f:
        return json.load(f)["podSpec"]


def podspec_schema() -> dict:
    """A private copy of the vendored ``core/v1`` PodSpec structural schema."""
    return copy.deepcopy(_podspec())


def _date_time() -> dict:
    return {"format": "date-time", "type": "string"}


def _string() -> dict:
    return {"type": "string"}


def status_schema() -> dict:
    """``NotebookStatus`` (``kf/api/v1/notebook_types.go:37-63``): conditions, readyReplicas,
    containerState (a ``core/v1`` ContainerState)."""
    condition = {"properties": {"lastProbeTime": _date_time(), "lastTransitionTime": _date_time(),
                                "message": _string(), "reason": _string(), "status": _string(), "type": _string()},
                 "required": ["status", "type"], "type": "object"}
    terminated = {"properties": {"containerID": _string(), "exitCode": {"format": "int32", "type": "integer"},
                                 "finishedAt": _date_time(), "message": _string(), "reason": _string(),
                                 "signal": {"format": "int32", "type": "integer"}, "startedAt": _date_time()},
                  "required": ["exitCode"], "type": "object"}
    return {"properties": {
        "conditions": {"items": condition, "type": "array"},
        "containerState": {"properties": {"running": {"properties": {"startedAt": _date_time()}, "type": "object"},
                                          "terminated": terminated,
                                          "waiting": {"properties": {"message": _string(), "reason": _string()},
                                                      "type": "object"}},
                           "type": "object"},
        "readyReplicas": {"format": "int32", "type": "integer"}},
        "required": ["conditions", "containerState", "readyReplicas"], "type": "object"}


def apply_validation_patches(schema: dict) -> dict:
    """``validation_patches.yaml``: containers ``minItems: 1``, items require ``name`` + ``image``."""
    containers = schema["properties"]["spec"]["properties"]["template"]["properties"]["spec"]["properties"]["containers"]
    containers["items"]["required"] = ["name", "image"]
    containers["minItems"] = 1
    return schema


def version_schema() -> dict:
    """The ``openAPIV3Schema`` every served version carries (identical across versions)."""
    spec = {"properties": {"template": {"properties": {"spec": podspec_schema()}, "type": "object"}},
            "type": "object"}
    return apply_validation_patches({"properties": {"apiVersion": _string(), "kind": _string(),
                                                    "metadata": {"type": "object"}, "spec": spec,
                                                    "status": status_schema()},
                                     "type": "object"})


def notebook_crd() -> dict:
    versions: List[Dict] = []
    for v in VERSIONS:
        versions.append({"name": v, "schema": {"openAPIV3Schema": version_schema()}, "served": True,
                         "storage": v == STORAGE_VERSION, "subresources": {"status": {}}})
    return {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
            "metadata": {"annotations": {"controller-gen.kubebuilder.io/version": "v0.18.0"},
                         "name": "notebooks.kubeflow.org"},
            # trivial_conversion_patch.yaml: identical schemas, no conversion webhook
            "spec": {"conversion": {"strategy": "None"}, "group": "kubeflow.org",
                     "names": {"kind": "Notebook", "listKind": "NotebookList", "plural": "notebooks",
                               "singular": "notebook"},
                     "scope": "Namespaced", "versions": versions}}
