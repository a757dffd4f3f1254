"""The ``kubeflow.org`` Notebook API: constants, status shapes and version conversion.

Wire schema (``kf/api/v1/notebook_types.go:26-84``)::

    spec:   {template: {spec: <corev1.PodSpec>}}
    status: {conditions: [{type, status, lastProbeTime, lastTransitionTime, reason, message}],
             readyReplicas: int32, containerState: <corev1.ContainerState>}

``conditions``, ``readyReplicas`` and ``containerState`` have no ``omitempty`` and are
always serialised; the condition's optional fields are omitted when empty.  v1 is the
storage version; v1alpha1 and v1beta1 carry the identical schema, and the CRD uses
``conversion.strategy: None`` (``kf/config/crd/patches/trivial_conversion_patch.yaml``)
so served versions differ only in ``apiVersion``.
"""

from __future__ import annotations

from typing import List, Optional

from ..utils.objutil import deepcopy_json
from ..utils.timeutil import rfc3339

GROUP = "kubeflow.org"
VERSIONS = ("v1", "v1alpha1", "v1beta1")
STORAGE_VERSION = "v1"
HUB_VERSION = "v1beta1"  # kf/api/v1beta1/notebook_conversion.go:19

# ---- annotations / labels shared by the three controllers
STOP_ANNOTATION = "kubeflow-resource-stopped"
LAST_ACTIVITY_ANNOTATION = "notebooks.kubeflow.org/last-activity"
LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION = "notebooks.kubeflow.org/last_activity_check_timestamp"
# the culler's bookkeeping, rewritten on every check of every running notebook
# (kf/controllers/culling_controller.go:171-196); no reconciler reads them, and the StatefulSet
# generator never copies them into the pod template (keys containing "notebook",
# kf/controllers/notebook_controller.go:488), so a change to these alone is not a reason to
# reconcile or to run the admission pipeline
CULLER_HEARTBEAT_ANNOTATIONS = frozenset({LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION})


def heartbeat_filter_enabled(env) -> bool:
    """``ODH_HEARTBEAT_FILTER=false`` turns the heartbeat filtering off (every culler write then
    reconciles kf and odh and runs the admission pipeline, as in the reference) — for A/B
    measurements only."""
    return (env.get("ODH_HEARTBEAT_FILTER") or "true").strip().lower() != "false"


ANNOTATION_REWRITE_URI = "notebooks.kubeflow.org/http-rewrite-uri"
ANNOTATION_HEADERS_REQUEST_SET = "notebooks.kubeflow.org/http-headers-request-set"
ANNOTATION_NOTEBOOK_RESTART = "notebooks.opendatahub.io/notebook-restart"
WORKBENCH_LABEL = "opendatahub.io/workbenches"
NOTEBOOK_NAME_LABEL = "notebook-name"
STATEFULSET_LABEL = "statefulset"
PREFIX_ENV_VAR = "NB_PREFIX"

DEFAULT_CONTAINER_PORT = 8888
DEFAULT_SERVING_PORT = 80
MAX_STATEFULSET_NAME_LENGTH = 52
DEFAULT_FS_GROUP = 100

# ---- MI355X placement: device-plugin resource and node-labeller keys
GPU_RESOURCE = "amd.com/gpu"
HBM_BYTES_PER_GPU = 288 * 10 ** 9
GPU_IDS_ANNOTATION = "amd.com/gpu-ids"  # written by our device plugin / node agent on the pod


def notebook(name: str, namespace: str, image: str = "rocm/pytorch:latest", gpus: int = 0,
             version: str = STORAGE_VERSION, labels: Optional[dict] = None, annotations: Optional[dict] = None,
             container_name: Optional[str] = None, extra_container: Optional[dict] = None) -> dict:
    """Build a Notebook object; ``gpus`` requests ``amd.com/gpu`` (limits == requests)."""
    c = {"name": container_name or name, "image": image}
    if gpus:
        c["resources"] = {"limits": {GPU_RESOURCE: str(gpus)}, "requests": {GPU_RESOURCE: str(gpus)}}
    if extra_container:
        c.update(extra_container)
    md = {"name": name, "namespace": namespace}
    if labels:
        md["labels"] = dict(labels)
    if annotations:
        md["annotations"] = dict(annotations)
    return {"apiVersion": f"{GROUP}/{version}", "kind": "Notebook", "metadata": md,
            "spec": {"template": {"spec": {"containers": [c]}}}}


def empty_status() -> dict:
    return {"conditions": [], "readyReplicas": 0, "containerState": {}}


def pod_cond_to_notebook_cond(podc: dict, now: Optional[str] = None) -> dict:
    """``PodCondToNotebookCond`` (``kf/controllers/notebook_controller.go:376-415``).

    Zero ``lastProbeTime`` / ``lastTransitionTime`` are stamped with "now".
    """
    now = now or rfc3339()
    cond = {}
    if podc.get("type"):
        cond["type"] = podc["type"]
    if podc.get("status"):
        cond["status"] = podc["status"]
    if podc.get("message"):
        cond["message"] = podc["message"]
    if podc.get("reason"):
        cond["reason"] = podc["reason"]
    cond["lastProbeTime"] = podc.get("lastProbeTime") or now
    cond["lastTransitionTime"] = podc.get("lastTransitionTime") or now
    return cond


def _convert_conditions(conds: Optional[List[dict]]) -> List[dict]:
    out = []
    for c in conds or []:
        n = {"type": c.get("type", "")}
        if c.get("lastProbeTime"):
            n["lastProbeTime"] = c["lastProbeTime"]
        if c.get("reason"):
            n["reason"] = c["reason"]
        if c.get("message"):
            n["message"] = c["message"]
        # NOTE: the reference's field copy omits Status and LastTransitionTime
        # (kf/api/v1/notebook_conversion.go:25-43) — kept for parity.
        n["status"] = ""
        out.append(n)
    return out


def convert(nb: dict, to_version: str, lossy: bool = False) -> dict:
    """Convert between served versions.

    ``lossy=False`` (default) is the ``conversion.strategy: None`` behaviour the CRD
    actually uses: only ``apiVersion`` changes.  ``lossy=True`` reproduces the
    ``ConvertTo``/``ConvertFrom`` hub conversion functions verbatim, including their
    dropping of ``Condition.status`` and ``Condition.lastTransitionTime``.
    """
    if to_version not in VERSIONS:
        raise ValueError(f"unsupported Notebook version {to_version}")
    out = deepcopy_json(nb)
    out["apiVersion"] = f"{GROUP}/{to_version}"
    if lossy:
        st = out.get("status") or {}
        if st:
            st["conditions"] = _convert_conditions(st.get("conditions"))
    return out


def container_for(nb: dict) -> Optional[dict]:
    """The notebook's main container: the one named like the Notebook."""
    name = (nb.get("metadata") or {}).get("name")
    for c in (((nb.get("spec") or {}).get("template") or {}).get("spec") or {}).get("containers") or []:
        if c.get("name") == name:
            return c
    return None


def pod_spec(nb: dict) -> dict:
    spec = nb.setdefault("spec", {})
    tmpl = spec.setdefault("template", {})
    return tmpl.setdefault("spec", {})


def gpu_request(pod_spec_: dict) -> int:
    """Total ``amd.com/gpu`` the pod asks for (limits win, as for extended resources)."""
    total = 0
    for c in pod_spec_.get("containers") or []:
        res = c.get("resources") or {}
        v = (res.get("limits") or {}).get(GPU_RESOURCE) or (res.get("requests") or {}).get(GPU_RESOURCE)
        if v:
            total += int(str(v))
    return total
