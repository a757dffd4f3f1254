"""Server-side defaulting, as kube-apiserver applies it when it decodes a write
(``k8s.io/kubernetes/pkg/apis/{core,apps}/v1/defaults.go`` + quantity canonicalisation).

Two users:

* both fake apiservers (``apiserver/store.py`` and, re-implemented in C++,
  ``testing/native/apiserver/apiserver.cpp``) default every Pod / StatefulSet / Deployment /
  Service they store, so controllers meet the same live objects envtest's real
  kube-apiserver hands them (``kf/controllers/suite_test.go:50-104``);
* the reconcile helpers (``utils/reconcilehelper.py``) default the *desired* object the
  same way before comparing it with the live one.  The reference compares the raw
  desired pod template against the defaulted live one (``common/reconcilehelper/util.go:107-134``),
  which differs on every pass against a real apiserver and issues a StatefulSet Update per
  reconcile; comparing like with like removes that write storm.

Only defaults that can appear in objects this control plane writes are implemented; the
function is idempotent (``apply(apply(x)) == apply(x)``).
"""

from __future__ import annotations

from typing import Optional

from ..utils.quantity import QuantityError, canonical, parse_quantity

_PROBE_DEFAULTS = {"timeoutSeconds": 1, "periodSeconds": 10, "successThreshold": 1, "failureThreshold": 3}


def _image_pull_policy(image: str) -> str:
    """``SetDefaults_Container``: ``Always`` for ``:latest`` or an untagged image, else ``IfNotPresent``."""
    if "@" in image:
        return "IfNotPresent"
    last = image.rsplit("/", 1)[-1]
    tag = last.rsplit(":", 1)[1] if ":" in last else ""
    return "Always" if tag in ("", "latest") else "IfNotPresent"


def _canon_resources(res: Optional[dict]) -> None:
    if not res:
        return
    for part in ("limits", "requests"):
        q = res.get(part)
        if not q:
            continue
        for k, v in list(q.items()):
            try:
                q[k] = canonical(parse_quantity(v))
            except (QuantityError, TypeError, ValueError):
                pass  # validation rejects it elsewhere; defaulting never fails


def _probe(p: Optional[dict]) -> None:
    if not p:
        return
    for k, v in _PROBE_DEFAULTS.items():
        p.setdefault(k, v)
    hg = p.get("httpGet")
    if hg is not None:
        hg.setdefault("path", "/")
        hg.setdefault("scheme", "HTTP")


def _container(c: dict) -> None:
    c.setdefault("terminationMessagePath", "/dev/termination-log")
    c.setdefault("terminationMessagePolicy", "File")
    if c.get("image") is not None:
        c.setdefault("imagePullPolicy", _image_pull_policy(c["image"]))
    for port in c.get("ports") or []:
        port.setdefault("protocol", "TCP")
    for e in c.get("env") or []:
        fr = (e.get("valueFrom") or {}).get("fieldRef")
        if fr is not None:
            fr.setdefault("apiVersion", "v1")
    c.setdefault("resources", {})
    _canon_resources(c["resources"])
    for k in ("livenessProbe", "readinessProbe", "startupProbe"):
        _probe(c.get(k))


def _volume(v: dict) -> None:
    for src in ("secret", "configMap"):
        if src in v and v[src] is not None:
            v[src].setdefault("defaultMode", 420)
    if "hostPath" in v and v["hostPath"] is not None:
        v["hostPath"].setdefault("type", "")
    if "emptyDir" in v and v["emptyDir"] is not None:
        sl = v["emptyDir"].get("sizeLimit")
        if sl is not None:
            try:
                v["emptyDir"]["sizeLimit"] = canonical(parse_quantity(sl))
            except (QuantityError, TypeError, ValueError):
                pass


def pod_spec(spec: dict) -> dict:
    """``SetDefaults_PodSpec`` + containers / volumes / probes."""
    spec.setdefault("restartPolicy", "Always")
    spec.setdefault("terminationGracePeriodSeconds", 30)
    spec.setdefault("dnsPolicy", "ClusterFirst")
    spec.setdefault("securityContext", {})
    spec.setdefault("schedulerName", "default-scheduler")
    spec.setdefault("enableServiceLinks", True)
    if spec.get("serviceAccountName") and not spec.get("serviceAccount"):
        spec["serviceAccount"] = spec["serviceAccountName"]  # deprecated mirror field
    for c in spec.get("initContainers") or []:
        _container(c)
    for c in spec.get("containers") or []:
        _container(c)
    for v in spec.get("volumes") or []:
        _volume(v)
    return spec


def pod_template(tmpl: dict) -> dict:
    tmpl.setdefault("metadata", {}).setdefault("creationTimestamp", None)
    pod_spec(tmpl.setdefault("spec", {}))
    return tmpl


def statefulset(obj: dict) -> dict:
    spec = obj.setdefault("spec", {})
    if spec.get("replicas") is None:
        spec["replicas"] = 1
    spec.setdefault("podManagementPolicy", "OrderedReady")
    us = spec.setdefault("updateStrategy", {})
    us.setdefault("type", "RollingUpdate")
    if us["type"] == "RollingUpdate":
        us.setdefault("rollingUpdate", {}).setdefault("partition", 0)
    spec.setdefault("revisionHistoryLimit", 10)
    ret = spec.setdefault("persistentVolumeClaimRetentionPolicy", {})
    ret.setdefault("whenDeleted", "Retain")
    ret.setdefault("whenScaled", "Retain")
    pod_template(spec.setdefault("template", {}))
    return obj


def deployment(obj: dict) -> dict:
    spec = obj.setdefault("spec", {})
    if spec.get("replicas") is None:
        spec["replicas"] = 1
    st = spec.setdefault("strategy", {})
    st.setdefault("type", "RollingUpdate")
    if st["type"] == "RollingUpdate":
        ru = st.setdefault("rollingUpdate", {})
        ru.setdefault("maxUnavailable", "25%")
        ru.setdefault("maxSurge", "25%")
    spec.setdefault("revisionHistoryLimit", 10)
    spec.setdefault("progressDeadlineSeconds", 600)
    pod_template(spec.setdefault("template", {}))
    return obj


def service(obj: dict) -> dict:
    """``SetDefaults_Service`` (+ the IP-family / traffic-policy defaulting of the REST
    strategy); the ClusterIP itself is allocated by the apiserver, not here."""
    spec = obj.setdefault("spec", {})
    spec.setdefault("type", "ClusterIP")
    spec.setdefault("sessionAffinity", "None")
    if spec["type"] in ("ClusterIP", "NodePort", "LoadBalancer") and spec.get("clusterIP") != "None":
        spec.setdefault("ipFamilies", ["IPv4"])
        spec.setdefault("ipFamilyPolicy", "SingleStack")
        spec.setdefault("internalTrafficPolicy", "Cluster")
    for p in spec.get("ports") or []:
        p.setdefault("protocol", "TCP")
        if p.get("targetPort") is None and p.get("port") is not None:
            p["targetPort"] = p["port"]
    return obj


def pod(obj: dict) -> dict:
    """``SetDefaults_Pod``: requests default to limits when unset, then the PodSpec defaults."""
    spec = obj.setdefault("spec", {})
    for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
        res = c.get("resources") or {}
        lim = res.get("limits") or {}
        if lim:
            req = res.setdefault("requests", {})
            for k, v in lim.items():
                req.setdefault(k, v)
            c["resources"] = res
    pod_spec(spec)
    return obj


BY_RESOURCE = {"statefulsets.apps": statefulset, "deployments.apps": deployment, "services": service, "pods": pod}


def apply(resource: str, obj: dict) -> dict:
    """Default ``obj`` (store key ``plural[.group]``, e.g. ``"statefulsets.apps"``) in place; returns it."""
    fn = BY_RESOURCE.get(resource)
    return fn(obj) if fn is not None else obj
