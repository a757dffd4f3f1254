"""Desired-vs-found field copying (``components/common/reconcilehelper/util.go``).

Each ``copy_*_fields(frm, to)`` copies the fields the controller owns from the desired
object ``frm`` onto the live object ``to`` and returns True when an Update is needed.
Semantics match the reference, including its one-sided label/annotation check (only
keys present on ``to`` are compared, util.go:107-134) — a label *added* to the desired
object alone does not force an update, but it is still copied over.

One deliberate fix: pod specs and Service ports are compared *after* kube-apiserver
defaulting of both sides (``models/defaults.py``).  The live object always carries the
server's defaults (``terminationMessagePath``, ``imagePullPolicy``, ``dnsPolicy``, port
``protocol``, canonical quantities, ...) and the freshly generated desired one never
does, so the reference's raw DeepEqual (util.go:126-130, 187-193) is false on every pass
and issues an Update per reconcile against a real apiserver.
"""

from __future__ import annotations

import json
from collections import OrderedDict
from typing import Callable, Optional

from ..models import defaults
from ..models import meta as m
from ..models.errors import is_not_found
from .objutil import deepcopy_json, ensure_dict


def _copy_meta(frm: dict, to: dict) -> bool:
    require = False
    fl, tl = m.labels(frm), m.labels(to)
    for k, v in tl.items():
        if fl.get(k) != v:
            require = True
    tm = ensure_dict(to, "metadata")
    if "labels" in (frm.get("metadata") or {}):
        tm["labels"] = deepcopy_json(frm["metadata"]["labels"])
    else:
        tm.pop("labels", None)
    fa, ta = m.annotations(frm), m.annotations(to)
    for k, v in ta.items():
        if fa.get(k) != v:
            require = True
    if "annotations" in (frm.get("metadata") or {}):
        tm["annotations"] = deepcopy_json(frm["metadata"]["annotations"])
    else:
        tm.pop("annotations", None)
    return require


_DEFAULTED: "OrderedDict[str, dict]" = OrderedDict()  # canonical JSON of a desired pod spec -> defaulted
_DEFAULTED_MAX = 1024


def _defaulted(spec: dict) -> dict:
    """``defaults.pod_spec`` of a desired spec, remembered by content: a notebook's desired spec
    is regenerated identical on every reconcile of one generation."""
    key = json.dumps(spec, sort_keys=True, separators=(",", ":"))
    hit = _DEFAULTED.get(key)
    if hit is None:
        hit = _DEFAULTED[key] = defaults.pod_spec(deepcopy_json(spec))
        if len(_DEFAULTED) > _DEFAULTED_MAX:
            _DEFAULTED.popitem(last=False)
    else:
        _DEFAULTED.move_to_end(key)
    return hit


def pod_specs_equal(desired: Optional[dict], live: Optional[dict]) -> bool:
    """Semantic pod-spec equality: both sides defaulted as kube-apiserver would.  The live side
    normally already is (the apiserver defaulted it on write), so it is defaulted here only
    when the defaulted desired spec does not equal it as it is."""
    if desired == live:
        return True
    if desired is None or live is None:
        return False
    d = _defaulted(desired)
    return d == live or d == defaults.pod_spec(deepcopy_json(live))


def _copy_pod_template_spec(frm: dict, to: dict) -> bool:
    require = _copy_meta(frm, to)
    fs, ts = frm.get("spec") or {}, ensure_dict(to, "spec")
    if fs.get("replicas") != ts.get("replicas"):
        ts["replicas"] = fs.get("replicas")
        require = True
    fpod = (fs.get("template") or {}).get("spec")
    tt = ensure_dict(ts, "template")
    if not pod_specs_equal(fpod, tt.get("spec")):
        require = True
        tt["spec"] = deepcopy_json(fpod)
    return require


def copy_statefulset_fields(frm: dict, to: dict) -> bool:
    """``CopyStatefulSetFields`` (util.go:107-134): labels, annotations, replicas, pod spec."""
    return _copy_pod_template_spec(frm, to)


def copy_deployment_fields(frm: dict, to: dict) -> bool:
    """``CopyDeploymentSetFields`` (util.go:136-162)."""
    return _copy_pod_template_spec(frm, to)


def _ports_equal(desired, live) -> bool:
    if desired == live:
        return True
    wrap = lambda ps: defaults.service({"spec": {"ports": deepcopy_json(ps or []), "clusterIP": "None"}})["spec"]["ports"]  # noqa: E731
    return wrap(desired) == wrap(live)


def copy_service_fields(frm: dict, to: dict) -> bool:
    """``CopyServiceFields`` (util.go:166-195): selector and ports only, never clusterIP."""
    require = _copy_meta(frm, to)
    fs, ts = frm.get("spec") or {}, ensure_dict(to, "spec")
    if ts.get("selector") != fs.get("selector"):
        require = True
    ts["selector"] = deepcopy_json(fs.get("selector"))
    if not _ports_equal(fs.get("ports"), ts.get("ports")):
        require = True
        ts["ports"] = deepcopy_json(fs.get("ports"))
    return require


def copy_virtual_service(frm: dict, to: dict) -> bool:
    """``CopyVirtualService`` (util.go:199-219): whole ``spec`` map."""
    fspec = frm.get("spec")
    if fspec is None:
        return False
    tspec = to.get("spec")
    if tspec is None:
        to["spec"] = deepcopy_json(fspec)
        return True
    if fspec != tspec:
        to["spec"] = deepcopy_json(fspec)
        return True
    return False


async def reconcile_object(client, desired: dict, copy_fields: Callable[[dict, dict], bool]) -> dict:
    """Generic get → create-if-missing → copy → update-if-changed (util.go:18-101)."""
    md = desired["metadata"]
    kind = f"{desired['apiVersion']}/{desired['kind']}"
    try:
        found = await client.get(kind, md["name"], md.get("namespace"))
    except Exception as e:
        if not is_not_found(e):
            raise
        return await client.create(deepcopy_json(desired))
    if copy_fields(desired, found):
        return await client.update(found)
    return found
