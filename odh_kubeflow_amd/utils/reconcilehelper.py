"""Desired-vs-found field copying (``components/common/reconcilehelper/util.go``).

Each ``copy_*_fields(frm, to)`` copies the fields the controller owns from the desired
object ``frm`` onto the live object ``to`` and returns True when an Update is needed.
Semantics match the reference exactly, including its one-sided label/annotation check
(only keys present on ``to`` are compared, util.go:107-134) — a label *added* to the
desired object alone does not force an update, but it is still copied over.
"""

from __future__ import annotations

from typing import Callable

from ..models import meta as m
from ..models.errors import is_not_found
from ..utils.objutil import deepcopy_json, ensure_dict


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


def copy_statefulset_fields(frm: dict, to: dict) -> bool:
    """``CopyStatefulSetFields`` (util.go:107-134): labels, annotations, replicas, pod spec."""
    require = _copy_meta(frm, to)
    fs, ts = frm.get("spec") or {}, ensure_dict(to, "spec")
    if fs.get("replicas") != ts.get("replicas"):
        ts["replicas"] = fs.get("replicas")
        require = True
    fpod = (fs.get("template") or {}).get("spec")
    tt = ensure_dict(ts, "template")
    if tt.get("spec") != fpod:
        require = True
    tt["spec"] = deepcopy_json(fpod)
    return require


def copy_deployment_fields(frm: dict, to: dict) -> bool:
    """``CopyDeploymentSetFields`` (util.go:136-162)."""
    require = _copy_meta(frm, to)
    fs, ts = frm.get("spec") or {}, ensure_dict(to, "spec")
    if fs.get("replicas") != ts.get("replicas"):
        ts["replicas"] = fs.get("replicas")
        require = True
    fpod = (fs.get("template") or {}).get("spec")
    tt = ensure_dict(ts, "template")
    if tt.get("spec") != fpod:
        require = True
    tt["spec"] = deepcopy_json(fpod)
    return require


def copy_service_fields(frm: dict, to: dict) -> bool:
    """``CopyServiceFields`` (util.go:166-195): selector and ports only, never clusterIP."""
    require = _copy_meta(frm, to)
    fs, ts = frm.get("spec") or {}, ensure_dict(to, "spec")
    if ts.get("selector") != fs.get("selector"):
        require = True
    ts["selector"] = deepcopy_json(fs.get("selector"))
    if ts.get("ports") != fs.get("ports"):
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
