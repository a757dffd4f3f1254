"""``metav1.ObjectMeta`` accessors for JSON-tree objects, plus ownerRef/finalizer helpers
(the ``controllerutil`` and ``metav1.IsControlledBy`` analogues)."""

from __future__ import annotations

from typing import Dict, List, Optional

from ..utils.objutil import ensure_dict


def meta(obj: dict) -> dict:
    return ensure_dict(obj, "metadata")


def name(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("name", "")


def namespace(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("namespace", "")


def uid(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("uid", "")


def resource_version(obj: dict) -> str:
    return (obj.get("metadata") or {}).get("resourceVersion", "")


def key(obj: dict) -> str:
    ns = namespace(obj)
    return f"{ns}/{name(obj)}" if ns else name(obj)


def labels(obj: dict) -> Dict[str, str]:
    return (obj.get("metadata") or {}).get("labels") or {}


def annotations(obj: dict) -> Dict[str, str]:
    return (obj.get("metadata") or {}).get("annotations") or {}


def ensure_labels(obj: dict) -> Dict[str, str]:
    m = meta(obj)
    if not isinstance(m.get("labels"), dict):
        m["labels"] = {}
    return m["labels"]


def ensure_annotations(obj: dict) -> Dict[str, str]:
    m = meta(obj)
    if not isinstance(m.get("annotations"), dict):
        m["annotations"] = {}
    return m["annotations"]


def has_annotation(obj: dict, k: str) -> bool:
    return k in annotations(obj)


def deletion_timestamp(obj: dict) -> Optional[str]:
    return (obj.get("metadata") or {}).get("deletionTimestamp")


def is_deleting(obj: dict) -> bool:
    return bool(deletion_timestamp(obj))


# ------------------------------------------------------------------ finalizers


def finalizers(obj: dict) -> List[str]:
    return list((obj.get("metadata") or {}).get("finalizers") or [])


def contains_finalizer(obj: dict, f: str) -> bool:
    return f in ((obj.get("metadata") or {}).get("finalizers") or [])


def add_finalizer(obj: dict, f: str) -> bool:
    m = meta(obj)
    fs = m.get("finalizers") or []
    if f in fs:
        return False
    m["finalizers"] = fs + [f]
    return True


def remove_finalizer(obj: dict, f: str) -> bool:
    m = meta(obj)
    fs = m.get("finalizers") or []
    if f not in fs:
        return False
    fs = [x for x in fs if x != f]
    if fs:
        m["finalizers"] = fs
    else:
        m.pop("finalizers", None)
    return True


# ------------------------------------------------------------------ owner references


def owner_reference(owner: dict, controller: bool = True, block_owner_deletion: bool = True) -> dict:
    return {
        "apiVersion": owner.get("apiVersion", ""),
        "kind": owner.get("kind", ""),
        "name": name(owner),
        "uid": uid(owner),
        "controller": controller,
        "blockOwnerDeletion": block_owner_deletion,
    }


class AlreadyOwnedError(ValueError):
    pass


def set_controller_reference(owner: dict, obj: dict) -> None:
    """``ctrl.SetControllerReference``: add a controller ownerRef, refusing a second controller."""
    m = meta(obj)
    if namespace(owner) and namespace(obj) and namespace(owner) != namespace(obj):
        raise ValueError("cross-namespace owner references are disallowed")
    refs = list(m.get("ownerReferences") or [])
    ref = owner_reference(owner)
    for i, r in enumerate(refs):
        if r.get("controller") and r.get("uid") != ref["uid"]:
            raise AlreadyOwnedError(f"object is already owned by another {r.get('kind')} controller {r.get('name')}")
        if r.get("uid") == ref["uid"] or (r.get("kind") == ref["kind"] and r.get("name") == ref["name"]
                                          and r.get("apiVersion", "").split("/")[0] == ref["apiVersion"].split("/")[0]):
            refs[i] = ref
            m["ownerReferences"] = refs
            return
    refs.append(ref)
    m["ownerReferences"] = refs


def controller_of(obj: dict) -> Optional[dict]:
    for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
        if r.get("controller"):
            return r
    return None


def is_controlled_by(obj: dict, owner: dict) -> bool:
    r = controller_of(obj)
    return bool(r) and r.get("uid") == uid(owner)
