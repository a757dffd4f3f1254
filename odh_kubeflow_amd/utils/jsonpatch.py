"""RFC 6902 JSON Patch and RFC 7386 JSON Merge Patch.

The mutating webhook answers the apiserver with a JSON patch computed between the
object it received and the object it mutated (reference:
``odh/controllers/notebook_webhook.go:498`` — ``admission.PatchResponseFromRaw``), and
the fake apiserver applies JSON / merge patches sent by controllers (for example the
lock removal merge patch at ``odh/controllers/notebook_controller.go:171-173``).

Objects are plain JSON trees (dict / list / str / int / float / bool / None).
"""

from __future__ import annotations

from typing import Any, List

from .objutil import deepcopy_json


class PatchError(ValueError):
    pass


def _escape(token: str) -> str:
    return token.replace("~", "~0").replace("/", "~1")


def _unescape(token: str) -> str:
    return token.replace("~1", "/").replace("~0", "~")


def _split(path: str) -> List[str]:
    if path == "":
        return []
    if not path.startswith("/"):
        raise PatchError(f"invalid JSON pointer {path!r}")
    return [_unescape(t) for t in path[1:].split("/")]


# --------------------------------------------------------------------------- create


def create_patch(src: Any, dst: Any) -> List[dict]:
    """Return a list of RFC 6902 operations turning ``src`` into ``dst``.

    Lists are diffed element-wise by index with trailing adds/removes; this is the
    same strategy gomodules.xyz/jsonpatch uses for the controller-runtime response
    and it keeps the patch small for the webhook's typical "append a container /
    volume / env var" mutations.
    """
    ops: List[dict] = []
    _diff(src, dst, "", ops)
    return ops


def _diff(a: Any, b: Any, path: str, ops: List[dict]) -> None:
    if a is b:
        return
    if type(a) is dict and type(b) is dict:
        for k, av in a.items():
            p = path + "/" + _escape(k)
            if k not in b:
                ops.append({"op": "remove", "path": p})
            else:
                bv = b[k]
                if av != bv:
                    _diff(av, bv, p, ops)
        for k, bv in b.items():
            if k not in a:
                ops.append({"op": "add", "path": path + "/" + _escape(k), "value": deepcopy_json(bv)})
        return
    if type(a) is list and type(b) is list:
        n = min(len(a), len(b))
        for i in range(n):
            if a[i] != b[i]:
                _diff(a[i], b[i], f"{path}/{i}", ops)
        # remove from the back so indices stay valid
        for i in range(len(a) - 1, n - 1, -1):
            ops.append({"op": "remove", "path": f"{path}/{i}"})
        for i in range(n, len(b)):
            ops.append({"op": "add", "path": f"{path}/-", "value": deepcopy_json(b[i])})
        return
    if a != b or type(a) is not type(b):
        ops.append({"op": "replace", "path": path, "value": deepcopy_json(b)})


# --------------------------------------------------------------------------- apply


def _index(t: str) -> int:
    """RFC 6901 array index: ``0`` or digits without a leading zero — ``int()`` would also
    take ``-1`` (Python's from-the-end indexing), ``+1``, `` 1`` and ``1_0``."""
    if not (t.isascii() and t.isdigit()) or (len(t) > 1 and t[0] == "0") or len(t) > 9:
        raise PatchError(f"bad list index {t!r}")
    return int(t)


def _resolve_parent(doc: Any, tokens: List[str]):
    cur = doc
    for t in tokens[:-1]:
        if isinstance(cur, dict):
            if t not in cur:
                raise PatchError(f"path segment {t!r} not found")
            cur = cur[t]
        elif isinstance(cur, list):
            i = _index(t)
            if i >= len(cur):
                raise PatchError(f"bad list index {t!r}")
            cur = cur[i]
        else:
            raise PatchError(f"cannot traverse into scalar at {t!r}")
    return cur


def _get(doc: Any, tokens: List[str]) -> Any:
    cur = doc
    for t in tokens:
        if isinstance(cur, dict):
            if t not in cur:
                raise PatchError(f"path segment {t!r} not found")
            cur = cur[t]
        elif isinstance(cur, list):
            i = _index(t)
            if i >= len(cur):
                raise PatchError(f"bad list index {t!r}")
            cur = cur[i]
        else:
            raise PatchError("cannot traverse into scalar")
    return cur


def _add(doc: Any, tokens: List[str], value: Any) -> Any:
    if not tokens:
        return value
    parent = _resolve_parent(doc, tokens)
    last = tokens[-1]
    if isinstance(parent, dict):
        parent[last] = value
    elif isinstance(parent, list):
        if last == "-":
            parent.append(value)
        else:
            idx = _index(last)
            if idx > len(parent):
                raise PatchError(f"list index {idx} out of range")
            parent.insert(idx, value)
    else:
        raise PatchError("cannot add into scalar")
    return doc


def _remove(doc: Any, tokens: List[str]) -> Any:
    if not tokens:
        raise PatchError("cannot remove document root")
    parent = _resolve_parent(doc, tokens)
    last = tokens[-1]
    if isinstance(parent, dict):
        if last not in parent:
            raise PatchError(f"remove: {last!r} not found")
        return parent.pop(last)
    if isinstance(parent, list):
        i = _index(last)
        if i >= len(parent):
            raise PatchError(f"remove: bad index {last!r}")
        return parent.pop(i)
    raise PatchError("cannot remove from scalar")


def json_equal(a: Any, b: Any) -> bool:
    """RFC 6902 ``test`` equality: numbers by value, booleans only equal booleans (Python's
    ``True == 1`` is not JSON's), objects regardless of member order."""
    if isinstance(a, bool) or isinstance(b, bool):
        return isinstance(a, bool) and isinstance(b, bool) and a == b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return a == b
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(json_equal(v, b[k]) for k, v in a.items())
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(json_equal(x, y) for x, y in zip(a, b))
    return type(a) is type(b) and a == b


def apply_patch(doc: Any, ops: List[dict], in_place: bool = False) -> Any:
    """Apply an RFC 6902 patch; raises PatchError (→ HTTP 422) on failure."""
    if not in_place:
        doc = deepcopy_json(doc)
    for op in ops:
        kind = op.get("op")
        tokens = _split(op.get("path", ""))
        if kind == "add":
            doc = _add(doc, tokens, deepcopy_json(op.get("value")))
        elif kind == "remove":
            _remove(doc, tokens)
        elif kind == "replace":
            if not tokens:
                doc = deepcopy_json(op.get("value"))
                continue
            _get(doc, tokens)  # must exist
            parent = _resolve_parent(doc, tokens)
            last = tokens[-1]
            if isinstance(parent, list):
                parent[int(last)] = deepcopy_json(op.get("value"))
            else:
                parent[last] = deepcopy_json(op.get("value"))
        elif kind == "move":
            frm = _split(op.get("from", ""))
            val = _remove(doc, frm)
            doc = _add(doc, tokens, val)
        elif kind == "copy":
            val = deepcopy_json(_get(doc, _split(op.get("from", ""))))
            doc = _add(doc, tokens, val)
        elif kind == "test":
            if not json_equal(_get(doc, tokens), op.get("value")):
                raise PatchError(f"test failed at {op.get('path')}")
        else:
            raise PatchError(f"unknown op {kind!r}")
    return doc


# --------------------------------------------------------------------------- merge patch


def apply_merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386: ``null`` deletes, objects merge recursively, anything else replaces."""
    if not isinstance(patch, dict):
        return deepcopy_json(patch)
    if not isinstance(target, dict):
        target = {}
    else:
        target = dict(target)
    for k, v in patch.items():
        if v is None:
            target.pop(k, None)
        elif isinstance(v, dict):
            target[k] = apply_merge_patch(target.get(k), v)
        else:
            target[k] = deepcopy_json(v)
    return target


def create_merge_patch(src: Any, dst: Any) -> Any:
    """Smallest merge patch turning ``src`` into ``dst`` (``client.MergeFrom`` analogue)."""
    if not (isinstance(src, dict) and isinstance(dst, dict)):
        return deepcopy_json(dst)
    out = {}
    for k, sv in src.items():
        if k not in dst:
            out[k] = None
        elif sv != dst[k]:
            dv = dst[k]
            if isinstance(sv, dict) and isinstance(dv, dict):
                out[k] = create_merge_patch(sv, dv)
            else:
                out[k] = deepcopy_json(dv)
    for k, dv in dst.items():
        if k not in src:
            out[k] = deepcopy_json(dv)
    return out


# --------------------------------------------------------------------------- strategic merge (subset)

# Merge keys for the core list fields a notebook PodSpec uses.  Kubernetes'
# strategic merge patch looks these up in the Go struct tags; we keep the subset
# that kubectl users actually patch on Notebooks/StatefulSets.
_SMP_MERGE_KEYS = {
    "containers": "name",
    "initContainers": "name",
    "ephemeralContainers": "name",
    "env": "name",
    "volumes": "name",
    "volumeMounts": "mountPath",
    "ports": "containerPort",
    "imagePullSecrets": "name",
    "tolerations": None,
    "finalizers": None,
    "ownerReferences": "uid",
    "conditions": "type",
}


def apply_strategic_merge_patch(target: Any, patch: Any) -> Any:
    """Strategic merge patch for the list fields in ``_SMP_MERGE_KEYS``.

    Lists with a merge key are merged element-wise (``$patch: delete`` removes an
    element); other lists are replaced, as in Kubernetes.
    """
    if not isinstance(patch, dict):
        return deepcopy_json(patch)
    if not isinstance(target, dict):
        target = {}
    else:
        target = dict(target)
    for k, v in patch.items():
        if k.startswith("$"):
            continue
        if v is None:
            target.pop(k, None)
        elif isinstance(v, dict):
            target[k] = apply_strategic_merge_patch(target.get(k), v)
        elif isinstance(v, list) and _SMP_MERGE_KEYS.get(k) and isinstance(target.get(k), list):
            key = _SMP_MERGE_KEYS[k]
            merged = [deepcopy_json(x) for x in target[k]]
            for item in v:
                if not isinstance(item, dict) or key not in item:
                    merged.append(deepcopy_json(item))
                    continue
                idx = next((i for i, e in enumerate(merged) if isinstance(e, dict) and e.get(key) == item[key]), None)
                if item.get("$patch") == "delete":
                    if idx is not None:
                        merged.pop(idx)
                    continue
                if idx is None:
                    merged.append(deepcopy_json(item))
                else:
                    merged[idx] = apply_strategic_merge_patch(merged[idx], item)
            target[k] = merged
        else:
            target[k] = deepcopy_json(v)
    return target
