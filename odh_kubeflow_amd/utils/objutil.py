"""Helpers for JSON-tree ("unstructured") Kubernetes objects.

Every object that flows through the framework is a plain ``dict`` in Kubernetes wire
form (``apiVersion``/``kind``/``metadata``/``spec``/``status``).  Copying those trees is
the dominant cost of an in-memory apiserver and of an informer cache, so
``deepcopy_json`` dispatches to the native ``_objcore`` extension (C++, built by
``__graft_entry__.build``) when it is importable and falls back to a tight Python
recursion otherwise.
"""

from __future__ import annotations

from typing import Any, Iterable, Optional


def _py_deepcopy_json(o: Any) -> Any:
    t = type(o)
    if t is dict:
        return {k: (v if type(v) in _SCALARS else _py_deepcopy_json(v)) for k, v in o.items()}
    if t is list:
        return [(v if type(v) in _SCALARS else _py_deepcopy_json(v)) for v in o]
    if t is tuple:
        return [_py_deepcopy_json(v) for v in o]
    return o


_SCALARS = frozenset((str, int, float, bool, type(None)))

try:  # native fast path (odh_kubeflow_amd/native/objcore.cpp)
    from ..native import _objcore  # type: ignore

    deepcopy_json = _objcore.deepcopy
    NATIVE_OBJCORE = True
except Exception:  # pragma: no cover - exercised when the extension is not built
    deepcopy_json = _py_deepcopy_json
    NATIVE_OBJCORE = False


def get_nested(obj: Any, *path: str, default: Any = None) -> Any:
    cur = obj
    for p in path:
        if not isinstance(cur, dict):
            return default
        cur = cur.get(p)
        if cur is None:
            return default
    return cur


def set_nested(obj: dict, value: Any, *path: str) -> None:
    cur = obj
    for p in path[:-1]:
        nxt = cur.get(p)
        if not isinstance(nxt, dict):
            nxt = {}
            cur[p] = nxt
        cur = nxt
    cur[path[-1]] = value


def ensure_dict(obj: dict, *path: str) -> dict:
    cur = obj
    for p in path:
        nxt = cur.get(p)
        if not isinstance(nxt, dict):
            nxt = {}
            cur[p] = nxt
        cur = nxt
    return cur


def ensure_list(obj: dict, *path: str) -> list:
    parent = ensure_dict(obj, *path[:-1]) if len(path) > 1 else obj
    cur = parent.get(path[-1])
    if not isinstance(cur, list):
        cur = []
        parent[path[-1]] = cur
    return cur


def prune_empty(o: Any) -> Any:
    """Drop ``None`` values and empty maps/lists, like Go's ``omitempty`` on marshal."""
    if isinstance(o, dict):
        out = {}
        for k, v in o.items():
            v = prune_empty(v)
            if v is None or (isinstance(v, (dict, list)) and not v):
                continue
            out[k] = v
        return out
    if isinstance(o, list):
        return [prune_empty(v) for v in o]
    return o


def _py_semantic_equal(a: Any, b: Any) -> bool:
    """``equality.Semantic.DeepEqual`` analogue: absent == empty for maps/lists/None."""
    return prune_empty(a) == prune_empty(b)


def _py_equal_except(a: dict, b: dict, keys) -> bool:
    ma, mb = dict(a.get("metadata") or {}), dict(b.get("metadata") or {})
    for k in keys:
        ma.pop(k, None)
        mb.pop(k, None)
    return ({**a, "metadata": ma} if "metadata" in a else a) == ({**b, "metadata": mb} if "metadata" in b else b)


if NATIVE_OBJCORE:
    semantic_equal = _objcore.semantic_equal
    equal_except = _objcore.equal_except
else:  # pragma: no cover
    semantic_equal = _py_semantic_equal
    equal_except = _py_equal_except


def find_by_name(items: Optional[Iterable[dict]], name: str) -> Optional[dict]:
    for it in items or ():
        if isinstance(it, dict) and it.get("name") == name:
            return it
    return None


def index_by_name(items: Optional[list], name: str) -> int:
    for i, it in enumerate(items or ()):
        if isinstance(it, dict) and it.get("name") == name:
            return i
    return -1
