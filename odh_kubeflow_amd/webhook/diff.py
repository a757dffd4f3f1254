"""First-difference reporter for the restart guard.

The reference reports the first differing path of two PodSpecs with a go-cmp reporter
(``odh/controllers/notebook_webhook_utils.go:27-80``) and stores it in the
``notebooks.opendatahub.io/update-pending`` annotation.  This walks two JSON values in
a deterministic order (mapping keys sorted, lists by index) and renders the first
difference as ``<path>: <a> != <b>``.
"""

from __future__ import annotations

import json
from typing import Any, Optional

_MISSING = object()


def _fmt(v: Any) -> str:
    if v is _MISSING:
        return "<missing>"
    try:
        return json.dumps(v, sort_keys=True, separators=(",", ":"))
    except (TypeError, ValueError):
        return repr(v)


def _first(a: Any, b: Any, path: str) -> Optional[str]:
    if a is _MISSING or b is _MISSING or type(a) is not type(b):
        if a == b and a is not _MISSING:
            return None
        return f"{path}: {_fmt(a)} != {_fmt(b)}"
    if isinstance(a, dict):
        for k in sorted(set(a) | set(b)):
            d = _first(a.get(k, _MISSING), b.get(k, _MISSING), f"{path}.{k}" if path else k)
            if d:
                return d
        return None
    if isinstance(a, list):
        for i in range(max(len(a), len(b))):
            d = _first(a[i] if i < len(a) else _MISSING, b[i] if i < len(b) else _MISSING, f"{path}[{i}]")
            if d:
                return d
        return None
    if a != b:
        return f"{path}: {_fmt(a)} != {_fmt(b)}"
    return None


def first_difference(a: Any, b: Any, root: str = "PodSpec") -> str:
    """Human-readable single line naming the first difference ('' when equal)."""
    try:
        return _first(a, b, root) or ""
    except RecursionError:
        return "failed to compute the reason for why there is a pending restart"
