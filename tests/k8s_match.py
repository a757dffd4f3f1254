"""``assert_matching_k8s_resource`` — the envtest suite's ``BeMatchingK8sResource``
matcher (``odh/controllers/matchers_test.go:79-491``): compare two objects with the
controller's own comparator and, on mismatch, fail with a full diff AND a minimized diff
— only the differences the comparator actually looks at (server-set metadata such as
``uid`` / ``resourceVersion`` / ``managedFields`` drops out).

A difference belongs to the minimized diff when applying it alone to ``expected`` makes
the comparator reject the result.
"""

from __future__ import annotations

import copy
import json
from typing import Any, Callable, List, Tuple

_MISSING = object()


def diff_paths(a: Any, b: Any, path: Tuple = ()) -> List[Tuple[Tuple, Any, Any]]:
    """Leaf differences ``(path, a_value, b_value)``; missing members are ``_MISSING``."""
    if isinstance(a, dict) and isinstance(b, dict):
        out = []
        for k in sorted(set(a) | set(b), key=str):
            out += diff_paths(a.get(k, _MISSING), b.get(k, _MISSING), path + (k,))
        return out
    if isinstance(a, list) and isinstance(b, list) and len(a) == len(b):
        out = []
        for i, (x, y) in enumerate(zip(a, b)):
            out += diff_paths(x, y, path + (i,))
        return out
    return [] if a == b else [(path, a, b)]


def _set(doc: Any, path: Tuple, value: Any) -> Any:
    if not path:
        return value
    cur = doc
    for k in path[:-1]:
        if isinstance(cur, dict) and k not in cur:
            cur[k] = {}
        cur = cur[k]
    if value is _MISSING:
        if isinstance(cur, dict):
            cur.pop(path[-1], None)
    else:
        cur[path[-1]] = value
    return doc


def _fmt(diffs) -> str:
    def v(x):
        return "<absent>" if x is _MISSING else json.dumps(x, sort_keys=True)
    return "\n".join(f"  {'.'.join(map(str, p)) or '<root>'}: -{v(a)} +{v(e)}" for p, a, e in diffs) or "  (none)"


def minimized_diff(actual: dict, expected: dict, comparator: Callable[[dict, dict], bool]):
    out = []
    for p, a, e in diff_paths(actual, expected):
        probe = _set(copy.deepcopy(expected), p, copy.deepcopy(a))
        if not comparator(expected, probe):
            out.append((p, a, e))
    return out


def assert_matching_k8s_resource(actual: dict, expected: dict, comparator: Callable[[dict, dict], bool]) -> None:
    if comparator(expected, actual):
        return
    full = diff_paths(actual, expected)
    raise AssertionError("resource does not match (comparator rejected it)\n"
                         f"full diff (-actual +expected):\n{_fmt(full)}\n"
                         f"minimized diff (-actual +expected):\n{_fmt(minimized_diff(actual, expected, comparator))}")
