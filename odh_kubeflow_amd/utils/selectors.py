"""Label and field selectors (``metav1.LabelSelector`` + the string query syntax).

The fake apiserver and the informer cache both filter List/Watch with these; the ODH
reconciler looks up its HTTPRoutes in the central namespace purely by label
(``odh/controllers/notebook_route.go:155-165``) because a cross-namespace ownerRef is
impossible.
"""

from __future__ import annotations

import re
from typing import Callable, Dict, List, Optional, Tuple

from .objutil import get_nested

Req = Tuple[str, str, Tuple[str, ...]]  # (key, op, values)

_TOKEN = re.compile(r"\s*([^,()!=\s]+(?:\([^)]*\))?)\s*")


def parse_label_selector(text: Optional[str]) -> List[Req]:
    """Parse ``a=b,c!=d,e in (x,y),f notin (z),g,!h`` into requirements."""
    reqs: List[Req] = []
    if not text:
        return reqs
    parts = _split_top(text)
    for p in parts:
        p = p.strip()
        if not p:
            continue
        m = re.match(r"^([\w./-]+)\s+(in|notin)\s+\(([^)]*)\)$", p)
        if m:
            vals = tuple(v.strip() for v in m.group(3).split(",") if v.strip())
            reqs.append((m.group(1), m.group(2), vals))
            continue
        if p.startswith("!"):
            reqs.append((p[1:].strip(), "!", ()))
            continue
        for op in ("==", "!=", "="):
            if op in p:
                k, v = p.split(op, 1)
                reqs.append((k.strip(), "!=" if op == "!=" else "=", (v.strip(),)))
                break
        else:
            reqs.append((p, "exists", ()))
    return reqs


def _split_top(text: str) -> List[str]:
    out, depth, cur = [], 0, []
    for ch in text:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return out


def selector_from_dict(sel: Optional[dict]) -> List[Req]:
    """Convert ``metav1.LabelSelector`` (matchLabels + matchExpressions) to requirements."""
    reqs: List[Req] = []
    if not sel:
        return reqs
    for k, v in (sel.get("matchLabels") or {}).items():
        reqs.append((k, "=", (v,)))
    for e in sel.get("matchExpressions") or []:
        op = {"In": "in", "NotIn": "notin", "Exists": "exists", "DoesNotExist": "!"}[e["operator"]]
        reqs.append((e["key"], op, tuple(e.get("values") or ())))
    return reqs


def match_labels(reqs: List[Req], labels: Optional[Dict[str, str]]) -> bool:
    labels = labels or {}
    for key, op, vals in reqs:
        has = key in labels
        if op == "=":
            if not has or labels[key] != vals[0]:
                return False
        elif op == "!=":
            if has and labels[key] == vals[0]:
                return False
        elif op == "in":
            if not has or labels[key] not in vals:
                return False
        elif op == "notin":
            if has and labels[key] in vals:
                return False
        elif op == "exists":
            if not has:
                return False
        elif op == "!":
            if has:
                return False
    return True


def format_label_selector(labels: Dict[str, str]) -> str:
    return ",".join(f"{k}={v}" for k, v in sorted(labels.items()))


def parse_field_selector(text: Optional[str]) -> List[Tuple[str, str, str]]:
    out = []
    if not text:
        return out
    for p in text.split(","):
        p = p.strip()
        if not p:
            continue
        if "!=" in p:
            k, v = p.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        else:
            k, v = p.split("==", 1) if "==" in p else p.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
    return out


def field_matcher(reqs: List[Tuple[str, str, str]]) -> Callable[[dict], bool]:
    paths = [(tuple(k.split(".")), op, v) for k, op, v in reqs]

    def match(obj: dict) -> bool:
        for path, op, v in paths:
            got = get_nested(obj, *path)
            got = "" if got is None else str(got)
            if (got == v) != (op == "="):
                return False
        return True

    return match
