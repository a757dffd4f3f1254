"""The CEL subset a MutatingWebhookConfiguration's ``matchConditions`` may use here.

kube-apiserver (``matchConditions``, GA in 1.30, beta and on by default since 1.28) calls a
webhook only when every condition evaluates to true; a condition that errors leaves the
decision to the webhook's ``failurePolicy`` (``Fail``: the request is refused; ``Ignore``:
the webhook is skipped).  The two test apiservers evaluate the subset this repository's
configurations use — ``has(<root>.<field>…)``, ``!``, ``&&``, ``||``, parentheses, ``true``
and ``false`` over the roots ``object`` and ``oldObject`` (null on CREATE) — and refuse any
other expression as a compile error rather than guess at it.  The native apiserver has the
same evaluator (``testing/native/apiserver/apiserver.cpp``, ``cel_*``).

CEL's logical operators absorb errors: ``false && <error>`` is false and
``true || <error>`` is true, whichever side errs.
"""

from __future__ import annotations

import re
from typing import Callable, List, Optional

ROOTS = ("object", "oldObject")
_TOKEN = re.compile(r"\s*(?:(\|\||&&|[!().])|([A-Za-z_][A-Za-z0-9_]*))")


class CelError(Exception):
    """A compile error (unsupported expression) or an evaluation error (no such key)."""


Condition = Callable[[Optional[dict], Optional[dict]], bool]


def _tokens(expr: str) -> List[str]:
    out, i = [], 0
    while i < len(expr):
        if expr[i:].strip() == "":
            break
        mo = _TOKEN.match(expr, i)
        if not mo:
            raise CelError(f"unsupported CEL at {expr[i:]!r}")
        out.append(mo.group(1) or mo.group(2))
        i = mo.end()
    return out


def compile_condition(expr: str) -> Condition:
    """``expr`` → ``f(object, oldObject)`` returning a bool or raising :class:`CelError`."""
    toks = _tokens(expr)
    pos = 0

    def peek():
        return toks[pos] if pos < len(toks) else None

    def take(want=None):
        nonlocal pos
        t = peek()
        if t is None or (want is not None and t != want):
            raise CelError(f"expected {want or 'a term'} in {expr!r}")
        pos += 1
        return t

    def disj():
        terms = [conj()]
        while peek() == "||":
            take()
            terms.append(conj())
        return terms[0] if len(terms) == 1 else ("or", terms)

    def conj():
        terms = [unary()]
        while peek() == "&&":
            take()
            terms.append(unary())
        return terms[0] if len(terms) == 1 else ("and", terms)

    def unary():
        if peek() == "!":
            take()
            return ("not", unary())
        return primary()

    def primary():
        t = take()
        if t == "(":
            e = disj()
            take(")")
            return e
        if t in ("true", "false"):
            return ("lit", t == "true")
        if t == "has":
            take("(")
            root = take()
            if root not in ROOTS:
                raise CelError(f"unsupported root {root!r} in {expr!r}")
            path = []
            while peek() == ".":
                take()
                f = take()
                if not re.fullmatch(r"[A-Za-z_][A-Za-z0-9_]*", f):
                    raise CelError(f"unsupported field {f!r} in {expr!r}")
                path.append(f)
            if not path:
                raise CelError(f"has() needs a field selection in {expr!r}")
            take(")")
            return ("has", root, path)
        raise CelError(f"unsupported CEL term {t!r} in {expr!r}")

    tree = disj()
    if pos != len(toks):
        raise CelError(f"trailing tokens in {expr!r}")

    def ev(n, obj, old):
        k = n[0]
        if k == "lit":
            return n[1]
        if k == "not":
            return not ev(n[1], obj, old)
        if k in ("and", "or"):
            absorbing = k == "or"  # true absorbs errors in ||, false in &&
            err = None
            for t in n[1]:
                try:
                    if ev(t, obj, old) == absorbing:
                        return absorbing
                except CelError as e:
                    err = e
            if err is not None:
                raise err
            return not absorbing
        cur = obj if n[1] == "object" else old
        if cur is None:
            raise CelError(f"{n[1]} is null")
        for f in n[2][:-1]:
            if not isinstance(cur, dict) or f not in cur:
                raise CelError(f"no such key: {f}")
            cur = cur[f]
        if not isinstance(cur, dict):
            raise CelError(f"has() on a non-map before {n[2][-1]}")
        return cur.get(n[2][-1]) is not None

    return lambda obj, old: ev(tree, obj, old)


def conditions_allow(conds: List[Condition], obj: Optional[dict], old: Optional[dict],
                     fail_closed: bool) -> bool:
    """Whether the webhook is called: every condition true.  Any false condition skips it,
    whatever the others do; otherwise an evaluation error refuses the request when
    ``fail_closed`` (raises :class:`CelError`) and skips the webhook when not."""
    err = None
    for c in conds:
        try:
            if not c(obj, old):
                return False
        except CelError as e:
            err = e
    if err is not None:
        if fail_closed:
            raise err
        return False
    return True
