"""Kubernetes ``resource.Quantity`` parsing and canonical formatting.

Used to validate the four auth-sidecar resource annotations (reference:
``odh/controllers/notebook_webhook.go:126-173``) and to size notebook pods for
MI355X (``amd.com/gpu`` counts, memory sized against 288 GB of HBM3E per device).
Values are held as exact ``fractions.Fraction`` so comparisons never round.
"""

from __future__ import annotations

import re
from fractions import Fraction

_BINARY = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DECIMAL = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
            "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
            "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}

_RE = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+))(?:([eE][+-]?\d+)|(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E))?$")


class QuantityError(ValueError):
    pass


class Quantity:
    __slots__ = ("value", "text", "binary", "_canon")

    def __init__(self, text: str):
        s = str(text).strip()
        m = _RE.match(s)
        if not m:
            raise QuantityError(f"quantities must match the regular expression '^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$': {text!r}")
        num, exp, suffix = m.group(1), m.group(2), m.group(3)
        v = Fraction(num)
        self.binary = False
        if exp:
            v *= Fraction(10) ** int(exp[1:])
        elif suffix:
            if suffix in _BINARY:
                v *= _BINARY[suffix]
                self.binary = True
            else:
                v *= _DECIMAL[suffix]
        self.value = v
        self.text = s
        self._canon = None

    def sign(self) -> int:
        return (self.value > 0) - (self.value < 0)

    def cmp(self, other: "Quantity") -> int:
        return (self.value > other.value) - (self.value < other.value)

    def __lt__(self, o):
        return self.value < o.value

    def __le__(self, o):
        return self.value <= o.value

    def __eq__(self, o):
        return isinstance(o, Quantity) and self.value == o.value

    def __hash__(self):
        return hash(self.value)

    def milli(self) -> int:
        return int(self.value * 1000)

    def __str__(self) -> str:
        return canonical(self)

    def __repr__(self) -> str:
        return f"Quantity({self.text!r})"


_QCACHE: dict = {}


def parse_quantity(text) -> Quantity:
    """Parsed quantities are immutable and the same few strings recur on every pod
    (``"1"``, ``"100m"``, ``"64Mi"``): memoized."""
    if type(text) is str:
        q = _QCACHE.get(text)
        if q is None:
            q = Quantity(text)
            if len(_QCACHE) > 4096:
                _QCACHE.clear()
            _QCACHE[text] = q
        return q
    return Quantity(text)


def canonical(q: Quantity) -> str:
    """Canonical string the apiserver would echo back (``"100m"``, ``"64Mi"``, ``"2"``).
    Computed once per (memoized, immutable) Quantity: the defaulting of every pod template
    the controllers compare asks for the same few values."""
    c = q._canon
    if c is None:
        c = q._canon = _canonical(q)
    return c


def _canonical(q: Quantity) -> str:
    v = q.value
    if v == 0:
        return "0"
    if q.binary:
        for suf in ("Ei", "Pi", "Ti", "Gi", "Mi", "Ki"):
            base = _BINARY[suf]
            if v % base == 0:
                return f"{v // base}{suf}"
        if v.denominator == 1:
            return str(v.numerator)
    if v.denominator == 1:
        n = v.numerator
        for suf, exp in (("E", 18), ("P", 15), ("T", 12), ("G", 9), ("M", 6), ("k", 3)):
            if n % (10 ** exp) == 0:
                return f"{n // 10 ** exp}{suf}"
        return str(n)
    for suf, scale in (("m", 1000), ("u", 10 ** 6), ("n", 10 ** 9)):
        x = v * scale
        if x.denominator == 1:
            return f"{x.numerator}{suf}"
    return f"{int(v * 10 ** 9)}n"


def to_bytes(text) -> int:
    return int(parse_quantity(text).value)
