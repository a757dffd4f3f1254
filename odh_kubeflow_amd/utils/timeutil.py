"""RFC3339 timestamps as the Go controllers format them (``time.RFC3339``, UTC ``Z``).

Culling compares annotation timestamps with second granularity
(``kf/controllers/culling_controller.go:514-517``); ``metav1.Time`` also serialises at
second precision.  A module-level clock indirection lets tests freeze or fast-forward
time without sleeping.
"""

from __future__ import annotations

import datetime as _dt
import time as _time
from typing import Callable, Optional

_clock: Callable[[], float] = _time.time


def set_clock(fn: Optional[Callable[[], float]]) -> None:
    global _clock
    _clock = fn or _time.time


def now() -> float:
    return _clock()


def rfc3339(ts: Optional[float] = None) -> str:
    if ts is None:
        ts = _clock()
    return _dt.datetime.fromtimestamp(int(ts), tz=_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def rfc3339_micro(ts: Optional[float] = None) -> str:
    if ts is None:
        ts = _clock()
    return _dt.datetime.fromtimestamp(ts, tz=_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_rfc3339(text: Optional[str]) -> Optional[float]:
    """Parse RFC3339 / RFC3339Nano (with ``Z`` or numeric offset); ``None`` on error."""
    if not text or not isinstance(text, str):
        return None
    s = text.strip()
    try:
        if s.endswith("Z") or s.endswith("z"):
            s = s[:-1] + "+00:00"
        # trim nanoseconds to microseconds for fromisoformat
        if "." in s:
            head, rest = s.split(".", 1)
            frac = ""
            i = 0
            while i < len(rest) and rest[i].isdigit():
                frac += rest[i]
                i += 1
            s = head + "." + (frac[:6].ljust(6, "0")) + rest[i:]
        d = _dt.datetime.fromisoformat(s)
        if d.tzinfo is None:
            return None
        return d.timestamp()
    except ValueError:
        return None
