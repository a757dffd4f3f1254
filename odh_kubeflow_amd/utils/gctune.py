"""Garbage-collector settings for long-running control-plane processes.

The controllers' objects are JSON trees freed by reference counting; CPython's cyclic
collector only finds garbage in the few framework objects that form cycles.  But a
generation-2 pass walks EVERY tracked container — with torch + ROCm loaded (the node agent
needs them) that is ~1M objects, 25–55 ms of a stopped event loop, which showed up as
80–135 ms create→Ready outliers in the benchmark (p50 3.5 ms).  The Go reference tunes its
collector the same way through ``GOMEMLIMIT`` (``odh/config/manager/manager.yaml:58-59``).

``tune()`` moves everything alive after start-up (imports, caches, compiled code) into the
permanent generation with ``gc.freeze()`` and raises the generation-0 threshold so young
collections run less often; cyclic garbage is still collected.
"""

from __future__ import annotations

import gc

DEFAULT_THRESHOLDS = (50_000, 20, 100)


def tune(thresholds=DEFAULT_THRESHOLDS) -> None:
    gc.collect()
    gc.freeze()
    gc.set_threshold(*thresholds)
