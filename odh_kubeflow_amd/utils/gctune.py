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

Every collection's pause is recorded (:data:`PAUSES`, installed by ``tune()``): the
managers export it as ``odh_gc_pause_seconds{generation}`` (Go's ``go_gc_duration_seconds``)
and on ``/debug/gc``, so a stopped event loop shows up by name instead of as an unexplained
admission or reconcile tail.
"""

from __future__ import annotations

import collections
import gc
import os
import sys
import time
from typing import Dict, List

DEFAULT_THRESHOLDS = (50_000, 20, 100)
_STALL_MS = float(os.environ.get("ODH_STALL_WATCHDOG_MS") or 0)
_BOUNDS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0)


class PauseRecorder:
    """``gc.callbacks`` hook: each collection's wall time and generation (the newest 4096),
    plus a per-generation histogram."""

    def __init__(self, keep: int = 4096):
        self.seq = 0
        self.recent = collections.deque(maxlen=keep)  # (seq, generation, seconds)
        self.counts: Dict[int, List[int]] = {g: [0] * (len(_BOUNDS) + 1) for g in range(3)}
        self.sums: Dict[int, float] = {g: 0.0 for g in range(3)}
        self._t0 = 0.0
        self.installed = False

    def __call__(self, phase: str, info: dict) -> None:
        if phase == "start":
            self._t0 = time.perf_counter()
            return
        d = time.perf_counter() - self._t0
        g = int(info.get("generation", 0))
        self.seq += 1
        self.recent.append((self.seq, g, d))
        self.sums[g] = self.sums.get(g, 0.0) + d
        if _STALL_MS and d * 1e3 >= _STALL_MS:  # diagnostics (ODH_STALL_WATCHDOG_MS)
            print(f"stall-watchdog: pid {os.getpid()} gc generation {g} took {d * 1e3:.1f} ms ending at "
                  f"{time.time():.6f}", file=sys.stderr, flush=True)
        b = self.counts.setdefault(g, [0] * (len(_BOUNDS) + 1))
        i = 0
        while i < len(_BOUNDS) and d > _BOUNDS[i]:
            i += 1
        b[i] += 1

    def install(self) -> "PauseRecorder":
        if not self.installed:
            gc.callbacks.append(self)
            self.installed = True
        return self

    def since(self, seq: int = 0) -> dict:
        """Pauses after ``seq``: ``{"seq": newest, "pauses": [[seq, generation, ms], ...]}``."""
        return {"seq": self.seq, "pauses": [[s, g, round(d * 1e3, 3)] for s, g, d in self.recent if s > seq]}

    def collect(self):
        """Prometheus collector: ``odh_gc_pause_seconds`` histogram per generation."""
        from prometheus_client.core import HistogramMetricFamily

        h = HistogramMetricFamily("odh_gc_pause_seconds", "Wall time of CPython cyclic-GC collections "
                                  "(the event loop is stopped for it)", labels=["generation"])
        for g in sorted(self.counts):
            acc, buckets = 0, []
            for bound, c in zip(_BOUNDS + (float("inf"),), self.counts[g]):
                acc += c
                buckets.append(("+Inf" if bound == float("inf") else repr(bound), acc))
            h.add_metric([str(g)], buckets, self.sums[g])
        yield h


PAUSES = PauseRecorder()


def tune(thresholds=DEFAULT_THRESHOLDS) -> None:
    gc.collect()
    gc.freeze()
    gc.set_threshold(*thresholds)
    PAUSES.install()
