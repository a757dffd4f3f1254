"""Rate-limited, de-duplicating work queue (client-go ``workqueue`` semantics on asyncio).

* An item is queued at most once; re-adding an item that a worker is processing marks
  it dirty and it is re-queued when the worker calls :meth:`done` — so one object is
  never reconciled by two workers at once, whatever ``MaxConcurrentReconciles`` is.
* :meth:`add_after` backs ``Result.requeue_after`` (the culler's
  ``RequeueAfter(IDLENESS_CHECK_PERIOD)``, ``kf/controllers/culling_controller.go:202``).
* :meth:`add_rate_limited` applies max(per-item exponential 5 ms→1000 s, 10 qps / 100
  burst token bucket) — controller-runtime's default controller rate limiter.
"""

from __future__ import annotations

import asyncio
import os
import sys
import time
from collections import deque
from typing import Any, Deque, Dict, Hashable, Optional, Set


# ODH_STALL_WATCHDOG_MS (diagnostics): items that wait in the queue, or are requeued with a
# delay (under a second), at least this long are reported to stderr
_STALL_MS = float(os.environ.get("ODH_STALL_WATCHDOG_MS") or 0)


def stall_report(what: str) -> None:
    print(f"stall-watchdog: pid {os.getpid()} {what} ending at {time.time():.6f}", file=sys.stderr, flush=True)


class ExponentialRateLimiter:
    def __init__(self, base: float = 0.005, cap: float = 1000.0):
        self.base, self.cap = base, cap
        self.failures: Dict[Hashable, int] = {}

    def when(self, item) -> float:
        n = self.failures.get(item, 0)
        self.failures[item] = n + 1
        return min(self.cap, self.base * (2 ** n))

    def forget(self, item) -> None:
        self.failures.pop(item, None)

    def num_requeues(self, item) -> int:
        return self.failures.get(item, 0)


class BucketRateLimiter:
    def __init__(self, qps: float = 10.0, burst: int = 100):
        self.qps, self.burst = qps, burst
        self.tokens = float(burst)
        self.last = time.monotonic()

    def when(self, item) -> float:
        now = time.monotonic()
        self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
        self.last = now
        self.tokens -= 1.0
        if self.tokens >= 0:
            return 0.0
        return -self.tokens / self.qps

    def forget(self, item) -> None:
        pass

    def num_requeues(self, item) -> int:
        return 0


class MaxOfRateLimiter:
    def __init__(self, *limiters):
        self.limiters = limiters

    def when(self, item) -> float:
        return max(l.when(item) for l in self.limiters)

    def forget(self, item) -> None:
        for l in self.limiters:
            l.forget(item)

    def num_requeues(self, item) -> int:
        return max(l.num_requeues(item) for l in self.limiters)


def default_controller_rate_limiter():
    return MaxOfRateLimiter(ExponentialRateLimiter(0.005, 1000.0), BucketRateLimiter(10.0, 100))


class ShutDown(Exception):
    pass


class WorkQueue:
    def __init__(self, name: str = "", rate_limiter=None, metrics=None):
        self.name = name
        self.rate_limiter = rate_limiter or default_controller_rate_limiter()
        self._queue: Deque[Any] = deque()
        self._dirty: Set[Any] = set()
        self._processing: Set[Any] = set()
        self._added_at: Dict[Any, float] = {}
        self._waiting: Dict[Any, asyncio.TimerHandle] = {}
        self._waiting_when: Dict[Any, float] = {}
        self._cond: Optional[asyncio.Condition] = None
        self._getters: Deque[asyncio.Future] = deque()
        self._shutdown = False
        self.metrics = metrics
        self.adds = 0

    # --------------------------------------------------------------- core

    def __len__(self) -> int:
        return len(self._queue)

    def add(self, item) -> None:
        if self._shutdown or item in self._dirty:
            return
        self.adds += 1
        self._dirty.add(item)
        if item in self._processing:
            return
        self._queue.append(item)
        self._added_at[item] = time.monotonic()
        if self.metrics:
            self.metrics.on_add(self.name, len(self._queue))
        self._wake()

    def _wake(self) -> None:
        while self._getters:
            fut = self._getters.popleft()
            if not fut.done():
                fut.set_result(None)
                return

    async def get(self):
        while not self._queue:
            if self._shutdown:
                raise ShutDown()
            fut = asyncio.get_running_loop().create_future()
            self._getters.append(fut)
            try:
                await fut
            except asyncio.CancelledError:
                if fut in self._getters:
                    self._getters.remove(fut)
                raise
        item = self._queue.popleft()
        self._processing.add(item)
        self._dirty.discard(item)
        t0 = self._added_at.pop(item, None)
        if _STALL_MS and t0 is not None and (time.monotonic() - t0) * 1e3 >= _STALL_MS:
            stall_report(f"queue {self.name}: {item} waited {(time.monotonic() - t0) * 1e3:.1f} ms for a worker")
        if self.metrics and t0 is not None:
            self.metrics.on_get(self.name, len(self._queue), time.monotonic() - t0)
        return item

    def done(self, item) -> None:
        self._processing.discard(item)
        if item in self._dirty:
            self._queue.append(item)
            self._added_at[item] = time.monotonic()
            self._wake()

    # --------------------------------------------------------------- delaying

    def add_after(self, item, delay: float) -> None:
        if self._shutdown:
            return
        if delay <= 0:
            self.add(item)
            return
        if _STALL_MS and _STALL_MS <= delay * 1e3 < 1000:
            stall_report(f"queue {self.name}: {item} requeued {delay * 1e3:.1f} ms ahead")
        loop = asyncio.get_running_loop()
        when = loop.time() + delay
        prev = self._waiting_when.get(item)
        if prev is not None and prev <= when:
            return
        h = self._waiting.pop(item, None)
        if h is not None:
            h.cancel()
        self._waiting_when[item] = when

        def fire():
            self._waiting.pop(item, None)
            self._waiting_when.pop(item, None)
            self.add(item)

        self._waiting[item] = loop.call_at(when, fire)

    # --------------------------------------------------------------- rate limiting

    def add_rate_limited(self, item) -> None:
        if self.metrics:
            self.metrics.on_retry(self.name)
        self.add_after(item, self.rate_limiter.when(item))

    def forget(self, item) -> None:
        self.rate_limiter.forget(item)

    def num_requeues(self, item) -> int:
        return self.rate_limiter.num_requeues(item)

    # --------------------------------------------------------------- lifecycle

    def shutdown(self) -> None:
        self._shutdown = True
        for h in self._waiting.values():
            h.cancel()
        self._waiting.clear()
        self._waiting_when.clear()
        while self._getters:
            fut = self._getters.popleft()
            if not fut.done():
                fut.set_result(None)

    @property
    def shutting_down(self) -> bool:
        return self._shutdown

    def pending(self, timers_within: Optional[float] = None) -> int:
        """Items queued, in process or waiting on a delay; ``timers_within``: only the delayed
        ones due within that many seconds (a requeue a period away is not outstanding work)."""
        n = len(self._queue) + len(self._processing)
        if timers_within is None or not self._waiting_when:
            return n + len(self._waiting)
        due = asyncio.get_running_loop().time() + timers_within
        return n + sum(1 for w in self._waiting_when.values() if w <= due)
