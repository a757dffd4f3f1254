"""``k8s.io/client-go/util/retry`` analogues.

``retry_on_conflict`` uses ``retry.DefaultRetry`` (5 steps, 10 ms, factor 1, jitter 0.1),
as every ``RetryOnConflict`` call site in the reference does — with one change: the first
retry reads live from the apiserver (see ``client.LIVE_READS``) and runs at once.  A
conflict almost always means the informer copy was one write behind; the reference pays
the 10 ms sleep and often a second conflict for it, on the create→Ready path.
"""

from __future__ import annotations

import asyncio
import random
from dataclasses import dataclass
from typing import Awaitable, Callable, TypeVar

from ..models.errors import is_conflict

T = TypeVar("T")


@dataclass
class Backoff:
    steps: int = 5
    duration: float = 0.010
    factor: float = 1.0
    jitter: float = 0.1
    cap: float = 0.0

    def delays(self):
        d = self.duration
        for _ in range(self.steps - 1):
            j = d + (random.random() * self.jitter * d if self.jitter > 0 else 0.0)
            yield j
            d = d * self.factor if self.factor else d
            if self.cap and d > self.cap:
                d = self.cap


DEFAULT_RETRY = Backoff(5, 0.010, 1.0, 0.1)
DEFAULT_BACKOFF = Backoff(4, 0.010, 5.0, 0.1)


async def retry_on_error(backoff: Backoff, retriable: Callable[[BaseException], bool],
                         fn: Callable[[], Awaitable[T]]) -> T:
    delays = backoff.delays()
    while True:
        try:
            return await fn()
        except Exception as e:
            if not retriable(e):
                raise
            try:
                d = next(delays)
            except StopIteration:
                raise e
            await asyncio.sleep(d)


async def retry_on_conflict(fn: Callable[[], Awaitable[T]], backoff: Backoff = DEFAULT_RETRY) -> T:
    from .client import LIVE_READS

    delays = backoff.delays()
    attempt = 0
    while True:
        tok = LIVE_READS.set(attempt > 0)
        try:
            return await fn()
        except Exception as e:
            if not is_conflict(e):
                raise
            try:
                d = next(delays)
            except StopIteration:
                raise e
            if attempt > 0:
                await asyncio.sleep(d)
            attempt += 1
        finally:
            LIVE_READS.reset(tok)
