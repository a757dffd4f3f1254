"""Event recorder (``record.EventRecorder`` analogue) writing ``core/v1`` Events.

Identical events (same involved object, type, reason, message, source) within the
aggregation window are folded into one Event whose ``count`` is bumped, as client-go's
event correlator does, so a hot reconcile loop cannot flood the store.  The events seen are
kept in an LRU of ``MAX_SEEN`` entries (client-go's correlator cache is an LRU of 4096), so
recording stays O(1) however many distinct events a long-running manager writes.  Writes
are fire-and-forget tasks: recording an event never blocks a reconcile.
"""

from __future__ import annotations

import asyncio
import logging
import time
import uuid
from collections import OrderedDict
from typing import Tuple

from ..models import meta as m
from ..models.errors import ApiError, is_not_found
from ..utils.timeutil import rfc3339

log = logging.getLogger(__name__)

NORMAL = "Normal"
WARNING = "Warning"


class EventRecorder:
    AGGREGATE_WINDOW = 600.0
    MAX_SEEN = 4096

    def __init__(self, client, component: str, host: str = ""):
        self.client = client
        self.component = component
        self.host = host
        self._seen: OrderedDict[Tuple, Tuple[str, str, int, float]] = OrderedDict()
        self._tasks: set = set()
        self.emitted = 0

    def event(self, obj: dict, etype: str, reason: str, message: str) -> None:
        self.emitted += 1
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            return
        t = loop.create_task(self._write(obj, etype, reason, message))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    def eventf(self, obj: dict, etype: str, reason: str, fmt: str, *args) -> None:
        self.event(obj, etype, reason, fmt % args if args else fmt)

    async def _write(self, obj: dict, etype: str, reason: str, message: str) -> None:
        ns = m.namespace(obj) or "default"
        inv = {"kind": obj.get("kind", ""), "namespace": m.namespace(obj), "name": m.name(obj), "uid": m.uid(obj),
               "apiVersion": obj.get("apiVersion", ""), "resourceVersion": m.resource_version(obj)}
        key = (inv["kind"], inv["namespace"], inv["name"], inv["uid"], etype, reason, message)
        now = time.time()
        seen = self._seen.get(key)
        try:
            if seen and now - seen[3] < self.AGGREGATE_WINDOW:
                ev_ns, ev_name, count, _ = seen
                count += 1
                try:
                    await self.client.patch("v1/Event", {"count": count, "lastTimestamp": rfc3339()},
                                            name=ev_name, namespace=ev_ns)
                    self._seen[key] = (ev_ns, ev_name, count, now)
                    self._seen.move_to_end(key)
                    return
                except ApiError as e:
                    if not is_not_found(e):
                        raise
            name = f"{m.name(obj)}.{uuid.uuid4().hex[:16]}"
            ev = {
                "apiVersion": "v1", "kind": "Event",
                "metadata": {"name": name, "namespace": ns},
                "involvedObject": inv, "reason": reason, "message": message, "type": etype,
                "source": {"component": self.component, **({"host": self.host} if self.host else {})},
                "firstTimestamp": rfc3339(), "lastTimestamp": rfc3339(), "eventTime": None, "count": 1,
                "reportingComponent": self.component, "reportingInstance": self.host,
            }
            await self.client.create(ev)
            self._seen[key] = (ns, name, 1, now)
            self._seen.move_to_end(key)
            while len(self._seen) > self.MAX_SEEN:  # the least recently seen goes first
                self._seen.popitem(last=False)
        except Exception as e:  # events are best effort
            log.debug("event write failed: %r", e)

    async def flush(self) -> None:
        if self._tasks:
            await asyncio.gather(*list(self._tasks), return_exceptions=True)
