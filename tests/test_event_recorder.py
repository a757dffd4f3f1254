"""The event recorder (``runtime/events.py``): identical events fold into one Event whose
count is bumped, and the correlation cache is an LRU of ``MAX_SEEN`` entries, so a
long-running manager records each event in O(1) (a full scan of the cache per event, once it
held 4096 events of the last 10 minutes, cost the culler process most of a core after a few
thousand notebooks)."""

from __future__ import annotations

import time

from odh_kubeflow_amd.runtime.events import EventRecorder


class _Client:
    def __init__(self):
        self.creates, self.patches = [], []

    async def create(self, obj):
        self.creates.append(obj)
        return obj

    async def patch(self, kind, body, name, namespace):
        self.patches.append((name, body["count"]))
        return body


def _pod(i: int) -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": f"nb-{i}-0", "namespace": "ns", "uid": f"u{i}", "resourceVersion": "1"}}


async def _record(rec: EventRecorder, objs, reason: str = "Started") -> None:
    for o in objs:
        rec.event(o, "Normal", reason, "started container")
    await rec.flush()


def test_identical_events_fold_into_one(run):
    async def go():
        c = _Client()
        rec = EventRecorder(c, "notebook-controller")
        await _record(rec, [_pod(1)] * 3)
        assert len(c.creates) == 1
        assert [n for _, n in c.patches] == [2, 3]
        await _record(rec, [_pod(1)], reason="Killing")  # another reason: another Event
        assert len(c.creates) == 2
    run(go())


def test_correlation_cache_is_a_bounded_lru(run):
    async def go():
        c = _Client()
        rec = EventRecorder(c, "notebook-controller")
        rec.MAX_SEEN = 64
        await _record(rec, [_pod(0)])
        for start in range(1, 1000, 50):
            await _record(rec, [_pod(0)] + [_pod(i) for i in range(start, start + 49)])
        assert len(rec._seen) == 64
        # the event seen again and again stayed in the cache: still one Event, its count bumped
        assert sum(1 for e in c.creates if e["involvedObject"]["name"] == "nb-0-0") == 1
        assert max(n for name, n in c.patches) == 21
        # an event evicted as least recently seen is a new Event when it comes back
        await _record(rec, [_pod(1)])
        assert sum(1 for e in c.creates if e["involvedObject"]["name"] == "nb-1-0") == 2
    run(go())


def test_recording_stays_constant_time_with_a_full_cache(run):
    async def go():
        c = _Client()
        rec = EventRecorder(c, "notebook-controller")

        async def per_event(lo: int, n: int) -> float:
            t0 = time.perf_counter()
            for i in range(lo, lo + n):
                rec.event(_pod(i), "Normal", "Started", "started container")
                if i % 256 == 0:
                    await rec.flush()
            await rec.flush()
            return (time.perf_counter() - t0) / n

        await per_event(0, rec.MAX_SEEN)  # fill the cache
        full = await per_event(10**6, 4000)  # every event now evicts one
        assert len(rec._seen) == rec.MAX_SEEN
        assert full < 0.5e-3, f"{full * 1e6:.0f} us per event with a full cache"
    run(go())


def test_no_running_loop_is_a_no_op():
    rec = EventRecorder(_Client(), "x")
    rec.event(_pod(1), "Normal", "Started", "m")
    assert rec.emitted == 1 and not rec._seen


def test_reemitter_caches_slim_events():
    """The re-emitter's cache keeps what it reads of a platform Event, and nothing else (its
    cache holds every Pod/StatefulSet Event of its namespaces until the Event expires)."""
    from odh_kubeflow_amd.controllers.notebook import slim_event

    ev = {"apiVersion": "v1", "kind": "Event",
          "metadata": {"name": "nb-0.1", "namespace": "ns", "uid": "u", "resourceVersion": "9",
                       "creationTimestamp": "2026-01-01T00:00:00Z", "managedFields": [{"manager": "x"}]},
          "involvedObject": {"kind": "Pod", "name": "nb-0", "namespace": "ns"},
          "reason": "Started", "message": "started container", "type": "Normal",
          "source": {"component": "kubelet", "host": "node"}, "count": 3,
          "firstTimestamp": "2026-01-01T00:00:00Z", "lastTimestamp": "2026-01-01T00:00:01Z",
          "reportingComponent": "kubelet", "reportingInstance": "node"}
    s = slim_event(ev)
    assert set(s) == {"apiVersion", "kind", "metadata", "involvedObject", "reason", "message", "type"}
    assert s["metadata"] == {"name": "nb-0.1", "namespace": "ns", "uid": "u", "resourceVersion": "9"}
    assert s["involvedObject"] is ev["involvedObject"]
