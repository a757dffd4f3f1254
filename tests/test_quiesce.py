"""``WorkQueue.pending`` / ``Manager.quiesce`` with a timer horizon: a delayed requeue a check
period away (the culler's next check of every notebook) is not outstanding work, so the
benchmark's pre-window quiesce does not leave the processes idle until it fires."""

from __future__ import annotations

import asyncio
import time

from odh_kubeflow_amd.runtime.controller import Controller, Request, Result
from odh_kubeflow_amd.runtime.manager import Manager
from odh_kubeflow_amd.runtime.workqueue import WorkQueue


def test_pending_counts_only_timers_due_within_the_horizon(run):
    async def go():
        q = WorkQueue("q")
        q.add_after("soon", 0.01)
        q.add_after("later", 5.0)
        assert q.pending() == 2
        assert q.pending(timers_within=0.05) == 1
        assert q.pending(timers_within=0.0) == 0
        q.add("now")
        assert q.pending(timers_within=0.0) == 1
        q.shutdown()
    run(go())


class _Src:
    last_event = 0.0


def test_quiesce_does_not_wait_for_a_requeue_a_period_away(run):
    async def go():
        mgr = Manager(client=None, reader=_Src(), source=None)
        c = Controller("culler", _requeue_later)
        mgr.controllers.append(c)
        c.queue.add_after(Request("ns", "nb"), 2.0)  # the next check, a period away
        assert not c.idle() and c.idle(0.05)
        t0 = time.monotonic()
        assert await mgr.quiesce(0.002, 1.0, timers_within=0.05)
        assert time.monotonic() - t0 < 0.5
        assert not await mgr.quiesce(0.002, 0.2)  # without the horizon it waits for the timer
        c.queue.shutdown()
    run(go())


async def _requeue_later(req) -> Result:
    await asyncio.sleep(0)
    return Result(requeue_after=2.0)
