"""Shared process plumbing for the ``cmd`` entry points: logging (zap-like, RFC3339
timestamps, development/production modes), signal handling and runnable wrappers."""

from __future__ import annotations

import asyncio
import logging
import signal
import sys
import time


class _RFC3339Formatter(logging.Formatter):
    def formatTime(self, record, datefmt=None):  # noqa: N802 (logging API)
        return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(record.created))


def setup_logging(debug: bool = False, development: bool = False) -> None:
    level = logging.DEBUG if (debug or development) else logging.INFO
    h = logging.StreamHandler(sys.stderr)
    if development:
        h.setFormatter(_RFC3339Formatter("%(asctime)s\t%(levelname)s\t%(name)s\t%(message)s"))
    else:
        h.setFormatter(_RFC3339Formatter('{"ts":"%(asctime)s","level":"%(levelname)s","logger":"%(name)s",'
                                         '"msg":"%(message)s"}'))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(level)
    logging.getLogger("aiohttp.access").setLevel(logging.WARNING)


def signal_event() -> asyncio.Event:
    """``ctrl.SetupSignalHandler``: set on SIGTERM / SIGINT."""
    ev = asyncio.Event()
    loop = asyncio.get_running_loop()
    for s in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(s, ev.set)
        except (NotImplementedError, RuntimeError):
            pass
    return ev


class ServerRunnable:
    """Adapter so servers (webhook, telemetry) join a manager's lifecycle."""

    def __init__(self, start, stop):
        self._start, self._stop = start, stop

    async def start(self):
        await self._start()

    async def stop(self):
        await self._stop()


def add_shard_flags(p) -> None:
    """``--shard``: run as one namespace shard of the control plane (see ``cmd/control_plane.py``)."""
    p.add_argument("--shard", default=None,
                   help="serve only namespaces labelled notebooks.amd.com/shard=<SHARD> (+ the controller "
                        "namespace); 'ordinal' takes it from the StatefulSet pod name (POD_NAME/HOSTNAME -<n>)")
    add_watch_scope_flag(p)


def add_watch_scope_flag(p) -> None:
    """``--cluster-wide-watches``: a process that serves a subset of the namespaces (a shard, a
    ``--workers`` worker) watches each kind once, cluster-wide, dropping the other namespaces'
    objects on arrival — instead of one watch per served namespace per kind."""
    p.add_argument("--cluster-wide-watches", action="store_true",
                   help="one cluster-wide watch per kind, filtered here by namespace, instead of a watch per "
                        "served namespace per kind (many namespaces per shard or worker)")


def resolve_shard(value, env=None):
    """The shard id for ``--shard`` (None: unsharded, the reference's cluster-wide manager)."""
    import os
    import re

    env = os.environ if env is None else env
    if value is None or value == "":
        return None
    if value == "ordinal":
        name = env.get("POD_NAME") or env.get("HOSTNAME") or ""
        mo = re.search(r"-(\d+)$", name)
        if not mo:
            raise SystemExit(f"--shard=ordinal: cannot read a StatefulSet ordinal from pod name {name!r}")
        return mo.group(1)
    if not re.fullmatch(r"[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?", value) or len(value) > 63:
        raise SystemExit(f"--shard={value!r} is not a valid label value")
    return value


def add_worker_flags(p) -> None:
    """``--workers W``: run the controllers in W namespace-partitioned child processes
    (:mod:`~odh_kubeflow_amd.runtime.workers`); ``--worker i/W`` is how the supervisor starts
    one of them."""
    import argparse

    p.add_argument("--workers", type=int, default=1,
                   help="controller worker processes, each serving the namespaces the supervisor assigns it "
                        "(fewest first, sticky; 1: in this process)")
    p.add_argument("--worker", default=None, help=argparse.SUPPRESS)


def add_debug_flags(p) -> None:
    """``--enable-debug-endpoints``: ``/debug/reconciles`` and ``/debug/quiesce`` on the
    metrics server (see :meth:`~odh_kubeflow_amd.runtime.manager.Manager.quiesce`)."""
    p.add_argument("--enable-debug-endpoints", action="store_true",
                   help="serve /debug/reconciles and /debug/quiesce on the metrics address (benchmarks, e2e)")


async def run_announcing_ready(mgr, stop) -> int:
    """``mgr.run_until(stop)``, printing ``ready`` on stdout once the servers are up and this
    replica leads (its informers synced and controllers started): the start-up handshake the
    benchmark and the multi-process tests wait for."""
    import asyncio

    async def announce():
        await mgr.started_event().wait()
        await mgr.elected.wait()
        print("ready", flush=True)

    t = asyncio.ensure_future(announce())
    try:
        return await mgr.run_until(stop)
    finally:
        t.cancel()
