"""Namespace-partitioned worker processes inside one manager Deployment (``--workers W``).

The reference runs each manager as one Go process whose controllers use one reconcile
worker each (``kf/main.go:87-98``, ``odh/main.go:155-192``).  A Python manager
is one event loop, so one manager process tops out at one core however many reconcile
workers it runs: measured on an MI355X box with the reference topology
(``config/overlays/mi355x``), the kf and odh managers each burnt ≈1 core at 4 notebook
streams and throughput stopped scaling (49 % efficiency, ``pass r3_p35``), with the
odh webhook's admissions queued behind the reconciles on the same loop.

``--workers W`` keeps the deployment unit — one Deployment, one replica, one leader lease,
one ``/metrics``, one webhook Service — and runs the controllers in ``W`` child processes of
it, each serving a set of namespaces the parent assigns:

* the parent (the **supervisor**) watches Namespaces and gives each new namespace to the
  worker holding the fewest (ties: the lowest index).  An assignment is sticky: it moves only
  when its worker is restarted, so a namespace is never served by two workers at once.  A
  hash of the name would need no coordination, but over the handful of namespaces a node's
  notebooks live in it is lumpy (``bench-0..3``: crc32 % 4 puts them on two of four workers);
* the assignments travel over the worker's stdin (``assign <ns>`` / ``release <ns>``, then
  ``sync`` once the initial set is sent) — nothing is written to the cluster, and the set is
  rebuilt from the Namespace list whenever the supervisor starts;
* a worker's informer cache lists and watches only its namespaces (one watch per namespace and
  kind, the machinery a shard uses — :class:`~odh_kubeflow_amd.runtime.informer.InformerCache`
  ``namespace_filter``), plus the controller namespace for the odh reconciler's central
  objects (HTTPRoutes, ImageStreams);
* its controllers drop every request for a namespace it does not serve
  (:attr:`WorkerAssignments.request_filter`): an HTTPRoute in the controller namespace maps to
  the notebook it routes to, which only that notebook's worker reconciles.

A notebook is therefore reconciled by exactly one process — the workqueue's "never two
workers on one object" guarantee holds across processes — and no object is written by two
workers.

The supervisor leads the manager's lease and starts the workers only once it leads; losing
the lease stops them and ends the process, as controller-runtime does.  A worker that dies
is restarted with back-off and given its namespaces again (``/healthz`` fails meanwhile).
The workers die with the supervisor (``PR_SET_PDEATHSIG``,
:mod:`~odh_kubeflow_amd.utils.procutil`, and end of stdin).  The supervisor's ``/metrics`` is
the sum of its own registry and the workers' (counters, histograms and the per-namespace
gauges are additive over disjoint namespace sets), and its ``/debug`` endpoints aggregate
theirs.  In the odh manager the supervisor also serves the mutating webhook, so admissions
never wait behind a reconcile.
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
import re
import subprocess
import sys
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

log = logging.getLogger("runtime.workers")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_worker(value: Optional[str]) -> Optional[Tuple[int, int]]:
    """``--worker i/W`` → ``(i, W)``; ``None`` / ``""`` → None (not a worker)."""
    if not value:
        return None
    mo = re.fullmatch(r"(\d+)/(\d+)", value.strip())
    if not mo or not 0 <= int(mo.group(1)) < int(mo.group(2)):
        raise SystemExit(f"--worker={value!r}: expected i/W with 0 <= i < W")
    return int(mo.group(1)), int(mo.group(2))


class WorkerAssignments:
    """A worker's side of the protocol: the namespaces it serves, kept current from stdin.

    Use :meth:`cache_options` for its informer cache and :attr:`request_filter` for its
    controllers, then add it to the manager as a runnable (``needs_leader=False``): its
    ``start`` returns once the supervisor's initial set has arrived (``sync``), before any
    controller starts, and end of stdin (the supervisor is gone) makes the manager exit."""

    def __init__(self, index: int, count: int, stream=None):
        self.index, self.count = index, count
        self.namespaces: set = set()
        self.cache = None  # InformerCache, set by the owner once built
        self.on_lost: Optional[Callable[[], None]] = None
        self._stream = stream
        self._task: Optional[asyncio.Task] = None
        self._synced: Optional[asyncio.Event] = None

    def cache_options(self, extra_namespaces: Iterable[str] = (), cluster_watch: bool = False) -> dict:
        from ..models import meta as m

        return {"namespace_filter": lambda ns: m.name(ns) in self.namespaces,
                "namespaces": [n for n in extra_namespaces if n], "cluster_watch": cluster_watch}

    def request_filter(self, req) -> bool:
        return not req.namespace or req.namespace in self.namespaces

    def apply(self, line: str) -> None:
        verb, _, ns = line.strip().partition(" ")
        if verb == "assign" and ns:
            self.namespaces.add(ns)
        elif verb == "release" and ns:
            self.namespaces.discard(ns)
        else:
            return
        if self.cache is not None:
            self.cache.refresh_namespace(ns)

    async def start(self) -> None:
        loop = asyncio.get_running_loop()
        self._synced = asyncio.Event()
        stream = self._stream or sys.stdin
        reader = asyncio.StreamReader()
        await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), stream)
        self._task = asyncio.ensure_future(self._read(reader))
        await self._synced.wait()

    async def _read(self, reader) -> None:
        while True:
            line = await reader.readline()
            if not line:
                break
            text = line.decode().strip()
            if text == "sync":
                self._synced.set()
            else:
                self.apply(text)
        log.error("worker %d/%d: supervisor gone (stdin closed); exiting", self.index, self.count)
        self._synced.set()
        if self.on_lost is not None:
            self.on_lost()

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()


def strip_flags(argv: Sequence[str], with_value: Iterable[str] = (), boolean: Iterable[str] = ()) -> List[str]:
    """``argv`` without the given flags (``--f v`` and ``--f=v`` spellings)."""
    wv, bo = set(with_value), set(boolean)
    out: List[str] = []
    skip = False
    for a in argv:
        if skip:
            skip = False
            continue
        name = a.split("=", 1)[0]
        if name in bo:
            continue
        if name in wv:
            skip = "=" not in a
            continue
        out.append(a)
    return out


def _free_port() -> int:
    from ..utils.procutil import listen_port

    return listen_port()


# ------------------------------------------------------------------ /metrics merge


_SAMPLE = re.compile(r"^([A-Za-z_:][A-Za-z0-9_:]*)(\{.*\})?\s+(\S+)(?:\s+\S+)?$")
# gauges that measure a share of the work each worker holds: the manager's is the sum
ADDITIVE_GAUGES = frozenset({"controller_runtime_max_concurrent_reconciles", "controller_runtime_active_workers",
                             "workqueue_depth", "workqueue_unfinished_work_seconds"})


def merge_metrics(texts: Sequence[str]) -> str:
    """Merge Prometheus text expositions of the same metrics from several processes: one
    HELP/TYPE per family; samples with the same name and labels are added for counters,
    histograms and summaries, and the largest is kept for gauges (a gauge is a level — two
    processes exporting ``last_notebook_culling_timestamp_seconds`` for the same notebook must
    not add up to twice the epoch) except the per-worker shares in :data:`ADDITIVE_GAUGES`
    (two workers of 8 concurrent reconciles each are 16), and for ``_created`` timestamps the
    earliest.  The families keep the order of their first appearance."""
    meta: Dict[str, List[str]] = {}
    order: List[str] = []
    samples: Dict[str, Dict[Tuple[str, str], float]] = {}
    fam_of: Dict[str, str] = {}
    types: Dict[str, str] = {}
    for text in texts:
        fam = None
        for line in text.splitlines():
            if not line:
                continue
            if line.startswith("#"):
                parts = line.split(None, 3)
                if len(parts) >= 3 and parts[1] in ("HELP", "TYPE"):
                    fam = parts[2]
                    if fam not in meta:
                        meta[fam] = []
                        order.append(fam)
                        samples[fam] = {}
                    if parts[1] == "TYPE" and len(parts) == 4:
                        types.setdefault(fam, parts[3].strip())
                    if not any(x.split(None, 2)[1] == parts[1] for x in meta[fam]):
                        meta[fam].append(line)
                continue
            mo = _SAMPLE.match(line)
            if not mo:
                continue
            name, labels, val = mo.group(1), mo.group(2) or "", mo.group(3)
            try:
                v = float(val)
            except ValueError:
                continue
            f = fam_of.get(name)
            if f is None:
                f = fam if fam is not None and name.startswith(fam) else name
                if f not in samples:
                    meta.setdefault(f, [])
                    order.append(f)
                    samples[f] = {}
                fam_of[name] = f
            key = (name, labels)
            prev = samples[f].get(key)
            if prev is None:
                samples[f][key] = v
            elif name.endswith("_created"):
                samples[f][key] = min(prev, v)  # a creation timestamp: the earliest, not a sum
            elif types.get(f) == "gauge" and f not in ADDITIVE_GAUGES:
                samples[f][key] = max(prev, v)
            else:
                samples[f][key] = prev + v
    out: List[str] = []
    for f in order:
        out.extend(meta.get(f, []))
        for (name, labels), v in samples[f].items():
            out.append(f"{name}{labels} {_fmt(v)}")
    return "\n".join(out) + "\n"


def _fmt(v: float) -> str:
    if v != v:  # NaN
        return "NaN"
    if v in (float("inf"), float("-inf")):
        return "+Inf" if v > 0 else "-Inf"
    return repr(float(v))


# ------------------------------------------------------------------ supervisor


class _Worker:
    def __init__(self, index: int, role: str = ""):
        self.index = index
        self.role = role  # "" or one of the supervisor's roles (all roles of an index share its namespaces)
        self.label = str(index) if not role else f"{index}_{role}"
        self.proc: Optional[subprocess.Popen] = None
        self.base = ""
        self.restarts = 0
        self.started_at = 0.0
        self.namespaces: set = set()
        self.pending = False  # exited and not yet running again (a failed restart is retried)

    def send(self, line: str) -> None:
        if self.proc is None or self.proc.stdin is None:
            return
        try:
            self.proc.stdin.write(line + "\n")
            self.proc.stdin.flush()
        except (BrokenPipeError, OSError, ValueError):
            pass  # the worker is gone: the watch loop restarts it with its namespaces


class WorkerSupervisor:
    """Starts, watches and stops the ``count`` worker processes of one manager.

    ``argv_for(i, metrics_addr)`` returns the worker's command-line arguments for
    ``python -m module``.  A manager runnable: the owning :class:`Manager` adds it with
    ``needs_leader=True``, so the workers run only while the supervisor leads.

    ``roles``: each of the ``count`` namespace slots is served by one process per role
    (``argv_for(i, metrics_addr, role)``), all given the slot's namespaces — the kf manager
    runs its notebook reconciler apart from its culler and event re-emitter this way
    (``--split-workers``), as a shard pod does."""

    def __init__(self, module: str, count: int, argv_for: Callable[..., List[str]],
                 env: Optional[Dict[str, str]] = None, name: str = "manager", start_timeout: float = 120.0,
                 restart_backoff: Tuple[float, float] = (0.5, 30.0), cache=None,
                 system_namespaces: Iterable[str] = (), roles: Sequence[str] = ("",)):
        self.cache = cache  # the supervisor's InformerCache: its Namespace watch drives the assignments
        self.owner: Dict[str, int] = {}
        self.system_namespaces = set(system_namespaces)
        self._system: set = set()
        self._unsub = None
        self.module = module
        self.count = int(count)
        self.argv_for = argv_for
        self.env = dict(os.environ if env is None else env)
        self.name = name
        self.start_timeout = start_timeout
        self.backoff0, self.backoff_max = restart_backoff
        self.roles = tuple(roles) or ("",)
        self.workers = [_Worker(i, r) for i in range(self.count) for r in self.roles]
        self._slots: Dict[int, List[_Worker]] = {}
        for w in self.workers:
            self._slots.setdefault(w.index, []).append(w)
        self._monitor: Optional[asyncio.Task] = None
        self._http = None
        self._stopping = False

    # -------------------------------------------------------------- lifecycle

    async def _spawn(self, w: _Worker) -> None:
        from ..utils.procutil import child_env

        port = _free_port()
        env = child_env({**self.env, "PYTHONPATH": ROOT + os.pathsep + self.env.get("PYTHONPATH", "")})
        extra = (w.role,) if w.role else ()
        args = [sys.executable, "-m", self.module, *self.argv_for(w.index, f"127.0.0.1:{port}", *extra)]
        w.proc = subprocess.Popen(args, cwd=ROOT, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  stderr=None, text=True)
        w.base = f"http://127.0.0.1:{port}"
        w.started_at = time.monotonic()
        for ns in sorted(w.namespaces):
            w.send(f"assign {ns}")
        w.send("sync")
        loop = asyncio.get_running_loop()
        try:
            line = await asyncio.wait_for(loop.run_in_executor(None, w.proc.stdout.readline), self.start_timeout)
        except asyncio.TimeoutError:
            line = ""
        if line.strip() != "ready":
            rc = w.proc.poll()
            w.proc.kill()
            raise RuntimeError(f"{self.name} worker {w.label}/{self.count} did not start (rc={rc})")
        # keep draining stdout so a chatty worker never blocks on a full pipe
        loop.run_in_executor(None, _drain, w.proc.stdout)
        log.info("%s worker %s/%d started (pid %d)", self.name, w.label, self.count, w.proc.pid)

    # -------------------------------------------------------------- namespace assignment

    def assign(self, ns: str) -> int:
        """Give ``ns`` to the worker serving the fewest user namespaces (sticky).  System
        namespaces (``default``, ``kube-*``, ``openshift*``, the controller's own) rarely hold a
        notebook: worker 0 serves them, and they do not count as load."""
        i = self.owner.get(ns)
        if i is None:
            if self.is_system(ns):
                i = 0
            else:
                i = min(self._slots, key=lambda k: (len(self._slots[k][0].namespaces - self._system), k))
            self.owner[ns] = i
            for w in self._slots[i]:
                w.namespaces.add(ns)
                w.send(f"assign {ns}")
        return i

    def is_system(self, ns: str) -> bool:
        if ns == "default" or ns in self.system_namespaces or ns.startswith(("kube-", "openshift")):
            self._system.add(ns)
            return True
        return False

    def release(self, ns: str) -> None:
        i = self.owner.pop(ns, None)
        if i is not None:
            for w in self._slots[i]:
                w.namespaces.discard(ns)
                w.send(f"release {ns}")

    def _on_namespace(self, etype: str, obj: dict, old) -> None:
        name = (obj.get("metadata") or {}).get("name", "")
        if etype == "DELETED":
            self.release(name)
        elif name:
            self.assign(name)

    def assignments(self) -> Dict[int, List[str]]:
        return {i: sorted(ws[0].namespaces) for i, ws in self._slots.items()}

    async def start(self) -> None:
        self._stopping = False
        if self.cache is not None and self._unsub is None:
            from ..models import kinds

            self._unsub = self.cache.subscribe(kinds.NAMESPACE, self._on_namespace)
            await self.cache.wait_synced([kinds.NAMESPACE])
        await asyncio.gather(*(self._spawn(w) for w in self.workers))
        self._monitor = asyncio.ensure_future(self._watch())

    async def _watch(self) -> None:
        """Restart a worker that exited, with exponential back-off (reset after a minute up).  A
        restart that fails (the new process never reports ``ready``) leaves the worker pending:
        every later pass tries again, each after a longer back-off, until one comes up."""
        delay: Dict[str, float] = {}
        while not self._stopping:
            await asyncio.sleep(0.2)
            for w in self.workers:
                if self._stopping:
                    return
                exited = w.proc is not None and w.proc.poll() is not None
                if not exited and not w.pending:
                    continue
                if exited:
                    up = time.monotonic() - w.started_at
                    d = self.backoff0 if up > 60 else min(self.backoff_max, delay.get(w.label, self.backoff0 / 2) * 2)
                    log.error("%s worker %s/%d exited (rc=%s); restarting in %.1f s", self.name, w.label, self.count,
                              w.proc.returncode, d)
                    w.proc = None
                    w.pending = True
                else:  # the last restart failed
                    d = min(self.backoff_max, delay.get(w.label, self.backoff0 / 2) * 2)
                delay[w.label] = d
                await asyncio.sleep(d)
                if self._stopping:
                    return
                w.restarts += 1
                try:
                    await self._spawn(w)
                    w.pending = False
                except Exception as e:  # noqa: BLE001 — pending: the next pass tries again
                    log.error("%s; retrying", e)
                    w.proc = None

    def alive(self) -> bool:
        return all(w.proc is not None and w.proc.poll() is None for w in self.workers)

    def pids(self) -> Dict[str, int]:
        return {f"worker_{w.label}": w.proc.pid for w in self.workers if w.proc is not None}

    async def stop(self) -> None:
        self._stopping = True
        if self._unsub is not None:
            self._unsub()
            self._unsub = None
        if self._monitor is not None:
            self._monitor.cancel()
            try:
                await self._monitor
            except (asyncio.CancelledError, Exception):
                pass
        procs = [w.proc for w in self.workers if w.proc is not None]
        for p in procs:
            if p.poll() is None:
                p.terminate()
            try:
                p.stdin.close()
            except (OSError, AttributeError):
                pass
        loop = asyncio.get_running_loop()
        for p in procs:
            try:
                await asyncio.wait_for(loop.run_in_executor(None, p.wait), 10)
            except asyncio.TimeoutError:
                p.kill()
        for w in self.workers:
            w.proc = None
        if self._http is not None:
            await self._http.close()
            self._http = None

    # -------------------------------------------------------------- aggregation

    async def _get(self, w: _Worker, path: str, timeout: float = 30.0) -> Optional[str]:
        import aiohttp

        if self._http is None:
            self._http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=60))
        if w.proc is None:
            return None
        try:
            async with self._http.get(w.base + path, timeout=aiohttp.ClientTimeout(total=timeout)) as r:
                return await r.text() if r.status == 200 else None
        except Exception:  # noqa: BLE001 — a restarting worker: missing from this scrape
            return None

    async def metrics_texts(self) -> List[str]:
        return [t for t in await asyncio.gather(*(self._get(w, "/metrics") for w in self.workers)) if t]

    async def debug(self, path: str, timeout: float = 30.0) -> List[dict]:
        return list((await self.debug_by_worker(path, timeout)).values())

    async def debug_by_worker(self, path: str, timeout: float = 30.0) -> Dict[str, dict]:
        """worker label (its index, ``<index>_<role>`` with roles) → its JSON answer (a worker
        restarting is missing)."""
        return await self.debug_each(lambda _i: path, timeout)

    async def debug_each(self, path_for: Callable[[int], str], timeout: float = 30.0) -> Dict[str, dict]:
        """worker label → its JSON answer to ``path_for(index)``."""
        docs = await asyncio.gather(*(self._get(w, path_for(w.index), timeout) for w in self.workers))
        return {w.label: json.loads(d) for w, d in zip(self.workers, docs) if d}


def _drain(stream) -> None:
    try:
        for _ in stream:
            pass
    except (OSError, ValueError):
        pass


def merge_counts(parts: Iterable[dict]) -> dict:
    """Sum nested ``{a: {b: n}}`` count dicts (reconcile breakdowns, IO counters)."""
    out: dict = {}
    for part in parts:
        for k, v in (part or {}).items():
            if isinstance(v, dict):
                out[k] = merge_counts([out.get(k) or {}, v])
            else:
                out[k] = out.get(k, 0) + v
    return out
