#!/usr/bin/env python3
"""Failover and cold start with a resident population.

    python tools/bench_failover.py --resident 1000 [--lease 15 --renew 10 --retry 2]

The reference's managers relist every watched kind before their first reconcile
(``kf/main.go:91-93``, ``odh/main.go:159-160``: controller-runtime starts the controllers'
informers when the replica is elected).  With R notebooks and their children in the cluster
that relist, and the resync it triggers (every object queued once), is what a takeover or a
restart costs.  This tool runs one control-plane shard (``cmd/control_plane.py``: a kf, an odh
and a webhook process, as the ``mi355x-sharded`` pod does, with ``--leader-elect``) plus a
standby replica of the kf and odh processes against the native apiserver and the node
platform, fills the cluster with R Ready notebooks (inject-auth: every child the odh path
makes), then measures:

* **takeover** — the kf and odh leaders are SIGKILLed (no lease release): time until each
  standby leads (lease expiry + the retry period), its first reconcile, and its queue drained
  (every Notebook reconciled once — the resync); the relist bytes the standby read at takeover
  (0: standbys keep warm caches, ``Manager.warm_standby``); its peak RSS;
* **cold start** — the new leaders are stopped gracefully (SIGTERM releases the lease, as a
  rolling update does) and fresh processes started: process start → caches synced → first
  reconcile → queue drained, and the relist bytes;
* after each, a new notebook's create→Ready (the control plane is serving again).

Prints one JSON line.  CPU-only (no GPU needed); numbers depend on the box.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from odh_kubeflow_amd.models import kinds  # noqa: E402
from odh_kubeflow_amd.models.notebook import notebook  # noqa: E402

NS = "bench-0"
CTRL_NS = "opendatahub"
ANN = {"notebooks.opendatahub.io/inject-auth": "true"}


def _rss_hwm_mib(pid: int):
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmHWM:"):
                    return round(int(line.split()[1]) / 1024.0, 1)
    except OSError:
        return None
    return None


class Replica:
    """A control-plane process launched here (a standby, or a fresh one after a restart)."""

    def __init__(self, name: str, module: str, argv, env):
        from odh_kubeflow_amd.parallel.shard import free_port

        self.name = name
        self.port = free_port()
        self.started = time.monotonic()
        self.proc = subprocess.Popen([sys.executable, "-m", module, *argv(self.port)], cwd=ROOT, env=env,
                                     stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        self.base = f"http://127.0.0.1:{self.port}"

    async def debug(self, http):
        try:
            async with http.get(self.base + "/debug/reconciles") as r:
                return json.loads(await r.text())
        except Exception:  # noqa: BLE001 — not serving yet
            return None


def _total(doc) -> int:
    return sum(sum(t.values()) for t in ((doc or {}).get("reconciles") or {}).values())


async def watch_replica(http, rep: Replica, t0: float, want: int, timeout: float = 300.0) -> dict:
    """Poll a replica until it leads, has reconciled, and has ``want`` reconciles with an empty
    queue: the times (s after ``t0``) of each, and what it read in lists."""
    out = {"lead_s": None, "first_reconcile_s": None, "drained_s": None}
    base = None
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        d = await rep.debug(http)
        now = time.monotonic() - t0
        if d is not None:
            if base is None:
                base = _total(d)
            if d.get("leader") and out["lead_s"] is None:
                out["lead_s"] = round(now, 3)
            n = _total(d) - base
            if n > 0 and out["first_reconcile_s"] is None:
                out["first_reconcile_s"] = round(now, 3)
            if d.get("leader") and n >= want and not d.get("pending"):
                out["drained_s"] = round(now, 3)
                out["reconciles"] = n
                out["list_bytes"] = ((d.get("io") or {}).get("bytes_in") or {}).get("LIST", 0)
                out["lists"] = (d.get("io") or {}).get("lists")
                break
        await asyncio.sleep(0.02)
    out["rss_hwm_mib"] = _rss_hwm_mib(rep.proc.pid)
    return out


async def run(args) -> dict:
    import aiohttp

    from odh_kubeflow_amd.parallel.platform import NodePlatform
    from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig, notebook_is_ready
    from odh_kubeflow_amd.runtime.informer import InformerCache
    from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
    from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS

    le = ["--leader-elect", "--leader-election-namespace", CTRL_NS,
          "--leader-election-lease-duration", f"{args.lease:g}", "--leader-election-renew-deadline", f"{args.renew:g}",
          "--leader-election-retry-period", f"{args.retry:g}"]
    base_env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
    native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
    platform = await NodePlatform(native.url, workers=args.platform_workers).start()
    shard = await ControlPlaneShard(ShardConfig(native.url, NS, shard="0", bootstrap=True, process=True,
                                                env={**base_env, "POD_NAME": "replica-0"},
                                                leader_elect_args=le)).start()
    http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30))
    out: dict = {"metric": "control-plane takeover and cold start with a resident population", "resident": args.resident,
                 "lease": {"duration_s": args.lease, "renew_deadline_s": args.renew, "retry_period_s": args.retry},
                 "layout": "one shard: kf | odh | webhook processes (cmd/control_plane.py --leader-elect) + a standby "
                           "kf and odh replica"}
    reps = []
    try:
        specs = {n: (mod, a, fl) for n, mod, a, fl in shard._specs(0)}
        env = {**os.environ, **base_env, "K8S_NAMESPACE": CTRL_NS,
               "PYTHONPATH": ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")}

        def spawn(name: str, pod: str) -> Replica:
            mod, a, fl = specs[name]
            return Replica(name, mod, lambda port: [*shard._common_flags(), fl, f"127.0.0.1:{port}", *a],
                           {**env, "POD_NAME": pod})

        leads = {"control_plane_kf": "kf", "control_plane_odh": "odh"}
        standbys = {n: spawn(n, "replica-1") for n in leads}
        reps += standbys.values()

        # ---- fill: R Ready notebooks with every child of the odh auth path
        fill = InformerCache(shard.rest, namespaces=[NS])
        for k in (kinds.NOTEBOOK, kinds.POD):
            await fill.ensure_informer(k)
        names = [f"res-{i}" for i in range(args.resident)]
        sem = asyncio.Semaphore(32)

        async def create(nm):
            nb = notebook(nm, NS, annotations=ANN)
            nb["spec"]["template"]["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "50m",
                                                                                        "memory": "256Mi"}}
            async with sem:
                await shard.admin.create(nb)
        t = time.monotonic()
        await asyncio.gather(*(create(nm) for nm in names))
        deadline = time.monotonic() + 600
        while not all(notebook_is_ready(fill.get(kinds.NOTEBOOK, nm, NS)) for nm in names):
            if time.monotonic() > deadline:
                raise RuntimeError("resident notebooks not Ready")
            await asyncio.sleep(0.05)
        out["fill_s"] = round(time.monotonic() - t, 3)
        await fill.stop()
        objects = {}
        for kind in (kinds.NOTEBOOK, kinds.STATEFUL_SET, kinds.POD, kinds.SERVICE, kinds.CONFIG_MAP,
                     kinds.SERVICE_ACCOUNT, kinds.NETWORK_POLICY, kinds.HTTP_ROUTE):
            objects[kinds_name(kind)] = len(await shard.rest.list(kind))
        out["objects"] = objects
        # every standby has synced its caches (warm standby) before the leaders go
        for rep in standbys.values():
            while (await rep.debug(http)) is None:
                await asyncio.sleep(0.05)
        await asyncio.sleep(1.0)
        for rep in standbys.values():
            d = await rep.debug(http)
            rep.bytes_before = ((d.get("io") or {}).get("bytes_in") or {}).get("LIST", 0)

        # ---- takeover: SIGKILL the leaders (no lease release)
        victims = [p for p in shard.procs if p.name in leads]
        t0 = time.monotonic()
        for p in victims:
            p.proc.send_signal(signal.SIGKILL)
        res = await asyncio.gather(*(watch_replica(http, standbys[n], t0, args.resident) for n in leads))
        take = {}
        for n, r in zip(leads, res):
            r["relist_bytes_at_takeover"] = (r.pop("list_bytes", 0) or 0) - standbys[n].bytes_before
            take[leads[n]] = r
        out["takeover_sigkill"] = take
        out["after_takeover_ready_ms"] = await new_notebooks(shard, "nb-after-takeover", 5)

        # ---- cold start: stop the new leaders gracefully (lease released), start fresh processes
        for rep in standbys.values():
            rep.proc.send_signal(signal.SIGTERM)
        for rep in standbys.values():
            rep.proc.wait(timeout=30)
        t0 = time.monotonic()
        fresh = {n: spawn(n, "replica-2") for n in leads}
        reps += fresh.values()
        res = await asyncio.gather(*(watch_replica(http, fresh[n], t0, args.resident) for n in leads))
        cold = {}
        for n, r in zip(leads, res):
            r["relist_bytes"] = r.pop("list_bytes", 0)
            cold[leads[n]] = r
        out["cold_start_graceful"] = cold
        out["after_cold_start_ready_ms"] = await new_notebooks(shard, "nb-after-restart", 5)
    finally:
        await http.close()
        for rep in reps:
            if rep.proc.poll() is None:
                rep.proc.terminate()
                try:
                    rep.proc.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    rep.proc.kill()
        await shard.stop()
        await platform.stop()
        await native.stop()
    return out


def kinds_name(kind) -> str:
    from odh_kubeflow_amd.models.scheme import SCHEME

    return SCHEME.resolve(kind).kind


async def new_notebooks(shard, prefix: str, n: int) -> dict:
    from odh_kubeflow_amd.parallel.bench_dist import _lifecycle, _pcts

    lat = []
    for i in range(n):
        ready_s, _gone, _pod = await _lifecycle(shard, f"{prefix}-{i}", dict(ANN), timeout=120)
        lat.append(ready_s * 1e3)
    return _pcts(lat, (0.5,))


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--resident", type=int, default=1000)
    p.add_argument("--lease", type=float, default=15.0, help="lease duration s (controller-runtime's default)")
    p.add_argument("--renew", type=float, default=10.0)
    p.add_argument("--retry", type=float, default=2.0)
    p.add_argument("--platform-workers", type=int, default=1)
    args = p.parse_args(argv)
    out = asyncio.run(run(args))
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
