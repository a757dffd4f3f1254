"""Leader election (``kf/main.go:91-93``, ``odh/main.go:159-160``): client-go observed-time
expiry (immune to clock skew between nodes) and fatal loss of leadership (the manager
exits non-zero like controller-runtime instead of idling with green probes)."""

import asyncio
import os
import subprocess
import sys
import time

from odh_kubeflow_amd.testing.apiserver.inprocess import in_process_manager
from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.runtime.leaderelection import LeaderElector
from odh_kubeflow_amd.utils.timeutil import rfc3339_micro

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lease(holder, renew, dur=1):
    return {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
            "metadata": {"name": "ctl", "namespace": "ns"},
            "spec": {"holderIdentity": holder, "renewTime": renew, "leaseDurationSeconds": dur}}


def test_skewed_holder_clock_does_not_expire_a_live_lease(run):
    """The holder's clock is an hour behind, so its renewTime always looks expired on the
    candidate's wall clock; it keeps renewing, so the candidate must not take the Lease.
    Once it stops renewing, the candidate takes over after one lease duration."""
    async def go():
        store = ObjectStore()
        cli = in_process_manager(store, name="t").client
        await cli.create(_lease("other", rfc3339_micro(time.time() - 3600)))
        stop = asyncio.Event()

        async def skewed_holder():
            while not stop.is_set():
                cur = await cli.get(kinds.LEASE, "ctl", "ns")
                cur["spec"]["renewTime"] = rfc3339_micro(time.time() - 3600)
                await cli.update(cur)
                await asyncio.sleep(0.1)
        task = asyncio.ensure_future(skewed_holder())
        le = LeaderElector(cli, "ctl", "ns", identity="me", lease_duration=1.0, renew_deadline=0.5, retry_period=0.05)
        t_end = time.monotonic() + 2.0
        while time.monotonic() < t_end:
            assert not await le.try_acquire_or_renew()
            await asyncio.sleep(0.05)
        stop.set()
        await task
        t0 = time.monotonic()
        while not await le.try_acquire_or_renew():
            await asyncio.sleep(0.05)
        waited = time.monotonic() - t0
        assert 0.8 <= waited < 2.0, waited
        assert (await cli.get(kinds.LEASE, "ctl", "ns"))["spec"]["holderIdentity"] == "me"
    run(go())


def test_released_lease_is_taken_immediately(run):
    async def go():
        store = ObjectStore()
        cli = in_process_manager(store, name="t").client
        await cli.create(_lease("", rfc3339_micro(), 1))
        le = LeaderElector(cli, "ctl", "ns", identity="me", lease_duration=15, renew_deadline=10, retry_period=1)
        assert await le.try_acquire_or_renew()
    run(go())


def test_manager_exits_when_leadership_is_lost(run):
    async def go():
        store = ObjectStore()
        admin = in_process_manager(store, name="admin").client
        le = LeaderElector(in_process_manager(store, name="le").client, "ctl", "ns", identity="me",
                           lease_duration=1.0, renew_deadline=0.4, retry_period=0.05)
        mgr = in_process_manager(store, name="kf", leader_elector=le)
        stop = asyncio.Event()
        runner = asyncio.ensure_future(mgr.run_until(stop))
        for _ in range(100):
            if mgr.elected is not None and mgr.elected.is_set():
                break
            await asyncio.sleep(0.02)
        assert mgr.elected.is_set() and all(fn() for fn in mgr.healthz.values())
        # another candidate steals the Lease (e.g. after a partition); renewals now fail
        cur = await admin.get(kinds.LEASE, "ctl", "ns")
        cur["spec"].update(holderIdentity="thief", renewTime=rfc3339_micro(), leaseDurationSeconds=30)
        await admin.update(cur)
        rc = await asyncio.wait_for(runner, 5)
        assert rc == 1 and mgr.fatal == "leader election lost" and le.lost
        assert not mgr.healthz["leader-election"]()
        assert not stop.is_set()
    run(go())


def test_kf_manager_process_exits_nonzero_on_lost_lease(tmp_path, run):
    from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig
    from tests.test_processes_e2e import free_port, spawn, wait_http

    api_port = free_port()
    master = f"http://127.0.0.1:{api_port}"
    logf = open(tmp_path / "procs.log", "wb")
    api = spawn(["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(api_port), "--no-openshift-apis"], log=logf)
    mgr = None
    try:
        async def go():
            nonlocal mgr
            await wait_http(master + "/healthz")
            c = RestClient(RestConfig(host=master))
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "opendatahub"}})
            mgr = subprocess.Popen(
                [sys.executable, "-m", "odh_kubeflow_amd.cmd.kf_manager", "--master", master, "--metrics-addr", "0",
                 "--probe-addr", "0", "--enable-leader-election", "--leader-election-lease-duration", "2",
                 "--leader-election-renew-deadline", "1", "--leader-election-retry-period", "0.1"],
                cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT, K8S_NAMESPACE="opendatahub"),
                stdout=logf, stderr=subprocess.STDOUT)
            lease = None
            for _ in range(300):
                try:
                    lease = await c.get(kinds.LEASE, "kubeflow-notebook-controller", "opendatahub")
                    if lease["spec"].get("holderIdentity"):
                        break
                except Exception:
                    pass
                await asyncio.sleep(0.05)
            lease["spec"].update(holderIdentity="thief", renewTime=rfc3339_micro(), leaseDurationSeconds=60)
            await c.update(lease)
            await c.close()
        run(go(), timeout=60)
        assert mgr.wait(15) == 1
    finally:
        for p in (mgr, api):
            if p is not None and p.poll() is None:
                p.terminate()
                p.wait(10)
        logf.close()
