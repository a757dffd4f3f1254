"""Lease-based leader election (``coordination.k8s.io/v1`` Lease), as controller-runtime
runs it for ``--enable-leader-election`` / ``--leader-elect``
(``kf/main.go:91-93`` ID ``kubeflow-notebook-controller``; ``odh/main.go:159-160``).

Active/passive: a candidate acquires the Lease when it is free or expired, renews it
every ``retry_period`` and must renew within ``renew_deadline`` or step down — the
manager then exits the process non-zero, as controller-runtime does, so the kubelet
restarts it as a fresh candidate.  Defaults are controller-runtime's: lease 15 s, renew
deadline 10 s, retry 2 s.  ``release()`` on shutdown clears the holder so a standby
takes over immediately (``LeaderElectionReleaseOnCancel``).

Expiry is judged like client-go's ``observedTime``: never by comparing the holder's
``renewTime`` (written with the holder's wall clock) against the local clock, but by how
long the Lease record has gone unchanged on this candidate's monotonic clock.  Clock skew
between nodes therefore cannot let a standby take a Lease that is still being renewed.
"""

from __future__ import annotations

import asyncio
import logging
import os
import socket
import time
import uuid
from typing import Awaitable, Callable, Optional

from ..models import kinds
from ..models.errors import ApiError, is_conflict, is_not_found
from ..utils.timeutil import rfc3339_micro

log = logging.getLogger("runtime.leaderelection")


def default_identity() -> str:
    """``<hostname>_<uuid>`` like controller-runtime; ``POD_NAME`` (downward API) names the
    pod instead of the container hostname when it is set."""
    return f"{os.environ.get('POD_NAME') or socket.gethostname()}_{uuid.uuid4()}"


class LeaderElector:
    def __init__(self, client, lease_name: str, namespace: str, identity: Optional[str] = None,
                 lease_duration: float = 15.0, renew_deadline: float = 10.0, retry_period: float = 2.0):
        if renew_deadline >= lease_duration:
            raise ValueError("renew_deadline must be shorter than lease_duration")
        self.client = client
        self.name = lease_name
        self.namespace = namespace
        self.identity = identity or default_identity()
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.is_leader = False
        self.transitions = 0
        self.lost = False
        self._observed = None  # (holder, renewTime, leaseDurationSeconds) last seen
        self._observed_at = 0.0  # time.monotonic() when that record was first seen

    def _spec(self, cur: Optional[dict]) -> dict:
        now = rfc3339_micro()
        spec = dict((cur or {}).get("spec") or {})
        if spec.get("holderIdentity") != self.identity:
            spec["acquireTime"] = now
            spec["leaseTransitions"] = int(spec.get("leaseTransitions") or 0) + (1 if cur else 0)
        spec["holderIdentity"] = self.identity
        spec["leaseDurationSeconds"] = int(self.lease_duration)
        spec["renewTime"] = now
        return spec

    async def try_acquire_or_renew(self) -> bool:
        try:
            cur = await self.client.get(kinds.LEASE, self.name, self.namespace)
        except ApiError as e:
            if not is_not_found(e):
                raise
            try:
                await self.client.create({"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                                          "metadata": {"name": self.name, "namespace": self.namespace},
                                          "spec": self._spec(None)})
                return True
            except ApiError as e2:
                log.debug("lease create lost: %r", e2)
                return False
        spec = cur.get("spec") or {}
        holder = spec.get("holderIdentity")
        record = (holder, spec.get("renewTime"), spec.get("leaseDurationSeconds"))
        if record != self._observed:
            self._observed, self._observed_at = record, time.monotonic()
        if holder and holder != self.identity:
            dur = float(spec.get("leaseDurationSeconds") or self.lease_duration)
            if time.monotonic() < self._observed_at + dur:
                return False  # held by a leader that renewed within the lease duration
        cur["spec"] = self._spec(cur)
        try:
            await self.client.update(cur)
            sp = cur["spec"]
            self._observed = (sp["holderIdentity"], sp["renewTime"], sp["leaseDurationSeconds"])
            self._observed_at = time.monotonic()
            return True
        except ApiError as e:
            if is_conflict(e):
                return False
            raise

    async def run(self, on_started: Callable[[], Awaitable[None]],
                  on_stopped: Callable[[], Awaitable[None]]) -> None:
        # acquire
        while True:
            try:
                if await self.try_acquire_or_renew():
                    break
            except Exception as e:
                log.warning("leader election: %r", e)
            await asyncio.sleep(self.retry_period)
        self.is_leader = True
        self.transitions += 1
        log.info("%s became leader of %s/%s", self.identity, self.namespace, self.name)
        await on_started()
        # renew
        last = time.monotonic()
        try:
            while True:
                await asyncio.sleep(self.retry_period)
                ok = False
                try:
                    ok = await self.try_acquire_or_renew()
                except Exception as e:
                    log.warning("lease renew failed: %r", e)
                if ok:
                    last = time.monotonic()
                elif time.monotonic() - last > self.renew_deadline:
                    log.error("failed to renew lease %s/%s within %.0fs", self.namespace, self.name,
                              self.renew_deadline)
                    break
        finally:
            was = self.is_leader
            self.is_leader = False
        if was:
            self.lost = True
            await on_stopped()

    async def release(self) -> None:
        if not self.transitions:
            return  # never led
        try:
            cur = await self.client.get(kinds.LEASE, self.name, self.namespace)
            if (cur.get("spec") or {}).get("holderIdentity") == self.identity:
                cur["spec"]["holderIdentity"] = ""
                cur["spec"]["leaseDurationSeconds"] = 1
                await self.client.update(cur)
        except Exception as e:
            log.debug("lease release failed: %r", e)
        self.is_leader = False


def namespace_from_env(default: str = "default") -> str:
    """``getControllerNamespace`` (``odh/main.go:103-115``): SA namespace file, then ``K8S_NAMESPACE``."""
    p = "/var/run/secrets/kubernetes.io/serviceaccount/namespace"
    try:
        with open(p) as f:
            ns = f.read().strip()
            if ns:
                return ns
    except OSError:
        pass
    return os.environ.get("K8S_NAMESPACE") or default
