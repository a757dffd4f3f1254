"""Launcher for the native C++ apiserver (``testing/native/apiserver/apiserver.cpp`` →
``testing/native/bin/odh-apiserver``).

The scheme (kinds, plurals, scope, versions, status subresource, installed CRDs) is
generated from :data:`~odh_kubeflow_amd.models.scheme.SCHEME` so both apiservers —
the in-process Python :class:`~odh_kubeflow_amd.testing.apiserver.store.ObjectStore` and the
native one — serve exactly the same API.  :class:`StoreView` gives tests and the
benchmark the ``peek`` / ``list_nocopy`` read helpers of the in-process store on top of
a watch-backed informer cache.
"""

from __future__ import annotations

import asyncio
import json
import os
import tempfile
from typing import Iterable, List, Optional

from ...models.scheme import SCHEME

HERE = os.path.dirname(os.path.abspath(__file__))
BINARY = os.path.join(os.path.dirname(HERE), "native", "bin", "odh-apiserver")


def scheme_config(uninstalled: Iterable[str] = (), gc: bool = False, token: Optional[str] = None,
                  history: int = 512) -> dict:
    skip = {SCHEME.resolve(k).key for k in uninstalled}
    res = []
    for i in SCHEME.all():
        res.append({"group": i.group, "kind": i.kind, "plural": i.plural, "singular": i.singular,
                    "listKind": i.list_kind, "versions": list(i.versions), "storageVersion": i.storage_version,
                    "namespaced": i.namespaced, "status": i.status_subresource, "installed": i.key not in skip})
    from ...models.crd import version_schema

    # CRD structural schemas: prune -> default -> validate, as models/openapi.py does in-process
    cfg = {"resources": res, "gc": gc, "history": history, "defaulting": True,
           "schemas": {"notebooks.kubeflow.org": version_schema()}}
    if token:
        cfg["token"] = token
    return cfg


def available() -> bool:
    return os.path.exists(BINARY)


class NativeApiServer:
    """``binary`` (or ``$ODH_APISERVER_BINARY``) selects another build of the server, e.g. the
    ThreadSanitizer one the race-detection test compiles; ``env`` is added to its environment.
    ``history`` (default ``$ODH_APISERVER_HISTORY`` or 512) bounds each resource's watch
    history in events."""

    def __init__(self, uninstalled: Iterable[str] = (), gc: bool = False, token: Optional[str] = None,
                 host: str = "127.0.0.1", port: int = 0, history: Optional[int] = None, binary: Optional[str] = None,
                 env: Optional[dict] = None, audit_log_path: Optional[str] = None, audit_policy=None,
                 write_latency_ms: float = 0.0):
        if history is None:
            history = int(os.environ.get("ODH_APISERVER_HISTORY") or 512)
        self.cfg = scheme_config(uninstalled, gc, token, history)
        self.write_latency_ms = float(write_latency_ms)  # etcd-like storage round trip per write
        if audit_log_path:  # kube-apiserver --audit-log-path / --audit-policy-file (apiserver/audit.py)
            from .audit import DEFAULT_POLICY, AuditPolicy

            pol = audit_policy or AuditPolicy.load(DEFAULT_POLICY)
            self.cfg["audit"] = {"path": os.path.abspath(audit_log_path), "policy": pol.to_json()}
        self.host = host
        self.port = port
        self.binary = binary or os.environ.get("ODH_APISERVER_BINARY") or BINARY
        self.env = env
        self.proc: Optional[asyncio.subprocess.Process] = None
        self._cfg_path: Optional[str] = None

    async def start(self) -> "NativeApiServer":
        from ...utils.procutil import child_env

        if self.binary == BINARY and not available():
            from ...ops.build import build

            build(verbose=False)
        fd, self._cfg_path = tempfile.mkstemp(prefix="odh-apiserver-", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(self.cfg, f)
        self.proc = await asyncio.create_subprocess_exec(
            self.binary, "--config", self._cfg_path, "--host", self.host, "--port", str(self.port),
            *(["--write-latency-ms", f"{self.write_latency_ms:g}"] if self.write_latency_ms > 0 else []),
            stdout=asyncio.subprocess.PIPE, env=child_env({**os.environ, **(self.env or {})}))
        line = await asyncio.wait_for(self.proc.stdout.readline(), 30)
        if not line.startswith(b"LISTENING"):
            raise RuntimeError(f"native apiserver failed to start: {line!r}")
        self.port = int(line.split()[1])
        return self

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    async def stats(self) -> dict:
        import aiohttp

        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30)) as s:
            async with s.get(self.url + "/metrics") as r:
                return await r.json(content_type=None)

    async def admissions(self, start: int = 0) -> dict:
        """Admission webhook calls from call ``start`` on: ``{"seq": next start, "us": [wall µs]}``."""
        import aiohttp

        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30)) as s:
            async with s.get(self.url + f"/debug/admissions?from={int(start)}") as r:
                return await r.json(content_type=None)

    async def set_write_latency(self, ms: float) -> None:
        """Change the etcd-like per-write storage latency while serving."""
        import aiohttp

        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30)) as s:
            async with s.post(self.url + "/debug/storage-latency", json={"ms": float(ms)}) as r:
                if r.status != 200:
                    raise RuntimeError(f"storage-latency: HTTP {r.status}: {await r.text()}")
        self.write_latency_ms = float(ms)

    async def stop(self) -> None:
        if self.proc is not None and self.proc.returncode is None:
            self.proc.terminate()
            try:
                await asyncio.wait_for(self.proc.wait(), 10)
            except asyncio.TimeoutError:
                self.proc.kill()
        if self._cfg_path and os.path.exists(self._cfg_path):
            os.unlink(self._cfg_path)


class StoreView:
    """Read-only ``ObjectStore``-like view (``peek``, ``list_nocopy``) over an informer cache."""

    def __init__(self, cache):
        self.cache = cache

    def peek(self, ref, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        return self.cache.get(ref, name, namespace)

    def list_nocopy(self, ref, namespace=None, label_selector=None, field_selector=None, owner_uid=None,
                    copy: bool = False, version=None) -> List[dict]:
        return self.cache.list(ref, namespace, label_selector, field_selector, owner_uid)
