"""Jupyter-server API subset served by notebook containers of the in-process node agent.

The culler polls ``/notebook/<ns>/<name>/api/kernels`` and ``/api/terminals``
(``kf/controllers/culling_controller.go:243-313``); the reference's e2e suite exercises
that against a real Jupyter image.  Here each started notebook pod gets a small aiohttp
server with the same JSON shapes (kernel ``id``/``name``/``last_activity``/
``execution_state``/``connections``; terminal ``name``/``last_activity``), whose state
tests and benchmarks drive directly (start a kernel, make it busy, go idle).
:class:`JupyterContainerRuntime` plugs it into ``GpuRuntime`` as the container runtime.
"""

from __future__ import annotations

import asyncio
import uuid
from typing import Dict, List, Optional, Sequence

from ..kubelet.node import ContainerHandle, ContainerRuntime
from ...models import meta as m
from ...utils.timeutil import rfc3339


class JupyterState:
    def __init__(self, prefix: str):
        self.prefix = prefix.rstrip("/")
        self.kernels: Dict[str, dict] = {}
        self.terminals: Dict[str, dict] = {}
        self.requests = 0

    def start_kernel(self, name: str = "python3", busy: bool = False) -> str:
        kid = str(uuid.uuid4())
        self.kernels[kid] = {"id": kid, "name": name, "last_activity": rfc3339(),
                             "execution_state": "busy" if busy else "idle", "connections": 1}
        return kid

    def set_kernel_state(self, kid: str, state: str, touch: bool = True) -> None:
        k = self.kernels[kid]
        k["execution_state"] = state
        if touch:
            k["last_activity"] = rfc3339()

    def set_kernel_last_activity(self, kid: str, ts: str) -> None:
        self.kernels[kid]["last_activity"] = ts

    def open_terminal(self, last_activity: Optional[str] = None) -> str:
        name = str(len(self.terminals) + 1)
        self.terminals[name] = {"name": name, "last_activity": last_activity or rfc3339()}
        return name


class JupyterServer:
    def __init__(self, prefix: str, host: str = "127.0.0.1", port: int = 0, info: Optional[dict] = None):
        self.state = JupyterState(prefix)
        self.host = host
        self.port = port
        self.info = info or {}  # extra fields of GET <prefix>/api (the workbench's start-up report)
        self._runner = None

    async def start(self) -> "JupyterServer":
        from aiohttp import web

        st = self.state

        async def kernels(_req):
            st.requests += 1
            return web.json_response(list(st.kernels.values()))

        async def terminals(_req):
            st.requests += 1
            return web.json_response(list(st.terminals.values()))

        async def api(_req):
            return web.json_response({"version": "2.14.0", **self.info})

        app = web.Application()
        app.router.add_get(st.prefix + "/api/kernels", kernels)
        app.router.add_get(st.prefix + "/api/terminals", terminals)
        app.router.add_get(st.prefix + "/api", api)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None


class JupyterProxy:
    """``kubectl proxy`` in front of every notebook's Jupyter server, for the culler's ``DEV``
    mode (``kf/controllers/culling_controller.go:249-256``: ``/api/v1/namespaces/<ns>/services/
    <nm>:http-<nm>/proxy/notebook/<ns>/<nm>/api/{kernels,terminals}``) — one process answering
    for R resident notebooks, where a :class:`JupyterServer` per pod would be R servers.

    Every notebook reports one idle kernel whose last activity is this proxy's start (and no
    terminals): a notebook nobody uses, so each check is the culler's plain heartbeat, never a
    cull while ``CULL_IDLE_TIME`` has not passed."""

    PATH = "/api/v1/namespaces/{ns}/services/{svc}/proxy/notebook/{ns2}/{nm}/api/{res}"

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.host = host
        self.port = port
        self.requests = 0
        self.started_at = rfc3339()
        self._runner = None

    async def start(self) -> "JupyterProxy":
        from aiohttp import web

        kernel = [{"id": "00000000-0000-0000-0000-000000000000", "name": "python3", "last_activity": self.started_at,
                   "execution_state": "idle", "connections": 0}]

        async def api(req):
            self.requests += 1
            res = req.match_info["res"]
            if res == "kernels":
                return web.json_response(kernel)
            if res == "terminals":
                return web.json_response([])
            raise web.HTTPNotFound()

        app = web.Application()
        app.router.add_get(self.PATH, api)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port, backlog=1024)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None


class JupyterContainerRuntime(ContainerRuntime):
    """Container runtime whose "notebook container" is a :class:`JupyterServer`."""

    def __init__(self, start_delay: float = 0.0, host: str = "127.0.0.1"):
        self.start_delay = start_delay
        self.host = host
        self.servers: Dict[str, JupyterServer] = {}

    async def start(self, pod: dict, devices: Sequence[int]) -> ContainerHandle:
        if self.start_delay:
            await asyncio.sleep(self.start_delay)
        nb = m.labels(pod).get("notebook-name") or m.name(pod)
        srv = await JupyterServer(f"/notebook/{m.namespace(pod)}/{nb}", self.host).start()
        key = f"{m.namespace(pod)}/{nb}"
        old = self.servers.pop(key, None)
        if old is not None:
            await old.stop()
        self.servers[key] = srv
        h = ContainerHandle(m.key(pod), devices, ip=self.host, port=srv.port, info={"notebook": key})
        return h

    async def stop(self, handle: ContainerHandle) -> None:
        key = handle.info.get("notebook")
        srv = self.servers.get(key)
        if srv is not None and srv.port == handle.port:
            self.servers.pop(key, None)
            await srv.stop()

    async def close(self) -> None:
        for s in list(self.servers.values()):
            await s.stop()
        self.servers.clear()

    def state(self, namespace: str, name: str) -> Optional[JupyterState]:
        s = self.servers.get(f"{namespace}/{name}")
        return s.state if s else None

    def all_states(self) -> List[JupyterState]:
        return [s.state for s in self.servers.values()]
