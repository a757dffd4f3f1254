"""Container runtime that runs each notebook container as a real process — TEST PLATFORM.

The fake kubelet's default runtime starts nothing, so pod start-up costs zero and a
"create → Ready" figure measures only the control plane (BASELINE config #1).  Configs
#2/#3 need the notebook's own start: this runtime spawns
:mod:`odh_kubeflow_amd.testing.notebook_server.workbench` per pod — the Jupyter API served,
and a first cell that imports PyTorch, initialises the HIP runtime on the pod's allocated
MI355X (``HIP_VISIBLE_DEVICES``, the device plugin's job) and runs a bf16 matmul — with the
container's env (``NB_PREFIX`` …) and reports the pod Ready once its readiness probe
(``GET <NB_PREFIX>/api``) answers.  ``gpu_init="first-cell"`` (default) runs that cell after
the server is Ready, as JupyterLab would (:meth:`first_cell` awaits it);
``"before-ready"`` holds readiness until the GPU is usable.  A pod's MI355X start-up probe init container
(``odh-gpu-probe``) runs first, as its own process on the same GPU.  Image pull and
container-runtime overheads are not included (no registry or container runtime on the
benchmark boxes).

The readiness probe is polled every ``probe_interval_s`` (20 ms) rather than at the
kubelet's ``periodSeconds`` granularity (≥ 1 s), to time the process itself.
"""

from __future__ import annotations

import asyncio
import json
import os
import sys
import time
from typing import Dict, Optional, Sequence

from ...models import meta as m
from .node import ContainerHandle, ContainerRuntime

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


class ProcessContainerRuntime(ContainerRuntime):
    def __init__(self, host: str = "127.0.0.1", matmul: int = 1024, ready_timeout_s: float = 300.0,
                 probe_interval_s: float = 0.02, visible_device=None, env: Optional[Dict[str, str]] = None,
                 gpu_init: str = "first-cell"):
        if gpu_init not in ("first-cell", "before-ready"):
            raise ValueError(f"gpu_init: {gpu_init!r}")
        self.host = host
        self.matmul = matmul
        self.gpu_init = gpu_init
        self.ready_timeout_s = ready_timeout_s
        self.probe_interval_s = probe_interval_s
        # node GPU index → the HIP device id the process should see (a 1-GPU box hosts all
        # eight "node GPUs" on its one device)
        self.visible_device = visible_device or (lambda d: d)
        self.exec_init = True  # the start-up probe init container runs as a process too
        self.env = env or {}
        self.procs: Dict[str, asyncio.subprocess.Process] = {}
        self.reports: Dict[str, dict] = {}

    def _container_env(self, pod: dict, devices: Sequence[int]) -> Dict[str, str]:
        env = {k: v for k, v in os.environ.items() if not k.startswith(("HIP_VISIBLE", "ROCR_VISIBLE", "CUDA_VISIBLE"))}
        c0 = ((pod.get("spec") or {}).get("containers") or [{}])[0]
        for e in c0.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
        if devices:
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(self.visible_device(d)) for d in devices)
        else:
            env["HIP_VISIBLE_DEVICES"] = ""  # a CPU pod sees no GPU
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        env.update(self.env)
        return env

    async def start(self, pod: dict, devices: Sequence[int]) -> ContainerHandle:
        import aiohttp

        from ...utils.procutil import child_env

        env = self._container_env(pod, devices)
        prefix = env.get("NB_PREFIX") or f"/notebook/{m.namespace(pod)}/{m.labels(pod).get('notebook-name', m.name(pod))}"
        t0 = time.perf_counter()
        proc = await asyncio.create_subprocess_exec(
            sys.executable, "-m", "odh_kubeflow_amd.testing.notebook_server.workbench", "--prefix", prefix,
            "--host", self.host, "--matmul", str(self.matmul if devices else 0),
            "--gpu-init", self.gpu_init,
            env=child_env(env), cwd=ROOT, stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.DEVNULL)
        key = m.key(pod)
        self.procs[key] = proc
        try:
            line = await asyncio.wait_for(proc.stdout.readline(), self.ready_timeout_s)
            report = json.loads(line.decode() or "{}")
            port = int(report["port"])
        except (asyncio.TimeoutError, ValueError, KeyError) as e:
            proc.kill()
            await proc.wait()
            raise RuntimeError(f"workbench of {key} did not start (rc={proc.returncode}): {e!r}")
        # readiness probe: GET <prefix>/api until 200
        url = f"http://{self.host}:{port}{prefix}/api"
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5)) as s:
            while True:
                try:
                    async with s.get(url) as r:
                        if r.status == 200:
                            break
                except aiohttp.ClientError:
                    pass
                if time.perf_counter() - t0 > self.ready_timeout_s:
                    raise RuntimeError(f"workbench of {key}: readiness probe failed")
                await asyncio.sleep(self.probe_interval_s)
        report["spawn_to_ready_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        self.reports[key] = report
        return ContainerHandle(key, devices, ip=self.host, port=port, info={"pid": proc.pid, "workbench": report})

    async def first_cell(self, key: str, timeout_s: Optional[float] = None) -> dict:
        """Wait for the workbench of pod ``key`` to finish its first cell (``first-cell``
        mode) and return the cell's timings; in ``before-ready`` mode the start-up report
        already holds them.  Call before the pod is stopped (``stop`` drains stdout)."""
        report = self.reports[key]
        if self.gpu_init == "before-ready" or "first_cell" in report:
            return report.get("first_cell", report)
        proc = self.procs[key]
        deadline = time.perf_counter() + (timeout_s or self.ready_timeout_s)
        cell = None
        while cell is None:  # skip anything else a library printed to stdout meanwhile
            line = await asyncio.wait_for(proc.stdout.readline(), max(0.0, deadline - time.perf_counter()))
            if not line:
                raise RuntimeError(f"workbench of {key} exited before its first cell (rc={proc.returncode})")
            try:
                msg = json.loads(line.decode())
            except ValueError:
                continue
            cell = msg.get("first_cell") if isinstance(msg, dict) else None
        report["first_cell"] = cell
        return cell

    async def stop(self, handle: ContainerHandle) -> None:
        proc = self.procs.get(handle.pod_key)
        if proc is None:
            return
        try:
            if proc.returncode is None:
                proc.terminate()
            try:
                await asyncio.wait_for(proc.communicate(), 10)  # drains stdout: the pipe transport closes
            except asyncio.TimeoutError:
                proc.kill()
                await proc.communicate()
        finally:
            # listed until it has exited and its pipes are closed
            if self.procs.get(handle.pod_key) is proc:
                self.procs.pop(handle.pod_key, None)

    async def close(self) -> None:
        for key in list(self.procs):
            await self.stop(ContainerHandle(key, []))
