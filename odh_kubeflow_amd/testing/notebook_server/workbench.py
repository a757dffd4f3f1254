"""A PyTorch-ROCm workbench process: what the notebook container runs, minus the image.

    python -m odh_kubeflow_amd.testing.notebook_server.workbench --prefix /notebook/<ns>/<name>

BASELINE configs #2/#3 time a notebook pod requesting ``amd.com/gpu`` becoming Ready on an
MI355X with a PyTorch-ROCm Jupyter image.  There is no container runtime or registry on
the benchmark boxes, so the test platform's process runtime
(:class:`~odh_kubeflow_amd.testing.kubelet.process_runtime.ProcessContainerRuntime`) starts this
program as the container's process instead: with the allocated GPU made visible
(``HIP_VISIBLE_DEVICES``, what the AMD device plugin's device mounts amount to) it serves
the Jupyter API the culler and the readiness probe use (``<prefix>/api``, ``/api/kernels``,
``/api/terminals``) and runs the user's first cell: import PyTorch, initialise the HIP
runtime on the GPU, a first bf16 matmul (hipBLASLt and the MFMA path loaded).

``--gpu-init`` decides when that first cell runs relative to readiness:

* ``first-cell`` (default) — JupyterLab's behaviour: the server listens and answers the
  readiness probe at once (a Jupyter server imports no PyTorch and touches no GPU); the
  first cell runs afterwards, as a user's would, and its timings appear on ``/api``.
* ``before-ready`` — the cell runs before the server listens, so Ready means "GPU usable"
  (round 2's workbench; kept for comparison).

It prints one JSON line with its port and start-up timings when it starts listening (until
then the readiness probe is refused, as with a real server) and, in ``first-cell`` mode, a
second line ``{"first_cell": {...}}`` when the cell has run.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import sys
import time

T_PROC = time.perf_counter()


def init_gpu(n: int) -> dict:
    t0 = time.perf_counter()
    import torch

    out = {"import_torch_ms": round((time.perf_counter() - t0) * 1e3, 1), "torch": torch.__version__,
           "hip": getattr(torch.version, "hip", None), "gpu": None}
    if torch.cuda.is_available() and n > 0:
        t1 = time.perf_counter()
        dev = torch.device("cuda", 0)
        torch.cuda.init()
        a = torch.randn((n, n), device=dev, dtype=torch.bfloat16)
        c = a @ a
        c.float().sum().item()  # synchronises
        props = torch.cuda.get_device_properties(0)
        out["gpu"] = torch.cuda.get_device_name(0)
        out["arch"] = getattr(props, "gcnArchName", "").split(":")[0]
        out["visible_devices"] = os.environ.get("HIP_VISIBLE_DEVICES")
        out["first_matmul_ms"] = round((time.perf_counter() - t1) * 1e3, 1)
        out["hbm_total_gib"] = round(props.total_memory / 2 ** 30, 1)
    return out


async def serve(prefix: str, host: str, info: dict, first_cell: int = -1) -> None:
    """Serve the Jupyter API; with ``first_cell >= 0`` run :func:`init_gpu` (matmul size
    ``first_cell``) once listening, off the event loop, and publish its timings."""
    from .jupyter import JupyterServer

    srv = await JupyterServer(prefix, host, 0, info=info).start()
    info["ready_ms"] = round((time.perf_counter() - T_PROC) * 1e3, 1)
    print(json.dumps({"port": srv.port, **info}), flush=True)
    if first_cell >= 0:
        try:
            cell = await asyncio.to_thread(init_gpu, first_cell)
        except Exception as e:  # a failing cell does not take the server down
            cell = {"error": f"{type(e).__name__}: {e}"}
        cell["first_cell_done_ms"] = round((time.perf_counter() - T_PROC) * 1e3, 1)
        info.update(cell)  # the dict GET <prefix>/api answers with
        print(json.dumps({"first_cell": cell}), flush=True)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for s in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(s, stop.set)
    await stop.wait()
    await srv.stop()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="workbench")
    ap.add_argument("--prefix", default=os.environ.get("NB_PREFIX", "/"))
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--matmul", type=int, default=1024, help="first bf16 matmul size (0: no GPU work)")
    ap.add_argument("--gpu-init", choices=("first-cell", "before-ready"), default="first-cell",
                    help="run the first cell (torch import, HIP init, matmul) after the server is Ready "
                         "(JupyterLab) or before it listens")
    a = ap.parse_args(argv)
    if a.gpu_init == "before-ready":
        info = init_gpu(a.matmul)
        info["gpu_init"] = a.gpu_init
        asyncio.run(serve(a.prefix, a.host, info))
    else:
        asyncio.run(serve(a.prefix, a.host, {"gpu_init": a.gpu_init}, first_cell=a.matmul))
    return 0


if __name__ == "__main__":
    sys.exit(main())
