"""``kubectl proxy`` + every notebook's Jupyter API as one process (TEST PLATFORM ONLY).

    python -m odh_kubeflow_amd.testing.cmd.jupyter_proxy --port 18001

The culler in ``DEV`` mode reaches each notebook's ``/api/kernels`` and ``/api/terminals``
through ``kubectl proxy`` (``kf/controllers/culling_controller.go:249-256``; the proxy
address is ``CULLER_DEV_PROXY_URL``, default ``http://localhost:8001``).  The benchmark's
resident-population block points the culler here
(:class:`~odh_kubeflow_amd.testing.notebook_server.jupyter.JupyterProxy`): hundreds of
running notebooks, each answering like an idle Jupyter server, without a server process per
pod.  Prints ``ready`` once it listens.
"""

from __future__ import annotations

import argparse
import asyncio
import sys


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-jupyter-proxy")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, required=True)
    return p.parse_args(argv)


async def amain(argv=None) -> int:
    from ...cmd.common import signal_event
    from ..notebook_server.jupyter import JupyterProxy

    args = parse(argv)
    proxy = await JupyterProxy(args.host, args.port).start()
    print("ready", flush=True)
    try:
        await signal_event().wait()
    finally:
        await proxy.stop()
    return 0


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
