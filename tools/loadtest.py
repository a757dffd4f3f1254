#!/usr/bin/env python3
"""Notebook load generator against any apiserver (kube-apiserver or ours).

Reference counterpart: ``kf/loadtest/start_notebooks.py:1-99`` applies N Notebook CRs
(+ PVCs) with ``kubectl`` and records nothing.  This one talks REST directly (kubeconfig,
in-cluster config or ``--server``), creates N notebooks requesting ``amd.com/gpu`` with
an optional PVC each, and measures create→Ready per notebook from a watch — so the same
numbers as ``bench.py`` can be taken on a real cluster.

    python tools/loadtest.py -l 8 -n loadtest --gpus 1                 # create + measure
    python tools/loadtest.py -l 8 -n loadtest -p delete                # clean up
    python tools/loadtest.py -l 8 -n loadtest --local                  # in-process cluster

Prints one JSON summary line (count, ready, p50/p95/max create→Ready ms, wall s).
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from odh_kubeflow_amd.models import kinds  # noqa: E402
from odh_kubeflow_amd.models.errors import ApiError, is_already_exists, is_not_found  # noqa: E402
from odh_kubeflow_amd.models.notebook import notebook  # noqa: E402

DEFAULT_IMAGE = "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_2.10"


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("-l", "--load", dest="num_notebooks", type=int, default=3, help="number of notebooks")
    p.add_argument("-n", "--namespace", default="kubeflow")
    p.add_argument("-p", "--operation", choices=("create", "delete"), default="create")
    p.add_argument("--gpus", type=int, default=1, help="amd.com/gpu per notebook (0 for CPU notebooks)")
    p.add_argument("--image", default=DEFAULT_IMAGE)
    p.add_argument("--pvc", action="store_true", help="give every notebook a 10Gi workspace PVC")
    p.add_argument("--inject-auth", action="store_true", help="set notebooks.opendatahub.io/inject-auth=true")
    p.add_argument("--timeout", type=float, default=300.0)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--server", default=None, help="apiserver URL (overrides kubeconfig)")
    p.add_argument("--local", action="store_true", help="run against an in-process cluster (no real cluster)")
    return p.parse_args(argv)


def _pvc(name: str, ns: str) -> dict:
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": ns},
            "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "10Gi"}}}}


def _ready(nb) -> bool:
    st = (nb or {}).get("status") or {}
    return st.get("readyReplicas") == 1 and any(
        c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])


async def run(args, client) -> dict:
    ns = args.namespace
    names = [f"jupyter-test-{i}" for i in range(args.num_notebooks)]
    if args.operation == "delete":
        n = 0
        for nm in names:
            for kind, obj in ((kinds.NOTEBOOK, nm), ("v1/PersistentVolumeClaim", f"{nm}-workspace")):
                try:
                    await client.delete(kind, obj, ns)
                    n += 1
                except ApiError as e:
                    if not is_not_found(e):
                        raise
        return {"deleted": n}
    try:
        await client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    except ApiError as e:
        if not is_already_exists(e):
            raise
    ready_at, t0 = {}, {}

    async def watch():
        async for et, obj in client.watch(kinds.NOTEBOOK, ns, "0"):
            nm = obj["metadata"]["name"]
            if nm in t0 and nm not in ready_at and _ready(obj):
                ready_at[nm] = time.perf_counter()

    wt = asyncio.ensure_future(watch())
    ann = {"notebooks.opendatahub.io/inject-auth": "true"} if args.inject_auth else None
    start = time.perf_counter()
    for nm in names:
        nb = notebook(nm, ns, image=args.image, gpus=args.gpus, annotations=ann)
        if args.pvc:
            await client.create(_pvc(f"{nm}-workspace", ns))
            spec = nb["spec"]["template"]["spec"]
            spec.setdefault("volumes", []).append({"name": "workspace",
                                                   "persistentVolumeClaim": {"claimName": f"{nm}-workspace"}})
            spec["containers"][0].setdefault("volumeMounts", []).append({"name": "workspace",
                                                                         "mountPath": "/home/jovyan"})
        t0[nm] = time.perf_counter()
        await client.create(nb)
    deadline = time.monotonic() + args.timeout
    while len(ready_at) < len(names) and time.monotonic() < deadline:
        await asyncio.sleep(0.01)
    wt.cancel()
    lat = sorted((ready_at[n] - t0[n]) * 1e3 for n in ready_at)

    def pct(q):
        return round(lat[min(len(lat) - 1, int(q * (len(lat) - 1) + 0.5))], 3) if lat else None

    return {"count": len(names), "ready": len(lat), "p50_ready_ms": pct(0.5), "p95_ready_ms": pct(0.95),
            "max_ready_ms": round(lat[-1], 3) if lat else None, "wall_s": round(time.perf_counter() - start, 3)}


async def amain(args) -> dict:
    if args.local:
        from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster

        async with LocalCluster(ClusterConfig(gpus_per_node=8, odh=True, webhook=True, transport="native",
                                              env={"SET_PIPELINE_RBAC": "false",
                                                   "SET_PIPELINE_SECRET": "false"})) as cl:
            return await run(args, cl.admin)
    from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig

    cfg = RestConfig(host=args.server) if args.server else RestConfig.load(kubeconfig=args.kubeconfig)
    client = RestClient(cfg)
    try:
        return await run(args, client)
    finally:
        await client.close()


def main(argv=None) -> int:
    args = parse(argv)
    out = asyncio.run(amain(args))
    print(json.dumps(out))
    return 0 if args.operation == "delete" or out.get("ready") == out.get("count") else 1


if __name__ == "__main__":
    sys.exit(main())
