#!/usr/bin/env python3
"""BASELINE config #4: the odh webhook path across 8 notebooks (auth sidecar + routing).

Every round creates 8 notebooks at once with ``notebooks.opendatahub.io/inject-auth``
against the native C++ apiserver, which calls the odh mutating webhook over HTTPS
(MutatingWebhookConfiguration with a self-signed caBundle, as the reference's kind CI
wires it).  The kf controller runs with ``USE_ISTIO=true`` (VirtualService per notebook)
and the odh controller creates the kube-rbac-proxy resources and the HTTPRoute.
Measured per notebook: the client-observed create latency (admission included), the
webhook's own handling time, and create → VirtualService / HTTPRoute / Ready.
(The north star says "OAuth-proxy"; the reference injects kube-rbac-proxy — SURVEY §0.4.)

    python tools/bench_webhook.py [--rounds 20]
"""
import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster  # noqa: E402
from odh_kubeflow_amd.models import kinds  # noqa: E402
from odh_kubeflow_amd.models.notebook import notebook  # noqa: E402
from odh_kubeflow_amd.webhook import notebook_webhook  # noqa: E402

N = 8
AUTH = {"notebooks.opendatahub.io/inject-auth": "true"}


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))], 3) if xs else None


async def run(args) -> dict:
    handle_ms = []
    orig = notebook_webhook.NotebookWebhook.handle

    async def timed(self, review):
        t = time.perf_counter()
        try:
            return await orig(self, review)
        finally:
            handle_ms.append((time.perf_counter() - t) * 1e3)
    notebook_webhook.NotebookWebhook.handle = timed

    env = {"USE_ISTIO": "true", "SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
    cfg = ClusterConfig(odh=True, webhook=True, transport=args.transport, env=env)
    create_ms, vs_ms, route_ms, ready_ms = [], [], [], []
    try:
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("wh")

            def vs_of(nm):
                return cl.store.peek(kinds.VIRTUAL_SERVICE, f"notebook-wh-{nm}", "wh")

            def route_of(nm):
                return cl.store.peek(kinds.HTTP_ROUTE, f"nb-wh-{nm}", cfg.controller_namespace)

            for rnd in range(args.warmup + args.rounds):
                names = [f"r{rnd}-nb{i}" for i in range(N)]
                t0 = {}
                done = {k: {} for k in ("create", "vs", "route", "ready")}

                async def create(nm):
                    t0[nm] = time.perf_counter()
                    out = await cl.admin.create(notebook(nm, "wh", gpus=1, annotations=AUTH))
                    done["create"][nm] = time.perf_counter()
                    containers = [c["name"] for c in out["spec"]["template"]["spec"]["containers"]]
                    assert containers == [nm, "kube-rbac-proxy"], containers  # mutated by admission
                if rnd == args.warmup:
                    handle_ms.clear()
                await asyncio.gather(*(create(nm) for nm in names))

                def poll():
                    now = time.perf_counter()
                    for nm in names:
                        if nm not in done["vs"] and vs_of(nm) is not None:
                            done["vs"][nm] = now
                        if nm not in done["route"] and route_of(nm) is not None:
                            done["route"][nm] = now
                        if nm not in done["ready"] and cl.notebook_ready(nm, "wh"):
                            done["ready"][nm] = now
                    return all(len(done[k]) == N for k in ("vs", "route", "ready"))
                if not await cl.wait_for(poll, 60, 0.0005):
                    raise RuntimeError({k: sorted(set(names) - set(v)) for k, v in done.items()})
                if rnd >= args.warmup:
                    for nm in names:
                        create_ms.append((done["create"][nm] - t0[nm]) * 1e3)
                        vs_ms.append((done["vs"][nm] - t0[nm]) * 1e3)
                        route_ms.append((done["route"][nm] - t0[nm]) * 1e3)
                        ready_ms.append((done["ready"][nm] - t0[nm]) * 1e3)
                await asyncio.gather(*(cl.admin.delete(kinds.NOTEBOOK, nm, "wh") for nm in names))
                if not await cl.wait_for(lambda: all(cl.store.peek(kinds.NOTEBOOK, nm, "wh") is None
                                                     for nm in names), 60):
                    raise RuntimeError("teardown did not finish")
            calls = cl.webhook.requests
    finally:
        notebook_webhook.NotebookWebhook.handle = orig
    return {"metric": "odh webhook path across 8 notebooks (kube-rbac-proxy sidecar + Istio VirtualService + "
                      "HTTPRoute)", "n_notebooks": N, "rounds": args.rounds,
            "transport": f"{args.transport} apiserver" + (", HTTPS admission webhook" if args.transport != "inprocess"
                                                          else ", in-process admission"),
            "create_admitted_ms_p50": pct(create_ms, 0.5), "create_admitted_ms_p95": pct(create_ms, 0.95),
            "webhook_handle_ms_p50": pct(handle_ms, 0.5), "webhook_handle_ms_p95": pct(handle_ms, 0.95),
            "webhook_calls_per_notebook": round(calls / (N * (args.rounds + args.warmup)), 2),
            "virtualservice_ms_p50": pct(vs_ms, 0.5), "httproute_ms_p50": pct(route_ms, 0.5),
            "ready_ms_p50": pct(ready_ms, 0.5), "ready_ms_p95": pct(ready_ms, 0.95),
            "mean_ready_ms": round(statistics.fmean(ready_ms), 3)}


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=20)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--transport", choices=("native", "http", "inprocess"), default="native")
    args = p.parse_args(argv)
    print(json.dumps(asyncio.run(run(args))), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
