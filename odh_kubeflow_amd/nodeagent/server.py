"""The production MI355X node agent: amdgpu telemetry + pod→GPU attribution over HTTP.

Read-only by construction — it holds **no Kubernetes client**: it never creates or patches a
Node, never writes pod status and needs no RBAC.  (The kubelet stand-in that does write pod
status lives in :mod:`odh_kubeflow_amd.testing.kubelet` and is test-harness only.)

Endpoints (``--port``, default 9464, exposed as a hostPort so the culler reaches the agent
of a pod's node at ``<pod.status.hostIP>:9464``):

* ``GET /gpu/activity?pod_uid=<uid>&namespace=<ns>&name=<pod>&window=<s>`` — the GPUs
  attributed to the pod (:mod:`.attribution`) and their busy percentage (mean/max over the
  window, from the native sampler ``ops/csrc/gpu_telemetry.cpp``), device VRAM and the VRAM
  held by the pod's own processes (KFD).  ``{"attributed": false, "n": 0}`` when no GPU is
  attributed; ``n == 0`` when no sample is readable — the culler treats both as "no data",
  never as idleness;
* ``GET /gpu/activity?devices=0,3&window=<s>`` — explicit telemetry indices (debugging);
* ``GET /gpu/pods`` — the attribution tables and per-source health;
* ``GET /gpu/devices``, ``GET /healthz``, ``GET /metrics`` (Prometheus text).

With a token file (``--token-file``, :mod:`.auth`) every endpoint but ``/healthz`` needs
``Authorization: Bearer <token>`` and answers 401 otherwise.

The agent serves HTTPS (``--tls-cert-dir``: ``tls.crt`` / ``tls.key`` — this node's own key
and certificate, which the DaemonSet's enrollment containers obtain through a CSR and renew,
``nodeagent/identity.py``; reloaded when renewed), so neither the bearer token nor a busy/idle
answer — on which a GPU notebook is culled or kept — crosses the node network in cleartext,
and the culler verifies the answer comes from the agent of the pod's own node (the signer's
CA from the ``mi355x-node-agent-ca`` ConfigMap, and the certificate's name
``<spec.nodeName>.mi355x-node-agent.nodes``).  Plain HTTP only with ``--insecure`` (tests,
development).
"""

from __future__ import annotations

import logging
from typing import Optional, Sequence

log = logging.getLogger("nodeagent")

DEFAULT_PORT = 9464


def aggregate_windows(telemetry, indices: Sequence[Optional[int]], window_s: float) -> Optional[dict]:
    """Combine per-device windows: the pod is as busy as its busiest GPU."""
    best = None
    n = 0
    vram = 0.0
    for idx in indices:
        if idx is None:
            continue
        w = telemetry.window(idx, window_s)
        if w is None or w.n == 0 or w.busy_mean < 0:
            continue
        n += w.n
        if w.vram_used_mean > 0:
            vram += w.vram_used_mean
        cand = {"busy_mean": w.busy_mean, "busy_max": w.busy_max}
        if best is None or cand["busy_mean"] > best["busy_mean"]:
            best = cand
    if best is None:
        return None
    best["vram_used_mean"] = vram
    best["n"] = n
    return best


class NodeTelemetryAgent:
    def __init__(self, telemetry, attributor=None, host: str = "0.0.0.0", port: int = DEFAULT_PORT,
                 token=None, tls_cert_dir: Optional[str] = None, cert_reload_s: float = 10.0):
        self.telemetry = telemetry
        self.tls = None
        if tls_cert_dir:
            from ..utils.tlsreload import ServingCert

            self.tls = ServingCert(tls_cert_dir, "node agent serving")
        self.cert_reload_s = cert_reload_s
        self.token = token  # nodeagent.auth.TokenFile, or None: unauthenticated
        self.refused = 0
        self.attributor = attributor
        self.host = host
        self.port = port
        self._runner = None
        self.queries = 0
        self.attributed_queries = 0

    async def activity(self, pod_uid: Optional[str], namespace: Optional[str], name: Optional[str],
                       window_s: float) -> dict:
        self.queries += 1
        if self.attributor is None:
            return {"attributed": False, "n": 0}
        pg = await self.attributor.lookup(pod_uid, namespace, name)
        if pg is None:
            return {"attributed": False, "n": 0}
        self.attributed_queries += 1
        devs = self.telemetry.devices()
        out = {"attributed": True, "devices": [devs[i].pci_bdf for i in pg.devices], "sources": pg.sources,
               "pod_vram_bytes": pg.pod_vram_bytes, "n": 0}
        agg = aggregate_windows(self.telemetry, pg.devices, window_s)
        if agg is not None:
            out.update(agg)
        return out

    def metrics_text(self) -> str:
        lines = ["# HELP amdgpu_busy_percent Latest gpu_busy_percent sample per GPU.",
                 "# TYPE amdgpu_busy_percent gauge"]
        vram = ["# HELP amdgpu_vram_used_bytes Latest mem_info_vram_used sample per GPU.",
                "# TYPE amdgpu_vram_used_bytes gauge"]
        for d in self.telemetry.devices():
            s = self.telemetry.read(d.index)
            lab = f'gpu="{d.index}",bdf="{d.pci_bdf}",render_minor="{d.render_minor}"'
            if s is not None and s["busy"] >= 0:
                lines.append(f"amdgpu_busy_percent{{{lab}}} {s['busy']}")
            if s is not None and s["vram_used"] >= 0:
                vram.append(f"amdgpu_vram_used_bytes{{{lab}}} {s['vram_used']}")
        lines += vram
        lines += ["# HELP odh_node_agent_activity_queries_total Culler activity queries served.",
                  "# TYPE odh_node_agent_activity_queries_total counter",
                  f"odh_node_agent_activity_queries_total {self.queries}",
                 "# HELP odh_node_agent_unauthorized_total Requests refused for a missing or wrong token.",
                 "# TYPE odh_node_agent_unauthorized_total counter",
                 f"odh_node_agent_unauthorized_total {self.refused}"]
        if self.attributor is not None:
            # a node silently falling back from the pod-resources API to the checkpoint shows here
            lines += ["# HELP odh_node_agent_attribution_source_up Pod->GPU attribution source readable at the "
                      "last refresh (1) or unavailable / failing (0).",
                      "# TYPE odh_node_agent_attribution_source_up gauge"]
            lines += [f'odh_node_agent_attribution_source_up{{source="{k}"}} {v}'
                      for k, v in sorted(self.attributor.source_health().items())]
            lines += ["# HELP odh_node_agent_attribution_refreshes_total Attribution table refreshes.",
                      "# TYPE odh_node_agent_attribution_refreshes_total counter",
                      f"odh_node_agent_attribution_refreshes_total {self.attributor.refreshes}"]
        return "\n".join(lines) + "\n"

    async def start(self) -> "NodeTelemetryAgent":
        from aiohttp import web

        async def activity(req):
            q = req.query
            try:
                window = float(q.get("window") or 60)
                if not 0 < window <= 86400:  # also refuses nan / inf
                    raise ValueError(window)
                devs = [int(x) for x in (q.get("devices") or "").split(",") if x.strip() != ""]
            except ValueError:
                return web.json_response({"error": "bad query"}, status=400)
            if devs:
                self.queries += 1
                n = len(self.telemetry.devices())
                if any(d < 0 or d >= n for d in devs):
                    return web.json_response({"error": "no such device"}, status=400)
                return web.json_response(aggregate_windows(self.telemetry, devs, window) or {"n": 0})
            if not (q.get("pod_uid") or (q.get("namespace") and q.get("name"))):
                return web.json_response({"error": "pod_uid or namespace+name required"}, status=400)
            return web.json_response(await self.activity(q.get("pod_uid"), q.get("namespace"), q.get("name"),
                                                         window))

        async def pods(_req):
            if self.attributor is None:
                return web.json_response({})
            return web.json_response(await self.attributor.all_pods())

        async def devices(_req):
            return web.json_response([{**d.__dict__, "pci_bdf": d.pci_bdf} for d in self.telemetry.devices()])

        async def healthz(_req):
            return web.Response(text="ok")

        async def metrics(_req):
            return web.Response(text=self.metrics_text(), content_type="text/plain")

        @web.middleware
        async def auth(req, handler):
            if self.token is not None and req.path != "/healthz" and \
                    not self.token.authorizes(req.headers.get("Authorization")):
                self.refused += 1
                return web.json_response({"error": "unauthorized"}, status=401,
                                         headers={"WWW-Authenticate": "Bearer"})
            return await handler(req)

        app = web.Application(middlewares=[auth])
        app.router.add_get("/gpu/activity", activity)
        app.router.add_get("/gpu/pods", pods)
        app.router.add_get("/gpu/devices", devices)
        app.router.add_get("/healthz", healthz)
        app.router.add_get("/metrics", metrics)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        ctx = self.tls.context() if self.tls is not None else None
        site = web.TCPSite(self._runner, self.host, self.port, ssl_context=ctx)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        if self.tls is not None:
            self.tls.watch(self.cert_reload_s)
        return self

    @property
    def scheme(self) -> str:
        return "https" if self.tls is not None else "http"

    async def stop(self) -> None:
        if self.tls is not None:
            self.tls.stop()
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None
