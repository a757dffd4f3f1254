"""Idle-notebook culler (reference ``kf/controllers/culling_controller.go``), with an
MI355X GPU-busy activity signal.

Annotation protocol — identical to the reference so existing tooling keeps working:

* ``notebooks.kubeflow.org/last-activity`` — RFC3339 of the last observed activity;
* ``notebooks.kubeflow.org/last_activity_check_timestamp`` — RFC3339 of the last check;
* ``kubeflow-resource-stopped`` = RFC3339 when culled (the kf reconciler then scales the
  StatefulSet to 0; removing the annotation resumes the notebook).

Per reconcile (:86-203): stopped → strip the two activity annotations; pod ``<nb>-0``
missing → strip them; initialise them; skip until ``IDLENESS_CHECK_PERIOD`` has passed
since the last check; sample activity; in one ``RetryOnConflict`` update set
last-activity, the check timestamp and — if idle for longer than ``CULL_IDLE_TIME`` —
the stop annotation; ``RequeueAfter(IDLENESS_CHECK_PERIOD)``.

Activity sources (``CULLING_ACTIVITY_SOURCE``):

* ``jupyter`` (default, the reference): ``GET .../api/kernels`` and ``.../api/terminals``
  (10 s timeout each); any non-idle kernel means "active now", otherwise the newest
  kernel/terminal ``last_activity`` is taken if it is newer than the annotation;
* ``amdgpu``: for a pod that requests ``amd.com/gpu``, the node agent of the pod's node
  (``http://<pod.status.hostIP>:CULLING_GPU_AGENT_PORT``, default 9464; ``nodeagent/``)
  is asked by pod UID which GPUs the kubelet gave the pod (pod-resources API /
  device-plugin checkpoint / KFD per-process sysfs — no pod annotation involved) and how
  busy they were over the last check period.  A mean busy percentage at or above
  ``CULLING_GPU_BUSY_THRESHOLD`` (default 5) means "active now".  Averaging over the whole
  window is the hysteresis: a single spike does not keep a notebook alive and a single
  idle sample does not cull it;
* ``combined``: active if either signal says so.

Resident VRAM is **not** activity by default.  A notebook that holds 200 GB of HBM3E at
0 % busy for ``CULL_IDLE_TIME`` (24 h by default) is exactly the waste culling exists to
reclaim: the memory is stranded for every other tenant of the GPU, and the state it holds
is what the user's PVC-backed home directory and checkpoints are for.  Interactive use
that keeps a model resident (occasional generation calls) shows up as busy samples and,
in ``combined`` mode, as Jupyter kernel activity.  Clusters that want the other policy set
``CULLING_GPU_VRAM_ACTIVE_BYTES`` (e.g. ``1e9``): the pod then counts as active while its
own processes hold at least that much VRAM (KFD per-process accounting, so a co-tenant's
memory on a shared GPU never keeps it alive).

Missing telemetry is never read as idleness: with no GPU samples the Jupyter signal is
used, and with neither the last-activity annotation is simply left alone (as the
reference does for HTTP errors, :258-270).  A Pending pod (image pull, init containers)
is not checked while it is plausibly still starting — younger than ``CULL_IDLE_TIME`` plus
``CULL_STARTUP_ALLOWANCE`` (minutes, default 10) and not stuck — and the idle clock of a
new pod starts no earlier than its first Ready transition: start-up time is not idle time.
A pod that cannot start (an init container such as ``amd-gpu-probe`` in back-off, an image
pull failing) or that outlived that bound holds its ``amd.com/gpu`` devices for nothing: it
is checked like any other pod, its idle clock running from the pod's creation, so a bad
GPU or a typo'd image never pins an MI355X for good.

Fixes over the reference: the two culling metrics are exported; the configuration is
an object (no package globals); sub-minute periods are available through
``IDLENESS_CHECK_PERIOD_SECONDS`` / ``CULL_IDLE_TIME_SECONDS`` for tests and benchmarks.
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
from dataclasses import dataclass
from typing import Any, Callable, Mapping, Optional, Sequence

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_not_found
from ..models.notebook import (LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, STOP_ANNOTATION,
                               gpu_request)
from ..nodeagent.identity import IDENTITY_DOMAIN
from ..nodeagent.identity import server_name as agent_server_name
from ..runtime.controller import Request, Result
from ..runtime.retry import retry_on_conflict
from ..utils.timeutil import now, parse_rfc3339, rfc3339

log = logging.getLogger("controllers.Culler")

DEFAULT_CULL_IDLE_TIME = "1440"
DEFAULT_IDLENESS_CHECK_PERIOD = "1"
DEFAULT_CLUSTER_DOMAIN = "cluster.local"
KERNEL_IDLE, KERNEL_BUSY, KERNEL_STARTING = "idle", "busy", "starting"
_ABSENT = object()


def _phase_of(namespace: str, name: str) -> float:
    """A notebook's fixed fraction of the check period.  blake2b, not crc32: CRC is linear, and
    the sequential names notebooks usually get (``nb-0`` … ``nb-999``) cluster under it — the
    fullest 10 s slot of a 60 s period held up to 1.7x the emptiest at R=1000, against 1.3x here."""
    import hashlib

    h = hashlib.blake2b(f"{namespace}/{name}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "big") / 2.0 ** 64


def env_default(env: Mapping[str, str], key: str, default: str) -> str:
    v = env.get(key)
    return v if v else default


@dataclass
class CullerConfig:
    cull_idle_time_s: float = 1440 * 60.0
    check_period_s: float = 60.0
    enable_culling: bool = False
    cluster_domain: str = DEFAULT_CLUSTER_DOMAIN
    dev: bool = False
    dev_proxy_url: str = "http://localhost:8001"  # DEV mode: the kubectl proxy the culler goes through
    activity_source: str = "jupyter"
    gpu_busy_threshold: float = 5.0
    gpu_agent_port: int = 9464
    gpu_agent_token_file: str = ""  # bearer token for the node agent (nodeagent/auth.py); "" = none
    gpu_agent_ca_file: str = ""  # the node agents' CA (HTTPS); "" with gpu_agent_insecure false: no GPU data
    gpu_agent_identity_domain: str = ""  # agent certificates name <node>.<this> (nodeagent/identity.py)
    gpu_agent_insecure: bool = False  # plain HTTP to the agents (tests, development)
    gpu_vram_active_bytes: float = 0.0  # 0: resident VRAM is not activity (see module docstring)
    http_timeout_s: float = 10.0
    startup_allowance_s: float = 600.0  # a Pending pod younger than cull_idle_time + this is not checked
    # write last_activity_check_timestamp on every k-th check of a notebook whose check changed
    # nothing else (1: every check, as the reference does) — see CullingReconciler.reconcile
    check_stamp_every: int = 1

    @classmethod
    def from_env(cls, env: Mapping[str, str] = os.environ) -> "CullerConfig":
        """``initGlobalVars`` (:525-558): a bad CULL_IDLE_TIME falls back to the default,
        a bad IDLENESS_CHECK_PERIOD is an error."""
        c = cls()
        c.dev = env_default(env, "DEV", "false") == "true"
        c.dev_proxy_url = env_default(env, "CULLER_DEV_PROXY_URL", c.dev_proxy_url).rstrip("/")
        raw = env_default(env, "CULL_IDLE_TIME", DEFAULT_CULL_IDLE_TIME)
        try:
            c.cull_idle_time_s = int(raw) * 60.0
        except ValueError:
            log.info("CULL_IDLE_TIME should be Int. Got %s instead. Using default value.", raw)
            c.cull_idle_time_s = int(DEFAULT_CULL_IDLE_TIME) * 60.0
        c.enable_culling = env_default(env, "ENABLE_CULLING", "false") == "true"
        c.cluster_domain = env_default(env, "CLUSTER_DOMAIN", DEFAULT_CLUSTER_DOMAIN)
        c.check_period_s = int(env_default(env, "IDLENESS_CHECK_PERIOD", DEFAULT_IDLENESS_CHECK_PERIOD)) * 60.0
        if env.get("IDLENESS_CHECK_PERIOD_SECONDS"):
            c.check_period_s = float(env["IDLENESS_CHECK_PERIOD_SECONDS"])
        if env.get("CULL_IDLE_TIME_SECONDS"):
            c.cull_idle_time_s = float(env["CULL_IDLE_TIME_SECONDS"])
        c.activity_source = env_default(env, "CULLING_ACTIVITY_SOURCE", "jupyter").strip().lower()
        if c.activity_source not in ("jupyter", "amdgpu", "combined"):
            raise ValueError(f"CULLING_ACTIVITY_SOURCE must be jupyter|amdgpu|combined, got {c.activity_source}")
        c.gpu_busy_threshold = float(env_default(env, "CULLING_GPU_BUSY_THRESHOLD", "5"))
        c.gpu_agent_port = int(env_default(env, "CULLING_GPU_AGENT_PORT", "9464"))
        c.gpu_agent_token_file = env.get("CULLING_GPU_AGENT_TOKEN_FILE", "")
        c.gpu_agent_ca_file = env.get("CULLING_GPU_AGENT_CA_FILE", "")
        c.gpu_agent_identity_domain = env_default(env, "CULLING_GPU_AGENT_IDENTITY_DOMAIN", IDENTITY_DOMAIN)
        c.gpu_agent_insecure = env_default(env, "CULLING_GPU_AGENT_INSECURE", "false").strip().lower() == "true"
        c.gpu_vram_active_bytes = float(env_default(env, "CULLING_GPU_VRAM_ACTIVE_BYTES", "0"))
        c.startup_allowance_s = float(env_default(env, "CULL_STARTUP_ALLOWANCE", "10")) * 60.0
        if env.get("CULL_STARTUP_ALLOWANCE_SECONDS"):
            c.startup_allowance_s = float(env["CULL_STARTUP_ALLOWANCE_SECONDS"])
        raw = env_default(env, "CULL_CHECK_STAMP_EVERY", "1")
        try:
            c.check_stamp_every = max(1, int(raw))
        except ValueError:
            raise ValueError(f"CULL_CHECK_STAMP_EVERY must be a positive integer, got {raw!r}")
        return c


# ------------------------------------------------------------------ pure helpers (unit-tested like the reference)


def stop_annotation_is_set(nb: dict) -> bool:
    return STOP_ANNOTATION in m.annotations(nb)


def annotations_exist(nb: dict) -> bool:
    a = m.annotations(nb)
    return LAST_ACTIVITY_ANNOTATION in a and LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION in a


def initialize_annotations(nb: dict, last_activity: Optional[str] = None) -> None:
    t = rfc3339()
    a = m.ensure_annotations(nb)
    a[LAST_ACTIVITY_ANNOTATION] = last_activity or t
    a[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION] = t


def remove_annotations(nb: dict) -> None:
    a = (nb.get("metadata") or {}).get("annotations")
    if a:
        a.pop(LAST_ACTIVITY_ANNOTATION, None)
        a.pop(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION, None)


def culling_check_period_has_passed(nb: dict, period_s: float) -> bool:
    raw = m.annotations(nb).get(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION)
    if raw is None:
        return False
    t = parse_rfc3339(raw)
    if t is None:
        t = -62135596800.0  # Go zero time: an unparsable stamp is "long ago"
    return t + period_s < now()


def notebook_is_idle(nb: dict, idle_s: float) -> bool:
    if stop_annotation_is_set(nb):
        return False
    t = parse_rfc3339(m.annotations(nb).get(LAST_ACTIVITY_ANNOTATION))
    if t is None:
        return False
    return now() > t + idle_s


def all_kernels_are_idle(kernels: Sequence[dict]) -> bool:
    return all(k.get("execution_state") == KERNEL_IDLE for k in kernels)


def most_recent_time(times: Sequence[str]) -> str:
    best = None
    for s in times:
        t = parse_rfc3339(s)
        if t is None:
            return ""
        if best is None or t > best:
            best = t
    return rfc3339(best) if best is not None else ""


def annotation_not_after(nb: dict, resource_time: str) -> bool:
    """``compareAnnotationTimeToResource``: True unless the annotation is newer."""
    a = parse_rfc3339(m.annotations(nb).get(LAST_ACTIVITY_ANNOTATION))
    t = parse_rfc3339(resource_time)
    if a is None or t is None:
        return False
    return not a > t


def update_from_kernels(nb: dict, kernels: Optional[Sequence[dict]]) -> bool:
    if not kernels:
        return False
    if not all_kernels_are_idle(kernels):
        m.ensure_annotations(nb)[LAST_ACTIVITY_ANNOTATION] = rfc3339()
        return False
    t = most_recent_time([k.get("last_activity", "") for k in kernels])
    if not t or not annotation_not_after(nb, t):
        return False
    m.ensure_annotations(nb)[LAST_ACTIVITY_ANNOTATION] = t
    return True


def update_from_terminals(nb: dict, terminals: Optional[Sequence[dict]]) -> bool:
    if not terminals:
        return False
    t = most_recent_time([x.get("last_activity", "") for x in terminals])
    if not t or not annotation_not_after(nb, t):
        return False
    m.ensure_annotations(nb)[LAST_ACTIVITY_ANNOTATION] = t
    return True


def update_check_timestamp(nb: dict) -> None:
    m.ensure_annotations(nb)[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION] = rfc3339()


def set_stop_annotation(nb: dict, metrics=None) -> None:
    t = now()
    m.ensure_annotations(nb)[STOP_ANNOTATION] = rfc3339(t)
    if metrics is not None:
        metrics.notebook_culling_count.labels(m.namespace(nb), m.name(nb)).inc()
        metrics.notebook_culling_timestamp.labels(m.namespace(nb), m.name(nb)).set(int(t))


def pod_is_starting(pod: dict) -> bool:
    """Pending: scheduling, image pull, init containers (``odh-gpu-probe``).  Nothing of the
    notebook runs yet, so nothing of it can be idle — for a while (:func:`pod_start_stuck`,
    :meth:`CullingReconciler.reconcile`)."""
    return (pod.get("status") or {}).get("phase") == "Pending"


# container waiting reasons the kubelet reports for a start that will not succeed by itself
STUCK_WAITING_REASONS = frozenset({
    "CrashLoopBackOff", "ImagePullBackOff", "ErrImagePull", "ErrImageNeverPull", "InvalidImageName",
    "CreateContainerConfigError", "CreateContainerError", "RunContainerError"})


def pod_start_stuck(pod: dict) -> bool:
    """The pod is Pending because something failed, not because it is still working: an init
    container exited non-zero (the kubelet restarts it with back-off — ``amd-gpu-probe`` on a bad
    GPU) or any container waits on a failing image pull / config."""
    st = pod.get("status") or {}
    for cs in st.get("initContainerStatuses") or []:
        state = cs.get("state") or {}
        if (state.get("waiting") or {}).get("reason") in STUCK_WAITING_REASONS:
            return True
        term = state.get("terminated") or (cs.get("lastState") or {}).get("terminated") or {}
        if term.get("exitCode") not in (None, 0):
            return True
    for cs in st.get("containerStatuses") or []:
        if ((cs.get("state") or {}).get("waiting") or {}).get("reason") in STUCK_WAITING_REASONS:
            return True
    return False


def pod_created_at(pod: dict) -> Optional[float]:
    return parse_rfc3339((pod.get("metadata") or {}).get("creationTimestamp"))


def pod_ready_since(pod: dict) -> Optional[float]:
    """When the pod last became Ready (its server came up), or None."""
    for c in ((pod.get("status") or {}).get("conditions") or []):
        if c.get("type") == "Ready" and c.get("status") == "True":
            return parse_rfc3339(c.get("lastTransitionTime"))
    return None


def update_from_pod_start(nb: dict, pod: dict) -> None:
    """The idle clock of a new pod starts no earlier than its server: a last-activity stamp
    older than the pod itself (left by an earlier pod of the notebook — a restart, a resume)
    is moved up to the pod's Ready transition.  Once per pod: after that the stamp is newer
    than the pod's creation, so a flapping readiness probe or a container restart (each a new
    Ready transition) never resets the clock again."""
    t = pod_ready_since(pod)
    a = parse_rfc3339(m.annotations(nb).get(LAST_ACTIVITY_ANNOTATION))
    born = pod_created_at(pod)
    if t is None or a is None or t <= a:
        return
    if born is not None and a >= born:
        return  # this pod's clock has started already
    m.ensure_annotations(nb)[LAST_ACTIVITY_ANNOTATION] = rfc3339(t)


def update_from_pod_creation(nb: dict, pod: dict) -> None:
    """A pod that never got going (stuck or over-long start): idle since it was created."""
    born = pod_created_at(pod)
    a = parse_rfc3339(m.annotations(nb).get(LAST_ACTIVITY_ANNOTATION))
    if born is not None and (a is None or a < born):
        m.ensure_annotations(nb)[LAST_ACTIVITY_ANNOTATION] = rfc3339(born)


def pod_requests_gpu(pod: Optional[dict]) -> bool:
    return gpu_request((pod or {}).get("spec") or {}) > 0


def gpu_says_active(data: dict, cfg: CullerConfig) -> bool:
    if data.get("busy_mean", -1) >= cfg.gpu_busy_threshold:
        return True
    vram = data.get("pod_vram_bytes")
    return cfg.gpu_vram_active_bytes > 0 and vram is not None and vram >= cfg.gpu_vram_active_bytes


# ------------------------------------------------------------------ activity sources


class JupyterActivity:
    """``getNotebookApiKernels`` / ``getNotebookApiTerminals`` over HTTP (10 s timeout).

    ``url_for(nb_name, namespace, resource, pod)`` may be overridden; by default it is the
    in-cluster Service URL, or the ``kubectl proxy`` URL in ``DEV`` mode (:243-273; the proxy's
    address is ``CULLER_DEV_PROXY_URL``, default ``http://localhost:8001`` as in the reference).  With
    ``use_pod_endpoint`` the node agent's ``amd.com/notebook-endpoint`` pod annotation is
    used (the in-process runtime serves the Jupyter API on an ephemeral port).
    """

    # plain-HTTP Jupyter endpoints go through lean keep-alive pools (runtime/http1.py: ~4x less
    # CPU per request than aiohttp, which matters when R notebooks are checked every period);
    # one pool per endpoint host, the least recently used dropped beyond MAX_POOLS
    MAX_POOLS = 256
    POOL_SIZE = 4

    def __init__(self, cfg: CullerConfig, url_for: Optional[Callable[..., str]] = None,
                 use_pod_endpoint: bool = False):
        from collections import OrderedDict

        self.cfg = cfg
        self.url_for = url_for or self.default_url
        self.use_pod_endpoint = use_pod_endpoint
        self._session = None
        self._pools: "OrderedDict[str, Any]" = OrderedDict()
        self.requests = 0

    def default_url(self, nm: str, ns: str, resource: str, pod: Optional[dict] = None) -> str:
        if self.use_pod_endpoint and pod is not None:
            ep = m.annotations(pod).get("amd.com/notebook-endpoint")
            if ep:
                return f"http://{ep}/notebook/{ns}/{nm}/api/{resource}"
        if self.cfg.dev:
            return (f"{self.cfg.dev_proxy_url}/api/v1/namespaces/{ns}/services/{nm}:http-{nm}/proxy/notebook/"
                    f"{ns}/{nm}/api/{resource}")
        return f"http://{nm}.{ns}.svc.{self.cfg.cluster_domain}/notebook/{ns}/{nm}/api/{resource}"

    def _pool(self, url: str):
        from urllib.parse import urlsplit

        from ..runtime.http1 import Http1Pool

        u = urlsplit(url)
        key = u.netloc
        pool = self._pools.get(key)
        if pool is None:
            pool = self._pools[key] = Http1Pool(f"http://{key}", size=self.POOL_SIZE)
            while len(self._pools) > self.MAX_POOLS:
                _k, old = self._pools.popitem(last=False)
                asyncio.ensure_future(old.close())
        else:
            self._pools.move_to_end(key)
        target = u.path + (f"?{u.query}" if u.query else "")
        return pool, target

    async def _get(self, url: str) -> Optional[Any]:
        self.requests += 1
        try:
            if url.startswith("http://"):
                pool, target = self._pool(url)
                status, body = await asyncio.wait_for(pool.request("GET", target), self.cfg.http_timeout_s)
            else:
                import aiohttp

                if self._session is None or self._session.closed:
                    self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.cfg.http_timeout_s))
                async with self._session.get(url) as resp:
                    status, body = resp.status, await resp.read()
            if status != 200:
                log.info("Warning: GET to %s: %d", url, status)
                return None
            return json.loads(body)
        except (asyncio.TimeoutError, OSError, ValueError, Exception) as e:  # noqa: B014 - any failure is "no data"
            log.debug("GET %s failed: %r", url, e)
            return None

    async def sample(self, nb: dict, pod: Optional[dict]):
        nm, ns = m.name(nb), m.namespace(nb)
        kernels, terminals = await asyncio.gather(self._get(self.url_for(nm, ns, "kernels", pod)),
                                                  self._get(self.url_for(nm, ns, "terminals", pod)))
        return (kernels if isinstance(kernels, list) else None), (terminals if isinstance(terminals, list) else None)

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
        for pool in self._pools.values():
            await pool.close()
        self._pools.clear()


class GpuActivity:
    """Base class: how busy the GPUs attributed to ``pod`` were over the last ``window_s``.

    Returns a dict with ``busy_mean`` / ``busy_max`` (percent), ``vram_used_mean`` (device)
    and ``pod_vram_bytes`` (the pod's own processes, KFD; ``None`` if unknown), or ``None``
    when nothing could be read — never interpreted as idle.
    """

    async def busy(self, pod: dict, window_s: float) -> Optional[dict]:
        raise NotImplementedError

    async def close(self) -> None:
        return None


def _usable(data: Optional[dict]) -> Optional[dict]:
    return data if data and data.get("n", 0) > 0 and data.get("busy_mean", -1) >= 0 else None


class LocalTelemetryActivity(GpuActivity):
    """In-process telemetry + attribution (a single-node setup running the culler next to the
    GPUs): :class:`~odh_kubeflow_amd.nodeagent.attribution.Attributor` resolves the pod."""

    def __init__(self, telemetry, attributor):
        self.telemetry = telemetry
        self.attributor = attributor

    async def busy(self, pod, window_s):
        from ..nodeagent.server import aggregate_windows

        pg = await self.attributor.lookup(m.uid(pod), m.namespace(pod), m.name(pod))
        if pg is None:
            return None
        agg = aggregate_windows(self.telemetry, pg.devices, window_s)
        if agg is not None:
            agg["pod_vram_bytes"] = pg.pod_vram_bytes
        return _usable(agg)


class NodeAgentActivity(GpuActivity):
    """Asks the node agent on the pod's node (``nodeagent/server.py``) — the telemetry and the
    kubelet's allocation records live next to the GPUs, not in the controller.

    The agent is a DaemonSet with a hostPort, so it is at ``<pod.status.hostIP>:<port>``;
    ``endpoint_for(pod) -> "host:port"`` overrides that (test harnesses whose fake nodes
    share one IP).

    Over HTTPS (``ca_file``): the agent's certificate must chain to that CA and name the pod's
    own node — ``<pod.spec.nodeName>.<identity_domain>``, issued to that node's agent alone
    (``nodeagent/identity.py``: a key per node, the node bound by the agent pod's token) — so
    the bearer token and the busy/idle answers never cross the node network in cleartext, and
    neither a spoofed agent nor another node's agent can cull or pin a notebook.  Without a CA
    the agents are not asked at all (no GPU data: the Jupyter signal decides) unless
    ``insecure``.
    """

    def __init__(self, port: int = 9464, timeout_s: float = 2.0,
                 endpoint_for: Optional[Callable[[dict], Optional[str]]] = None, token_file: str = "",
                 ca_file: str = "", identity_domain: str = "", insecure: bool = False):
        self.port = port
        self.token = None
        if token_file:
            from ..nodeagent.auth import TokenFile

            self.token = TokenFile(token_file)
        self.ssl = None
        if ca_file:
            from ..utils.tlsreload import client_context

            self.ssl = client_context(ca_file)
        self.identity_domain = identity_domain or IDENTITY_DOMAIN
        self.insecure = insecure
        self.timeout_s = timeout_s
        self.endpoint_for = endpoint_for or self.default_endpoint
        self._session = None
        self.requests = 0
        self.refused_cleartext = 0
        self.no_node = 0  # pods without spec.nodeName: no agent identity to verify

    def default_endpoint(self, pod: dict) -> Optional[str]:
        """``<hostIP>:<port>`` of the pod's node agent; IPv6 literals are bracketed
        (``[fd00::5]:9464``), as an URL authority needs them on v6 / dual-stack-v6 clusters."""
        host = (pod.get("status") or {}).get("hostIP")
        if not host:
            return None
        import ipaddress

        try:
            if ipaddress.ip_address(host).version == 6:
                host = f"[{host}]"
        except ValueError:
            pass  # a hostname: used as is
        return f"{host}:{self.port}"

    async def busy(self, pod, window_s):
        import urllib.parse

        import aiohttp

        ep = self.endpoint_for(pod)
        if not ep:
            return None
        if self.ssl is None and not self.insecure:
            if not self.refused_cleartext:
                log.warning("no node-agent CA (CULLING_GPU_AGENT_CA_FILE): GPU activity is not queried over plain "
                            "HTTP; culling falls back to the Jupyter signal")
            self.refused_cleartext += 1
            return None
        node = (pod.get("spec") or {}).get("nodeName")
        if self.ssl is not None and not node:
            self.no_node += 1
            return None
        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout_s))
        q = urllib.parse.urlencode({"pod_uid": m.uid(pod), "namespace": m.namespace(pod), "name": m.name(pod),
                                    "window": window_s})
        self.requests += 1
        try:
            headers = self.token.header() if self.token is not None else None
            scheme = "https" if self.ssl is not None else "http"
            tls = ({"ssl": self.ssl, "server_hostname": agent_server_name(node, self.identity_domain)}
                   if self.ssl is not None else {})
            async with self._session.get(f"{scheme}://{ep}/gpu/activity?{q}", headers=headers, **tls) as resp:
                if resp.status != 200:
                    return None
                data = await resp.json()
        except Exception:  # agent down / unreachable: no data, never idleness
            return None
        return _usable(data)

    async def close(self):
        if self._session is not None:
            await self._session.close()


# ------------------------------------------------------------------ reconciler


class CullingReconciler:
    NAME = "Culler"

    def __init__(self, client, reader, metrics=None, env: Optional[Mapping[str, str]] = None, activity=None,
                 config: Optional[CullerConfig] = None, jupyter: Optional[JupyterActivity] = None):
        self.client = client
        self.reader = reader
        self.metrics = metrics
        self.env = env if env is not None else os.environ
        self.cfg = config or CullerConfig.from_env(self.env)
        self.gpu: Optional[GpuActivity] = activity
        if self.gpu is None and self.cfg.activity_source in ("amdgpu", "combined"):
            self.gpu = NodeAgentActivity(port=self.cfg.gpu_agent_port, token_file=self.cfg.gpu_agent_token_file,
                                         ca_file=self.cfg.gpu_agent_ca_file,
                                         identity_domain=self.cfg.gpu_agent_identity_domain,
                                         insecure=self.cfg.gpu_agent_insecure)
        self.jupyter = jupyter or JupyterActivity(self.cfg, use_pod_endpoint=self.env.get(
            "CULLER_USE_POD_ENDPOINT", "false") == "true")
        self.culled = 0
        self.checks = 0
        self.stamps_skipped = 0  # checks whose only change, the check stamp, was not written
        # (namespace, name) -> when this process last checked the notebook (whole seconds): the
        # schedule when the stored stamp is older (CULL_CHECK_STAMP_EVERY > 1)
        self._checked: dict = {}
        from collections import deque
        self.recent = deque(maxlen=64)  # (time, notebook, gpu_active, kernels, terminals) — debugging aid
        # per cull: which signal decided it ("amdgpu" = an attributed GPU sample said idle;
        # "jupyter" = the kernel/terminal activity, also when the GPU had no sample)
        self.cull_log = deque(maxlen=1024)

    def _cached(self, kind, name: str, namespace: str) -> Optional[dict]:
        """The informer's copy, zero-copy and read-only (None when this process's cache does not
        hold ``namespace``: the caller reads through the client instead)."""
        covers = getattr(self.reader, "covers", None)
        if covers is not None and not covers(kind, namespace):
            return None
        return self.reader.get(kind, name, namespace)

    async def _read(self, kind, name: str, namespace: str) -> Optional[dict]:
        covers = getattr(self.reader, "covers", None)
        if covers is not None and covers(kind, namespace):
            return self.reader.get(kind, name, namespace)
        return await self.client.get_or_none(kind, name, namespace)

    # the annotations only the culler writes (see _update)
    OWN_ANNOTATIONS = frozenset((LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION))

    async def _update(self, req: Request, mutate: Callable[[dict], None], precondition: bool = True) -> None:
        """``RetryOnConflict{Get; mutate; Update}`` (:106-112, :171-196), written as a merge patch
        of the annotations the culler changed, preconditioned on the resourceVersion it read —
        the same optimistic concurrency as the reference's Update, without re-sending (and the
        apiserver re-validating) the whole pod template on every check of every notebook.  A
        mutation that changes nothing writes nothing (kube-apiserver skips no-op updates too),
        and a notebook being deleted is not written at all.

        ``precondition=False`` (the first annotations of a notebook, written the moment its pod
        is up): a patch that sets only the culler's own activity annotations, which nobody else
        writes, goes without the precondition.  Preconditioned, it conflicted with the notebook
        controller's status write of the same moment on every notebook, and its retry then
        landed on notebooks being deleted.  The periodic checks keep it: the precondition is
        also what lets the client recognise the write's watch echo as its own."""
        from ..runtime.client import LIVE_READS

        async def fn():
            cur = None if LIVE_READS.get() else self._cached(kinds.NOTEBOOK_V1BETA1, req.name, req.namespace)
            if cur is None:
                cur = await self.client.get(kinds.NOTEBOOK_V1BETA1, req.name, req.namespace)
            if m.is_deleting(cur):
                return
            md = cur.get("metadata") or {}
            before = md.get("annotations") or {}
            view = {"metadata": {"name": md.get("name"), "namespace": md.get("namespace"),
                                 "annotations": dict(before)}}
            mutate(view)
            after = view["metadata"].get("annotations") or {}
            diff = {k: v for k, v in after.items() if before.get(k, _ABSENT) != v}
            diff.update({k: None for k in before if k not in after})
            if not diff:
                return
            meta = {"annotations": diff}
            if precondition or not all(k in self.OWN_ANNOTATIONS and v is not None for k, v in diff.items()):
                meta["resourceVersion"] = md.get("resourceVersion")
            try:
                await self.client.patch(kinds.NOTEBOOK_V1BETA1, {"metadata": meta}, "merge",
                                        name=req.name, namespace=req.namespace)
            except ApiError as e:
                if not is_not_found(e):  # deleted meanwhile: nothing to annotate
                    raise

        await retry_on_conflict(fn)

    async def reconcile(self, req: Request) -> Result:
        nb = await self._read(kinds.NOTEBOOK_V1BETA1, req.name, req.namespace)
        if nb is None or m.is_deleting(nb):
            self._checked.pop((req.namespace, req.name), None)
            return Result()
        if stop_annotation_is_set(nb):
            if annotations_exist(nb) or any(k in m.annotations(nb) for k in (
                    LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION)):
                await self._update(req, remove_annotations)
            return Result()
        pod = await self._read(kinds.POD, m.name(nb) + "-0", req.namespace)
        if pod is None:
            if any(k in m.annotations(nb) for k in (LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION)):
                await self._update(req, remove_annotations)
            # the reference waits for the next Notebook event (its unconditional status write
            # follows the pod's creation); status writes are gated on change here, and a pod
            # that never leaves Pending changes no status, so look again after a period
            return Result(requeue_after=self.cfg.check_period_s)
        starting = pod_is_starting(pod)
        if starting:
            # Unlike the reference (:86-203), the idle clock waits for the server: an image
            # pull or init container slower than CULL_IDLE_TIME would otherwise cull a
            # notebook nobody could use yet (no Jupyter, no GPU process to sample).  But only
            # while it may still come up: a start that failed (init container in back-off,
            # image pull failing) or outlived CULL_IDLE_TIME + CULL_STARTUP_ALLOWANCE holds the
            # pod's GPUs for nothing, and is culled from the pod's creation on.
            born = pod_created_at(pod)
            young = born is None or now() - born < self.cfg.cull_idle_time_s + self.cfg.startup_allowance_s
            if young and not pod_start_stuck(pod):
                return Result(requeue_after=self.cfg.check_period_s)
        if not annotations_exist(nb):
            born = pod_created_at(pod) if starting else None
            await self._update(req, lambda cur: initialize_annotations(
                cur, rfc3339(born) if born is not None else None), precondition=False)
            nb = await self._read(kinds.NOTEBOOK_V1BETA1, req.name, req.namespace)
            if nb is None:
                return Result()
        key = (req.namespace, req.name)
        mem = self._checked.get(key)
        if not culling_check_period_has_passed(nb, self.cfg.check_period_s) or (
                mem is not None and mem + self.cfg.check_period_s >= now()):
            stored = parse_rfc3339(m.annotations(nb).get(LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION))
            last = max([t for t in (stored, mem) if t is not None], default=now())
            return Result(requeue_after=self._next_check(req, last))

        self.checks += 1
        active_now, kernels, terminals, signals = await self.sample(nb, pod)
        self.recent.append((rfc3339(), str(req), active_now, kernels, terminals))
        culled, skipped = [], []
        every = self.cfg.check_stamp_every

        def apply(cur: dict) -> None:
            culled.clear()
            skipped.clear()
            ann = m.annotations(cur)
            before = {k: ann.get(k) for k in (LAST_ACTIVITY_ANNOTATION, LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION,
                                               STOP_ANNOTATION)}
            if active_now:
                m.ensure_annotations(cur)[LAST_ACTIVITY_ANNOTATION] = rfc3339()
            else:
                update_from_kernels(cur, kernels)
                update_from_terminals(cur, terminals)
                if starting:
                    update_from_pod_creation(cur, pod)
                else:
                    update_from_pod_start(cur, pod)
            update_check_timestamp(cur)
            if notebook_is_idle(cur, self.cfg.cull_idle_time_s):
                set_stop_annotation(cur, self.metrics)
                culled.append(True)
            if every > 1:
                # The reference rewrites the check stamp on every check (:171-196); nothing but
                # its own schedule reads it, and that is kept here in memory.  When the check
                # changed nothing else, the stamp is written only in this notebook's slot of an
                # `every`-period cycle (its slot: a second hash of its key, independent of its phase in
                # the period, so R idle notebooks write
                # R/every stamps per period, evenly, not all in the same period).  An idle
                # notebook costs the apiserver, the webhook and every Notebook watcher one write
                # per `every` checks instead of one per check.  The stamp stays an RFC 3339
                # instant at most `every` periods (and a half) old, which any reader — a
                # reference culler taking over — takes as "check now".
                after = m.annotations(cur)
                stored = parse_rfc3339(before[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION])
                p = self.cfg.check_period_s
                t = now()
                my_slot = int(_phase_of(req.name, req.namespace) * every)
                if (after.get(LAST_ACTIVITY_ANNOTATION) == before[LAST_ACTIVITY_ANNOTATION]
                        and after.get(STOP_ANNOTATION) == before[STOP_ANNOTATION] and stored is not None
                        and t - stored < (every + 0.5) * p and int(t // p) % every != my_slot):
                    after[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION] = before[LAST_ACTIVITY_CHECK_TIMESTAMP_ANNOTATION]
                    skipped.append(True)

        await self._update(req, apply)
        self._checked[key] = float(int(now()))
        if skipped:
            self.stamps_skipped += 1
        if culled:
            self.culled += 1
            self.cull_log.append({"notebook": str(req), "at": rfc3339(), **signals})
            log.info("Notebook %s/%s culled (idle for %.0f s): %s", req.namespace, req.name,
                     self.cfg.cull_idle_time_s, ", ".join(f"{k}={v}" for k, v in signals.items()))
        return Result(requeue_after=self._next_check(req, float(int(now()))))

    def _next_check(self, req: Request, last_check: float) -> float:
        """Seconds until this notebook's next check: the first slot of its phase at or after
        ``last_check`` (the stamp, RFC3339 whole seconds) + the period.  Each notebook's checks
        land on a fixed phase of the period (a hash of its key), so R resident notebooks are
        checked evenly spread, R / period per second.  The reference requeues each after exactly
        the period (:200-202), so notebooks reconciled together — all of them when the manager
        starts — stay checked together: R writes in one burst every period, which is when every
        new notebook's create→Ready waits behind them.  The first aligned check may come up to one
        period later than the reference's; every later one comes exactly a period apart."""
        p = self.cfg.check_period_s
        if p <= 0:
            return p
        phase = _phase_of(req.namespace, req.name) * p
        target = last_check + p + 0.001  # strictly past the period at the wake-up
        k = -(-(target - phase) // p)  # ceil
        return max(0.001, phase + k * p - now())

    async def sample(self, nb: dict, pod: dict):
        """Returns ``(gpu_says_active, kernels, terminals, signals)``; ``signals`` says what each
        source reported (``amdgpu``: ``busy`` / ``idle`` with the mean busy %, or ``no-sample``;
        ``jupyter``: ``sampled`` / ``unreachable`` / not consulted) — the record of which signal
        a cull rests on."""
        src = self.cfg.activity_source
        gpu_active = False
        gpu_data = None
        signals = {}
        if src in ("amdgpu", "combined") and self.gpu is not None and pod_requests_gpu(pod):
            gpu_data = await self.gpu.busy(pod, self.cfg.check_period_s)
            if gpu_data is not None:
                gpu_active = gpu_says_active(gpu_data, self.cfg)
                signals["amdgpu"] = f"{'busy' if gpu_active else 'idle'} {gpu_data.get('busy_mean', 0):.0f}%"
            else:
                signals["amdgpu"] = "no-sample"
        kernels = terminals = None
        if src in ("jupyter", "combined") or gpu_data is None:
            kernels, terminals = await self.jupyter.sample(nb, pod)
            signals["jupyter"] = "sampled" if kernels is not None or terminals is not None else "unreachable"
        return gpu_active, kernels, terminals, signals

    async def close(self) -> None:
        await self.jupyter.close()
        if self.gpu is not None:
            await self.gpu.close()

    def setup_with_manager(self, mgr, max_concurrent: Optional[int] = None):
        b = mgr.builder().named(self.NAME).for_(kinds.NOTEBOOK_V1BETA1)
        if max_concurrent is not None:
            b.with_options(max_concurrent_reconciles=max_concurrent)
        c = b.complete(self)
        mgr.add(_Closer(self), needs_leader=False)
        return c


class _Closer:
    def __init__(self, r):
        self.r = r

    async def start(self):
        return None

    async def stop(self):
        await self.r.close()
