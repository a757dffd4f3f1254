"""REST client for a (real or in-process) Kubernetes apiserver — the ``client-go`` rest
layer the reference managers use through controller-runtime.

* :class:`RestConfig` — host, bearer token, TLS (CA / client cert / insecure) and the
  client-side ``QPS`` / ``Burst`` limiter of ``kf/main.go:71-85`` (``--qps`` /
  ``--burst``).  Loaders: :meth:`RestConfig.from_kubeconfig` (``$KUBECONFIG`` /
  ``~/.kube/config``, current context), :meth:`RestConfig.in_cluster` (service-account
  token + CA), :meth:`RestConfig.load` (explicit > kubeconfig > in-cluster, like
  ``ctrl.GetConfigOrDie``).
* :class:`RestClient` — the async :class:`~odh_kubeflow_amd.runtime.client.Client`
  interface over HTTP(S): CRUD, ``status`` subresource, the three patch types,
  ``DeleteOptions``, list with selectors, and :meth:`RestClient.watch` streaming
  ``WatchEvent`` lines.  Errors come back as the ``ApiError`` subclasses.
"""

from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
import ssl
import tempfile
import time
from dataclasses import dataclass, field
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple

try:  # native JSON (native/objcore.cpp): decoding with shared subtrees for watches, compact encoding
    from ..native._objcore import dumps as _dumps
    from ..native._objcore import loads_event as _loads_event
    from ..native._objcore import loads_shared as _loads_shared

    def loads_json(raw):
        try:
            return _loads_shared(raw)
        except ValueError:
            return json.loads(raw)  # json's own verdict (and its NaN / Infinity literals)

    def dumps_json(obj) -> bytes:
        """Compact JSON bytes of a request or response body (7x json.dumps on the control
        plane's objects); anything but a plain JSON tree goes through json.dumps."""
        try:
            return _dumps(obj)
        except (TypeError, ValueError):
            return json.dumps(obj, separators=(",", ":")).encode()
except ImportError:  # pragma: no cover - the extension is not built
    _loads_event = None
    loads_json = json.loads

    def dumps_json(obj) -> bytes:
        return json.dumps(obj, separators=(",", ":")).encode()

from ..models.errors import ApiError, Gone, InternalError
from ..models.scheme import SCHEME, ResourceInfo
from ..utils.selectors import format_label_selector
from .client import Client, _refresh, _version_of

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
log = logging.getLogger("runtime.rest")


def default_user_agent() -> str:
    """client-go's ``rest.DefaultKubernetesUserAgent``: ``<binary>/<version> (<os>/<arch>)
    <project>`` — the program name, so an apiserver audit log tells the processes apart
    (``control_plane``, ``scheduler``, ``odh_manager`` …)."""
    import platform
    import sys

    main = sys.modules.get("__main__")
    spec = getattr(main, "__spec__", None)
    prog = (spec.name.rsplit(".", 1)[-1] if spec is not None and spec.name else
            os.path.splitext(os.path.basename(sys.argv[0] if sys.argv and sys.argv[0] else "python"))[0])
    arch = {"x86_64": "amd64", "aarch64": "arm64"}.get(platform.machine(), platform.machine() or "unknown")
    return f"{prog or 'python'}/v0.0.0 ({sys.platform}/{arch}) odh-kubeflow-amd"


@dataclass
class RestConfig:
    host: str
    token: Optional[str] = None
    ca_file: Optional[str] = None
    ca_data: Optional[str] = None
    cert_file: Optional[str] = None
    key_file: Optional[str] = None
    insecure: bool = False
    qps: float = 0.0  # 0 = unlimited (controller-runtime defaults 20/30 on real clusters: pass --qps/--burst)
    burst: int = 0
    user_agent: str = field(default_factory=lambda: default_user_agent())
    extra: dict = field(default_factory=dict)
    # a bearer token file re-read while the process runs (in-cluster: the projected, rotated
    # ServiceAccount token; kubeconfig: ``tokenFile``) — see FileTokenSource
    token_file: Optional[str] = None

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.host.startswith("https"):
            return None
        if self.insecure:
            ctx = ssl.create_default_context()
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE  # lint: allow python-ssl-verify-disabled — kubeconfig insecure-skip-tls-verify
        else:
            ctx = ssl.create_default_context(cafile=self.ca_file, cadata=self.ca_data)
        if self.cert_file:
            ctx.load_cert_chain(self.cert_file, self.key_file)
        return ctx

    @classmethod
    def in_cluster(cls) -> "RestConfig":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if not host or not port:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        token_file = os.path.join(SA_DIR, "token")
        with open(token_file) as f:
            token = f.read().strip()
        if ":" in host:
            host = f"[{host}]"
        return cls(host=f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"),
                   token_file=token_file)

    @classmethod
    def from_kubeconfig(cls, path: Optional[str] = None, context: Optional[str] = None) -> "RestConfig":
        import yaml

        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        with open(path) as f:
            kc = yaml.safe_load(f) or {}
        ctx_name = context or kc.get("current-context")
        ctx = next((c["context"] for c in kc.get("contexts") or [] if c.get("name") == ctx_name), None)
        if ctx is None:
            raise RuntimeError(f"context {ctx_name!r} not found in {path}")
        cl = next((c["cluster"] for c in kc.get("clusters") or [] if c.get("name") == ctx.get("cluster")), {})
        user = next((u["user"] for u in kc.get("users") or [] if u.get("name") == ctx.get("user")), {})
        cfg = cls(host=cl.get("server", ""), token=user.get("token"), insecure=bool(cl.get("insecure-skip-tls-verify")))
        if cl.get("certificate-authority-data"):
            cfg.ca_data = base64.b64decode(cl["certificate-authority-data"]).decode()
        elif cl.get("certificate-authority"):
            cfg.ca_file = cl["certificate-authority"]
        for key, attr in (("client-certificate", "cert_file"), ("client-key", "key_file")):
            if user.get(key):
                setattr(cfg, attr, user[key])
            elif user.get(key + "-data"):
                fd, p = tempfile.mkstemp(prefix="odh-kc-")
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(user[key + "-data"]))
                setattr(cfg, attr, p)
        if user.get("tokenFile"):
            cfg.token_file = user["tokenFile"]
            with open(cfg.token_file) as f:
                cfg.token = f.read().strip()
        return cfg

    @classmethod
    def load(cls, master: Optional[str] = None, kubeconfig: Optional[str] = None) -> "RestConfig":
        if master:
            return cls(host=master, token=os.environ.get("KUBE_TOKEN"))
        if kubeconfig or os.environ.get("KUBECONFIG") or os.path.exists(os.path.expanduser("~/.kube/config")):
            return cls.from_kubeconfig(kubeconfig)
        return cls.in_cluster()


class FileTokenSource:
    """A bearer token read from a file and re-read while the process runs — client-go's
    ``cachingFileTokenSource`` (``transport/token_source.go``), which every controller-runtime
    manager of the reference gets through ``ctrl.GetConfigOrDie()`` (``kf/main.go:79-85``,
    ``odh/main.go:117-160``) for its in-cluster ``BearerTokenFile``.  The kubelet rotates a
    projected ServiceAccount token hourly (and a bound token expires unless the cluster
    extends it); a token read once at start-up starts failing with 401 after that.

    The file is re-read at most every ``period_s`` (client-go: one minute), and at once by
    :meth:`refresh` after a 401.  A failed read keeps the last good token (client-go logs
    and keeps serving the cached one)."""

    PERIOD_S = 60.0

    def __init__(self, path: str, initial: Optional[str] = None, period_s: float = PERIOD_S,
                 clock=time.monotonic):
        self.path = path
        self.period_s = period_s
        self._clock = clock
        self._token = initial or None
        self._read_at = clock() if self._token else float("-inf")
        self.reads = 0

    def token(self) -> Optional[str]:
        if self._clock() - self._read_at >= self.period_s:
            self._read()
        return self._token

    def refresh(self) -> bool:
        """Re-read now; True when the token changed (a request that got 401 is worth retrying)."""
        old = self._token
        self._read()
        return self._token != old

    def _read(self) -> None:
        self._read_at = self._clock()
        self.reads += 1
        try:
            with open(self.path) as f:
                tok = f.read().strip()
        except OSError as e:
            log.warning("cannot re-read the bearer token file %s (keeping the cached token): %s", self.path, e)
            return
        if tok:
            self._token = tok


class TokenBucket:
    """client-go's flowcontrol token bucket (``QPS`` refill, ``Burst`` capacity)."""

    def __init__(self, qps: float, burst: int):
        self.qps = qps
        self.capacity = max(1, burst or int(qps) or 1)
        self.tokens = float(self.capacity)
        self.t = time.monotonic()

    async def take(self) -> None:
        if self.qps <= 0:
            return
        while True:
            now = time.monotonic()
            self.tokens = min(self.capacity, self.tokens + (now - self.t) * self.qps)
            self.t = now
            if self.tokens >= 1:
                self.tokens -= 1
                return
            await asyncio.sleep((1 - self.tokens) / self.qps)


def _info_and_version(ref) -> Tuple[ResourceInfo, str]:
    info = SCHEME.resolve(ref)
    return info, _version_of(ref) or info.storage_version


class RestClient(Client):
    GET_RETRIES = 10

    def __init__(self, config: RestConfig, pool: int = 64):
        self.config = config
        self.base = config.host.rstrip("/")
        self._ssl = config.ssl_context()
        self._session = None
        self._pool = pool
        self._bucket = TokenBucket(config.qps, config.burst)
        self.requests = 0
        self.by_verb: Dict[str, int] = {}  # requests per HTTP method (watches counted as WATCH)
        self.bytes_in: Dict[str, int] = {}  # response body bytes: "LIST" (lists + relists) and "other"
        from collections import deque

        self.get_ms = deque(maxlen=8192)  # wall time of the recent GETs (ms): the live-read latency
        self.retries = 0  # GETs retried after a connection reset / EOF
        self.user = config.user_agent
        self._discovery: dict = {}  # "group/version" -> (fetched_at, set(plurals))
        self.tokens: Optional[FileTokenSource] = (FileTokenSource(config.token_file, config.token)
                                                  if config.token_file else None)
        self._sent_token: Optional[str] = None  # the token in the pool's Authorization header
        self.token_retries = 0  # requests / watches retried after a 401 with a re-read token

    def _bearer(self) -> Optional[str]:
        return self.tokens.token() if self.tokens is not None else self.config.token

    def _http(self):
        from .http1 import Http1Pool

        tok = self._bearer()
        if self._session is None:
            headers = {"User-Agent": self.config.user_agent}
            if tok:
                headers["Authorization"] = f"Bearer {tok}"
            self._session = Http1Pool(self.base, self._ssl, headers, size=self._pool, spare=2)
            self._sent_token = tok
        elif tok != self._sent_token:  # the token file was rotated
            self._session.set_header("Authorization", f"Bearer {tok}" if tok else None)
            self._sent_token = tok
        return self._session

    def _unauthorized_retry(self, status: int, sent: Optional[str]) -> bool:
        """A 401 while the token comes from a file: re-read it at once; retry iff the current
        token differs from the one the request carried (a concurrent request may have re-read
        the rotated file already)."""
        if status != 401 or self.tokens is None:
            return False
        self.tokens.refresh()
        if self.tokens.token() == sent:
            return False
        self.token_retries += 1
        return True

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
            self._session = None

    def path(self, info: ResourceInfo, version: str, namespace: Optional[str], name: Optional[str] = None,
             sub: Optional[str] = None) -> str:
        return self.base + info.path(version, namespace if info.namespaced else None, name, sub)

    async def request(self, method: str, url: str, body: Any = None, params: Optional[dict] = None,
                      content_type: str = "application/json", count_as: str = "other") -> dict:
        from urllib.parse import urlencode

        await self._bucket.take()
        self.requests += 1
        self.by_verb[method] = self.by_verb.get(method, 0) + 1
        data = None if body is None else dumps_json(body)
        target = url[len(self.base):] if url.startswith(self.base) else url
        if params:
            target += ("&" if "?" in target else "?") + urlencode(params)
        t0 = time.perf_counter()
        status, raw, sent = await self._roundtrip(method, target, data, content_type if data is not None else None)
        if self._unauthorized_retry(status, sent):
            status, raw, _ = await self._roundtrip(method, target, data, content_type if data is not None else None)
        if method == "GET":
            self.get_ms.append((time.perf_counter() - t0) * 1e3)
        if raw:
            self.bytes_in[count_as] = self.bytes_in.get(count_as, 0) + len(raw)
        try:
            out = loads_json(raw) if raw else {}
        except ValueError:
            out = {"message": raw[:200].decode(errors="replace")}
        if status >= 400:
            if isinstance(out, dict) and out.get("kind") == "Status":
                err = ApiError.from_status(out, status)
            else:
                err = ApiError.from_status({"code": status, "message": str(out)}, status)
            if status == 404 and err.reason != "NoKindMatch":
                await self._maybe_no_match(url, err)
            raise err
        return out

    async def _roundtrip(self, method: str, target: str, data: Optional[bytes],
                         content_type: Optional[str]) -> Tuple[int, bytes, Optional[str]]:
        """(status, body, the bearer token the request was sent with)."""
        from .http1 import HttpError

        for attempt in range(self.GET_RETRIES + 1):
            try:
                pool = self._http()
                sent = self._sent_token  # the header the next line writes (no await in between)
                status, raw = await pool.request(method, target, data, content_type)
                return status, raw, sent
            except HttpError as e:
                # client-go retries a GET whose connection was reset or hit EOF mid-response
                # (rest/request.go: IsConnectionReset || IsProbableEOF, up to maxRetries=10);
                # writes are not retried here — the reconcile's own requeue does that
                if method != "GET" or attempt == self.GET_RETRIES or not isinstance(
                        e.__cause__, (asyncio.IncompleteReadError, ConnectionResetError, BrokenPipeError,
                                      ConnectionAbortedError)):
                    raise InternalError(str(e))
                self.retries += 1
                await asyncio.sleep(min(0.5, 0.01 * (2 ** attempt)))
        raise InternalError("unreachable")

    async def _served(self, group: str, version: str) -> Optional[set]:
        """Plurals the server serves for ``group/version`` — ``None`` when discovery itself
        failed (connection dropped, 5xx): unknown is neither cached nor taken as "not
        served", or one dropped connection would turn every 404 into NoKindMatch for the
        cache lifetime."""
        key = f"{group}/{version}"
        hit = self._discovery.get(key)
        if hit is not None and time.monotonic() - hit[0] < 30.0:
            return hit[1]
        path = f"/apis/{group}/{version}" if group else f"/api/{version}"
        try:
            status, raw = await self._http().request("GET", path)
            if status == 404:
                doc = {}
            elif status == 200:
                doc = json.loads(raw) if raw else {}
            else:
                return None
        except Exception:  # noqa: BLE001 — discovery is best effort; the 404 stands
            return None
        plurals = {r.get("name") for r in (doc or {}).get("resources") or []}
        self._discovery[key] = (time.monotonic(), plurals)
        return plurals

    async def _maybe_no_match(self, url: str, err: ApiError) -> None:
        """A 404 on a resource type the server does not serve is ``meta.NoKindMatchError``
        (controller-runtime learns that from the RESTMapper's discovery)."""
        from ..models.scheme import parse_path
        from ..models.errors import NoKindMatch

        pp = parse_path(url[len(self.base):].split("?", 1)[0])
        if pp is None:
            return
        served = await self._served(pp.info.group, pp.version)
        if served is not None and pp.info.plural not in served:
            raise NoKindMatch(pp.info.kind)

    # -------------------------------------------------------------- Client interface

    async def get(self, kind, name, namespace=None):
        info, v = _info_and_version(kind)
        return await self.request("GET", self.path(info, v, namespace, name))

    async def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None):
        items, _ = await self.list_rv(kind, namespace, labels, fields)
        if owner_uid is not None:
            items = [o for o in items if any(r.get("uid") == owner_uid for r in
                                             (o.get("metadata") or {}).get("ownerReferences") or [])]
        return items

    async def list_rv(self, kind, namespace=None, labels=None, fields=None) -> Tuple[List[dict], str]:
        info, v = _info_and_version(kind)
        params = {}
        if labels:
            params["labelSelector"] = format_label_selector(labels) if isinstance(labels, dict) else labels
        if fields:
            params["fieldSelector"] = fields
        out = await self.request("GET", self.path(info, v, namespace), params=params or None, count_as="LIST")
        items = out.get("items") or []
        av = info.api_version(v)
        for o in items:
            o.setdefault("apiVersion", av)
            o.setdefault("kind", info.kind)
        return items, (out.get("metadata") or {}).get("resourceVersion", "")

    async def create(self, obj):
        info, v = _info_and_version(obj)
        ns = (obj.get("metadata") or {}).get("namespace")
        return _refresh(obj, await self.request("POST", self.path(info, v, ns), obj))

    async def update(self, obj):
        info, v = _info_and_version(obj)
        md = obj.get("metadata") or {}
        return _refresh(obj, await self.request("PUT", self.path(info, v, md.get("namespace"), md.get("name")), obj))

    async def update_status(self, obj):
        info, v = _info_and_version(obj)
        md = obj.get("metadata") or {}
        return _refresh(obj, await self.request("PUT", self.path(info, v, md.get("namespace"), md.get("name"),
                                                                 "status"), obj))

    async def patch(self, obj_or_kind, patch, patch_type="merge", name=None, namespace=None, subresource=None):
        if isinstance(obj_or_kind, dict):
            name = name or obj_or_kind["metadata"]["name"]
            namespace = namespace or obj_or_kind["metadata"].get("namespace")
        info, v = _info_and_version(obj_or_kind)
        ctype = {"merge": "application/merge-patch+json", "json": "application/json-patch+json",
                 "strategic": "application/strategic-merge-patch+json"}.get(patch_type, patch_type)
        out = await self.request("PATCH", self.path(info, v, namespace, name, subresource), patch, content_type=ctype)
        if isinstance(obj_or_kind, dict):
            return _refresh(obj_or_kind, out)
        return out

    async def delete(self, obj_or_kind, name=None, namespace=None, preconditions=None, propagation="Background"):
        if isinstance(obj_or_kind, dict):
            name = name or obj_or_kind["metadata"]["name"]
            namespace = namespace or obj_or_kind["metadata"].get("namespace")
        info, v = _info_and_version(obj_or_kind)
        body = {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": propagation}
        if preconditions:
            body["preconditions"] = preconditions
        return await self.request("DELETE", self.path(info, v, namespace, name), body)

    # -------------------------------------------------------------- watch

    async def watch(self, kind, namespace=None, resource_version: Optional[str] = None, labels=None, fields=None,
                    timeout_s: int = 300, bookmarks: bool = True) -> AsyncIterator[Tuple[str, dict]]:
        """Yield ``(type, object)``; raises :class:`Gone` when the RV is too old."""
        async for batch in self.watch_batches(kind, namespace, resource_version, labels, fields, timeout_s,
                                              bookmarks):
            for ev in batch:
                yield ev

    async def watch_batches(self, kind, namespace=None, resource_version: Optional[str] = None, labels=None,
                            fields=None, timeout_s: int = 300, bookmarks: bool = True,
                            lookup=None) -> AsyncIterator[List[Tuple[str, dict]]]:
        """Yield the ``(type, object)`` events of each arrival as one list (an informer applies
        them in one go); raises :class:`Gone` when the RV is too old — after yielding the
        events that preceded the ERROR in its batch.

        ``lookup(namespace, name)``: the caller's current copy of an object (an informer's
        store).  Events are decoded natively (``native/objcore.cpp`` ``loads_event``) against
        it: the subtrees a change leaves alone are the stored ones, not new copies."""
        from urllib.parse import urlencode

        info, v = _info_and_version(kind)
        params = {"watch": "true", "timeoutSeconds": str(timeout_s)}
        if resource_version:
            params["resourceVersion"] = resource_version
        if bookmarks:
            params["allowWatchBookmarks"] = "true"
        if labels:
            params["labelSelector"] = format_label_selector(labels) if isinstance(labels, dict) else labels
        if fields:
            params["fieldSelector"] = fields
        await self._bucket.take()
        self.requests += 1
        self.by_verb["WATCH"] = self.by_verb.get("WATCH", 0) + 1
        target = self.path(info, v, namespace)[len(self.base):] + "?" + urlencode(params)
        pool = self._http()
        sent = self._sent_token
        status, _headers, stream = await pool.stream("GET", target)
        if status == 401 and self.tokens is not None:
            await stream.read_all()
            stream.close()
            if self._unauthorized_retry(status, sent):  # rotated token: reopen once with the new one
                status, _headers, stream = await self._http().stream("GET", target)
            else:
                status, _headers, stream = 401, _headers, None
        if stream is None:
            raise ApiError.from_status({"code": 401, "reason": "Unauthorized", "message": "Unauthorized"}, 401)
        if status >= 400:
            raw = await stream.read_all()
            try:
                raise ApiError.from_status(json.loads(raw), status)
            except ValueError:
                raise InternalError(raw[:200].decode(errors="replace"))
        loads = json.loads
        native = _loads_event
        try:
            async for lines in stream.batches():
                out = []
                err = None
                for line in lines:
                    if not line or line.isspace():
                        continue
                    if native is not None:
                        try:
                            et, obj = native(line, lookup)
                        except ValueError:  # beyond the native decoder (NaN literals): json's verdict
                            ev = loads(line)
                            et, obj = ev.get("type"), ev.get("object") or {}
                    else:
                        ev = loads(line)
                        et, obj = ev.get("type"), ev.get("object") or {}
                    if et == "ERROR":
                        err = ApiError.from_status(obj)
                        break
                    out.append((et, obj))
                if out:
                    yield out
                if err is not None:
                    if err.code == 410:
                        raise Gone(err.message)
                    raise err
        finally:
            stream.close()
