"""Kubernetes REST + watch front end for :class:`~odh_kubeflow_amd.testing.apiserver.store.ObjectStore`.

This is the out-of-process half of the envtest substitute: the
managers, the webhook and the node agents talk to it exactly as they talk to a real
kube-apiserver — through :class:`~odh_kubeflow_amd.runtime.rest.RestClient` over
HTTP(S) with the standard URL layout, ``metav1.Status`` errors, list/watch with
``resourceVersion`` resumption (410 ``Gone`` when too old), label/field selectors, the
``status`` subresource, merge / JSON / strategic-merge patches, ``DeleteOptions``,
discovery documents and ``MutatingWebhookConfiguration``-driven HTTPS admission
webhooks (``failurePolicy`` honoured).

Routes:

* ``/api``, ``/apis``, ``/api/v1``, ``/apis/<g>/<v>`` — discovery;
* ``/api/v1[/namespaces/<ns>]/<plural>[/<name>[/<sub>]]``;
* ``/apis/<g>/<v>[/namespaces/<ns>]/<plural>[/<name>[/<sub>]]``;
* ``/healthz``, ``/readyz``, ``/livez``, ``/version``.
"""

from __future__ import annotations

import asyncio
import base64
import json
import logging
import ssl
import time
import uuid
from typing import Callable, Dict, List, Optional

from aiohttp import web

from ...models import meta as m
from ...models.errors import ApiError, BadRequest, InternalError, NotFound
from ...models.scheme import SCHEME, ParsedPath, ResourceInfo, parse_path  # noqa: F401  (re-exported)
from ...utils import jsonpatch
from ...utils.celmatch import CelError, Condition, compile_condition, conditions_allow
from ...utils.selectors import match_labels, selector_from_dict
from .store import ObjectStore

log = logging.getLogger("apiserver.http")

PATCH_TYPES = {
    "application/merge-patch+json": "merge",
    "application/json-patch+json": "json",
    "application/strategic-merge-patch+json": "strategic",
    "application/apply-patch+yaml": "merge",
}


def _dumps(o) -> bytes:
    return json.dumps(o, separators=(",", ":")).encode()


def _status_response(e: ApiError) -> web.Response:
    return web.Response(status=e.code, body=_dumps(e.to_status()), content_type="application/json")


class WebhookDispatcher:
    """Calls HTTPS mutating webhooks registered through ``MutatingWebhookConfiguration``.

    ``clientConfig.url`` is used as is; ``clientConfig.service`` is resolved through
    ``service_resolver(namespace, name, port) -> "host:port"`` (tests / local clusters).
    """

    def __init__(self, store: ObjectStore, service_resolver: Optional[Callable[[str, str, int], str]] = None):
        self.store = store
        self.service_resolver = service_resolver
        self._session = None
        self._registered: Dict[str, List[str]] = {}
        self.calls = 0

    def start(self) -> None:
        self.store.watch("admissionregistration.k8s.io/v1/MutatingWebhookConfiguration", self._on_mwc)
        for obj in self.store.list_nocopy("admissionregistration.k8s.io/v1/MutatingWebhookConfiguration"):
            self._on_mwc("ADDED", obj, None)

    def _on_mwc(self, etype: str, obj: dict, old: Optional[dict]) -> None:
        cfg_name = m.name(obj)
        for hname in self._registered.pop(cfg_name, []):
            self.store.remove_mutating_admission(hname)
        if etype == "DELETED":
            return
        names = []
        for wh in obj.get("webhooks") or []:
            hname = f"{cfg_name}/{wh.get('name', '')}"
            self.store.add_mutating_admission(hname, self._matcher(wh), self._handler(wh))
            names.append(hname)
        self._registered[cfg_name] = names

    @staticmethod
    def _matcher(wh: dict):
        rules = wh.get("rules") or []

        def match(info: ResourceInfo, op: str) -> bool:
            for r in rules:
                ops = r.get("operations") or []
                if "*" not in ops and op not in ops:
                    continue
                groups = r.get("apiGroups") or []
                if "*" not in groups and info.group not in groups:
                    continue
                res = r.get("resources") or []
                if "*" not in res and info.plural not in res:
                    continue
                return True
            return False

        return match

    def _url(self, wh: dict) -> str:
        cc = wh.get("clientConfig") or {}
        if cc.get("url"):
            return cc["url"]
        svc = cc.get("service") or {}
        port = int(svc.get("port") or 443)
        hostport = (self.service_resolver(svc.get("namespace", ""), svc.get("name", ""), port)
                    if self.service_resolver else f"{svc.get('name')}.{svc.get('namespace')}.svc:{port}")
        return f"https://{hostport}{svc.get('path') or '/'}"

    def _handler(self, wh: dict):
        fail_closed = (wh.get("failurePolicy") or "Fail") == "Fail"
        timeout = float(wh.get("timeoutSeconds") or 10)
        cc = wh.get("clientConfig") or {}
        ctx = None
        if cc.get("caBundle"):
            ctx = ssl.create_default_context(cadata=base64.b64decode(cc["caBundle"]).decode())
        name = wh.get("name", "")
        ns_sel = selector_from_dict(wh.get("namespaceSelector")) if wh.get("namespaceSelector") else None
        obj_sel = selector_from_dict(wh.get("objectSelector")) if wh.get("objectSelector") else None
        conds = [_condition(c) for c in wh.get("matchConditions") or []]

        def selected(info: ResourceInfo, obj: dict, old: Optional[dict]) -> bool:
            if obj_sel is not None and not match_labels(obj_sel, m.labels(obj)) and not (
                    old is not None and match_labels(obj_sel, m.labels(old))):
                return False
            if ns_sel is None:
                return True
            if info.kind == "Namespace" and not info.group:
                return match_labels(ns_sel, m.labels(obj))
            if not info.namespaced:
                return True
            ns = self.store.peek("v1/Namespace", m.namespace(obj))
            labels = m.labels(ns) if ns is not None else {"kubernetes.io/metadata.name": m.namespace(obj)}
            return match_labels(ns_sel, labels)

        async def handler(op, info, obj, old):
            import aiohttp

            if not selected(info, obj, old):
                return obj
            try:
                if not conditions_allow(conds, obj, old, fail_closed):
                    return obj
            except CelError as e:
                raise InternalError(f'failed calling webhook "{name}": matchConditions: {e}')

            if self._session is None or self._session.closed:
                # admission calls carry the webhook's own timeoutSeconds; this bounds anything else
                self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30))
            review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                      "request": {"uid": str(uuid.uuid4()), "operation": op, "name": m.name(obj),
                                  "namespace": m.namespace(obj), "object": obj, "oldObject": old,
                                  "kind": {"group": info.group, "version": info.storage_version, "kind": info.kind},
                                  "resource": {"group": info.group, "version": info.storage_version,
                                               "resource": info.plural}}}
            self.calls += 1
            try:
                async with self._session.post(self._url(wh), data=_dumps(review), ssl=ctx if ctx else None,
                                              headers={"Content-Type": "application/json"},
                                              timeout=aiohttp.ClientTimeout(total=timeout)) as resp:
                    body = await resp.json(content_type=None)
            except Exception as e:
                if fail_closed:
                    raise InternalError(f'failed calling webhook "{name}": {e}')
                log.warning("webhook %s failed (ignored): %s", name, e)
                return obj
            out = (body or {}).get("response") or {}
            if not out.get("allowed"):
                st = out.get("status") or {}
                raise InternalError(f'admission webhook "{name}" denied the request: {st.get("message", "")}')
            if out.get("patch"):
                obj = jsonpatch.apply_patch(obj, json.loads(base64.b64decode(out["patch"])))
            return obj

        return handler

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()


def _condition(mc) -> "Condition":
    """One ``matchConditions`` entry; an expression outside the evaluated CEL subset errors at
    every evaluation (``failurePolicy`` decides), as an uncompilable one would."""
    try:
        return compile_condition(str((mc or {}).get("expression", "")))
    except CelError as e:
        def bad(obj, old, e=e):
            raise e
        return bad


class ApiServer:
    """aiohttp application serving an :class:`ObjectStore`."""

    ADMIN = {"username": "system:admin", "groups": ["system:masters", "system:authenticated"]}

    def __init__(self, store: ObjectStore, token: Optional[str] = None,
                 service_resolver: Optional[Callable[[str, str, int], str]] = None, audit=None,
                 users: Optional[Dict[str, dict]] = None):
        self.store = store
        self.token = token
        # bearer token -> user info ({"username", "uid", "groups", "extra"}): who a request is
        # from, as kube-apiserver's authenticators say — stamped into a CertificateSigningRequest's
        # spec on create (a client cannot claim someone else's identity there); no authorization
        self.users = dict(users or {})
        self.audit = audit  # apiserver.audit.AuditLogger (DEBUG_WRITE_AUDITLOG)
        self.webhooks = WebhookDispatcher(store, service_resolver)
        self._runner: Optional[web.AppRunner] = None
        self.port = 0
        self.host = "127.0.0.1"
        self.requests = 0
        self.watches = 0
        self._watch_tasks: set = set()
        self._closing = asyncio.Event() if False else None

    # -------------------------------------------------------------- lifecycle

    def app(self) -> web.Application:
        app = web.Application(client_max_size=64 * 1024 * 1024)
        for p in ("/healthz", "/readyz", "/livez"):
            app.router.add_get(p, self._ok)
        app.router.add_get("/version", self._version)
        app.router.add_route("*", "/{tail:.*}", self._dispatch)
        return app

    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context: Optional[ssl.SSLContext] = None):
        self._closing = asyncio.Event()
        self.webhooks.start()
        self._runner = web.AppRunner(self.app(), access_log=None, handler_cancellation=True)
        await self._runner.setup()
        site = web.TCPSite(self._runner, host, port, ssl_context=ssl_context, backlog=1024)
        await site.start()
        self.host = host
        self.port = site._server.sockets[0].getsockname()[1]
        self.scheme = "https" if ssl_context else "http"
        return self

    @property
    def url(self) -> str:
        return f"{getattr(self, 'scheme', 'http')}://{self.host}:{self.port}"

    async def stop(self) -> None:
        if self._closing is not None:
            self._closing.set()
        for t in list(self._watch_tasks):
            t.cancel()
        await self.webhooks.close()
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None

    def rotate_token(self, token: str) -> None:
        """Accept only ``token`` from now on and end the open watches — a rotated (or expired
        bound) ServiceAccount token: every client must re-authenticate, a watch included when
        it re-opens."""
        self.token = token
        for t in list(self._watch_tasks):
            t.cancel()

    # -------------------------------------------------------------- handlers

    async def _ok(self, _req):
        return web.Response(text="ok")

    async def _version(self, _req):
        return web.json_response({"major": "1", "minor": "32", "gitVersion": "v1.32.8-odh-kubeflow-amd",
                                  "platform": "linux/amd64"})

    def _authorized(self, req: web.Request) -> bool:
        auth = req.headers.get("Authorization", "")
        if self.users and auth.startswith("Bearer ") and auth[7:] in self.users:
            return True
        if not self.token:
            return True
        return auth == f"Bearer {self.token}"

    def _user(self, req: web.Request) -> dict:
        auth = req.headers.get("Authorization", "")
        return self.users.get(auth[7:], self.ADMIN) if auth.startswith("Bearer ") else self.ADMIN

    async def _dispatch(self, req: web.Request) -> web.StreamResponse:
        self.requests += 1
        if not self._authorized(req):
            return web.Response(status=401, body=_dumps({"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                                         "message": "Unauthorized", "reason": "Unauthorized",
                                                         "code": 401}), content_type="application/json")
        path = req.path
        try:
            if req.method == "GET":
                disc = self._discovery(path)
                if disc is not None:
                    return web.Response(body=_dumps(disc), content_type="application/json")
            pp = parse_path(path)
            if pp is None:
                raise NotFound("path", path)
            if pp.version not in pp.info.versions:
                raise NotFound(pp.info.plural, f"version {pp.version}")
            if pp.info.namespaced is False and pp.namespace:
                raise BadRequest(f"{pp.info.plural} is not namespaced")
        except ApiError as e:
            return _status_response(e)
        if self.audit is None:
            return await self._resource_or_status(req, pp)
        from .audit import _now, verb_of

        received = _now()
        watch = req.method == "GET" and req.query.get("watch") in ("1", "true", "True")
        body = None
        if req.method in ("POST", "PUT", "PATCH") and req.can_read_body:
            try:
                body = json.loads(await req.read() or b"null")
            except ValueError:
                body = None
        verb = verb_of(req.method, pp.name or "", watch)
        common = dict(verb=verb, uri=str(req.rel_url), user="system:admin",
                      user_agent=req.headers.get("User-Agent", ""), group=pp.info.group, version=pp.version,
                      resource=pp.info.plural, namespace=pp.namespace or "", name=pp.name or "",
                      subresource=pp.sub or "", request_obj=body, received=received)
        if watch:  # a stream: logged when it starts
            self.audit.log(code=200, stage="ResponseStarted", **common)
            return await self._resource_or_status(req, pp)
        resp = await self._resource_or_status(req, pp)
        out = None
        if isinstance(resp, web.Response) and resp.body is not None:
            try:
                out = json.loads(resp.body)
            except (ValueError, TypeError):
                out = None
        if verb == "create" and not common["name"] and resp.status < 300 and isinstance(out, dict):
            common["name"] = (out.get("metadata") or {}).get("name") or ""  # as kube-apiserver's objectRef
        self.audit.log(code=resp.status, response_obj=out, **common)
        return resp

    async def _resource_or_status(self, req: web.Request, pp: ParsedPath) -> web.StreamResponse:
        try:
            return await self._resource(req, pp)
        except ApiError as e:
            return _status_response(e)
        except (ValueError, json.JSONDecodeError) as e:
            return _status_response(BadRequest(str(e)))

    def _discovery(self, path: str) -> Optional[dict]:
        p = path.rstrip("/")
        infos = SCHEME.all()
        if p == "/api":
            return {"kind": "APIVersions", "versions": ["v1"],
                    "serverAddressByClientCIDRs": [{"clientCIDR": "0.0.0.0/0", "serverAddress": "127.0.0.1"}]}
        if p == "/apis":
            groups: Dict[str, List[str]] = {}
            for i in infos:
                if i.group and i.key in self.store.installed:
                    for v in i.versions:
                        if v not in groups.setdefault(i.group, []):
                            groups[i.group].append(v)
            return {"kind": "APIGroupList", "apiVersion": "v1", "groups": [
                {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in vs],
                 "preferredVersion": {"groupVersion": f"{g}/{vs[0]}", "version": vs[0]}} for g, vs in sorted(groups.items())]}
        segs = [s for s in p.split("/") if s]
        if len(segs) == 2 and segs[0] == "api":
            group, version = "", segs[1]
        elif len(segs) == 3 and segs[0] == "apis":
            group, version = segs[1], segs[2]
        else:
            return None
        res = []
        for i in infos:
            if i.group == group and version in i.versions and i.key in self.store.installed:
                verbs = ["create", "delete", "get", "list", "patch", "update", "watch"]
                res.append({"name": i.plural, "singularName": i.singular, "namespaced": i.namespaced, "kind": i.kind,
                            "verbs": verbs, "shortNames": list(i.short_names)})
                if i.status_subresource:
                    res.append({"name": f"{i.plural}/status", "singularName": "", "namespaced": i.namespaced,
                                "kind": i.kind, "verbs": ["get", "patch", "update"]})
        if not res:
            return None
        return {"kind": "APIResourceList", "apiVersion": "v1",
                "groupVersion": f"{group}/{version}" if group else version, "resources": res}

    async def _body(self, req: web.Request) -> dict:
        raw = await req.read()
        if not raw:
            return {}
        return json.loads(raw)

    async def _resource(self, req: web.Request, pp: ParsedPath) -> web.StreamResponse:
        info, version, ns, name, sub = pp.info, pp.version, pp.namespace, pp.name, pp.sub
        q = req.query
        st = self.store
        if sub not in (None, "status") and not (sub == "approval" and info.kind == "CertificateSigningRequest"):
            raise NotFound(info.plural, f"{name}/{sub}")
        method = req.method
        if method == "GET" and name is None:
            if q.get("watch") in ("1", "true", "True"):
                return await self._watch(req, info, version, ns)
            items, rv = await st.list(info, ns, q.get("labelSelector") or None, q.get("fieldSelector") or None,
                                      version=version)
            body = {"kind": info.list_kind, "apiVersion": info.api_version(version),
                    "metadata": {"resourceVersion": rv}, "items": items}
            return web.Response(body=_dumps(body), content_type="application/json")
        if method == "GET":
            obj = await st.get(info, name, ns, version=version)
            return web.Response(body=_dumps(obj), content_type="application/json")
        if method == "POST" and name is None:
            obj = await self._body(req)
            obj.setdefault("apiVersion", info.api_version(version))
            obj.setdefault("kind", info.kind)
            if info.kind == "CertificateSigningRequest":  # the requester, from authentication
                u = self._user(req)
                spec = obj.setdefault("spec", {})
                for k in ("username", "uid", "groups", "extra"):
                    spec.pop(k, None)
                    if u.get(k):
                        spec[k] = u[k]
            dry = q.get("dryRun") == "All"
            out = await st.create(obj, namespace=ns, dry_run=dry)
            out["apiVersion"] = info.api_version(version)
            return web.Response(status=201, body=_dumps(out), content_type="application/json")
        if method == "PUT" and name:
            obj = await self._body(req)
            obj.setdefault("apiVersion", info.api_version(version))
            obj.setdefault("kind", info.kind)
            md = obj.setdefault("metadata", {})
            if md.get("name") and md["name"] != name:
                raise BadRequest("the name of the object does not match the name on the URL")
            md["name"] = name
            if ns:
                md.setdefault("namespace", ns)
            out = await st.update(obj, subresource=sub, namespace=ns)
            out["apiVersion"] = info.api_version(version)
            return web.Response(body=_dumps(out), content_type="application/json")
        if method == "PATCH" and name:
            ctype = req.headers.get("Content-Type", "application/merge-patch+json").split(";")[0].strip()
            ptype = PATCH_TYPES.get(ctype)
            if ptype is None:
                return web.Response(status=415, body=_dumps({"kind": "Status", "apiVersion": "v1",
                                                             "status": "Failure", "code": 415,
                                                             "reason": "UnsupportedMediaType",
                                                             "message": f"unsupported patch type {ctype}"}),
                                    content_type="application/json")
            patch = json.loads(await req.read() or b"{}")
            out = await st.patch(info, name, ns, patch, ptype, subresource=sub)
            out["apiVersion"] = info.api_version(version)
            return web.Response(body=_dumps(out), content_type="application/json")
        if method == "DELETE" and name:
            opts = await self._body(req)
            prop = opts.get("propagationPolicy") or q.get("propagationPolicy") or "Background"
            out = await st.delete(info, name, ns, opts.get("preconditions"), prop)
            return web.Response(body=_dumps(out), content_type="application/json")
        return web.Response(status=405, body=_dumps({"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                                     "code": 405, "reason": "MethodNotAllowed",
                                                     "message": f"{method} not allowed"}),
                            content_type="application/json")

    async def _watch(self, req: web.Request, info: ResourceInfo, version: str, ns: Optional[str]):
        q = req.query
        rv = q.get("resourceVersion")
        timeout = float(q.get("timeoutSeconds") or 1800)
        bookmarks = q.get("allowWatchBookmarks") in ("true", "1")
        av = info.api_version(version)
        queue: asyncio.Queue = asyncio.Queue()

        def cb(etype, obj, old):
            queue.put_nowait((etype, obj))

        resp = web.StreamResponse(headers={"Content-Type": "application/json", "Transfer-Encoding": "chunked"})
        try:
            if rv in (None, "", "0"):
                # "get state and start at most recent": synthetic ADDED for current objects
                initial = self.store.list_nocopy(info, ns, q.get("labelSelector") or None,
                                                 q.get("fieldSelector") or None)
                cancel = self.store.watch(info, cb, namespace=ns, label_selector=q.get("labelSelector") or None,
                                          field_selector=q.get("fieldSelector") or None)
                for o in initial:
                    queue.put_nowait(("ADDED", o))
            else:
                cancel = self.store.watch(info, cb, namespace=ns, label_selector=q.get("labelSelector") or None,
                                          field_selector=q.get("fieldSelector") or None, resource_version=rv)
        except ApiError as e:
            await resp.prepare(req)
            await resp.write(_dumps({"type": "ERROR", "object": e.to_status()}) + b"\n")
            await resp.write_eof()
            return resp
        self.watches += 1
        await resp.prepare(req)
        deadline = time.monotonic() + timeout
        task = asyncio.current_task()
        self._watch_tasks.add(task)
        try:
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    etype, obj = await asyncio.wait_for(queue.get(), timeout=min(left, 10.0))
                except asyncio.TimeoutError:
                    if bookmarks:
                        bm = {"kind": info.kind, "apiVersion": av,
                              "metadata": {"resourceVersion": self.store.resource_version}}
                        await resp.write(_dumps({"type": "BOOKMARK", "object": bm}) + b"\n")
                    continue
                chunks = []
                while True:
                    o = obj if obj.get("apiVersion") == av else {**obj, "apiVersion": av}
                    chunks.append(_dumps({"type": etype, "object": o}))
                    if queue.empty() or len(chunks) >= 256:
                        break
                    etype, obj = queue.get_nowait()
                await resp.write(b"\n".join(chunks) + b"\n")
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            cancel()
            self._watch_tasks.discard(task)
        try:
            await resp.write_eof()
        except Exception:
            pass
        return resp


async def serve(store: ObjectStore, host: str = "127.0.0.1", port: int = 0, token: Optional[str] = None,
                ssl_context: Optional[ssl.SSLContext] = None, **kw) -> ApiServer:
    return await ApiServer(store, token=token, **kw).start(host, port, ssl_context)
