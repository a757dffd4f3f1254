"""The ODH mutating admission webhook for ``kubeflow.org/v1 notebooks``
(reference ``odh/controllers/notebook_webhook.go``, registered at
``/mutate-notebook-v1`` with ``failurePolicy: Fail``, ``sideEffects: None``).

``Handle`` pipeline (:352-499), in order:

1. CREATE → inject the reconciliation lock (``kubeflow-resource-stopped:
   odh-notebook-controller-lock``) so the pod cannot start before the ODH reconciler
   has run;
2. CREATE/UPDATE → resolve the image from the ImageStream named by
   ``notebooks.opendatahub.io/last-image-selection`` (span events
   ``imagestream-not-found`` / ``imagestream-tag-not-found``), mount the trusted-CA
   bundle, sync + mount the pipeline runtime-images ConfigMap, [``SET_PIPELINE_SECRET``]
   sync + mount the Elyra secret, mount/unmount the Feast config;
3. ``inject-auth`` → kube-rbac-proxy sidecar;
4. ``INJECT_CLUSTER_PROXY_ENV`` + cluster ``Proxy`` → HTTP(S)_PROXY / NO_PROXY env;
5. restart guard: on UPDATE of a running notebook, webhook-only pod-template changes
   are reverted and reported in ``notebooks.opendatahub.io/update-pending``;
6. respond with an RFC 6902 JSONPatch from the request object to the mutated one.

Differences (internal, not observable): the cluster proxy values are returned, not
stored in a package-global map written by concurrent requests (:66, :340-342 — a data
race in the reference); the webhook client is uncached for ConfigMaps/Secrets like
the reference manager's (``odh/main.go:178-185``).
"""

from __future__ import annotations

import asyncio
import base64
import json
import logging
import os
from collections import OrderedDict
from typing import Dict, Mapping, Optional, Tuple

from ..controllers.odh import auth, certs, dspa_secret, feast, runtime_images
from ..controllers.odh.constants import (ANNOTATION_NOTEBOOK_RESTART, ANNOTATION_UPDATE_PENDING,
                                         ANNOTATION_VALUE_RECONCILIATION_LOCK, IMAGE_STREAM_NOT_FOUND_EVENT,
                                         IMAGE_STREAM_TAG_NOT_FOUND_EVENT, INTERNAL_REGISTRY,
                                         LAST_IMAGE_SELECTION_ANNOTATION, STOP_ANNOTATION,
                                         WORKBENCH_IMAGE_NAMESPACE_ANNOTATION)
from ..controllers.odh.podspec import add_missing_env, notebook_container
from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_not_found
from ..runtime.client import CONFIRM_ABSENCE
from ..runtime.rest import dumps_json
from ..tracing import current_span, get_tracer
from ..utils import jsonpatch
from ..utils.objutil import deepcopy_json, semantic_equal
from .diff import first_difference

log = logging.getLogger("webhook.notebook")
tracer = get_tracer("opendatahub.io/kubeflow/components/odh-notebook-controller/controllers/notebook_webhook.go")

WEBHOOK_PATH = "/mutate-notebook-v1"
PROXY_ENV_ORDER = ("HTTP_PROXY", "HTTPS_PROXY", "NO_PROXY")


class AdmissionError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


def validate_gpu_resources(nb: dict) -> None:
    """``amd.com/gpu`` is an extended resource: whole numbers, never overcommitted, so a
    request needs an equal limit (the pod-validation rules kube-apiserver applies when
    the StatefulSet controller creates the pod).  Checked at admission so a bad Notebook
    is refused up front instead of leaving a StatefulSet that can never create its pod."""
    from ..models.notebook import GPU_RESOURCE

    spec = ((nb.get("spec") or {}).get("template") or {}).get("spec") or {}
    for i, c in enumerate(spec.get("containers") or []):
        res = c.get("resources") or {}
        req = (res.get("requests") or {}).get(GPU_RESOURCE)
        lim = (res.get("limits") or {}).get(GPU_RESOURCE)
        path = f"spec.template.spec.containers[{i}].resources"
        for kind_, v in (("limits", lim), ("requests", req)):
            if v is not None and not str(v).strip().isdigit():
                raise AdmissionError(400, f'{path}.{kind_}[{GPU_RESOURCE}]: Invalid value: "{v}": must be an integer')
        if req is not None and lim is None:
            raise AdmissionError(400, f"{path}.limits: Required value: Limit must be set for non overcommitable "
                                      f"resources ({GPU_RESOURCE})")
        if req is not None and int(str(req)) != int(str(lim)):
            raise AdmissionError(400, f'{path}.requests[{GPU_RESOURCE}]: Invalid value: "{req}": must be equal to '
                                      f"{GPU_RESOURCE} limit of {lim}")


def _gpu_resources(nb: Optional[dict]) -> list:
    from ..models.notebook import GPU_RESOURCE

    spec = (((nb or {}).get("spec") or {}).get("template") or {}).get("spec") or {}
    out = []
    for c in spec.get("containers") or []:
        res = (c.get("resources") if isinstance(c, dict) else None) or {}
        out.append(((res.get("requests") or {}).get(GPU_RESOURCE), (res.get("limits") or {}).get(GPU_RESOURCE)))
    return out


def gpu_validation_applies(operation: str, nb: dict, old: Optional[dict]) -> bool:
    """Whether :func:`validate_gpu_resources` judges this admission: a CREATE, or an UPDATE
    that changes some container's ``amd.com/gpu`` request or limit — never an update of a
    Notebook being deleted.

    The check is this webhook's own (the reference's ``Handle`` denies none of these paths,
    ``odh/controllers/notebook_webhook.go:352-499``), so it must never wedge a Notebook that
    is already stored: one that predates the webhook (a takeover from the reference's
    controllers) must stay finalizable, cullable and unlockable — the controllers' finalizer,
    stop-annotation and lock writes leave the GPU fields as they were."""
    if operation == "CREATE":
        return True
    if operation != "UPDATE" or m.is_deleting(nb):
        return False
    return old is None or _gpu_resources(nb) != _gpu_resources(old)


_HEARTBEAT_META_SKIP = frozenset({"annotations", "resourceVersion", "managedFields", "generation"})


def culler_heartbeat_only(nb: dict, old: Optional[dict]) -> bool:
    """An UPDATE of a running notebook whose only change is the culler's activity bookkeeping
    (``CULLER_HEARTBEAT_ANNOTATIONS``; the culler writes it on every check of every notebook,
    ``kf/controllers/culling_controller.go:171-196``).

    For such an update the reference's pipeline can only end one of two ways: its mutations
    leave the pod template alone, or the restart guard reverts them (the notebook runs and the
    culler did not touch the template, :505-564) — apart from refreshing
    ``update-pending``, the response is empty.  Such an update skips the pipeline while the
    webhook's inputs are unchanged since the notebook's last full admission
    (``NotebookWebhook._heartbeat_settled``), so R resident notebooks do not cost R
    admissions' worth of ConfigMap reads per check period; once an input changed, the next
    heartbeat runs the pipeline and refreshes ``update-pending``.  A stopped or restarting
    notebook (no restart guard) always takes the full pipeline."""
    from ..controllers.odh.constants import ANNOTATION_NOTEBOOK_RESTART as RESTART
    from ..models.notebook import CULLER_HEARTBEAT_ANNOTATIONS
    from ..runtime.controller import maps_differ

    if old is None:
        return False
    md, om = nb.get("metadata") or {}, old.get("metadata") or {}
    ann, oann = md.get("annotations") or {}, om.get("annotations") or {}
    if STOP_ANNOTATION in ann or RESTART in ann:
        return False
    if ann == oann or maps_differ(ann, oann, CULLER_HEARTBEAT_ANNOTATIONS):
        return False  # no heartbeat change, or something else changed too
    for k in md.keys() | om.keys():
        if k not in _HEARTBEAT_META_SKIP and md.get(k) != om.get(k):
            return False
    return nb.get("spec") == old.get("spec")


def inject_reconciliation_lock(nb: dict) -> None:
    m.ensure_annotations(nb)[STOP_ANNOTATION] = ANNOTATION_VALUE_RECONCILIATION_LOCK


def _parse_go_bool(raw: str) -> Optional[bool]:
    v = raw.strip()
    if v in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if v in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    return None


def created_time(raw) -> float:
    """An ImageStream tag item's ``created`` (a ``metav1.Time``, RFC 3339) as seconds since the
    epoch, so items are ordered by instant as the reference's ``Time.After`` orders them
    (``odh/controllers/notebook_webhook.go:860-864``) — not by string, which misorders
    ``+02:00`` against ``Z`` and fractional against whole seconds.  Absent or unparsable:
    the zero time, i.e. oldest."""
    import datetime

    if not isinstance(raw, str) or not raw:
        return float("-inf")
    s = raw.strip()
    if s[-1:] in ("Z", "z"):
        s = s[:-1] + "+00:00"
    head, dot, rest = s.partition(".")
    if dot:  # fromisoformat (3.10) takes 3 or 6 fractional digits only: normalise to 6
        i = 0
        while i < len(rest) and rest[i].isdigit():
            i += 1
        s = head + "." + (rest[:i] + "000000")[:6] + rest[i:]
    try:
        t = datetime.datetime.fromisoformat(s)  # any single character separates date and time
    except ValueError:
        return float("-inf")
    if t.tzinfo is None:
        return float("-inf")  # RFC 3339 requires an offset
    return t.timestamp()


async def set_container_image_from_registry(client, nb: dict, controller_namespace: str) -> None:
    """``SetContainerImageFromRegistry`` (:787-894)."""
    span = current_span()
    ann = m.annotations(nb)
    selection = ann.get(LAST_IMAGE_SELECTION_ANNOTATION)
    if selection is None:
        return
    c = notebook_container(nb)
    if c is None:
        raise AdmissionError(500, f"no container found matching the notebook name {m.name(nb)}")
    if INTERNAL_REGISTRY in (c.get("image") or ""):
        return
    parts = selection.split(":")
    if len(parts) != 2:
        raise AdmissionError(500, "invalid image selection format")
    is_name, tag_name = parts
    image_ns = ann.get(WORKBENCH_IMAGE_NAMESPACE_ANNOTATION)
    if image_ns is None or not image_ns.strip():
        image_ns = controller_namespace
    try:
        ist = await client.get(kinds.IMAGE_STREAM, is_name, image_ns)
    except ApiError as e:
        if is_not_found(e):
            span.add_event(IMAGE_STREAM_NOT_FOUND_EVENT)
        else:
            log.error("error getting ImageStream %s/%s: %s", image_ns, is_name, e)
        return
    tags = (ist.get("status") or {}).get("tags")
    if tags is None:
        span.add_event(IMAGE_STREAM_TAG_NOT_FOUND_EVENT)
        raise AdmissionError(500, "ImageStream has no status or tags")
    for tag in tags:
        if tag.get("tag") != tag_name:
            continue
        items = tag.get("items") or []
        if not items:
            continue
        newest = sorted(items, key=lambda it: created_time(it.get("created")), reverse=True)[0]
        # the reference writes Containers[0] (:868) — preserved
        nb["spec"]["template"]["spec"]["containers"][0]["image"] = newest.get("dockerImageReference", "")
        for e in c.get("env") or []:
            if e.get("name") == "JUPYTER_IMAGE":
                e["value"] = selection
                break
        return
    span.add_event(IMAGE_STREAM_TAG_NOT_FOUND_EVENT)


async def cluster_proxy_env(client) -> Optional[Dict[str, str]]:
    """``ClusterWideProxyIsEnabled`` (:328-349) without the shared global map."""
    try:
        proxies = await client.list(kinds.PROXY)
    except ApiError:
        return None
    for p in proxies:
        if m.name(p) == "cluster":
            st = p.get("status") or {}
            if st.get("httpProxy") and st.get("httpsProxy") and st.get("noProxy"):
                return {"HTTP_PROXY": st["httpProxy"], "HTTPS_PROXY": st["httpsProxy"], "NO_PROXY": st["noProxy"]}
    return None


def inject_proxy_config_env_vars(nb: dict, values: Mapping[str, str]) -> None:
    c = notebook_container(nb)
    if c is not None:
        add_missing_env(c, values, order=[k for k in PROXY_ENV_ORDER if k in values])


class NotebookWebhook:
    MEMO_CAP = 262144  # notebooks whose last full admission is remembered (a few hundred bytes each)

    def __init__(self, client, namespace: str, kube_rbac_proxy_image: str, env: Optional[Mapping[str, str]] = None,
                 reader=None):
        self.client = client
        self.namespace = namespace
        self.kube_rbac_proxy_image = kube_rbac_proxy_image
        self.env = env if env is not None else os.environ
        self.requests = 0
        self.denied = 0
        self.heartbeats = 0  # culler heartbeat updates answered without the pipeline
        self.heartbeats_full = 0  # ... and those that took it (inputs changed since the last one)
        from ..models.notebook import heartbeat_filter_enabled

        self.heartbeat_fast_path = heartbeat_filter_enabled(self.env)
        # the cache the inputs' versions are read from (see _inputs_token)
        self._reader = reader if reader is not None else getattr(client, "reader", None)
        # uid -> (inputs token, notebook token) of the notebook's last full UPDATE admission
        # whose answer was empty: the stored notebook is the pipeline's fixed point for them
        self._fixed: "OrderedDict[str, tuple]" = OrderedDict()
        self._informers_started: set = set()
        self._informer_tasks: list = []

    # -------------------------------------------------------------- heartbeat fast path

    def _inputs_token(self, nb: dict) -> Optional[tuple]:
        """The versions of everything the pipeline reads besides the Notebook itself, from the
        webhook's cache — no request: the kube-rbac-proxy image, the namespace's three
        ConfigMaps (``odh-trusted-ca-bundle``, ``workbench-trusted-ca-bundle``,
        ``pipeline-runtime-images``), the ImageStreams (runtime images and
        ``last-image-selection``), and, when their features are on, the cluster Proxy and the
        Elyra inputs (DSPA, its S3 Secret, ``ds-pipeline-config``, Gateway, Routes).  ``None``
        when the cache cannot vouch for one of them (not synced yet, or a namespace outside
        a sharded cache): the admission then takes the full pipeline, whose reads start the
        informers the next token needs."""
        r = self._reader
        kind_version = getattr(r, "kind_version", None)
        watching = getattr(r, "watching", None)
        if kind_version is None or watching is None:
            return None
        ns = m.namespace(nb)
        if not watching(kinds.CONFIG_MAP, ns):
            self._start_informer(kinds.CONFIG_MAP)
            return None
        parts: list = [self.kube_rbac_proxy_image]
        for name in (certs.ODH_CONFIGMAP_NAME, certs.WORKBENCH_CA_CONFIGMAP_NAME, runtime_images.RUNTIME_IMAGES_CONFIGMAP):
            o = r.get(kinds.CONFIG_MAP, name, ns)
            parts.append(None if o is None else m.resource_version(o))
        ann = m.annotations(nb)
        if LAST_IMAGE_SELECTION_ANNOTATION in ann:
            image_ns = (ann.get(WORKBENCH_IMAGE_NAMESPACE_ANNOTATION) or "").strip() or self.namespace
            covers = getattr(r, "covers", None)
            if covers is not None and not covers(kinds.IMAGE_STREAM, image_ns):
                return None
        global_kinds = [kinds.IMAGE_STREAM]
        raw = self.env.get("INJECT_CLUSTER_PROXY_ENV")
        if raw is not None and _parse_go_bool(raw):
            global_kinds.append(kinds.PROXY)
        elyra = (self.env.get("SET_PIPELINE_SECRET") or "").strip().lower() == "true"
        if elyra:
            global_kinds += [kinds.DSPA, kinds.GATEWAY, kinds.ROUTE]
        for k in global_kinds:
            v = kind_version(k)
            if v is None:
                return None
            parts.append(v)
        if elyra:
            if not watching(kinds.SECRET, ns):
                self._start_informer(kinds.SECRET)
                return None
            dspa = r.get(kinds.DSPA, dspa_secret.DSPA_INSTANCE_NAME, ns)
            s3 = ((((dspa or {}).get("spec") or {}).get("objectStorage") or {}).get("externalStorage") or {}) \
                .get("s3CredentialsSecret") or {}
            for name in (dspa_secret.ELYRA_SECRET_NAME, s3.get("secretName")):
                o = r.get(kinds.SECRET, name, ns) if name else None
                parts.append(None if o is None else m.resource_version(o))
        return tuple(parts)

    def _start_informer(self, kind) -> None:
        """Start watching ``kind`` (once) so that later tokens can vouch for it: the webhook
        reads ConfigMaps and Secrets live (``odh/main.go:178-185``), so nothing else starts
        their data-stripped informers in a webhook-only process.  In the background: this
        admission does not wait for the list."""
        ensure = getattr(self._reader, "ensure_informer", None)
        if ensure is None or kind in self._informers_started:
            return
        self._informers_started.add(kind)

        async def run():
            try:
                await ensure(kind)
            except Exception as e:  # noqa: BLE001 — the token stays None: full pipeline
                log.info("webhook: cannot watch %s for the heartbeat fast path: %s", kind, e)
        self._informer_tasks.append(asyncio.ensure_future(run()))

    @staticmethod
    def _notebook_token(nb: dict) -> Optional[tuple]:
        """What the pipeline reads of the Notebook: its spec (through ``generation``), its labels
        (the Feast mount follows one) and its annotations other than the culler's heartbeat pair."""
        from ..models.notebook import CULLER_HEARTBEAT_ANNOTATIONS

        md = nb.get("metadata") or {}
        gen = md.get("generation")
        if gen is None:
            return None
        ann = md.get("annotations") or {}
        return (md.get("uid"), gen, tuple(sorted((k, v) for k, v in ann.items()
                                                 if k not in CULLER_HEARTBEAT_ANNOTATIONS)),
                tuple(sorted((md.get("labels") or {}).items())))

    def _heartbeat_settled(self, obj: dict) -> bool:
        """A heartbeat may skip the pipeline iff the notebook is, as stored, the pipeline's
        fixed point for the inputs as they are now: then the reference's full run (which it
        makes on every culler write, ``odh/controllers/notebook_webhook.go:477-490``) would
        answer with an empty patch too.  After any input changed — a new kube-rbac-proxy
        image, a CA bundle or runtime-images ConfigMap edited — the next heartbeat runs the
        pipeline and its restart guard, so ``update-pending`` appears within one culler
        check period, as in the reference."""
        uid = m.uid(obj)
        memo = self._fixed.get(uid) if uid else None
        if memo is None or memo[1] != self._notebook_token(obj):
            return False
        return memo[0] is not None and memo[0] == self._inputs_token(obj)

    def _remember_fixed_point(self, obj: dict, inputs: Optional[tuple]) -> None:
        uid = m.uid(obj)
        tok = self._notebook_token(obj)
        if not uid or inputs is None or tok is None:
            return
        self._fixed[uid] = (inputs, tok)
        self._fixed.move_to_end(uid)
        if len(self._fixed) > self.MEMO_CAP:
            self._fixed.popitem(last=False)

    def forget(self, uid: str) -> None:
        self._fixed.pop(uid, None)

    async def mutate(self, operation: str, nb: dict, old: Optional[dict], name: str = "",
                     namespace: str = "") -> dict:
        """Return the mutated notebook (``nb`` is not modified)."""
        with tracer.start_span("handleFunc", {"notebook": name or m.name(nb), "namespace": namespace or m.namespace(nb),
                                              "operation": operation}, new_root=True):
            original = nb
            if gpu_validation_applies(operation, nb, old):
                validate_gpu_resources(nb)
            nb = deepcopy_json(nb)
            if operation == "CREATE":
                inject_reconciliation_lock(nb)
            if operation in ("CREATE", "UPDATE"):
                prefetch = getattr(self.client, "prefetch", None)
                if prefetch is not None:  # the two ConfigMaps every admission reads, at once
                    ns = m.namespace(nb) or namespace
                    await prefetch([(kinds.CONFIG_MAP, certs.ODH_CONFIGMAP_NAME, ns),
                                    (kinds.CONFIG_MAP, runtime_images.RUNTIME_IMAGES_CONFIGMAP, ns)])
                await set_container_image_from_registry(self.client, nb, self.namespace)
                await certs.check_and_mount_ca_cert_bundle(self.client, nb)
                try:
                    await runtime_images.sync_runtime_images_configmap(self.client, m.namespace(nb), self.namespace)
                except Exception as e:  # degrade: mount whatever exists
                    log.error("failed to sync runtime images ConfigMap: %s", e)
                await runtime_images.mount_pipeline_runtime_images(self.client, nb)
                if (self.env.get("SET_PIPELINE_SECRET") or "").strip().lower() == "true":
                    try:
                        await dspa_secret.sync_elyra_runtime_config_secret(self.client, nb)
                    except Exception as e:
                        log.error("failed to sync Elyra runtime config secret: %s", e)
                    await dspa_secret.mount_elyra_runtime_config_secret(self.client, nb)
                if feast.is_feast_enabled(nb):
                    try:
                        feast.new_feast_config(nb)
                    except ValueError as e:
                        log.info("unable to mount Feast config volume: %s", e)
                elif feast.is_feast_mounted(nb):
                    feast.unmount_feast_config(nb)
            if auth.kube_rbac_proxy_injection_enabled(nb):
                try:
                    auth.inject_kube_rbac_proxy(nb, self.kube_rbac_proxy_image)
                except auth.SidecarResourceError as e:
                    raise AdmissionError(500, f"invalid kube-rbac-proxy resource configuration: {e}")
            raw = self.env.get("INJECT_CLUSTER_PROXY_ENV")
            if raw is not None and _parse_go_bool(raw):
                vals = await cluster_proxy_env(self.client)
                if vals:
                    inject_proxy_config_env_vars(nb, vals)
            nb, reason = self.maybe_restart_running_notebook(operation, original, nb, old)
            ann = m.ensure_annotations(nb)
            if reason:
                ann[ANNOTATION_UPDATE_PENDING] = reason
            else:
                ann.pop(ANNOTATION_UPDATE_PENDING, None)
            return nb

    def maybe_restart_running_notebook(self, operation: str, updated: dict, mutated: dict,
                                       old: Optional[dict]) -> Tuple[dict, str]:
        """``maybeRestartRunningNotebook`` (:505-564)."""
        with tracer.start_span("maybeRestartRunningNotebook"):
            if operation == "CREATE":
                return mutated, ""
            if m.has_annotation(mutated, STOP_ANNOTATION) or m.has_annotation(mutated, ANNOTATION_NOTEBOOK_RESTART):
                return mutated, ""
            if old is None:
                return mutated, ""

            def tmpl(o):
                return (((o or {}).get("spec") or {}).get("template") or {}).get("spec") or {}

            if not semantic_equal(tmpl(old), tmpl(updated)):
                return mutated, ""  # the user's change already restarts the pod
            if semantic_equal(tmpl(old), tmpl(mutated)):
                return mutated, ""
            diff = first_difference(tmpl(mutated), tmpl(updated))
            log.info("update blocked, webhook would change the pod template of a running notebook: %s", diff)
            mutated["spec"]["template"]["spec"] = deepcopy_json(tmpl(updated))
            return mutated, diff or "failed to compute the reason for why there is a pending restart"

    # -------------------------------------------------------------- AdmissionReview v1

    async def handle(self, review: dict) -> dict:
        """AdmissionReview v1 request → AdmissionReview response with a JSONPatch."""
        self.requests += 1
        req = review.get("request") if isinstance(review, dict) else None
        if not isinstance(req, dict):  # not an AdmissionReview: deny, never raise
            self.denied += 1
            return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                    "response": {"uid": "", "allowed": False,
                                 "status": {"code": 400, "message": "request is not an AdmissionReview"}}}
        uid = req.get("uid", "") if isinstance(req.get("uid", ""), str) else ""
        resp = {"uid": uid, "allowed": True}
        try:
            obj = req.get("object")
            if not isinstance(obj, dict):
                raise AdmissionError(400, "there is no content to decode")
            old = req.get("oldObject") if isinstance(req.get("oldObject"), dict) else None
            # the culler's heartbeat first, before the shape check: the object is the stored
            # (admitted, schema-valid) old one but for two annotations, so it decodes iff their
            # values are strings — the one check left at 1000 heartbeats a second
            op = req.get("operation", "")
            beat = op == "UPDATE" and self.heartbeat_fast_path and heartbeat_update(obj, old)
            if beat and self._heartbeat_settled(obj):
                self.heartbeats += 1
                return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}
            if beat:
                self.heartbeats_full += 1
            bad = undecodable(obj)
            if bad:  # the reference's typed decode (admission.Decoder) refuses these
                raise AdmissionError(400, f"cannot decode Notebook: {bad}")
            inputs = self._inputs_token(obj) if op == "UPDATE" and self.heartbeat_fast_path else None
            tok = CONFIRM_ABSENCE.set(set())  # one-shot decision: absent objects are confirmed live, once
            try:
                mutated = await self.mutate(op, obj, old, req.get("name", ""), req.get("namespace", ""))
            finally:
                CONFIRM_ABSENCE.reset(tok)
            ops = jsonpatch.create_patch(obj, mutated)
            if ops:
                resp["patchType"] = "JSONPatch"
                resp["patch"] = base64.b64encode(dumps_json(ops)).decode()
            elif inputs is not None:
                self._remember_fixed_point(obj, inputs)
        except AdmissionError as e:
            self.denied += 1
            resp = {"uid": uid, "allowed": False, "status": {"code": e.code, "message": str(e)}}
        except ApiError as e:
            self.denied += 1
            resp = {"uid": uid, "allowed": False, "status": {"code": 500, "message": str(e)}}
        return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}


def heartbeat_update(obj: dict, old: Optional[dict]) -> bool:
    """:func:`culler_heartbeat_only` for an object not yet shape-checked: any shape it cannot
    read, or a heartbeat annotation that is not a string, is not a heartbeat (the full path,
    shape check first, answers it)."""
    from ..models.notebook import CULLER_HEARTBEAT_ANNOTATIONS

    try:
        if not culler_heartbeat_only(obj, old):
            return False
        ann = obj["metadata"]["annotations"]
        return isinstance(ann, dict) and all(isinstance(ann[k], str) for k in CULLER_HEARTBEAT_ANNOTATIONS if k in ann)
    except (AttributeError, KeyError, TypeError):
        return False


def undecodable(obj: dict) -> Optional[str]:
    """Where ``obj`` does not have the Notebook's JSON shape along the paths the webhook
    reads (the Go webhook decodes into ``nbv1.Notebook`` first and answers 400 on a type
    mismatch); ``None`` when it does."""
    def is_map(v, of_str=False):
        return v is None or (isinstance(v, dict) and (not of_str or all(isinstance(x, str) for x in v.values())))

    def is_list_of_maps(v):
        return v is None or (isinstance(v, list) and all(isinstance(x, dict) for x in v))

    md = obj.get("metadata")
    if not is_map(md):
        return "metadata"
    for k in ("annotations", "labels"):
        if not is_map((md or {}).get(k), of_str=True):
            return f"metadata.{k}"
    if not isinstance((md or {}).get("name", ""), str) or not isinstance((md or {}).get("namespace", ""), str):
        return "metadata.name"
    spec = obj.get("spec")
    if not is_map(spec):
        return "spec"
    tmpl = (spec or {}).get("template")
    if not is_map(tmpl):
        return "spec.template"
    ps = (tmpl or {}).get("spec")
    if not is_map(ps):
        return "spec.template.spec"
    for k in ("containers", "initContainers", "volumes", "imagePullSecrets", "tolerations"):
        if not is_list_of_maps((ps or {}).get(k)):
            return f"spec.template.spec.{k}"
    for i, c in enumerate((ps or {}).get("containers") or []):
        for k in ("env", "volumeMounts", "ports", "envFrom"):
            if not is_list_of_maps(c.get(k)):
                return f"spec.template.spec.containers[{i}].{k}"
        res = c.get("resources")
        if not is_map(res) or not all(is_map(v) for v in (res or {}).values()):
            return f"spec.template.spec.containers[{i}].resources"
        if not isinstance(c.get("name", ""), str) or not isinstance(c.get("image", ""), str):
            return f"spec.template.spec.containers[{i}].name"
    return None


def matches(info, operation: str) -> bool:
    """``rules: kubeflow.org/v1 notebooks CREATE,UPDATE`` (config/webhook/manifests.yaml)."""
    return info.key == "notebooks.kubeflow.org" and operation in ("CREATE", "UPDATE")


# The configuration's matchConditions: the apiserver does not call the webhook for a Notebook
# that is being deleted.  Its last writes (the controllers' finalizer removals) have nothing to
# inject into a pod template that is going away: one admission round trip fewer on every
# deletion.  The reference's configuration has none (odh/config/webhook/manifests.yaml), so its
# webhook runs the whole pipeline on those writes too.  A terminating Notebook is never
# validated either (gpu_validation_applies).
MATCH_CONDITIONS = [{"name": "not-terminating", "expression": "!has(object.metadata.deletionTimestamp)"}]


def register_in_process(store, webhook: NotebookWebhook, name: str = "notebooks.opendatahub.io") -> None:
    """Install the webhook as a mutating admission plugin of the in-process apiserver.

    The store calls it exactly like the apiserver calls the HTTPS endpoint: an
    AdmissionReview in, a JSONPatch out (applied to the request object); a denial
    fails the write (``failurePolicy: Fail``).
    """
    import uuid

    from ..models.errors import InternalError

    from ..utils.celmatch import compile_condition, conditions_allow

    conds = [compile_condition(c["expression"]) for c in MATCH_CONDITIONS]

    async def handler(op, info, obj, old):
        if not conditions_allow(conds, obj, old, fail_closed=True):
            return obj
        review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                  "request": {"uid": str(uuid.uuid4()), "operation": op, "name": m.name(obj),
                              "namespace": m.namespace(obj), "object": obj, "oldObject": old,
                              "kind": {"group": info.group, "version": "v1", "kind": info.kind},
                              "resource": {"group": info.group, "version": "v1", "resource": info.plural}}}
        out = (await webhook.handle(review))["response"]
        if not out.get("allowed"):
            st = out.get("status") or {}
            raise InternalError(f'admission webhook "{name}" denied the request: {st.get("message", "")}')
        if out.get("patch"):
            ops = json.loads(base64.b64decode(out["patch"]))
            obj = jsonpatch.apply_patch(obj, ops)
        return obj

    store.add_mutating_admission(name, matches, handler)
