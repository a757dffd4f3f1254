"""Core Notebook reconciler — the upstream Kubeflow notebook controller
(``kf/controllers/notebook_controller.go``), re-built for an 8×MI355X node.

Per reconcile of a Notebook (reference ``Reconcile`` :93-297):

1. skip objects being deleted (:138-140);
2. generate the StatefulSet (``generate_statefulset``, :433-523) — replicas 0 while the
   ``kubeflow-resource-stopped`` annotation is present (the culler's STOP and the odh
   reconciliation lock share it), ``generateName: nb-`` for names > 52 chars;
3. find the StatefulSet **through the owner-UID index** instead of listing every
   StatefulSet in the namespace (:157-170), create it or copy owned fields onto it;
4. reconcile the Service (port 80 → first container port) and, with ``USE_ISTIO=true``,
   the Istio VirtualService (:558-699);
5. mirror pod ``<sts>-0`` into ``status`` — written **only when it changed
   semantically** (the reference writes it unconditionally every pass, :299-313, and
   its ``metav1.Now()`` stamping makes every pass a new write that re-triggers both
   controllers);
6. honour ``notebooks.opendatahub.io/notebook-restart`` by deleting the pod (:262-294).

``amd.com/gpu`` requests/limits pass through verbatim; with ``GPU_NODE_SELECTOR=true``
pods that request GPUs also get the AMD node-labeller selector and the
``amd.com/gpu`` toleration so they land on MI355X nodes.  With
``GPU_SHM_SIZE_PER_GPU`` (e.g. ``16Gi``) a GPU notebook without its own ``/dev/shm``
gets a memory-backed one of that size per GPU: PyTorch DataLoader workers and RCCL's
intra-node transport live there, and the container default (64 MiB) breaks both.  The
``amd.com/shm-size`` annotation overrides the size (``0`` turns it off).  With
``amd.com/gpu-probe: "true"`` on the Notebook (or ``GPU_STARTUP_PROBE=true`` for every GPU
notebook) the pod gets the ``amd-gpu-probe`` init container: the MI355X start-up probe
(``odh-gpu-probe``, ``GPU_PROBE_IMAGE``) on the GPUs the device plugin gives it, before the
notebook container starts.

Event re-emission (:97-126) runs as its own small controller
(:class:`NotebookEventReemitter`) instead of sharing the Notebook work queue — the
TODO at :96 of the reference.
"""

from __future__ import annotations

import json
import logging
import os
import re
from typing import List, Mapping, Optional, Tuple

from ..models import kinds
from ..models import meta as m
from ..models.errors import ApiError, is_already_exists, is_not_found
from ..models.scheme import SCHEME
from ..models.notebook import (ANNOTATION_HEADERS_REQUEST_SET, ANNOTATION_NOTEBOOK_RESTART, ANNOTATION_REWRITE_URI,
                               CULLER_HEARTBEAT_ANNOTATIONS, DEFAULT_CONTAINER_PORT, DEFAULT_FS_GROUP,
                               DEFAULT_SERVING_PORT, GPU_RESOURCE, MAX_STATEFULSET_NAME_LENGTH, NOTEBOOK_NAME_LABEL,
                               PREFIX_ENV_VAR, STATEFULSET_LABEL, STOP_ANNOTATION, WORKBENCH_LABEL, gpu_request,
                               heartbeat_filter_enabled, pod_cond_to_notebook_cond)
from ..runtime.controller import Request, Result, controller_owner_alive, fields_changed, maps_differ, pred_funcs
from ..utils.objutil import deepcopy_json, semantic_equal
from ..utils.reconcilehelper import copy_service_fields, copy_statefulset_fields, copy_virtual_service

log = logging.getLogger("controllers.Notebook")

NOTEBOOK_KIND = kinds.NOTEBOOK_V1BETA1  # the kf controller works on the hub version (notebook_controller.go:31)


# ------------------------------------------------------------------ generators


def set_prefix_env_var(nb: dict, container: dict) -> None:
    """``setPrefixEnvVar`` (:417-431).

    The reference assigns to the range-loop copy, so an existing ``NB_PREFIX`` keeps
    its user-provided value; that observable behaviour is preserved.
    """
    prefix = f"/notebook/{m.namespace(nb)}/{m.name(nb)}"
    env = container.setdefault("env", [])
    for e in env:
        if e.get("name") == PREFIX_ENV_VAR:
            return
    env.append({"name": PREFIX_ENV_VAR, "value": prefix})


def _gpu_placement(pod_spec: dict) -> None:
    """MI355X placement: node-labeller selector + toleration for pods requesting amd.com/gpu."""
    if gpu_request(pod_spec) <= 0:
        return
    sel = pod_spec.setdefault("nodeSelector", {})
    sel.setdefault("amd.com/gpu.family", "AI")
    tol = pod_spec.setdefault("tolerations", [])
    if not any(t.get("key") == GPU_RESOURCE for t in tol):
        tol.append({"key": GPU_RESOURCE, "operator": "Exists", "effect": "NoSchedule"})


SHM_SIZE_ANNOTATION = "amd.com/shm-size"
SHM_VOLUME = "dshm"
_SIZE_RE = re.compile(r"^\s*(\d+)\s*([KMGT]i)?\s*$")


def _gpu_shm(nb: dict, pod_spec: dict, per_gpu: str) -> None:
    """Memory-backed ``/dev/shm`` sized per GPU for notebooks that request ``amd.com/gpu``."""
    ngpu = gpu_request(pod_spec)
    containers = pod_spec.get("containers") or []
    if ngpu <= 0 or not containers:
        return
    size = (m.annotations(nb).get(SHM_SIZE_ANNOTATION) or "").strip()
    if not size:
        mm = _SIZE_RE.match(per_gpu or "")
        if not mm:
            return
        size = f"{int(mm.group(1)) * ngpu}{mm.group(2) or ''}"
    if size in ("0", "none", "off"):
        return
    if any(vm.get("mountPath") == "/dev/shm" for c in containers for vm in c.get("volumeMounts") or []):
        return  # the user sized it already
    vols = pod_spec.setdefault("volumes", [])
    if any(v.get("name") == SHM_VOLUME for v in vols):
        return
    vols.append({"name": SHM_VOLUME, "emptyDir": {"medium": "Memory", "sizeLimit": size}})
    containers[0].setdefault("volumeMounts", []).append({"name": SHM_VOLUME, "mountPath": "/dev/shm"})


def parse_env_pairs(raw: str) -> List[Tuple[str, str]]:
    """``"K1=v1,K2=v2"`` → [(K1, v1), (K2, v2)] (blank and malformed entries skipped)."""
    out = []
    for item in (raw or "").split(","):
        k, sep, v = item.strip().partition("=")
        if sep and k.strip():
            out.append((k.strip(), v.strip()))
    return out


def _multi_gpu_env(pod_spec: dict, raw: str) -> None:
    """Collective-library environment defaults (``MULTI_GPU_ENV``) for notebooks that request
    2+ ``amd.com/gpu``: their RCCL collectives run over the node's xGMI links, and the
    settings that path needs on a given fleet (e.g. dmabuf-only IPC hosts) are set once by
    the operator instead of in every notebook.  A variable the user already set wins."""
    containers = pod_spec.get("containers") or []
    if gpu_request(pod_spec) < 2 or not containers:
        return
    env = containers[0].setdefault("env", [])
    have = {e.get("name") for e in env}
    for k, v in parse_env_pairs(raw):
        if k not in have:
            env.append({"name": k, "value": v})
            have.add(k)


def parse_gids(raw: str) -> List[int]:
    """``GPU_DEVICE_GROUPS``: ``"44,110"`` (or ``"video=44,render=110"``) → [44, 110]; entries
    that are not non-negative integers are skipped."""
    out: List[int] = []
    for item in (raw or "").split(","):
        v = item.strip().rpartition("=")[2].strip()
        if v.isdigit() and int(v) not in out:
            out.append(int(v))
    return out


def _gpu_device_groups(pod_spec: dict, raw: str) -> None:
    """The device plugin hands ``/dev/kfd`` and ``/dev/dri/renderD*`` to the container with the
    host's owner and mode — typically ``root:render 0660`` (the ``video`` group on older
    hosts).  A container running as a non-root user (the probe as 65532, notebook images as
    1000) opens them only as a member of that group, so pods that request ``amd.com/gpu`` get
    the operator's ``GPU_DEVICE_GROUPS`` as ``securityContext.supplementalGroups`` (they apply
    to every container of the pod, init containers included).  A value the user set wins."""
    gids = parse_gids(raw)
    if not gids or gpu_request(pod_spec) <= 0:
        return
    sc = pod_spec.get("securityContext")
    if sc is None:
        sc = pod_spec["securityContext"] = {}
    if sc.get("supplementalGroups") is None:
        sc["supplementalGroups"] = gids


GPU_PROBE_ANNOTATION = "amd.com/gpu-probe"
GPU_PROBE_CONTAINER = "amd-gpu-probe"
DEFAULT_GPU_PROBE_IMAGE = "quay.io/opendatahub/odh-kubeflow-amd-gpu-probe:main"  # manifests pin the release
GPU_PROBE_TIMEOUT_MS = "30000"
GPU_PROBE_RCCL_MIB = "64"  # all-reduce size of the RCCL step (annotation value "rccl")


def gpu_probe_enabled(nb: dict, pod_spec: dict, env: Mapping[str, str] = os.environ) -> bool:
    """The MI355X start-up probe runs for notebooks that request ``amd.com/gpu`` when the
    Notebook says ``amd.com/gpu-probe: "true"`` (or ``"rccl"``), or when the operator turned
    it on for every GPU notebook (``GPU_STARTUP_PROBE=true``) and the Notebook does not say
    ``"false"``.  Off by default (never on the reconcile path, opt-in)."""
    if gpu_request(pod_spec) <= 0:
        return False
    v = (m.annotations(nb).get(GPU_PROBE_ANNOTATION) or "").strip().lower()
    if v in ("true", "rccl", "false"):
        return v != "false"
    return env.get("GPU_STARTUP_PROBE", "false") == "true"


def gpu_probe_rccl(nb: dict, ngpu: int, env: Mapping[str, str] = os.environ) -> bool:
    """Whether the probe also runs its RCCL all-reduce over the pod's GPUs (SURVEY §7.0.4's
    collective readiness check): ``amd.com/gpu-probe: "rccl"``, or ``GPU_PROBE_RCCL=true`` for
    every probed notebook with 2+ GPUs (a single GPU has nothing to all-reduce with)."""
    v = (m.annotations(nb).get(GPU_PROBE_ANNOTATION) or "").strip().lower()
    return v == "rccl" or (ngpu >= 2 and env.get("GPU_PROBE_RCCL", "false") == "true")


def gpu_probe_init_container(ngpu: int, env: Mapping[str, str] = os.environ, rccl: bool = False) -> dict:
    """Init container that proves the pod's GPUs healthy before the notebook starts.

    ``odh-gpu-probe`` (``ops/csrc/probe_cli.cpp``, torch-free) runs the bf16 MFMA GEMM checked
    in registers and the HBM3E pattern sweep on every GPU the device plugin gives the pod, and
    with 2+ GPUs reads the xGMI ring between them (``rccl``: plus an RCCL all-reduce over all
    of them, ``--rccl-mib``); non-zero exit keeps the pod in Init, and its
    JSON verdict is the container's termination message.  It asks for the same
    ``amd.com/gpu`` count as the notebook: the kubelet device manager hands an init
    container's devices on to the app containers, so the GPUs probed are the GPUs the
    notebook gets, and the pod's effective request (max of init and app) does not grow."""
    n = str(ngpu)
    args = ["--json", "/dev/termination-log", "--timeout-ms", env.get("GPU_PROBE_TIMEOUT_MS") or GPU_PROBE_TIMEOUT_MS]
    if rccl:
        args += ["--rccl-mib", GPU_PROBE_RCCL_MIB]
    return {
        "name": GPU_PROBE_CONTAINER,
        "image": env.get("GPU_PROBE_IMAGE") or DEFAULT_GPU_PROBE_IMAGE,
        "command": ["odh-gpu-probe"],
        "args": args,
        "resources": {"limits": {GPU_RESOURCE: n, "cpu": "1", "memory": "2Gi"},
                      "requests": {GPU_RESOURCE: n, "cpu": "100m", "memory": "256Mi"}},
        "terminationMessagePolicy": "FallbackToLogsOnError",
        "securityContext": {"allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}},
    }


def _gpu_probe(nb: dict, pod_spec: dict, env: Mapping[str, str]) -> None:
    if not gpu_probe_enabled(nb, pod_spec, env):
        return
    inits = pod_spec.setdefault("initContainers", [])
    if any(c.get("name") == GPU_PROBE_CONTAINER for c in inits):
        return  # the user brought their own
    n = gpu_request(pod_spec)
    # before any init container that uses the GPU
    inits.insert(0, gpu_probe_init_container(n, env, rccl=gpu_probe_rccl(nb, n, env)))


def generate_statefulset(nb: dict, is_generate_name: bool, env: Mapping[str, str] = os.environ) -> dict:
    """``generateStatefulSet`` (:433-523)."""
    name, ns = m.name(nb), m.namespace(nb)
    replicas = 0 if m.has_annotation(nb, STOP_ANNOTATION) else 1
    if is_generate_name:
        md = {"generateName": "nb-", "namespace": ns}
    else:
        md = {"name": name, "namespace": ns, "labels": {}}
    pod_spec = deepcopy_json((((nb.get("spec") or {}).get("template") or {}).get("spec")) or {})
    tmpl_labels = {STATEFULSET_LABEL: name, NOTEBOOK_NAME_LABEL: name, WORKBENCH_LABEL: "true"}
    nb_labels = m.labels(nb)
    if nb_labels:
        md.setdefault("labels", {}).update(nb_labels)
        tmpl_labels.update(nb_labels)
    tmpl_ann = {k: v for k, v in m.annotations(nb).items() if "kubectl" not in k and "notebook" not in k}
    sts = {
        "apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": md,
        "spec": {
            "replicas": replicas,
            "selector": {"matchLabels": {STATEFULSET_LABEL: name}},
            "template": {"metadata": {"labels": tmpl_labels, "annotations": tmpl_ann}, "spec": pod_spec},
        },
    }
    containers = pod_spec.get("containers") or []
    if containers:
        c = containers[0]
        if not c.get("workingDir"):
            c["workingDir"] = "/home/jovyan"
        if c.get("ports") is None:
            c["ports"] = [{"containerPort": DEFAULT_CONTAINER_PORT, "name": "notebook-port", "protocol": "TCP"}]
        set_prefix_env_var(nb, c)
    add_fs = env.get("ADD_FSGROUP")
    if add_fs is None or add_fs == "true":
        if pod_spec.get("securityContext") is None:
            pod_spec["securityContext"] = {"fsGroup": DEFAULT_FS_GROUP}
    if env.get("GPU_NODE_SELECTOR", "false") == "true":
        _gpu_placement(pod_spec)
    if env.get("GPU_SHM_SIZE_PER_GPU"):
        _gpu_shm(nb, pod_spec, env["GPU_SHM_SIZE_PER_GPU"])
    if env.get("MULTI_GPU_ENV"):
        _multi_gpu_env(pod_spec, env["MULTI_GPU_ENV"])
    if env.get("GPU_DEVICE_GROUPS"):
        _gpu_device_groups(pod_spec, env["GPU_DEVICE_GROUPS"])
    _gpu_probe(nb, pod_spec, env)
    return sts


def generate_service(nb: dict) -> dict:
    """``generateService`` (:525-552): ClusterIP, ``http-notebook`` port 80 → container port."""
    port = DEFAULT_CONTAINER_PORT
    containers = ((((nb.get("spec") or {}).get("template") or {}).get("spec")) or {}).get("containers") or []
    if containers and containers[0].get("ports") is not None:
        ports = containers[0]["ports"]
        if ports:
            port = int(ports[0].get("containerPort", DEFAULT_CONTAINER_PORT))
    return {
        "apiVersion": "v1", "kind": "Service",
        "metadata": {"name": m.name(nb), "namespace": m.namespace(nb)},
        "spec": {
            "type": "ClusterIP",
            "selector": {STATEFULSET_LABEL: m.name(nb)},
            "ports": [{"name": "http-notebook", "port": DEFAULT_SERVING_PORT, "targetPort": port, "protocol": "TCP"}],
        },
    }


def virtual_service_name(nb_name: str, namespace: str) -> str:
    return f"notebook-{namespace}-{nb_name}"


def generate_virtual_service(nb: dict, env: Mapping[str, str] = os.environ) -> dict:
    """``generateVirtualService`` (:558-658)."""
    name, ns = m.name(nb), m.namespace(nb)
    prefix = f"/notebook/{ns}/{name}/"
    ann = m.annotations(nb)
    rewrite = ann.get(ANNOTATION_REWRITE_URI) or prefix
    domain = env.get("CLUSTER_DOMAIN", "cluster.local") if "CLUSTER_DOMAIN" in env else "cluster.local"
    service = f"{name}.{ns}.svc.{domain}"
    headers = {}
    raw = ann.get(ANNOTATION_HEADERS_REQUEST_SET)
    if raw:
        # json.Unmarshal into map[string]string (:605-613): a number or an object value is a
        # type error and the whole map falls back to {}; a null value is the zero string
        try:
            parsed = json.loads(raw)
        except ValueError:
            parsed = None
        if isinstance(parsed, dict) and all(v is None or isinstance(v, str) for v in parsed.values()):
            headers = {k: "" if v is None else v for k, v in parsed.items()}
    return {
        "apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService",
        "metadata": {"name": virtual_service_name(name, ns), "namespace": ns},
        "spec": {
            "hosts": [env.get("ISTIO_HOST") or "*"],
            "gateways": [env.get("ISTIO_GATEWAY") or "kubeflow/kubeflow-gateway"],
            "http": [{
                "headers": {"request": {"set": headers}},
                "match": [{"uri": {"prefix": prefix}}],
                "rewrite": {"uri": rewrite},
                "route": [{"destination": {"host": service, "port": {"number": DEFAULT_SERVING_PORT}}}],
            }],
        },
    }


# ------------------------------------------------------------------ status


def create_notebook_status(nb: dict, sts: Optional[dict], pod: Optional[dict], now: Optional[str] = None) -> dict:
    """``createNotebookStatus`` (:315-374)."""
    status = {"conditions": [], "readyReplicas": int(((sts or {}).get("status") or {}).get("readyReplicas", 0) or 0),
              "containerState": {}}
    pst = (pod or {}).get("status") or {}
    if not pst:
        return status
    cur_state = ((nb.get("status") or {}).get("containerState")) or {}
    for cs in pst.get("containerStatuses") or []:
        if cs.get("name") != m.name(nb):
            continue
        state = cs.get("state") or {}
        if not state and not cur_state:
            continue
        status["containerState"] = deepcopy_json(state)
        break
    status["conditions"] = [pod_cond_to_notebook_cond(c, now) for c in pst.get("conditions") or []]
    return status


def notebook_status_ready(status: dict) -> bool:
    """readyReplicas ≥ 1 and a ``Ready=True`` condition mirrored from the pod."""
    return bool((status or {}).get("readyReplicas")) and any(
        c.get("type") == "Ready" and c.get("status") == "True" for c in (status or {}).get("conditions") or [])


def _cond_key(c: dict):
    return (c.get("type"), c.get("status"), c.get("reason"), c.get("message"))


def status_equal(a: Optional[dict], b: Optional[dict]) -> bool:
    """Two Notebook statuses say the same: absent, ``null``, ``0`` replicas, ``[]`` conditions
    and ``{}`` containerState are one zero value (Go's ``NotebookStatus{}``).  A new Notebook's
    first pass — StatefulSet created, no pod yet — computes exactly that zero value, and
    writing it would be a status write (and an event in every Notebook watcher) that tells no
    reader anything; the first write is the one that carries the pod's state."""
    def norm(s):
        s = dict(s or {})
        s["readyReplicas"] = int(s.get("readyReplicas") or 0)
        return s
    return semantic_equal(norm(a), norm(b))


def merge_status_timestamps(old: dict, new: dict) -> dict:
    """Keep the previous probe/transition stamps for conditions that did not change, so a
    pod condition without timestamps does not turn every reconcile into a status write."""
    prev = {_cond_key(c): c for c in (old or {}).get("conditions") or []}
    for c in new.get("conditions") or []:
        p = prev.get(_cond_key(c))
        if p is not None:
            for f in ("lastProbeTime", "lastTransitionTime"):
                if p.get(f):
                    c[f] = p[f]
    return new


# ------------------------------------------------------------------ reconciler


class NotebookReconciler:
    def __init__(self, client, reader, recorder, metrics=None, env: Optional[Mapping[str, str]] = None,
                 unconditional_status: bool = False, owner_index: bool = True, event_filters: bool = True):
        self.client = client
        self.reader = reader
        self.recorder = recorder
        self.metrics = metrics
        self.env = env if env is not None else os.environ
        self.unconditional_status = unconditional_status  # reference-emulation knob
        self.owner_index = owner_index
        self.event_filters = event_filters  # False: reconcile on every event, as the reference
        self.status_writes = 0

    async def _find_statefulset(self, nb: dict, ns: str) -> Optional[dict]:
        if self.owner_index:
            items = await self.client.list(kinds.STATEFUL_SET, ns, owner_uid=m.uid(nb))
        else:
            items = await self.client.list(kinds.STATEFUL_SET, ns)
        for sts in items:
            if m.is_controlled_by(sts, nb):
                return sts
        return None

    async def reconcile(self, req: Request) -> Result:
        try:
            nb = await self.client.get(NOTEBOOK_KIND, req.name, req.namespace)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            raise
        if m.is_deleting(nb):
            return Result()

        is_generate_name = len(m.name(nb)) > MAX_STATEFULSET_NAME_LENGTH
        ss = generate_statefulset(nb, is_generate_name, self.env)
        m.set_controller_reference(nb, ss)
        found = await self._find_statefulset(nb, req.namespace)
        just_created = False
        if found is None:
            if self.metrics:
                self.metrics.notebook_creation.labels(req.namespace).inc()
            try:
                found = await self.client.create(ss)
            except ApiError:
                if self.metrics:
                    self.metrics.notebook_fail_creation.labels(req.namespace).inc()
                raise
            just_created = True
        # pod template labels follow when the replica count changes (:188-194)
        if ss["spec"]["replicas"] != (found.get("spec") or {}).get("replicas"):
            ftmpl = found["spec"].setdefault("template", {}).setdefault("metadata", {})
            if ftmpl.get("labels") != ss["spec"]["template"]["metadata"]["labels"]:
                ftmpl["labels"] = deepcopy_json(ss["spec"]["template"]["metadata"]["labels"])
        if not just_created:
            if is_generate_name:
                # desired object has no name; keep the live identity
                ss["metadata"]["name"] = m.name(found)
            if copy_statefulset_fields(ss, found):
                found = await self.client.update(found)

        svc = generate_service(nb)
        m.set_controller_reference(nb, svc)
        try:
            found_svc = await self.client.get(kinds.SERVICE, m.name(svc), req.namespace)
            if copy_service_fields(svc, found_svc):
                await self.client.update(found_svc)
        except ApiError as e:
            if not is_not_found(e):
                raise
            try:
                await self.client.create(svc)
            except ApiError as e2:
                if not is_already_exists(e2):
                    raise

        if self.env.get("USE_ISTIO") == "true":
            await self.reconcile_virtual_service(nb)

        pod = await self.client.get_or_none(kinds.POD, f"{m.name(found)}-0", req.namespace)

        status = create_notebook_status(nb, found, pod)
        old_status = nb.get("status") or {}
        if self.metrics is not None and notebook_status_ready(status) and not notebook_status_ready(old_status):
            self.metrics.observe_ready(nb, pod)
        if self.unconditional_status:
            nb["status"] = status
            self.status_writes += 1
            await self.client.update_status(nb)
        else:
            merge_status_timestamps(old_status, status)
            if not status_equal(status, old_status):
                # The whole status is recomputed from the pod each pass, so it is written as a
                # JSON-patch replacement without a resourceVersion precondition: a concurrent
                # metadata write (odh lock removal, culler annotations) cannot turn it into a
                # 409 + requeue the way the reference's Status().Update does.
                self.status_writes += 1
                await self.client.patch(nb, [{"op": "add", "path": "/status", "value": status}], "json",
                                        subresource="status")

        ann = m.annotations(nb)
        if ann.get(ANNOTATION_NOTEBOOK_RESTART) == "true":
            log.info("restart annotation set on %s", req)
            pod = await self.client.get_or_none(kinds.POD, f"{m.name(nb)}-0", req.namespace)
            if pod is not None:
                try:
                    await self.client.delete(pod)
                except ApiError as e:
                    if not is_not_found(e):
                        raise
            m.ensure_annotations(nb).pop(ANNOTATION_NOTEBOOK_RESTART, None)
            await self.client.update(nb)
        return Result()

    async def reconcile_virtual_service(self, nb: dict) -> None:
        vs = generate_virtual_service(nb, self.env)
        m.set_controller_reference(nb, vs)
        found = await self.client.get_or_none(kinds.VIRTUAL_SERVICE, m.name(vs), m.namespace(nb))
        if found is None:
            await self.client.create(vs)
            return
        if copy_virtual_service(vs, found):
            await self.client.update(found)

    # -------------------------------------------------------------- wiring

    def setup_with_manager(self, mgr, max_concurrent: Optional[int] = None):
        """``SetupWithManager`` (:778-826): For Notebook, Owns STS/Service, Pods by label.

        The reference registers these watches without predicates, so every status write,
        finalizer edit and child deletion queues a reconcile that finds nothing to do.
        With ``event_filters`` each watch passes only the changes the reconcile reads:

        * Notebook — spec (generation), labels, annotations (stop/restart/lock), creation;
          not its own status writes, odh's finalizer edits, the culler's activity heartbeat
          (``last-activity`` / ``last_activity_check_timestamp``, rewritten every check of
          every running notebook), or deletion (nothing to do on a deleting Notebook,
          :138-140; GC removes the children);
        * StatefulSet — spec/metadata drift and ``status.readyReplicas`` (the only STS
          status the Notebook status mirrors, :301-312); deletion only while its Notebook
          is alive (drift → recreate);
        * Service — the Notebook's own Service (name == Notebook name, :525-552), spec or
          metadata drift; not odh's ``<nb>-kube-rbac-proxy`` Service it also controls;
        * Pod — conditions / container statuses (what ``createNotebookStatus`` copies,
          :315-374) and label moves; deletion only while the Notebook is alive.
        """

        def map_pod(pod: dict):
            return [Request(m.namespace(pod), m.labels(pod)[NOTEBOOK_NAME_LABEL])]

        def pod_is_labeled(etype, obj, old):
            return NOTEBOOK_NAME_LABEL in m.labels(obj)

        nb_preds, sts_preds, svc_preds, pod_preds = [], [], [], [pod_is_labeled]
        if self.event_filters:
            reader = self.reader
            drift = ("spec", "metadata.labels", "metadata.annotations", "metadata.ownerReferences")
            nb_changed = fields_changed("metadata.generation", "metadata.labels")

            def nb_update(o, old):
                if m.is_deleting(o):
                    return False
                if nb_changed("MODIFIED", o, old):
                    return True
                # the culler's per-check heartbeat alone changes nothing this reconcile
                # reads or generates (the STS template never carries "notebook" keys, :488)
                return maps_differ(m.annotations(old), m.annotations(o), ignore)
            ignore = CULLER_HEARTBEAT_ANNOTATIONS if heartbeat_filter_enabled(self.env) else frozenset()
            nb_preds = [pred_funcs(update=nb_update, delete=lambda o: False)]
            sts_drift = fields_changed(*drift)

            def sts_changed(etype, sts, old):
                if etype != "MODIFIED" or old is None or sts_drift(etype, sts, old):
                    return True
                ready = lambda o: int(((o.get("status") or {}).get("readyReplicas")) or 0)  # noqa: E731
                return ready(sts) != ready(old)
            sts_preds = [sts_changed, controller_owner_alive(reader, NOTEBOOK_KIND)]

            def own_service(etype, svc, old):
                for r in (svc.get("metadata") or {}).get("ownerReferences") or []:
                    if r.get("controller"):
                        return r.get("name") == m.name(svc)
                return False
            svc_preds = [own_service, fields_changed(*drift), controller_owner_alive(reader, NOTEBOOK_KIND)]

            def pod_nb_alive(etype, pod, old):
                if etype != "DELETED":
                    return True
                nb = reader.get(NOTEBOOK_KIND, m.labels(pod).get(NOTEBOOK_NAME_LABEL, ""), m.namespace(pod))
                return nb is not None and not m.is_deleting(nb)

            def pod_status_known(etype, pod, old):
                # a pod the StatefulSet controller just created has no status: nothing to mirror
                return etype != "ADDED" or bool((pod.get("status") or {}).get("conditions"))
            pod_preds += [fields_changed("status.conditions", "status.containerStatuses",
                                         f"metadata.labels.{NOTEBOOK_NAME_LABEL}"),
                          pod_nb_alive, pod_status_known]

        b = (mgr.builder().named("notebook-controller").for_(NOTEBOOK_KIND, nb_preds)
             .owns(kinds.STATEFUL_SET, sts_preds).owns(kinds.SERVICE, svc_preds)
             .watches(kinds.POD, map_pod, pod_preds))
        if self.env.get("USE_ISTIO") == "true":
            b.owns(kinds.VIRTUAL_SERVICE, [fields_changed("spec", "metadata.labels"),
                                           controller_owner_alive(self.reader, NOTEBOOK_KIND)]
                   if self.event_filters else [])
        if max_concurrent is not None:
            b.with_options(max_concurrent_reconciles=max_concurrent)
        return b.complete(self)


# ------------------------------------------------------------------ event re-emission


def nb_name_from_involved_object(reader, obj_ref: dict) -> Optional[str]:
    """``nbNameFromInvolvedObject`` (:705-729)."""
    kind, name, ns = obj_ref.get("kind"), obj_ref.get("name", ""), obj_ref.get("namespace", "")
    if kind == "StatefulSet":
        return name
    if kind == "Pod":
        pod = reader.get(kinds.POD, name, ns)
        if pod is not None:
            return m.labels(pod).get(NOTEBOOK_NAME_LABEL)
    return None


# what the re-emitter reads of an Event: its cache holds every Pod/StatefulSet Event of its
# namespaces until the Event expires (kube-apiserver's --event-ttl, an hour), so it keeps
# only these (a third of a full Event's size)
_EVENT_FIELDS = ("apiVersion", "kind", "involvedObject", "reason", "message", "type")
_EVENT_META = ("name", "namespace", "uid", "resourceVersion")


def slim_event(ev: dict) -> dict:
    """The re-emitter's cache transform for Events."""
    md = ev.get("metadata") or {}
    out = {k: ev[k] for k in _EVENT_FIELDS if k in ev}
    out["metadata"] = {k: md[k] for k in _EVENT_META if k in md}
    return out


class NotebookEventReemitter:
    """Re-emits Pod/StatefulSet events onto their Notebook as ``Reissued from <kind>/<name>: <msg>``."""

    def __init__(self, client, reader, recorder):
        self.client = client
        self.reader = reader
        self.recorder = recorder
        self.reemitted = 0

    def _relevant(self, ev: dict) -> bool:
        inv = ev.get("involvedObject") or {}
        if inv.get("kind") not in ("Pod", "StatefulSet"):
            return False
        nb_name = nb_name_from_involved_object(self.reader, inv)
        if not nb_name:
            return False
        return self.reader.get(NOTEBOOK_KIND, nb_name, m.namespace(ev)) is not None

    async def reconcile(self, req: Request) -> Result:
        ev = await self.client.get_or_none(kinds.EVENT, req.name, req.namespace)
        if ev is None:
            return Result()
        inv = ev.get("involvedObject") or {}
        nb_name = nb_name_from_involved_object(self.reader, inv)
        if not nb_name:
            return Result()
        nb = await self.client.get_or_none(NOTEBOOK_KIND, nb_name, req.namespace)
        if nb is None:
            return Result()
        self.reemitted += 1
        self.recorder.event(nb, ev.get("type", "Normal"), ev.get("reason", ""),
                            f"Reissued from {str(inv.get('kind', '')).lower()}/{inv.get('name', '')}: {ev.get('message', '')}")
        return Result()

    # the re-emitter's own output (and every other Notebook event) never reaches it: the
    # apiserver filters the Event watch (kubectl get events --field-selector semantics)
    EVENT_FIELD_SELECTOR = "involvedObject.kind!=Notebook"

    def setup_with_manager(self, mgr, max_concurrent: Optional[int] = None):
        pred = pred_funcs(create=lambda o: self._relevant(o), update=lambda o, old: self._relevant(o),
                          delete=lambda o: False)
        cache = getattr(mgr, "cache", None) or mgr.reader
        if hasattr(cache, "set_field_selector"):
            cache.set_field_selector(kinds.EVENT, self.EVENT_FIELD_SELECTOR)
        transforms = getattr(cache, "transforms", None)
        if transforms is not None:
            transforms.setdefault(SCHEME.resolve(kinds.EVENT).key, slim_event)
        b = mgr.builder().named("notebook-events").for_(kinds.EVENT, [pred])
        if max_concurrent is not None:
            b.with_options(max_concurrent_reconciles=max_concurrent)
        return b.complete(self)
