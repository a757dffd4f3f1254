"""kube-rbac-proxy auth for notebooks (``notebooks.opendatahub.io/inject-auth=true``).

Admission side (reference ``odh/controllers/notebook_webhook.go:117-326``):
:func:`parse_and_validate_auth_sidecar_resources` and :func:`inject_kube_rbac_proxy`
build the ``kube-rbac-proxy`` sidecar (8443 TLS → ``http://127.0.0.1:8888/``, health on
8444, SubjectAccessReview config + serving-cert volumes) and point the pod at a
dedicated ServiceAccount ``<name>``.

Reconciler side (``odh/controllers/notebook_kube_rbac_auth.go``): the ServiceAccount,
the ``<name>-kube-rbac-proxy`` Service (8443, OpenShift serving-cert annotation), the
``<name>-kube-rbac-proxy-config`` ConfigMap (SAR rule ``get notebooks/<name>``), the
cluster-scoped ``<name>-rbac-<ns>-auth-delegator`` ClusterRoleBinding (cannot be
owned → cleaned up explicitly) and the auth HTTPRoute.
"""

from __future__ import annotations

import functools
import logging
from typing import Mapping

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_not_found
from ...utils.quantity import QuantityError, canonical, parse_quantity
from .constants import (ANNOTATION_AUTH_SIDECAR_CPU_LIMIT, ANNOTATION_AUTH_SIDECAR_CPU_REQUEST,
                        ANNOTATION_AUTH_SIDECAR_MEMORY_LIMIT, ANNOTATION_AUTH_SIDECAR_MEMORY_REQUEST,
                        ANNOTATION_INJECT_AUTH, CONTAINER_NAME_KUBE_RBAC_PROXY, DEFAULT_AUTH_SIDECAR_CPU_LIMIT,
                        DEFAULT_AUTH_SIDECAR_CPU_REQUEST, DEFAULT_AUTH_SIDECAR_MEMORY_LIMIT,
                        DEFAULT_AUTH_SIDECAR_MEMORY_REQUEST, KUBE_RBAC_PROXY_CONFIG_FILE,
                        KUBE_RBAC_PROXY_CONFIG_MOUNT_PATH, KUBE_RBAC_PROXY_CONFIG_SUFFIX,
                        KUBE_RBAC_PROXY_CONFIG_VOLUME, KUBE_RBAC_PROXY_HEALTH_PORT, KUBE_RBAC_PROXY_PORT,
                        KUBE_RBAC_PROXY_SERVICE_PORT_NAME, KUBE_RBAC_PROXY_SERVICE_SUFFIX,
                        KUBE_RBAC_PROXY_TLS_MOUNT_PATH, KUBE_RBAC_PROXY_TLS_SECRET_SUFFIX,
                        KUBE_RBAC_PROXY_TLS_VOLUME, NOTEBOOK_PORT)
from .podspec import containers, pod_spec, upsert_by_name, volumes

log = logging.getLogger("controllers.odh.auth")


def parse_bool(v) -> bool:
    """``strconv.ParseBool`` (invalid → False)."""
    return str(v).strip() in ("1", "t", "T", "TRUE", "true", "True")


def kube_rbac_proxy_injection_enabled(nb: dict) -> bool:
    v = m.annotations(nb).get(ANNOTATION_INJECT_AUTH, "")
    return bool(v) and parse_bool(v)


class SidecarResourceError(ValueError):
    pass


def parse_and_validate_auth_sidecar_resources(nb: dict) -> dict:
    """Annotations → requests/limits with defaults 100m / 64Mi; rejects negatives and request > limit."""
    ann = m.annotations(nb)
    cpu_req, mem_req, cpu_lim, mem_lim = _sidecar_resources(*(ann.get(k) or None for k in _SIDECAR_KEYS))
    return {"requests": {"cpu": cpu_req, "memory": mem_req}, "limits": {"cpu": cpu_lim, "memory": mem_lim}}


_SIDECAR_KEYS = (ANNOTATION_AUTH_SIDECAR_CPU_REQUEST, ANNOTATION_AUTH_SIDECAR_MEMORY_REQUEST,
                 ANNOTATION_AUTH_SIDECAR_CPU_LIMIT, ANNOTATION_AUTH_SIDECAR_MEMORY_LIMIT)
_SIDECAR_DEFAULTS = (DEFAULT_AUTH_SIDECAR_CPU_REQUEST, DEFAULT_AUTH_SIDECAR_MEMORY_REQUEST,
                     DEFAULT_AUTH_SIDECAR_CPU_LIMIT, DEFAULT_AUTH_SIDECAR_MEMORY_LIMIT)


@functools.lru_cache(maxsize=256)
def _sidecar_resources(*raws) -> tuple:
    """Canonical (cpu request, memory request, cpu limit, memory limit) for the four raw
    annotation values (None = default).  Memoised: the webhook evaluates this on every
    CREATE/UPDATE admission and nearly every notebook carries the same (usually no) values."""
    qs = []
    for key, raw, default in zip(_SIDECAR_KEYS, raws, _SIDECAR_DEFAULTS):
        if raw:
            try:
                q = parse_quantity(raw.strip())
            except (QuantityError, ValueError) as e:
                raise SidecarResourceError(f"invalid value for annotation '{key}': '{raw}': {e}")
            if q.sign() < 0:
                raise SidecarResourceError(f"annotation '{key}' value '{raw}' cannot be negative")
        else:
            q = parse_quantity(default)
        qs.append(q)
    cpu_req, mem_req, cpu_lim, mem_lim = qs
    if cpu_req.cmp(cpu_lim) > 0:
        raise SidecarResourceError(f"CPU request ({canonical(cpu_req)}) cannot be greater than CPU limit "
                                   f"({canonical(cpu_lim)})")
    if mem_req.cmp(mem_lim) > 0:
        raise SidecarResourceError(f"memory request ({canonical(mem_req)}) cannot be greater than memory limit "
                                   f"({canonical(mem_lim)})")
    return canonical(cpu_req), canonical(mem_req), canonical(cpu_lim), canonical(mem_lim)


def kube_rbac_proxy_container(image: str, resources: dict) -> dict:
    probe = lambda delay: {  # noqa: E731
        "httpGet": {"path": "/healthz", "port": KUBE_RBAC_PROXY_HEALTH_PORT, "scheme": "HTTPS"},
        "initialDelaySeconds": delay, "timeoutSeconds": 1, "periodSeconds": 5,
        "successThreshold": 1, "failureThreshold": 3}
    return {
        "name": CONTAINER_NAME_KUBE_RBAC_PROXY,
        "image": image,
        "imagePullPolicy": "Always",
        "args": [
            f"--secure-listen-address=0.0.0.0:{KUBE_RBAC_PROXY_PORT}",
            f"--upstream=http://127.0.0.1:{NOTEBOOK_PORT}/",
            "--logtostderr=true",
            "--v=10",
            f"--proxy-endpoints-port={KUBE_RBAC_PROXY_HEALTH_PORT}",
            f"--config-file={KUBE_RBAC_PROXY_CONFIG_MOUNT_PATH}/{KUBE_RBAC_PROXY_CONFIG_FILE}",
            f"--tls-cert-file={KUBE_RBAC_PROXY_TLS_MOUNT_PATH}/tls.crt",
            f"--tls-private-key-file={KUBE_RBAC_PROXY_TLS_MOUNT_PATH}/tls.key",
            "--auth-header-fields-enabled=true",
            "--auth-header-user-field-name=X-Auth-Request-User",
            "--auth-header-groups-field-name=X-Auth-Request-Groups",
        ],
        "ports": [{"name": KUBE_RBAC_PROXY_SERVICE_PORT_NAME, "containerPort": KUBE_RBAC_PROXY_PORT,
                   "protocol": "TCP"}],
        "livenessProbe": probe(30),
        "readinessProbe": probe(5),
        "resources": resources,
        "volumeMounts": [
            {"name": KUBE_RBAC_PROXY_CONFIG_VOLUME, "mountPath": KUBE_RBAC_PROXY_CONFIG_MOUNT_PATH},
            {"name": KUBE_RBAC_PROXY_TLS_VOLUME, "mountPath": KUBE_RBAC_PROXY_TLS_MOUNT_PATH},
        ],
    }


def inject_kube_rbac_proxy(nb: dict, image: str) -> None:
    """Upsert the sidecar + its two volumes and set ``serviceAccountName=<name>``.

    Raises :class:`SidecarResourceError` (leaving ``nb`` untouched) on bad annotations.
    """
    resources = parse_and_validate_auth_sidecar_resources(nb)
    upsert_by_name(containers(nb), kube_rbac_proxy_container(image, resources))
    name = m.name(nb)
    upsert_by_name(volumes(nb), {"name": KUBE_RBAC_PROXY_CONFIG_VOLUME,
                                 "configMap": {"name": name + KUBE_RBAC_PROXY_CONFIG_SUFFIX, "defaultMode": 420}})
    upsert_by_name(volumes(nb), {"name": KUBE_RBAC_PROXY_TLS_VOLUME,
                                 "secret": {"secretName": name + KUBE_RBAC_PROXY_TLS_SECRET_SUFFIX,
                                            "defaultMode": 420}})
    pod_spec(nb)["serviceAccountName"] = name


# ------------------------------------------------------------------ reconciler side


def new_service_account(nb: dict) -> dict:
    return {"apiVersion": "v1", "kind": "ServiceAccount",
            "metadata": {"name": m.name(nb), "namespace": m.namespace(nb), "labels": {"notebook-name": m.name(nb)}}}


def new_kube_rbac_proxy_service(nb: dict) -> dict:
    name = m.name(nb)
    return {
        "apiVersion": "v1", "kind": "Service",
        "metadata": {"name": name + KUBE_RBAC_PROXY_SERVICE_SUFFIX, "namespace": m.namespace(nb),
                     "labels": {"notebook-name": name},
                     "annotations": {"service.beta.openshift.io/serving-cert-secret-name":
                                     name + KUBE_RBAC_PROXY_TLS_SECRET_SUFFIX}},
        "spec": {"ports": [{"name": KUBE_RBAC_PROXY_SERVICE_PORT_NAME, "port": KUBE_RBAC_PROXY_PORT,
                            "targetPort": KUBE_RBAC_PROXY_SERVICE_PORT_NAME, "protocol": "TCP"}],
                 "selector": {"statefulset": name}},
    }


def kube_rbac_proxy_config_text(nb: dict) -> str:
    return ("authorization:\n  resourceAttributes:\n    verb: get\n    resource: notebooks\n"
            f"    apiGroup: kubeflow.org\n    name: {m.name(nb)}\n    namespace: {m.namespace(nb)}")


def new_kube_rbac_proxy_configmap(nb: dict) -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": m.name(nb) + KUBE_RBAC_PROXY_CONFIG_SUFFIX, "namespace": m.namespace(nb),
                         "labels": {"notebook-name": m.name(nb)}},
            "data": {KUBE_RBAC_PROXY_CONFIG_FILE: kube_rbac_proxy_config_text(nb)}}


def crb_name(nb: dict) -> str:
    return f"{m.name(nb)}-rbac-{m.namespace(nb)}-auth-delegator"


def new_kube_rbac_proxy_crb(nb: dict) -> dict:
    return {
        "apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
        "metadata": {"name": crb_name(nb), "labels": {"opendatahub.io/component": "notebook-controller",
                                                      "opendatahub.io/namespace": m.namespace(nb)}},
        "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "system:auth-delegator"},
        "subjects": [{"kind": "ServiceAccount", "name": m.name(nb), "namespace": m.namespace(nb)}],
    }


async def _create_owned_if_missing(client, nb: dict, kind: str, desired: dict, owned: bool = True):
    try:
        return await client.get(kind, m.name(desired), m.namespace(desired) or None)
    except ApiError as e:
        if not is_not_found(e):
            raise
    if owned:
        m.set_controller_reference(nb, desired)
    try:
        await client.create(desired)
    except ApiError as e:
        if not is_already_exists(e):
            raise
    return None


async def reconcile_notebook_service_account(client, nb: dict) -> None:
    await _create_owned_if_missing(client, nb, kinds.SERVICE_ACCOUNT, new_service_account(nb))


async def reconcile_kube_rbac_proxy_service(client, nb: dict) -> None:
    await _create_owned_if_missing(client, nb, kinds.SERVICE, new_kube_rbac_proxy_service(nb))


async def reconcile_kube_rbac_proxy_configmap(client, nb: dict) -> None:
    desired = new_kube_rbac_proxy_configmap(nb)
    found = await _create_owned_if_missing(client, nb, kinds.CONFIG_MAP, desired)
    if found is None:
        return
    if (found.get("data") or {}) != desired["data"] or (m.labels(found) or {}) != m.labels(desired):
        found["data"] = desired["data"]
        found["metadata"]["labels"] = dict(m.labels(desired))
        await client.update(found)


async def reconcile_kube_rbac_proxy_crb(client, nb: dict) -> None:
    await _create_owned_if_missing(client, nb, kinds.CLUSTER_ROLE_BINDING, new_kube_rbac_proxy_crb(nb), owned=False)


async def cleanup_kube_rbac_proxy_crb(client, nb: dict) -> None:
    try:
        await client.delete(kinds.CLUSTER_ROLE_BINDING, crb_name(nb))
    except ApiError as e:
        if not is_not_found(e):
            raise


def sidecar_image(env: Mapping[str, str], default: str) -> str:
    return env.get("KUBE_RBAC_PROXY_IMAGE") or default
