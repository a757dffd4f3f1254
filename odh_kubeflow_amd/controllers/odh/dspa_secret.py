"""Elyra KFP runtime Secret (reference ``odh/controllers/notebook_dspa_secret.go``).

With ``SET_PIPELINE_SECRET=true`` the webhook and the reconciler keep Secret
``ds-pipeline-config`` (key ``odh_dsp.json``) in the notebook namespace in sync with
the namespace's DataSciencePipelinesApplication ``dspa``: API endpoint, COS
endpoint/bucket/credentials, and a public endpoint
``https://<gateway host>/external/elyra/<ns>`` where the host comes from the
``openshift-ingress/data-science-gateway`` listener or, failing that, from the Route
owned by the Gateway's ``GatewayConfig`` owner.  The Secret is owned by the DSPA.
The webhook mounts it at ``/opt/app-root/runtimes``.
"""

from __future__ import annotations

import base64
import logging
from typing import Optional

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_no_match, is_not_found
from ...runtime.client import get_live
from .constants import (DEFAULT_GATEWAY_NAME, DEFAULT_GATEWAY_NAMESPACE, DSPA_INSTANCE_NAME, ELYRA_MOUNT_PATH,
                        ELYRA_SECRET_NAME, ELYRA_VOLUME_NAME, MANAGED_BY_KEY, MANAGED_BY_VALUE)
from .podspec import add_if_absent, containers, volumes
from .runtime_images import go_json

log = logging.getLogger("controllers.odh.dspa")


class ElyraConfigError(ValueError):
    pass


async def _get_optional(client, kind: str, name: str, namespace: Optional[str]) -> Optional[dict]:
    try:
        return await client.get(kind, name, namespace)
    except ApiError as e:
        if is_not_found(e) or is_no_match(e):
            return None
        raise


async def get_dspa_instance(client, namespace: str) -> Optional[dict]:
    return await _get_optional(client, kinds.DSPA, DSPA_INSTANCE_NAME, namespace)


async def get_gateway_instance(client) -> Optional[dict]:
    return await _get_optional(client, kinds.GATEWAY, DEFAULT_GATEWAY_NAME, DEFAULT_GATEWAY_NAMESPACE)


def gateway_config_owner_name(gw: Optional[dict]) -> str:
    for r in (gw or {}).get("metadata", {}).get("ownerReferences") or []:
        if r.get("kind") == "GatewayConfig":
            return r.get("name", "")
    return ""


async def hostname_from_route(client, gateway_config_name: str) -> str:
    if not gateway_config_name:
        return ""
    try:
        routes = await client.list(kinds.ROUTE, DEFAULT_GATEWAY_NAMESPACE)
    except ApiError as e:
        if is_no_match(e):
            return ""
        raise
    for r in routes:
        for ref in (r.get("metadata") or {}).get("ownerReferences") or []:
            if ref.get("kind") == "GatewayConfig" and ref.get("name") == gateway_config_name:
                return (r.get("spec") or {}).get("host") or ""
    return ""


async def hostname_for_public_endpoint(client, gw: Optional[dict]) -> str:
    if gw is None:
        return ""
    listeners = (gw.get("spec") or {}).get("listeners") or []
    host = ""
    if listeners and listeners[0].get("hostname"):
        host = listeners[0]["hostname"]
    if not host:
        owner = gateway_config_owner_name(gw)
        if owner:
            try:
                host = await hostname_from_route(client, owner)
            except ApiError as e:
                log.error("failed to get hostname from Route: %s", e)
                host = ""
    return host


def _b64d(v: str) -> str:
    try:
        return base64.b64decode(v).decode()
    except (ValueError, UnicodeDecodeError):
        return v


async def extract_elyra_runtime_config_info(client, gw: Optional[dict], dspa: dict, nb: dict) -> dict:
    api_endpoint = ((((dspa.get("status") or {}).get("components") or {}).get("apiServer") or {})
                    .get("externalUrl") or "")
    ext = (((dspa.get("spec") or {}).get("objectStorage") or {}).get("externalStorage") or {})
    host = ext.get("host") or ""
    if not host:
        raise ElyraConfigError("invalid DSPA CR: missing or invalid 'host'")
    scheme = ext.get("scheme") or "https"
    bucket = ext.get("bucket") or ""
    if not bucket:
        raise ElyraConfigError("invalid DSPA CR: missing or invalid 'bucket'")
    creds = ext.get("s3CredentialsSecret") or {}
    secret_name, ukey, pkey = creds.get("secretName", ""), creds.get("accessKey", ""), creds.get("secretKey", "")
    try:
        sec = await client.get(kinds.SECRET, secret_name, m.namespace(nb))
    except ApiError as e:
        raise ElyraConfigError(f"failed to get secret '{secret_name}': {e}")
    data = sec.get("data") or {}
    if ukey not in data:
        raise ElyraConfigError(f"missing key '{ukey}' in secret '{secret_name}'")
    if pkey not in data:
        raise ElyraConfigError(f"missing key '{pkey}' in secret '{secret_name}'")
    md = {
        "tags": [], "display_name": "Pipeline", "engine": "Argo", "runtime_type": "KUBEFLOW_PIPELINES",
        "auth_type": "KUBERNETES_SERVICE_ACCOUNT_TOKEN", "cos_auth_type": "KUBERNETES_SECRET",
        "api_endpoint": api_endpoint, "cos_endpoint": f"{scheme}://{host}", "cos_bucket": bucket,
        "cos_username": _b64d(data[ukey]), "cos_password": _b64d(data[pkey]), "cos_secret": secret_name,
    }
    hostname = await hostname_for_public_endpoint(client, gw)
    if hostname:
        md["public_api_endpoint"] = f"https://{hostname}/external/elyra/{m.namespace(nb)}"
    return {"display_name": "Pipeline", "schema_name": "kfp", "metadata": md}


async def sync_elyra_runtime_config_secret(client, nb: dict) -> None:
    gw = await get_gateway_instance(client)
    dspa = await get_dspa_instance(client, m.namespace(nb))
    if dspa is None:
        return
    info = await extract_elyra_runtime_config_info(client, gw, dspa, nb)
    payload = base64.b64encode(go_json(info).encode()).decode()
    desired_data = {"odh_dsp.json": payload}
    desired = {
        "apiVersion": "v1", "kind": "Secret", "type": "Opaque",
        "metadata": {"name": ELYRA_SECRET_NAME, "namespace": m.namespace(nb),
                     "labels": {MANAGED_BY_KEY: MANAGED_BY_VALUE},
                     "ownerReferences": [{"apiVersion": dspa.get("apiVersion", ""),
                                          "kind": "DataSciencePipelinesApplication", "name": m.name(dspa),
                                          "uid": m.uid(dspa), "controller": True, "blockOwnerDeletion": False}]},
        "data": desired_data,
    }
    try:
        existing = await client.get(kinds.SECRET, ELYRA_SECRET_NAME, m.namespace(nb))
    except ApiError as e:
        if not is_not_found(e):
            raise
        try:
            await client.create(desired)
            return
        except ApiError as e2:
            if not is_already_exists(e2):
                raise
        # created meanwhile by another actor (inside the informer's lag): reconcile ITS data
        # like any existing Secret's instead of leaving it as found
        existing = await get_live(client, kinds.SECRET, ELYRA_SECRET_NAME, m.namespace(nb))
    if (existing.get("data") or {}) != desired_data or m.labels(existing).get(MANAGED_BY_KEY) != MANAGED_BY_VALUE:
        existing["metadata"]["labels"] = dict(desired["metadata"]["labels"])
        existing["data"] = desired_data
        await client.update(existing)


async def mount_elyra_runtime_config_secret(client, nb: dict) -> None:
    try:
        sec = await client.get(kinds.SECRET, ELYRA_SECRET_NAME, m.namespace(nb))
    except ApiError as e:
        if is_not_found(e):
            return
        raise
    if m.labels(sec).get(MANAGED_BY_KEY) != MANAGED_BY_VALUE or not sec.get("data"):
        return
    add_if_absent(volumes(nb), {"name": ELYRA_VOLUME_NAME, "secret": {"secretName": ELYRA_SECRET_NAME,
                                                                      "optional": True}})
    for c in containers(nb):
        add_if_absent(c.setdefault("volumeMounts", []), {"name": ELYRA_VOLUME_NAME, "mountPath": ELYRA_MOUNT_PATH},
                      also_match=("mountPath", ELYRA_MOUNT_PATH))
