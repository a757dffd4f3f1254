"""Trusted-CA bundle for workbenches (reference ``odh/controllers/notebook_controller.go:504-704``
and the webhook half ``notebook_webhook.go:618-781``).

* :func:`create_notebook_cert_configmap` concatenates the valid PEM certificates of
  ``odh-trusted-ca-bundle`` (``ca-bundle.crt``, ``odh-ca-bundle.crt``),
  ``kube-root-ca.crt`` (``ca.crt``) and ``openshift-service-ca.crt``
  (``service-ca.crt``) into ``workbench-trusted-ca-bundle``.
* :func:`is_configmap_deleted` / :func:`unset_notebook_cert_config` un-mount the bundle
  (volume, mount, env) when it disappears while a notebook still uses it.
* :func:`check_and_mount_ca_cert_bundle` / :func:`inject_cert_config` are the admission
  side: ensure the bundle exists and mount it at
  ``/etc/pki/tls/custom-certs/ca-bundle.crt`` with the six CA env vars.

Certificates are validated by parsing them with OpenSSL through the ``ssl`` module
(``x509.ParseCertificate`` in the reference); ``cryptography`` is not available.
"""

from __future__ import annotations

import base64
import logging
import re
import ssl
from typing import List, Optional

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_not_found
from ...runtime.client import get_live
from .constants import (CA_ENV_VARS, CA_KEY, CA_MOUNT_PATH, CA_VOLUME_NAME, MANAGED_BY_KEY, MANAGED_BY_VALUE,
                        ODH_CONFIGMAP_NAME, SELF_SIGNED_CONFIGMAP_NAME, SERVICE_CA_CONFIGMAP_NAME,
                        WORKBENCH_CA_CONFIGMAP_NAME)
from .podspec import add_missing_env, notebook_container, upsert_by_name, volumes

log = logging.getLogger("controllers.odh.certs")

_PEM_RE = re.compile(r"-----BEGIN ([A-Z0-9 ]+)-----\s*(.*?)\s*-----END \1-----", re.S)

CONFIGMAP_FILES = ((ODH_CONFIGMAP_NAME, ("ca-bundle.crt", "odh-ca-bundle.crt")),
                   (SELF_SIGNED_CONFIGMAP_NAME, ("ca.crt",)),
                   (SERVICE_CA_CONFIGMAP_NAME, ("service-ca.crt",)))


def first_pem_block(data: str):
    """``pem.Decode``: the first PEM block as (type, der bytes), or (None, None)."""
    mt = _PEM_RE.search(data)
    if not mt:
        return None, None
    try:
        der = base64.b64decode("".join(mt.group(2).split()), validate=True)
    except (ValueError, base64.binascii.Error):
        return None, None
    return mt.group(1), der


def is_valid_certificate(pem_text: str) -> bool:
    """First PEM block is a CERTIFICATE that OpenSSL can parse."""
    typ, der = first_pem_block(pem_text)
    if typ != "CERTIFICATE" or not der:
        return False
    block = "-----BEGIN CERTIFICATE-----\n" + base64.encodebytes(der).decode() + "-----END CERTIFICATE-----\n"
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
    try:
        ctx.load_verify_locations(cadata=block)
    except (ssl.SSLError, ValueError):
        return False
    return True


async def create_notebook_cert_configmap(client, nb: dict) -> None:
    ns = m.namespace(nb)
    pool: List[str] = []
    for cm_name, files in CONFIGMAP_FILES:
        try:
            cm = await client.get(kinds.CONFIG_MAP, cm_name, ns)
        except ApiError as e:
            if is_not_found(e) and cm_name == ODH_CONFIGMAP_NAME:
                return
            log.info("unable to fetch ConfigMap %s/%s", ns, cm_name)
            continue
        data = cm.get("data") or {}
        for f in files:
            present = f in data
            cert = (data.get(f) or "").strip()
            if not present or (f == "ca-bundle.crt" and cert == ""):
                return  # reference: no bundle to build (created by inject-ca-bundle instead)
            if not cert:
                continue
            typ, _ = first_pem_block(cert)
            if typ == "CERTIFICATE":
                if not is_valid_certificate(cert):
                    log.error("error parsing certificate %s/%s", cm_name, f)
                    continue
                pool.append(cert)
            elif cert:
                log.info("invalid certificate format in %s/%s", cm_name, f)
    if not pool:
        return
    desired = {"apiVersion": "v1", "kind": "ConfigMap",
               "metadata": {"name": WORKBENCH_CA_CONFIGMAP_NAME, "namespace": ns,
                            "labels": {MANAGED_BY_KEY: MANAGED_BY_VALUE}},
               "data": {CA_KEY: "\n".join(pool)}}
    try:
        found = await client.get(kinds.CONFIG_MAP, WORKBENCH_CA_CONFIGMAP_NAME, ns)
    except ApiError as e:
        if not is_not_found(e):
            return  # the reference swallows non-NotFound read errors here
        try:
            await client.create(desired)
            return
        except ApiError as e2:
            if not is_already_exists(e2):
                raise
        found = await get_live(client, kinds.CONFIG_MAP, WORKBENCH_CA_CONFIGMAP_NAME, ns)  # created meanwhile
    if (found.get("data") or {}) != desired["data"]:
        found["data"] = desired["data"]
        await client.update(found)


async def is_configmap_deleted(client, nb: dict) -> bool:
    try:
        await client.get(kinds.CONFIG_MAP, WORKBENCH_CA_CONFIGMAP_NAME, m.namespace(nb))
        return False
    except ApiError:
        pass
    for v in (((nb.get("spec") or {}).get("template") or {}).get("spec") or {}).get("volumes") or []:
        if (v.get("configMap") or {}).get("name") == WORKBENCH_CA_CONFIGMAP_NAME:
            return True
    return False


async def unset_notebook_cert_config(client, nb: dict) -> None:
    """Merge-patch away the CA env vars, the ``trusted-ca`` mount and the bundle volume."""
    from ...utils.jsonpatch import create_merge_patch
    from ...utils.objutil import deepcopy_json

    new = deepcopy_json(nb)
    changed = False
    c = notebook_container(new)
    if c is not None:
        env = c.get("env") or []
        kept = [e for e in env if e.get("name") not in CA_ENV_VARS]
        if env:
            c["env"] = kept
        mounts = c.get("volumeMounts") or []
        keptm = [vm for vm in mounts if vm.get("name") != CA_VOLUME_NAME]
        if mounts:
            c["volumeMounts"] = keptm
        changed = True
    vols = (((new.get("spec") or {}).get("template") or {}).get("spec") or {}).get("volumes") or []
    for i, v in enumerate(vols):
        if (v.get("configMap") or {}).get("name") == WORKBENCH_CA_CONFIGMAP_NAME:
            del vols[i]
            changed = True
            break
    if not changed:
        return
    patch = create_merge_patch({"spec": nb.get("spec")}, {"spec": new.get("spec")})
    if patch:
        await client.patch(nb, patch, "merge")


# ------------------------------------------------------------------ admission side


async def check_and_mount_ca_cert_bundle(client, nb: dict) -> None:
    ns = m.namespace(nb)
    try:
        odh = await client.get(kinds.CONFIG_MAP, ODH_CONFIGMAP_NAME, ns)
    except ApiError:
        return  # feature disabled by the operator
    try:
        await client.get(kinds.CONFIG_MAP, WORKBENCH_CA_CONFIGMAP_NAME, ns)
    except ApiError:
        cm = {"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": WORKBENCH_CA_CONFIGMAP_NAME, "namespace": ns,
                           "labels": {MANAGED_BY_KEY: MANAGED_BY_VALUE}},
              "data": {CA_KEY: (odh.get("data") or {}).get(CA_KEY, "")}}
        try:
            await client.create(cm)
        except ApiError:
            log.info("failed to create %s in %s", WORKBENCH_CA_CONFIGMAP_NAME, ns)
            return
    inject_cert_config(nb, WORKBENCH_CA_CONFIGMAP_NAME)


def inject_cert_config(nb: dict, configmap_name: str) -> None:
    upsert_by_name(volumes(nb), {"name": CA_VOLUME_NAME,
                                 "configMap": {"name": configmap_name, "optional": True,
                                               "items": [{"key": CA_KEY, "path": CA_KEY}]}})
    c = notebook_container(nb)
    if c is None:
        return
    add_missing_env(c, {k: CA_MOUNT_PATH for k in CA_ENV_VARS}, order=CA_ENV_VARS)
    upsert_by_name(c.setdefault("volumeMounts", []),
                   {"name": CA_VOLUME_NAME, "readOnly": True, "mountPath": CA_MOUNT_PATH, "subPath": CA_KEY})


def notebook_uses_bundle(nb: dict) -> bool:
    return any((v.get("configMap") or {}).get("name") == WORKBENCH_CA_CONFIGMAP_NAME
               for v in (((nb.get("spec") or {}).get("template") or {}).get("spec") or {}).get("volumes") or [])


def bundle_data(cm: Optional[dict]) -> str:
    return ((cm or {}).get("data") or {}).get(CA_KEY, "")
