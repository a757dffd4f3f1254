"""Pipeline runtime-images ConfigMap (reference ``odh/controllers/notebook_runtime.go``).

ImageStreams labelled ``opendatahub.io/runtime-image=true`` in the controller namespace
are flattened into ConfigMap ``pipeline-runtime-images`` in the notebook namespace:
one key ``<sanitised display_name>.json`` per tag, value = the tag's first
``opendatahub.io/runtime-image-metadata`` entry with ``metadata.image_name`` set to the
tag's ``from.name``.  The webhook creates it before mounting (RHOAIENG-24545 race fix)
and mounts it read-only at ``/opt/app-root/pipeline-runtimes/`` on every container.
"""

from __future__ import annotations

import json
import logging
import re

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_no_match, is_not_found
from ...runtime.client import get_live
from .constants import (MANAGED_BY_KEY, MANAGED_BY_VALUE, RUNTIME_IMAGE_LABEL, RUNTIME_IMAGE_METADATA_ANNOTATION,
                        RUNTIME_IMAGES_CONFIGMAP, RUNTIME_IMAGES_MOUNT_PATH, RUNTIME_IMAGES_VOLUME)
from .podspec import add_if_absent, containers, volumes

log = logging.getLogger("controllers.odh.runtime")

_INVALID = re.compile(r"[^-._a-zA-Z0-9]+")
_MULTIDASH = re.compile(r"-+")


def go_json(o) -> str:
    """``json.Marshal`` of a ``map[string]interface{}``: sorted keys, compact, HTML-escaped."""
    s = json.dumps(o, sort_keys=True, separators=(",", ":"), ensure_ascii=False)
    return s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")


def format_key_name(display_name: str) -> str:
    s = _INVALID.sub("-", display_name.lower())
    s = _MULTIDASH.sub("-", s).strip("-")
    return s + ".json" if s else ""


def parse_runtime_image_metadata(raw: str, image_url: str) -> str:
    try:
        arr = json.loads(raw)
    except ValueError:
        return "{}"
    if not isinstance(arr, list) or not arr or not isinstance(arr[0], dict):
        return "{}"
    first = arr[0]
    md = first.get("metadata")
    if isinstance(md, dict):
        md["image_name"] = image_url
    return go_json(first)


def extract_display_name(metadata: str) -> str:
    try:
        d = json.loads(metadata)
    except ValueError:
        return ""
    v = d.get("display_name") if isinstance(d, dict) else None
    return v if isinstance(v, str) else ""


def runtime_images_data(image_streams) -> dict:
    data = {}
    for ist in image_streams:
        if m.labels(ist).get(RUNTIME_IMAGE_LABEL) != "true":
            continue
        tags = (ist.get("spec") or {}).get("tags") or []
        if not tags:
            log.error("ImageStream %s labeled as runtime-image has no tags", m.name(ist))
            continue
        for tag in tags:
            raw = (tag.get("annotations") or {}).get(RUNTIME_IMAGE_METADATA_ANNOTATION) or "[]"
            url = (tag.get("from") or {}).get("name")
            if not url:
                log.error("failed to extract image URL from ImageStream %s tag %s", m.name(ist), tag.get("name"))
                continue
            md = parse_runtime_image_metadata(raw, url)
            dn = extract_display_name(md)
            if dn:
                key = format_key_name(dn)
                if key:
                    data[key] = md
    return data


async def sync_runtime_images_configmap(client, notebook_namespace: str, controller_namespace: str) -> None:
    try:
        streams = await client.list(kinds.IMAGE_STREAM, controller_namespace)
    except ApiError as e:
        if not is_no_match(e):
            raise
        streams = []  # vanilla Kubernetes: no image.openshift.io API, nothing to publish
    data = runtime_images_data(streams)
    try:
        existing = await client.get(kinds.CONFIG_MAP, RUNTIME_IMAGES_CONFIGMAP, notebook_namespace)
    except ApiError as e:
        if not is_not_found(e):
            raise
        existing = None
    if not data:
        return  # never create an empty ConfigMap, never clear an existing one
    if existing is not None:
        if (existing.get("data") or {}) != data:
            existing["data"] = data
            await client.update(existing)
        return
    try:
        await client.create({"apiVersion": "v1", "kind": "ConfigMap",
                             "metadata": {"name": RUNTIME_IMAGES_CONFIGMAP, "namespace": notebook_namespace,
                                          "labels": {MANAGED_BY_KEY: MANAGED_BY_VALUE}},
                             "data": data})
    except ApiError as e:
        if not is_already_exists(e):
            raise
        # created meanwhile (a concurrent admission or reconcile): bring ITS data up to date
        existing = await get_live(client, kinds.CONFIG_MAP, RUNTIME_IMAGES_CONFIGMAP, notebook_namespace)
        if (existing.get("data") or {}) != data:
            existing["data"] = data
            await client.update(existing)


async def mount_pipeline_runtime_images(client, nb: dict) -> None:
    try:
        cm = await client.get(kinds.CONFIG_MAP, RUNTIME_IMAGES_CONFIGMAP, m.namespace(nb))
    except ApiError as e:
        if is_not_found(e):
            return
        raise
    if not cm.get("data"):
        return
    add_if_absent(volumes(nb), {"name": RUNTIME_IMAGES_VOLUME,
                                "configMap": {"name": RUNTIME_IMAGES_CONFIGMAP, "optional": True}})
    for c in containers(nb):
        add_if_absent(c.setdefault("volumeMounts", []),
                      {"name": RUNTIME_IMAGES_VOLUME, "mountPath": RUNTIME_IMAGES_MOUNT_PATH})
