"""Feast config mount (reference ``odh/controllers/notebook_feast_config.go``).

Label ``opendatahub.io/feast-integration=true`` → ConfigMap ``<name>-feast-config``
mounted read-only at ``/opt/app-root/src/feast-config`` on the notebook container
(volume ``odh-feast-config``).  Removing the label un-mounts it.
"""

from __future__ import annotations

from ...models import meta as m
from .constants import FEAST_CONFIGMAP_SUFFIX, FEAST_LABEL, FEAST_MOUNT_PATH, FEAST_VOLUME_NAME
from .podspec import notebook_container, remove_by_name, upsert_by_name, volumes


def is_feast_enabled(nb: dict) -> bool:
    return m.labels(nb).get(FEAST_LABEL) == "true"


def is_feast_mounted(nb: dict) -> bool:
    return any(v.get("name") == FEAST_VOLUME_NAME
               for v in (((nb.get("spec") or {}).get("template") or {}).get("spec") or {}).get("volumes") or [])


def mount_feast_config(nb: dict, configmap_name: str) -> None:
    upsert_by_name(volumes(nb), {"name": FEAST_VOLUME_NAME, "configMap": {"name": configmap_name}})
    c = notebook_container(nb)
    if c is None:
        raise ValueError(f"notebook image container not found {m.name(nb)}")
    upsert_by_name(c.setdefault("volumeMounts", []),
                   {"name": FEAST_VOLUME_NAME, "readOnly": True, "mountPath": FEAST_MOUNT_PATH})


def unmount_feast_config(nb: dict) -> None:
    spec = ((nb.get("spec") or {}).get("template") or {}).get("spec") or {}
    remove_by_name(spec.get("volumes"), FEAST_VOLUME_NAME)
    c = notebook_container(nb)
    if c is not None:
        remove_by_name(c.get("volumeMounts"), FEAST_VOLUME_NAME)


def new_feast_config(nb: dict) -> None:
    try:
        mount_feast_config(nb, m.name(nb) + FEAST_CONFIGMAP_SUFFIX)
    except ValueError as e:
        raise ValueError(f"error mounting Feast config volume: {e}")
