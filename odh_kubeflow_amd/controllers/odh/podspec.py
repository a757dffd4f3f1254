"""Pod-spec editing helpers shared by the webhook mutations and the ODH reconciler.

The reference repeats one idiom many times: "replace the element with this ``name`` if
present, else append" for containers, volumes, volume mounts and env vars (e.g.
``odh/controllers/notebook_webhook.go:273-319,716-779``).  Some call sites update an
existing env var through a Go range copy, so an env var that already exists keeps its
*old* value; :func:`add_missing_env` reproduces that observable behaviour.
"""

from __future__ import annotations

from typing import Iterable, List, Mapping, Optional, Tuple

from ...models import meta as m


def pod_spec(nb: dict) -> dict:
    return nb.setdefault("spec", {}).setdefault("template", {}).setdefault("spec", {})


def containers(nb: dict) -> List[dict]:
    return pod_spec(nb).setdefault("containers", [])


def volumes(nb: dict) -> List[dict]:
    return pod_spec(nb).setdefault("volumes", [])


def notebook_container(nb: dict) -> Optional[dict]:
    """The container named like the Notebook (the reference's ``container.Name == notebook.Name``)."""
    for c in (((nb.get("spec") or {}).get("template") or {}).get("spec") or {}).get("containers") or []:
        if c.get("name") == m.name(nb):
            return c
    return None


def upsert_by_name(items: List[dict], item: dict) -> bool:
    """Replace the element with ``item['name']`` or append; returns True when appended."""
    for i, x in enumerate(items):
        if x.get("name") == item["name"]:
            items[i] = item
            return False
    items.append(item)
    return True


def add_if_absent(items: List[dict], item: dict, also_match: Optional[Tuple[str, str]] = None) -> bool:
    for x in items:
        if x.get("name") == item["name"]:
            return False
        if also_match and x.get(also_match[0]) == also_match[1]:
            return False
    items.append(item)
    return True


def remove_by_name(items: Optional[List[dict]], name: str, first_only: bool = True) -> bool:
    if not items:
        return False
    removed = False
    i = 0
    while i < len(items):
        if items[i].get("name") == name:
            del items[i]
            removed = True
            if first_only:
                return True
            continue
        i += 1
    return removed


def add_missing_env(container: dict, env: Mapping[str, str], order: Optional[Iterable[str]] = None) -> bool:
    """Append env vars that are not present; existing ones keep their value (range-copy quirk)."""
    cur = container.setdefault("env", [])
    have = {e.get("name") for e in cur}
    changed = False
    for k in (order or sorted(env)):
        if k not in have:
            cur.append({"name": k, "value": env[k]})
            changed = True
    if not cur:
        container.pop("env", None)
    return changed
