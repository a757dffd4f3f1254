"""Structural-schema processing of custom resources, as kube-apiserver does it for an
``apiextensions.k8s.io/v1`` CRD on every write: **prune → default → validate**.

* pruning drops fields the schema does not know (unless ``x-kubernetes-preserve-unknown-fields``)
  and ``null`` values of non-nullable fields;
* defaulting fills ``default`` values of absent properties (e.g. ``ports[].protocol: TCP``
  in the PodSpec schema);
* validation checks ``type`` (with ``x-kubernetes-int-or-string``), ``format`` int32/int64,
  ``required``, ``items``, ``additionalProperties``, ``pattern``, ``minItems``/``maxItems``,
  ``enum`` and the list semantics ``x-kubernetes-list-type: set|map`` (+ ``list-map-keys``).

``metadata`` is the apiserver's own business (never pruned beyond its ``type: object``).
Error strings follow the apiserver's field-error format
(``<path>: Invalid value: ...: <path> in body must be of type integer: "string"``).
Used by both fake apiservers with :func:`odh_kubeflow_amd.models.crd.version_schema`.
"""

from __future__ import annotations

import copy
import re
from typing import Any, Dict, List, Optional

_INT32 = (-2 ** 31, 2 ** 31 - 1)
_INT64 = (-2 ** 63, 2 ** 63 - 1)
_PATTERNS: Dict[str, "re.Pattern"] = {}


def _type_name(v: Any) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, int):
        return "integer"
    if isinstance(v, float):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    return "object"


def _fmt(v: Any) -> str:
    if isinstance(v, str):
        return f'"{v}"'
    if isinstance(v, (dict, list)):
        return '"' + _type_name(v) + '"'
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _type_ok(schema: dict, v: Any) -> bool:
    if schema.get("x-kubernetes-int-or-string"):
        return (isinstance(v, int) and not isinstance(v, bool)) or isinstance(v, str)
    t = schema.get("type")
    if t is None:
        return True
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool) or (isinstance(v, float) and v.is_integer())
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return _type_name(v) == t


def prune(schema: dict, value: Any, root: bool = True) -> Any:
    """Drop unknown fields and non-nullable nulls, in place; returns ``value``."""
    if isinstance(value, dict):
        if schema.get("x-kubernetes-preserve-unknown-fields"):
            return value
        props = schema.get("properties") or {}
        addl = schema.get("additionalProperties")
        for k in list(value):
            v = value[k]
            if root and k in ("apiVersion", "kind", "metadata"):
                continue  # the apiserver's own fields
            # a known property, else the additionalProperties schema; an object schema with
            # neither keeps no fields at all
            sub = props.get(k) if k in props else (addl if isinstance(addl, dict) else None)
            if sub is None:
                if addl is not True:
                    del value[k]
                continue
            if v is None and not sub.get("nullable"):
                del value[k]
                continue
            prune(sub, v, False)
    elif isinstance(value, list):
        item = schema.get("items")
        if isinstance(item, dict):
            for v in value:
                prune(item, v, False)
    return value


def default(schema: dict, value: Any) -> Any:
    """Fill ``default`` of absent properties, in place (after pruning)."""
    if isinstance(value, dict):
        for k, sub in (schema.get("properties") or {}).items():
            if k not in value and "default" in sub:
                value[k] = copy.deepcopy(sub["default"])
            if k in value:
                default(sub, value[k])
        addl = schema.get("additionalProperties")
        if isinstance(addl, dict):
            for v in value.values():
                default(addl, v)
    elif isinstance(value, list):
        item = schema.get("items")
        if isinstance(item, dict):
            for v in value:
                default(item, v)
    return value


def validate(schema: dict, value: Any, path: str = "") -> List[str]:
    errs: List[str] = []
    if not _type_ok(schema, value):
        want = "integer or string" if schema.get("x-kubernetes-int-or-string") else schema.get("type")
        return [f"{path}: Invalid value: {_fmt(value)}: {path} in body must be of type {want}: "
                f'"{_type_name(value)}"']
    fmt = schema.get("format")
    if fmt in ("int32", "int64") and isinstance(value, (int, float)) and not isinstance(value, bool):
        lo, hi = _INT32 if fmt == "int32" else _INT64
        if not lo <= value <= hi:
            errs.append(f"{path}: Invalid value: {value}: {path} in body should be a valid {fmt}")
    if "enum" in schema and value not in schema["enum"]:
        errs.append(f"{path}: Unsupported value: {_fmt(value)}: supported values: "
                    + ", ".join(_fmt(x) for x in schema["enum"]))
    pat = schema.get("pattern")
    if pat and isinstance(value, str):
        rx = _PATTERNS.get(pat)
        if rx is None:
            rx = _PATTERNS[pat] = re.compile(pat)
        if not rx.search(value):
            errs.append(f"{path}: Invalid value: {_fmt(value)}: {path} in body should match '{pat}'")
    if isinstance(value, dict):
        props = schema.get("properties") or {}
        for r in schema.get("required") or []:
            if r not in value:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        addl = schema.get("additionalProperties")
        for k, v in value.items():
            sub = props.get(k) if k in props else (addl if isinstance(addl, dict) else None)
            if sub is not None and not (not path and k == "metadata"):
                errs.extend(validate(sub, v, f"{path}.{k}" if path else k))
    elif isinstance(value, list):
        if "minItems" in schema and len(value) < schema["minItems"]:
            errs.append(f"{path}: Invalid value: {len(value)}: {path} in body should have at least "
                        f"{schema['minItems']} items")
        if "maxItems" in schema and len(value) > schema["maxItems"]:
            errs.append(f"{path}: Too many: {len(value)}: must have at most {schema['maxItems']} items")
        lt = schema.get("x-kubernetes-list-type")
        if lt == "set":
            seen = []
            for i, v in enumerate(value):
                if v in seen:
                    errs.append(f"{path}[{i}]: Duplicate value: {_fmt(v)}")
                seen.append(v)
        elif lt == "map":
            keys = schema.get("x-kubernetes-list-map-keys") or []
            seen_k = set()
            for i, v in enumerate(value):
                if isinstance(v, dict):
                    k = tuple(repr(v.get(x)) for x in keys)
                    if k in seen_k:
                        errs.append(f"{path}[{i}]: Duplicate value: "
                                    + "{" + ", ".join(f'"{x}":{_fmt(v.get(x))}' for x in keys) + "}")
                    seen_k.add(k)
        item = schema.get("items")
        if isinstance(item, dict):
            for i, v in enumerate(value):
                errs.extend(validate(item, v, f"{path}[{i}]"))
    return errs


def process(schema: dict, obj: dict) -> List[str]:
    """prune → default → validate ``obj`` in place; returns the field errors (empty: valid)."""
    prune(schema, obj)
    default(schema, obj)
    return validate(schema, obj)


def crd_version_schema(crd: dict, version: str) -> dict:
    for v in crd["spec"]["versions"]:
        if v["name"] == version:
            return v["schema"]["openAPIV3Schema"]
    raise KeyError(version)


def first_error(errs: List[str]) -> Optional[str]:
    if not errs:
        return None
    return errs[0] if len(errs) == 1 else f"[{', '.join(errs)}]"
