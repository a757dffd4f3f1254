"""Structural OpenAPI v3 validation for CRD schemas (the subset kube-apiserver enforces
for ``apiextensions.k8s.io/v1`` structural schemas: ``type``, ``properties``,
``required``, ``items``, ``minItems``/``maxItems``, ``enum``, ``format: int32``,
``x-kubernetes-preserve-unknown-fields``).  Used to check objects against the generated
``notebooks.kubeflow.org`` CRD; errors read like the apiserver's field errors."""

from __future__ import annotations

from typing import Any, List

_TYPES = {"object": dict, "array": list, "string": str, "boolean": bool}


def validate(schema: dict, value: Any, path: str = "") -> List[str]:
    errs: List[str] = []
    t = schema.get("type")
    if t == "integer":
        if not isinstance(value, int) or isinstance(value, bool):
            return [f"{path}: Invalid value: {value!r}: must be of type integer"]
        if schema.get("format") == "int32" and not (-2 ** 31 <= value < 2 ** 31):
            errs.append(f"{path}: Invalid value: {value}: must fit in int32")
    elif t == "number":
        if not isinstance(value, (int, float)) or isinstance(value, bool):
            return [f"{path}: Invalid value: {value!r}: must be of type number"]
    elif t in _TYPES:
        if not isinstance(value, _TYPES[t]):
            return [f"{path}: Invalid value: {type(value).__name__}: must be of type {t}"]
    if "enum" in schema and value not in schema["enum"]:
        errs.append(f"{path}: Unsupported value: {value!r}")
    if isinstance(value, dict):
        props = schema.get("properties") or {}
        for r in schema.get("required") or []:
            if r not in value:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        for k, v in value.items():
            if k in props:
                errs.extend(validate(props[k], v, f"{path}.{k}" if path else k))
    if isinstance(value, list):
        if "minItems" in schema and len(value) < schema["minItems"]:
            errs.append(f"{path}: Invalid value: {len(value)}: should have at least {schema['minItems']} items")
        if "maxItems" in schema and len(value) > schema["maxItems"]:
            errs.append(f"{path}: Too many: {len(value)}: must have at most {schema['maxItems']} items")
        item = schema.get("items")
        if item:
            for i, v in enumerate(value):
                errs.extend(validate(item, v, f"{path}[{i}]"))
    return errs


def crd_version_schema(crd: dict, version: str) -> dict:
    for v in crd["spec"]["versions"]:
        if v["name"] == version:
            return v["schema"]["openAPIV3Schema"]
    raise KeyError(version)
