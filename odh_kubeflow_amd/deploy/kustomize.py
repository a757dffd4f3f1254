"""A small kustomize renderer for checking the generated ``config/`` tree offline.

``kubectl kustomize`` / ``kustomize build`` are not available here, and the reference
ships its deployment as kustomize overlays (``kf/config/overlays/*``,
``odh/config/**``).  This renders the subset of kustomize the generated tree uses, with
kustomize's semantics, so tests can assert on what ``kubectl apply -k`` would apply:

* ``resources`` (files and directories, built recursively, base first);
* ``configMapGenerator`` (``envs`` files, ``literals``; ``behavior`` create / merge /
  replace against a base ConfigMap found by its original name) with
  ``generatorOptions.disableNameSuffixHash`` (the tree always disables the hash);
* ``patches`` (inline JSON6902 op lists or strategic-merge documents; ``target`` by
  ``kind`` / ``name`` regex anchored as kustomize anchors it, ``^(?:…)$``, matched
  against a resource's current and original names — a target that matches several
  resources patches all of them, and a JSON6902 ``replace`` on a missing path fails,
  exactly the failure mode a too-broad regex has in real kustomize);
* ``images`` (``name`` → ``newName`` / ``newTag`` / ``digest`` on every container and init
  container image of a pod template; the release tooling sets the tag there);
* ``namespace`` and ``namePrefix`` with the name-reference fix-ups kustomize applies
  (ConfigMap/Secret refs in pod templates, ServiceAccount names, RBAC subjects and
  roleRefs, webhook ``clientConfig.service``), CRDs and cluster roles' aggregation
  untouched.

Anything outside this subset raises :class:`KustomizeError` rather than being ignored.
"""

from __future__ import annotations

import copy
import os
import re
from typing import Dict, List, Optional

import yaml

from ..utils.jsonpatch import PatchError, apply_patch, apply_strategic_merge_patch

CLUSTER_SCOPED = {"CustomResourceDefinition", "ClusterRole", "ClusterRoleBinding", "Namespace",
                  "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration", "PriorityClass"}
KNOWN_KEYS = {"apiVersion", "kind", "resources", "namespace", "namePrefix", "patches", "configMapGenerator",
              "generatorOptions", "images"}


class KustomizeError(ValueError):
    pass


class _Res:
    __slots__ = ("obj", "names")

    def __init__(self, obj: dict):
        self.obj = obj
        self.names = [obj["metadata"]["name"]]  # original first, then every rename

    @property
    def kind(self) -> str:
        return self.obj["kind"]

    @property
    def name(self) -> str:
        return self.obj["metadata"]["name"]

    def rename(self, new: str) -> None:
        self.obj["metadata"]["name"] = new
        self.names.append(new)


def _load_docs(path: str) -> List[dict]:
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _env_file(path: str) -> Dict[str, str]:
    out = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            k, sep, v = line.partition("=")
            if not sep:
                raise KustomizeError(f"{path}: not KEY=VALUE: {line!r}")
            out[k] = v
    return out


def _pod_spec(obj: dict) -> Optional[dict]:
    kind = obj.get("kind")
    spec = obj.get("spec") or {}
    if kind in ("Deployment", "StatefulSet", "DaemonSet", "ReplicaSet"):
        return ((spec.get("template") or {}).get("spec"))
    if kind == "Job":
        return (spec.get("template") or {}).get("spec")
    if kind == "CronJob":
        return ((((spec.get("jobTemplate") or {}).get("spec") or {}).get("template") or {}).get("spec"))
    if kind == "Pod":
        return spec
    return None


def _fix_references(resources: List[_Res], renames: Dict[tuple, str], namespace: Optional[str]) -> None:
    """kustomize's nameReference + namespace fix-ups for the references the tree uses."""
    def ren(kind: str, name: Optional[str]) -> Optional[str]:
        return renames.get((kind, name), name)

    for r in resources:
        o = r.obj
        ps = _pod_spec(o)
        if ps is not None:
            if ps.get("serviceAccountName"):
                ps["serviceAccountName"] = ren("ServiceAccount", ps["serviceAccountName"])
            for v in ps.get("volumes") or []:
                if "configMap" in v:
                    v["configMap"]["name"] = ren("ConfigMap", v["configMap"].get("name"))
                if "secret" in v:
                    v["secret"]["secretName"] = ren("Secret", v["secret"].get("secretName"))
            for c in (ps.get("containers") or []) + (ps.get("initContainers") or []):
                for ef in c.get("envFrom") or []:
                    if "configMapRef" in ef:
                        ef["configMapRef"]["name"] = ren("ConfigMap", ef["configMapRef"].get("name"))
                    if "secretRef" in ef:
                        ef["secretRef"]["name"] = ren("Secret", ef["secretRef"].get("name"))
                for e in c.get("env") or []:
                    vf = e.get("valueFrom") or {}
                    if "configMapKeyRef" in vf:
                        vf["configMapKeyRef"]["name"] = ren("ConfigMap", vf["configMapKeyRef"].get("name"))
                    if "secretKeyRef" in vf:
                        vf["secretKeyRef"]["name"] = ren("Secret", vf["secretKeyRef"].get("name"))
        if r.kind in ("RoleBinding", "ClusterRoleBinding"):
            rr = o.get("roleRef") or {}
            rr["name"] = ren(rr.get("kind"), rr.get("name"))
            for s in o.get("subjects") or []:
                if s.get("kind") == "ServiceAccount":
                    s["name"] = ren("ServiceAccount", s.get("name"))
                    if namespace is not None:
                        s["namespace"] = namespace
        if r.kind in ("MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"):
            for w in o.get("webhooks") or []:
                svc = (w.get("clientConfig") or {}).get("service")
                if svc:
                    svc["name"] = ren("Service", svc.get("name"))
                    if namespace is not None:
                        svc["namespace"] = namespace
        if r.kind == "StatefulSet" and (o.get("spec") or {}).get("serviceName"):
            o["spec"]["serviceName"] = ren("Service", o["spec"]["serviceName"])


def split_image(image: str):
    """``(name, tag, digest)`` of an image reference (a registry port is not a tag)."""
    name, digest = (image.split("@", 1) + [None])[:2]
    tag = None
    slash = name.rfind("/")
    colon = name.rfind(":")
    if colon > slash:
        name, tag = name[:colon], name[colon + 1:]
    return name, tag, digest


def _apply_images(resources: List[_Res], images: List[dict], kpath: str) -> None:
    for spec in images:
        if "name" not in spec:
            raise KustomizeError(f"{kpath}: images entry without name: {spec}")
        unknown = set(spec) - {"name", "newName", "newTag", "digest"}
        if unknown:
            raise KustomizeError(f"{kpath}: unsupported images fields {sorted(unknown)}")
        for r in resources:
            ps = _pod_spec(r.obj)
            if ps is None:
                continue
            for c in (ps.get("containers") or []) + (ps.get("initContainers") or []):
                name, tag, digest = split_image(c.get("image") or "")
                if name != spec["name"]:
                    continue
                name = spec.get("newName", name)
                if "digest" in spec:
                    c["image"] = f"{name}@{spec['digest']}"
                elif "newTag" in spec:
                    c["image"] = f"{name}:{spec['newTag']}"
                else:
                    c["image"] = name + (f":{tag}" if tag else "") + (f"@{digest}" if digest else "")


def _matches(res: _Res, target: dict) -> bool:
    for k in target:
        if k not in ("kind", "name", "group", "version"):
            raise KustomizeError(f"unsupported patch target key {k!r}")
    if "kind" in target and not re.fullmatch(f"(?:{target['kind']})", res.kind):
        return False
    if "name" in target and not any(re.fullmatch(f"(?:{target['name']})", n) for n in res.names):
        return False
    return True


def build(path: str) -> List[dict]:
    """Render the kustomization in directory ``path`` to a list of objects."""
    return [r.obj for r in _build(os.path.abspath(path))]


def _build(d: str) -> List[_Res]:
    kpath = os.path.join(d, "kustomization.yaml")
    if not os.path.exists(kpath):
        raise KustomizeError(f"no kustomization.yaml in {d}")
    with open(kpath) as f:
        k = yaml.safe_load(f) or {}
    unknown = set(k) - KNOWN_KEYS
    if unknown:
        raise KustomizeError(f"{kpath}: unsupported fields {sorted(unknown)}")
    resources: List[_Res] = []
    for ref in k.get("resources") or []:
        p = os.path.normpath(os.path.join(d, ref))
        if os.path.isdir(p):
            resources.extend(_build(p))
        elif os.path.isfile(p):
            resources.extend(_Res(copy.deepcopy(o)) for o in _load_docs(p))
        else:
            raise KustomizeError(f"{kpath}: resource {ref} not found")

    opts = k.get("generatorOptions") or {}
    for g in k.get("configMapGenerator") or []:
        data: Dict[str, str] = {}
        for e in g.get("envs") or []:
            data.update(_env_file(os.path.join(d, e)))
        for lit in g.get("literals") or []:
            key, sep, val = lit.partition("=")
            if not sep:
                raise KustomizeError(f"{kpath}: literal {lit!r} is not KEY=VALUE")
            data[key] = val
        behavior = g.get("behavior", "create")
        if behavior == "create":
            if not opts.get("disableNameSuffixHash"):
                raise KustomizeError(f"{kpath}: name-suffix hashes are not modelled; disable them")
            resources.append(_Res({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": g["name"]},
                                   "data": data}))
        elif behavior in ("merge", "replace"):
            hits = [r for r in resources if r.kind == "ConfigMap" and r.names[0] == g["name"]]
            if len(hits) != 1:
                raise KustomizeError(f"{kpath}: {behavior} of ConfigMap {g['name']}: {len(hits)} base matches")
            if behavior == "merge":
                hits[0].obj.setdefault("data", {}).update(data)
            else:
                hits[0].obj["data"] = data
        else:
            raise KustomizeError(f"{kpath}: unknown generator behavior {behavior!r}")

    for p in k.get("patches") or []:
        if "path" in p:
            with open(os.path.join(d, p["path"])) as f:
                body = yaml.safe_load(f)
        else:
            body = yaml.safe_load(p["patch"])
        target = p.get("target")
        if isinstance(body, list):  # JSON6902
            if not target:
                raise KustomizeError(f"{kpath}: a JSON6902 patch needs a target")
            hits = [r for r in resources if _matches(r, target)]
            if not hits:
                raise KustomizeError(f"{kpath}: patch target {target} matches nothing")
            for r in hits:
                try:
                    r.obj = apply_patch(r.obj, body)
                except PatchError as e:
                    raise KustomizeError(f"{kpath}: patch {target} on {r.kind}/{r.name}: {e}") from e
        elif isinstance(body, dict):  # strategic merge
            tgt = target or {"kind": body.get("kind"), "name": (body.get("metadata") or {}).get("name")}
            hits = [r for r in resources if _matches(r, {k2: v for k2, v in tgt.items() if v})]
            if not hits:
                raise KustomizeError(f"{kpath}: strategic-merge patch {tgt} matches nothing")
            for r in hits:
                if body.get("$patch") == "delete":
                    resources.remove(r)
                    continue
                patch = {k2: v for k2, v in body.items() if k2 not in ("apiVersion", "kind")}
                patch.get("metadata", {}).pop("name", None)
                r.obj = apply_strategic_merge_patch(r.obj, patch)
        else:
            raise KustomizeError(f"{kpath}: unsupported patch body")

    if k.get("images"):
        _apply_images(resources, k["images"], kpath)

    ns = k.get("namespace")
    prefix = k.get("namePrefix") or ""
    renames: Dict[tuple, str] = {}
    if prefix:
        for r in resources:
            if r.kind == "CustomResourceDefinition":
                continue
            old = r.name
            r.rename(prefix + old)
            renames[(r.kind, old)] = r.name
    if ns is not None:
        for r in resources:
            if r.kind not in CLUSTER_SCOPED:
                r.obj["metadata"]["namespace"] = ns
    if renames or ns is not None:
        _fix_references(resources, renames, ns)
    return resources
