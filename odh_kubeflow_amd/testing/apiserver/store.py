"""In-memory Kubernetes apiserver: the envtest substitute.

What it reproduces, because the controllers and their tests depend on it:

* ``metadata.resourceVersion`` (one global counter), ``uid``, ``creationTimestamp``,
  ``generation`` (bumped on spec changes and on deletion), ``generateName``;
* optimistic concurrency — an update carrying a stale resourceVersion is a 409
  ``Conflict`` (what ``retry.RetryOnConflict`` exists for, e.g.
  ``kf/controllers/culling_controller.go:171-196``);
* the ``status`` subresource: the main endpoint ignores status, ``/status`` ignores
  everything else;
* finalizers and ``deletionTimestamp`` (objects with finalizers linger until the last
  finalizer is removed; no new finalizer may be added while deleting);
* no-op writes do not bump the resourceVersion or emit watch events (the real
  apiserver short-circuits them, which keeps ``CopyStatefulSetFields`` updates cheap);
* merge-patch, JSON-patch and a strategic-merge subset;
* label / field selector List and Watch, with an event history for resumption;
* mutating admission (in-process handlers or HTTPS webhooks) on CREATE/UPDATE;
* CRD installation state (uninstalled kinds raise ``NoKindMatch``);
* kube-apiserver defaulting of Pods, StatefulSets, Deployments and Services on every write
  (``models/defaults.py``), so controllers see the same live objects as on a real cluster;
* optionally, ownerReference garbage collection. envtest has no GC
  (``kf/controllers/notebook_controller_bdd_test.go:73-76``), so it is off by default.

Objects handed to watch subscribers are the stored objects themselves and must be
treated as read-only; every object returned by a read is a private copy.
"""

from __future__ import annotations

import itertools
import logging
import random
import threading
import uuid
from collections import deque
from dataclasses import dataclass
from typing import Any, Awaitable, Callable, Deque, Dict, List, Optional, Tuple

from ...models import defaults
from ...models import meta as m
from ...models.errors import (AlreadyExists, ApiError, BadRequest, Conflict, Forbidden, Gone, Invalid, NoKindMatch,
                             NotFound)
from ...models.scheme import OPTIONAL_CRDS, SCHEME, ResourceInfo
from ...utils import jsonpatch
from ...utils.objutil import deepcopy_json, equal_except
from ...utils.selectors import field_matcher, match_labels, parse_field_selector, parse_label_selector, selector_from_dict
from ...utils.timeutil import rfc3339

log = logging.getLogger(__name__)

ADDED, MODIFIED, DELETED, BOOKMARK = "ADDED", "MODIFIED", "DELETED", "BOOKMARK"

# admission handler: (operation, info, new_obj, old_obj, user) -> mutated obj (or raises ApiError)
AdmissionHandler = Callable[[str, ResourceInfo, dict, Optional[dict]], Awaitable[dict]]
WatchCallback = Callable[[str, dict, Optional[dict]], None]


@dataclass
class _Watcher:
    wid: int
    resource: str
    namespace: Optional[str]
    label_reqs: list
    field_match: Optional[Callable[[dict], bool]]
    callback: WatchCallback

    def wants(self, obj: dict) -> bool:
        md = obj.get("metadata") or {}
        if self.namespace and md.get("namespace") != self.namespace:
            return False
        if self.label_reqs and not match_labels(self.label_reqs, md.get("labels")):
            return False
        if self.field_match is not None and not self.field_match(obj):
            return False
        return True


def _rand_suffix(n: int = 5) -> str:
    return "".join(random.choices("bcdfghjklmnpqrstvwxz2456789", k=n))


_COMPARE_SKIP = ("resourceVersion", "managedFields", "generation")


def _strip_for_compare(obj: dict) -> dict:
    md = dict(obj.get("metadata") or {})
    for k in ("resourceVersion", "managedFields", "generation"):
        md.pop(k, None)
    out = dict(obj)
    out["metadata"] = md
    return out


def _spec_part(obj: dict) -> dict:
    return {k: v for k, v in obj.items() if k not in ("metadata", "status", "apiVersion", "kind")}


_INFO_BY_KEY = {i.key: i for i in SCHEME.all()}


class ObjectStore:
    """The apiserver's storage + request-handling semantics, in process."""

    HISTORY = 4096

    def __init__(self, gc: bool = False, install_all_crds: bool = True, strict_namespaces: bool = False,
                 defaulting: bool = True):
        self._lock = threading.RLock()
        # kube-apiserver defaulting of Pods / StatefulSets / Deployments / Services (models/defaults.py)
        self.defaulting = defaulting
        self._data: Dict[str, Dict[Tuple[str, str], dict]] = {}
        self._rv = 0
        self._history: Dict[str, Deque[Tuple[int, str, dict, Optional[dict]]]] = {}
        self._watchers: Dict[str, Dict[int, _Watcher]] = {}
        self._wid = itertools.count(1)
        self._owner_index: Dict[str, set] = {}  # owner uid -> {(resource, ns, name)}
        self._uids: Dict[str, Tuple[str, str, str]] = {}  # uid -> (resource, ns, name): GC lookups in O(1)
        self.gc_enabled = gc
        self.strict_namespaces = strict_namespaces
        self.installed = {i.key for i in SCHEME.all()} if install_all_crds else {
            i.key for i in SCHEME.all() if i.key not in OPTIONAL_CRDS}
        self.mutating: List[Tuple[str, Callable[[ResourceInfo, str], bool], AdmissionHandler]] = []
        self.validators: Dict[str, Callable[[dict], Optional[str]]] = {}
        self.request_count = 0
        self.write_count = 0
        self._register_default_validators()

    # ------------------------------------------------------------------ config

    def install_crd(self, ref) -> None:
        self.installed.add(SCHEME.resolve(ref).key)

    def uninstall_crd(self, ref) -> None:
        self.installed.discard(SCHEME.resolve(ref).key)

    def add_mutating_admission(self, name: str, matcher: Callable[[ResourceInfo, str], bool],
                               handler: AdmissionHandler) -> None:
        self.mutating.append((name, matcher, handler))

    def remove_mutating_admission(self, name: str) -> None:
        self.mutating = [x for x in self.mutating if x[0] != name]

    def _register_default_validators(self) -> None:
        """The CRD's structural schema (``models/crd.py``: the reference's full PodSpec schema
        + ``validation_patches.yaml``): prune → default → validate on every Notebook write."""
        from ...models import crd, openapi

        schema = crd.version_schema()

        def notebook(obj: dict) -> Optional[str]:
            return openapi.first_error(openapi.process(schema, obj))

        self.validators["notebooks.kubeflow.org"] = notebook

    # ------------------------------------------------------------------ helpers

    def _info(self, ref) -> ResourceInfo:
        try:
            info = SCHEME.resolve(ref)
        except KeyError:
            raise NoKindMatch(str(ref))
        if info.key not in self.installed:
            raise NoKindMatch(info.kind)
        return info

    def _bucket(self, info: ResourceInfo) -> Dict[Tuple[str, str], dict]:
        b = self._data.get(info.key)
        if b is None:
            b = self._data[info.key] = {}
        return b

    def _next_rv(self) -> int:
        self._rv += 1
        return self._rv

    @property
    def resource_version(self) -> str:
        return str(self._rv)

    def kind_version(self, ref) -> Tuple[int, bool]:
        """A token that changes whenever an object of ``ref``'s kind does (or the kind gets
        installed / uninstalled): the resourceVersion of its last event."""
        info = SCHEME.resolve(ref)
        hist = self._history.get(info.key)
        return (hist[-1][0] if hist else 0, info.key in self.installed)

    def _out(self, info: ResourceInfo, obj: dict, version: Optional[str]) -> dict:
        o = deepcopy_json(obj)
        if version and version != info.storage_version:
            o["apiVersion"] = info.api_version(version)
        return o

    def _ns(self, info: ResourceInfo, namespace: Optional[str]) -> str:
        if not info.namespaced:
            return ""
        if not namespace:
            raise BadRequest(f"namespace is required for {info.plural}")
        return namespace

    def _emit(self, info: ResourceInfo, etype: str, obj: dict, old: Optional[dict]) -> None:
        hist = self._history.get(info.key)
        if hist is None:
            hist = self._history[info.key] = deque(maxlen=self.HISTORY)
        rv = int(obj["metadata"]["resourceVersion"])
        hist.append((rv, etype, obj, old))
        for w in list(self._watchers.get(info.key, {}).values()):
            if w.wants(obj) or (old is not None and w.wants(old)):
                try:
                    w.callback(etype, obj, old)
                except Exception:  # a broken subscriber must not break writes
                    log.exception("watch callback failed")

    def _index_owner(self, info: ResourceInfo, obj: dict, remove: bool = False) -> None:
        k = (info.key, m.namespace(obj), m.name(obj))
        for r in (obj.get("metadata") or {}).get("ownerReferences") or []:
            u = r.get("uid")
            if not u:
                continue
            s = self._owner_index.setdefault(u, set())
            if remove:
                s.discard(k)
                if not s:
                    self._owner_index.pop(u, None)
            else:
                s.add(k)

    async def _admit(self, op: str, info: ResourceInfo, obj: dict, old: Optional[dict]) -> dict:
        for _, matcher, handler in self.mutating:
            if matcher(info, op):
                obj = await handler(op, info, obj, old)
        self._validate(info, obj)
        return obj

    def _validate(self, info: ResourceInfo, obj: dict) -> None:
        v = self.validators.get(info.key)
        if v is not None:
            err = v(obj)
            if err:
                raise Invalid(info.singular if info.group == "" else f"{info.kind}.{info.group}", m.name(obj), err)

    def _check_namespace(self, info: ResourceInfo, ns: str) -> None:
        if self.strict_namespaces and info.namespaced:
            nsb = self._data.get("namespaces", {})
            if ("", ns) not in nsb:
                raise NotFound("namespaces", ns)

    def _defaults(self, info: ResourceInfo, obj: dict) -> None:
        """kube-apiserver defaulting (``models/defaults.py``) + ClusterIP allocation."""
        if self.defaulting:
            defaults.apply(info.key, obj)
        if info.key == "services":
            spec = obj.setdefault("spec", {})
            spec.setdefault("type", "ClusterIP")
            if spec.get("type") == "ClusterIP" and not spec.get("clusterIP"):
                ip = f"10.96.{(self._rv >> 8) & 255}.{self._rv & 255 or 1}"
                spec["clusterIP"] = ip
                spec["clusterIPs"] = [ip]
        elif info.key == "namespaces":
            m.ensure_labels(obj)["kubernetes.io/metadata.name"] = m.name(obj)
            obj.setdefault("status", {"phase": "Active"})
        elif info.key == "serviceaccounts":
            pass

    # ------------------------------------------------------------------ reads

    async def get(self, ref, name: str, namespace: Optional[str] = None, version: Optional[str] = None) -> dict:
        info = self._info(ref)
        self.request_count += 1
        ns = self._ns(info, namespace) if info.namespaced else ""
        obj = self._bucket(info).get((ns, name))
        if obj is None:
            raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
        return self._out(info, obj, version)

    def peek(self, ref, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        """Read the stored object without copying (read-only; for in-process caches)."""
        info = self._info(ref)
        return self._bucket(info).get((namespace or "" if info.namespaced else "", name))

    async def list(self, ref, namespace: Optional[str] = None, label_selector=None, field_selector=None,
                   version: Optional[str] = None, owner_uid: Optional[str] = None) -> Tuple[List[dict], str]:
        info = self._info(ref)
        self.request_count += 1
        return self.list_nocopy(info, namespace, label_selector, field_selector, owner_uid, copy=True,
                                version=version), str(self._rv)

    def list_nocopy(self, ref, namespace=None, label_selector=None, field_selector=None, owner_uid=None,
                    copy: bool = False, version: Optional[str] = None) -> List[dict]:
        info = self._info(ref)
        if isinstance(label_selector, dict):
            reqs = selector_from_dict({"matchLabels": label_selector})
        elif isinstance(label_selector, str):
            reqs = parse_label_selector(label_selector)
        else:
            reqs = label_selector or []
        fmatch = field_matcher(parse_field_selector(field_selector)) if field_selector else None
        bucket = self._bucket(info)
        if owner_uid is not None:
            keys = [(ns, n) for (res, ns, n) in self._owner_index.get(owner_uid, ()) if res == info.key]
            cands = [bucket[k] for k in keys if k in bucket]
        elif namespace and info.namespaced:
            cands = [o for (ns, _), o in bucket.items() if ns == namespace]
        else:
            cands = list(bucket.values())
        out = []
        for o in cands:
            md = o.get("metadata") or {}
            if namespace and info.namespaced and md.get("namespace") != namespace:
                continue
            if reqs and not match_labels(reqs, md.get("labels")):
                continue
            if fmatch is not None and not fmatch(o):
                continue
            out.append(self._out(info, o, version) if copy else o)
        out.sort(key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))
        return out

    # ------------------------------------------------------------------ writes

    async def create(self, obj: dict, namespace: Optional[str] = None, dry_run: bool = False) -> dict:
        info = self._info(obj)
        self.request_count += 1
        version = obj.get("apiVersion", "").rpartition("/")[2] or info.storage_version
        obj = deepcopy_json(obj)
        md = obj.setdefault("metadata", {})
        if info.namespaced:
            ns = md.get("namespace") or namespace
            if not ns:
                raise BadRequest("the namespace of the object must be set")
            if namespace and md.get("namespace") and namespace != md["namespace"]:
                raise BadRequest("the namespace of the provided object does not match the namespace sent on the request")
            md["namespace"] = ns
        else:
            md.pop("namespace", None)
            ns = ""
        if md.get("resourceVersion"):
            raise BadRequest("resourceVersion should not be set on objects to be created")
        if not md.get("name"):
            gen = md.get("generateName")
            if not gen:
                raise Invalid(info.kind, "", "metadata.name: Required value: name or generateName is required")
            md["name"] = gen + _rand_suffix()
        obj["apiVersion"] = info.api_version()
        obj = await self._admit("CREATE", info, obj, None)
        with self._lock:
            self._check_namespace(info, ns)
            bucket = self._bucket(info)
            k = (ns, obj["metadata"]["name"])
            if k in bucket:
                raise AlreadyExists(info.plural if not info.group else f"{info.plural}.{info.group}", k[1])
            md = obj["metadata"]
            md["uid"] = str(uuid.uuid4())
            md["creationTimestamp"] = rfc3339()
            md.pop("deletionTimestamp", None)
            if "spec" in obj or info.status_subresource:
                md["generation"] = 1
            if info.status_subresource and info.group:  # CRDs drop status on create
                obj.pop("status", None)
            self._defaults(info, obj)
            if dry_run:
                return self._out(info, obj, version)
            md["resourceVersion"] = str(self._next_rv())
            bucket[k] = obj
            self._uids[md["uid"]] = (info.key, ns, k[1])
            self._index_owner(info, obj)
            self.write_count += 1
            self._emit(info, ADDED, obj, None)
            out = self._out(info, obj, version)
            refs = md.get("ownerReferences")
            if self.gc_enabled and refs and not any(self._owner_live(r) for r in refs):
                # GC "absent owner": a dependent created after its owners are gone is collected
                try:
                    self._sync_delete(info, ns, k[1])
                except ApiError:
                    pass
            return out

    async def update(self, obj: dict, subresource: Optional[str] = None, namespace: Optional[str] = None) -> dict:
        info = self._info(obj)
        self.request_count += 1
        version = obj.get("apiVersion", "").rpartition("/")[2] or info.storage_version
        new = deepcopy_json(obj)
        md = new.setdefault("metadata", {})
        ns = (md.get("namespace") or namespace or "") if info.namespaced else ""
        name = md.get("name")
        if not name:
            raise BadRequest("name is required")
        cur = self._bucket(info).get((ns, name))
        if cur is None:
            raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
        new["apiVersion"] = info.api_version()
        if subresource in ("status", "approval"):  # CSR approval: status.conditions
            merged = deepcopy_json(cur)
            if "status" in new:
                merged["status"] = new["status"]
            else:
                merged.pop("status", None)
            merged["metadata"]["resourceVersion"] = md.get("resourceVersion", "")
            new = merged
            self._validate(info, new)
        else:
            if info.status_subresource:
                if "status" in cur:
                    new["status"] = deepcopy_json(cur["status"])
                else:
                    new.pop("status", None)
            new = await self._admit("UPDATE", info, new, cur)
        return self._commit_update(info, cur, new, version)

    def _commit_update(self, info: ResourceInfo, cur: dict, new: dict, version: str) -> dict:
        with self._lock:
            md = new["metadata"]
            ns, name = m.namespace(cur), m.name(cur)
            live = self._bucket(info).get((ns, name))
            if live is None:
                raise NotFound(info.plural, name)
            rv = md.get("resourceVersion")
            if rv and rv != live["metadata"]["resourceVersion"]:
                raise Conflict(info.plural if not info.group else f"{info.plural}.{info.group}", name)
            lmd = live["metadata"]
            # immutable / server-owned metadata
            for k in ("uid", "creationTimestamp", "deletionTimestamp", "deletionGracePeriodSeconds"):
                if k in lmd:
                    md[k] = lmd[k]
                else:
                    md.pop(k, None)
            md["namespace"] = lmd.get("namespace") if info.namespaced else md.pop("namespace", None)
            if not info.namespaced:
                md.pop("namespace", None)
            md["name"] = lmd["name"]
            if lmd.get("deletionTimestamp"):
                added = set(md.get("finalizers") or []) - set(lmd.get("finalizers") or [])
                if added:
                    raise Forbidden(f"no new finalizers can be added if the object is being deleted, found new "
                                    f"finalizers {sorted(added)}")
            if self.defaulting and info.key in defaults.BY_RESOURCE:
                defaults.apply(info.key, new)
                if info.key == "services":  # the allocated ClusterIP is immutable
                    for k in ("clusterIP", "clusterIPs"):
                        if k in (live.get("spec") or {}) and not (new.get("spec") or {}).get(k):
                            new.setdefault("spec", {})[k] = deepcopy_json(live["spec"][k])
            if "generation" in lmd:
                md["generation"] = lmd["generation"]
                if _spec_part(new) != _spec_part(live):
                    md["generation"] = lmd["generation"] + 1
            md["resourceVersion"] = lmd["resourceVersion"]
            if equal_except(new, live, _COMPARE_SKIP):
                return self._out(info, live, version)  # no-op write
            # finalizer-driven removal
            if lmd.get("deletionTimestamp") and not md.get("finalizers"):
                md["resourceVersion"] = str(self._next_rv())
                return self._remove(info, live, new, version)
            md["resourceVersion"] = str(self._next_rv())
            self._index_owner(info, live, remove=True)
            self._bucket(info)[(ns, name)] = new
            self._index_owner(info, new)
            self.write_count += 1
            self._emit(info, MODIFIED, new, live)
            return self._out(info, new, version)

    async def patch(self, ref, name: str, namespace: Optional[str], patch: Any, patch_type: str = "merge",
                    subresource: Optional[str] = None) -> dict:
        """Patches without a resourceVersion precondition retry on a concurrent write
        (the apiserver's GuaranteedUpdate loop) instead of surfacing a Conflict."""
        precond = isinstance(patch, dict) and bool((patch.get("metadata") or {}).get("resourceVersion"))
        for attempt in range(17):
            try:
                return await self._patch_once(ref, name, namespace, patch, patch_type, subresource)
            except Conflict:
                if precond or attempt == 16:
                    raise
        raise AssertionError("unreachable")

    async def _patch_once(self, ref, name: str, namespace: Optional[str], patch: Any, patch_type: str,
                          subresource: Optional[str]) -> dict:
        info = self._info(ref)
        self.request_count += 1
        ns = self._ns(info, namespace) if info.namespaced else ""
        cur = self._bucket(info).get((ns, name))
        if cur is None:
            raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
        base = deepcopy_json(cur)
        try:
            if patch_type in ("merge", "application/merge-patch+json"):
                new = jsonpatch.apply_merge_patch(base, patch)
            elif patch_type in ("json", "application/json-patch+json"):
                new = jsonpatch.apply_patch(base, patch, in_place=True)
            elif patch_type in ("strategic", "application/strategic-merge-patch+json"):
                new = jsonpatch.apply_strategic_merge_patch(base, patch)
            else:
                raise BadRequest(f"unsupported patch type {patch_type}")
        except jsonpatch.PatchError as e:
            raise Invalid(info.kind, name, str(e))
        nmd = new.setdefault("metadata", {})
        # a patch that carries a resourceVersion is a precondition, otherwise it applies to latest
        if not (isinstance(patch, dict) and (patch.get("metadata") or {}).get("resourceVersion")):
            nmd["resourceVersion"] = cur["metadata"]["resourceVersion"]
        if subresource in ("status", "approval"):  # CSR approval: status.conditions
            merged = deepcopy_json(cur)
            merged["status"] = new.get("status")
            merged["metadata"]["resourceVersion"] = nmd["resourceVersion"]
            new = merged
            self._validate(info, new)
        else:
            if info.status_subresource:
                if "status" in cur:
                    new["status"] = deepcopy_json(cur["status"])
                else:
                    new.pop("status", None)
            new = await self._admit("UPDATE", info, new, cur)
        return self._commit_update(info, cur, new, info.storage_version)

    async def delete(self, ref, name: str, namespace: Optional[str] = None, preconditions: Optional[dict] = None,
                     propagation: str = "Background") -> dict:
        info = self._info(ref)
        self.request_count += 1
        ns = self._ns(info, namespace) if info.namespaced else ""
        with self._lock:
            cur = self._bucket(info).get((ns, name))
            if cur is None:
                raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
            if preconditions:
                if preconditions.get("uid") and preconditions["uid"] != m.uid(cur):
                    raise Conflict(info.plural, name, "Precondition failed: UID in precondition does not match")
                if preconditions.get("resourceVersion") and preconditions["resourceVersion"] != m.resource_version(cur):
                    raise Conflict(info.plural, name, "Precondition failed: resourceVersion does not match")
            fins = cur["metadata"].get("finalizers") or []
            if propagation == "Foreground" and self.gc_enabled and "foregroundDeletion" not in fins:
                fins = fins + ["foregroundDeletion"]
            if fins:
                if cur["metadata"].get("deletionTimestamp"):
                    return self._out(info, cur, None)
                new = deepcopy_json(cur)
                new["metadata"]["finalizers"] = fins
                new["metadata"]["deletionTimestamp"] = rfc3339()
                new["metadata"]["deletionGracePeriodSeconds"] = 0
                if "generation" in new["metadata"]:
                    new["metadata"]["generation"] += 1
                new["metadata"]["resourceVersion"] = str(self._next_rv())
                self._bucket(info)[(ns, name)] = new
                self.write_count += 1
                self._emit(info, MODIFIED, new, cur)
                if "foregroundDeletion" in fins:
                    self._gc_dependents(m.uid(cur))
                return self._out(info, new, None)
            cur2 = deepcopy_json(cur)
            cur2["metadata"]["resourceVersion"] = str(self._next_rv())
            return self._remove(info, cur, cur2, None)

    def _remove(self, info: ResourceInfo, live: dict, final: dict, version: Optional[str]) -> dict:
        ns, name = m.namespace(live), m.name(live)
        self._bucket(info).pop((ns, name), None)
        self._uids.pop(m.uid(live), None)
        self._index_owner(info, live, remove=True)
        self.write_count += 1
        self._emit(info, DELETED, final, live)
        if self.gc_enabled:
            self._gc_dependents(m.uid(live))
            self._gc_foreground_owners(final)
        return self._out(info, final, version)

    # ------------------------------------------------------------------ garbage collection

    def _gc_dependents(self, owner_uid: str) -> None:
        deps = list(self._owner_index.get(owner_uid, ()))
        for res, ns, name in deps:
            info = _INFO_BY_KEY.get(res)
            if info is None:
                continue
            obj = self._bucket(info).get((ns, name))
            if obj is None:
                continue
            refs = [r for r in obj["metadata"].get("ownerReferences") or [] if r.get("uid") != owner_uid]
            # only collect when no other live owner remains
            if refs and any(self._uid_exists(r.get("uid")) for r in refs):
                continue
            try:
                self._sync_delete(info, ns, name)
            except ApiError:
                pass

    def _uid_exists(self, u: str) -> bool:
        return u in self._uids

    def _owner_live(self, ref: dict) -> bool:
        """True unless ``ref`` names a kind this store serves and no object has its uid
        (an owner of an unknown kind cannot be verified, so it counts as live)."""
        if self._uid_exists(ref.get("uid")):
            return True
        try:
            SCHEME.resolve(f"{ref.get('apiVersion', '')}/{ref.get('kind', '')}")
        except Exception:
            return True
        return False

    def _gc_foreground_owners(self, removed: dict) -> None:
        for r in removed["metadata"].get("ownerReferences") or []:
            u = r.get("uid")
            loc = self._uids.get(u)
            if loc is None:
                continue
            info = _INFO_BY_KEY.get(loc[0])
            if info is None:
                continue
            for (ns, name), o in ((loc[1:], self._bucket(info).get(loc[1:])),):
                if o is None:
                    continue
                if "foregroundDeletion" in (o["metadata"].get("finalizers") or []):
                        if not self._owner_index.get(u):
                            new = deepcopy_json(o)
                            new["metadata"]["finalizers"] = [f for f in new["metadata"]["finalizers"]
                                                             if f != "foregroundDeletion"]
                            new["metadata"]["resourceVersion"] = str(self._next_rv())
                            if not new["metadata"]["finalizers"]:
                                self._remove(info, o, new, None)
                            else:
                                self._bucket(info)[(ns, name)] = new
                                self._emit(info, MODIFIED, new, o)

    def _sync_delete(self, info: ResourceInfo, ns: str, name: str) -> None:
        cur = self._bucket(info).get((ns, name))
        if cur is None:
            return
        if cur["metadata"].get("finalizers"):
            if cur["metadata"].get("deletionTimestamp"):
                return
            new = deepcopy_json(cur)
            new["metadata"]["deletionTimestamp"] = rfc3339()
            new["metadata"]["resourceVersion"] = str(self._next_rv())
            self._bucket(info)[(ns, name)] = new
            self._emit(info, MODIFIED, new, cur)
            return
        final = deepcopy_json(cur)
        final["metadata"]["resourceVersion"] = str(self._next_rv())
        self._remove(info, cur, final, None)

    # ------------------------------------------------------------------ watch

    def watch(self, ref, callback: WatchCallback, namespace: Optional[str] = None, label_selector=None,
              field_selector=None, resource_version: Optional[str] = None,
              initial: bool = False) -> Callable[[], None]:
        """Subscribe to events; replays history after ``resource_version`` (410 if too old).

        ``initial`` first delivers every stored object the watch selects as ADDED — an
        informer's initial list, so a controller started against existing objects reconciles
        each of them once (controller-runtime's Kind source) — atomically with the subscribe,
        so nothing written in between is missed or seen twice.

        Returns an ``unsubscribe`` function.
        """
        info = self._info(ref)
        if isinstance(label_selector, dict):
            reqs = selector_from_dict({"matchLabels": label_selector})
        elif isinstance(label_selector, str):
            reqs = parse_label_selector(label_selector)
        else:
            reqs = label_selector or []
        fm = field_matcher(parse_field_selector(field_selector)) if field_selector else None
        w = _Watcher(next(self._wid), info.key, namespace if info.namespaced else None, reqs, fm, callback)
        with self._lock:
            if resource_version not in (None, "", "0"):
                since = int(resource_version)
                hist = self._history.get(info.key) or deque()
                if hist and since < hist[0][0] - 1 and since < self._rv - len(hist):
                    raise Gone()
                for rv, et, obj, old in list(hist):
                    if rv > since and (w.wants(obj) or (old is not None and w.wants(old))):
                        callback(et, obj, old)
            elif initial:
                for obj in list(self._bucket(info).values()):
                    if w.wants(obj):
                        callback("ADDED", obj, None)
            self._watchers.setdefault(info.key, {})[w.wid] = w

        def cancel() -> None:
            self._watchers.get(info.key, {}).pop(w.wid, None)

        return cancel

    # ------------------------------------------------------------------ stats / debug

    def count(self, ref=None) -> int:
        if ref is None:
            return sum(len(b) for b in self._data.values())
        return len(self._bucket(self._info(ref)))

    def dump(self) -> Dict[str, List[dict]]:
        return {k: [deepcopy_json(o) for o in b.values()] for k, b in self._data.items()}
