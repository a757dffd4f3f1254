"""Group/version/kind registry — the analogue of the controller-runtime ``Scheme``.

The kf manager registers the Notebook v1, v1alpha1 and v1beta1 types
(``kf/main.go:45-53``); the odh manager additionally registers Gateway API v1 and
v1beta1, OpenShift config/image/oauth/route and the DSPA API (``odh/main.go:62-75``).
Here each kind maps to a REST resource (plural, scope, subresources) so the fake
apiserver, the REST client and the informer cache all agree on URLs and semantics.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple


@dataclass(frozen=True)
class GVK:
    group: str
    version: str
    kind: str

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    def __str__(self) -> str:
        return f"{self.api_version}, Kind={self.kind}"


@dataclass
class ResourceInfo:
    group: str
    kind: str
    plural: str
    namespaced: bool
    versions: Tuple[str, ...]
    storage_version: str
    status_subresource: bool = False
    list_kind: str = ""
    singular: str = ""
    short_names: Tuple[str, ...] = field(default_factory=tuple)

    @property
    def key(self) -> str:
        """Store key: ``plural.group`` (``pods`` for the core group)."""
        return f"{self.plural}.{self.group}" if self.group else self.plural

    def gvk(self, version: Optional[str] = None) -> GVK:
        return GVK(self.group, version or self.storage_version, self.kind)

    def api_version(self, version: Optional[str] = None) -> str:
        return self.gvk(version).api_version

    def path(self, version: Optional[str] = None, namespace: Optional[str] = None, name: Optional[str] = None,
             subresource: Optional[str] = None) -> str:
        v = version or self.storage_version
        base = f"/apis/{self.group}/{v}" if self.group else f"/api/{v}"
        if self.namespaced and namespace:
            base += f"/namespaces/{namespace}"
        base += f"/{self.plural}"
        if name:
            base += f"/{name}"
            if subresource:
                base += f"/{subresource}"
        return base


class Scheme:
    def __init__(self) -> None:
        self._by_kind: Dict[Tuple[str, str], ResourceInfo] = {}
        self._by_plural: Dict[Tuple[str, str], ResourceInfo] = {}
        self._str_cache: Dict[str, ResourceInfo] = {}

    def register(self, info: ResourceInfo) -> ResourceInfo:
        if not info.list_kind:
            info.list_kind = info.kind + "List"
        if not info.singular:
            info.singular = info.kind.lower()
        self._by_kind[(info.group, info.kind)] = info
        self._by_plural[(info.group, info.plural)] = info
        return info

    def for_kind(self, group: str, kind: str) -> Optional[ResourceInfo]:
        return self._by_kind.get((group, kind))

    def for_plural(self, group: str, plural: str) -> Optional[ResourceInfo]:
        return self._by_plural.get((group, plural))

    def for_api_version(self, api_version: str, kind: str) -> Optional[ResourceInfo]:
        group = api_version.rsplit("/", 1)[0] if "/" in api_version else ""
        return self._by_kind.get((group, kind))

    def for_object(self, obj: dict) -> Optional[ResourceInfo]:
        return self.for_api_version(obj.get("apiVersion", ""), obj.get("kind", ""))

    def resolve(self, ref) -> ResourceInfo:
        """Accept a ResourceInfo, a GVK, ``"group/version/Kind"`` / ``"v1/Kind"`` or an object."""
        if type(ref) is str:  # the hot path: kind constants, ~700 calls per notebook lifecycle
            hit = self._str_cache.get(ref)
            if hit is not None:
                return hit
        elif isinstance(ref, ResourceInfo):
            return ref
        if isinstance(ref, GVK):
            info = self.for_kind(ref.group, ref.kind)
        elif isinstance(ref, dict):
            info = self.for_object(ref)
        elif isinstance(ref, str):
            api_version, _, kind = ref.rpartition("/")
            info = self.for_api_version(api_version, kind)
        else:
            info = None
        if info is None:
            raise KeyError(f"no kind registered for {ref!r}")
        if isinstance(ref, str):
            self._str_cache[ref] = info
        return info

    def all(self):
        return list(self._by_kind.values())


def _builtin(s: Scheme) -> None:
    R = ResourceInfo
    for info in (
        R("", "Pod", "pods", True, ("v1",), "v1", True, short_names=("po",)),
        R("", "Service", "services", True, ("v1",), "v1", True, short_names=("svc",)),
        R("", "ServiceAccount", "serviceaccounts", True, ("v1",), "v1", short_names=("sa",)),
        R("", "ConfigMap", "configmaps", True, ("v1",), "v1", short_names=("cm",)),
        R("", "Secret", "secrets", True, ("v1",), "v1"),
        R("", "Event", "events", True, ("v1",), "v1", short_names=("ev",)),
        R("", "Namespace", "namespaces", False, ("v1",), "v1", True, short_names=("ns",)),
        R("", "Node", "nodes", False, ("v1",), "v1", True, short_names=("no",)),
        R("", "Endpoints", "endpoints", True, ("v1",), "v1", short_names=("ep",)),
        R("", "PersistentVolumeClaim", "persistentvolumeclaims", True, ("v1",), "v1", True, short_names=("pvc",)),
        R("apps", "StatefulSet", "statefulsets", True, ("v1",), "v1", True, short_names=("sts",)),
        R("apps", "Deployment", "deployments", True, ("v1",), "v1", True, short_names=("deploy",)),
        R("apps", "DaemonSet", "daemonsets", True, ("v1",), "v1", True, short_names=("ds",)),
        R("networking.k8s.io", "NetworkPolicy", "networkpolicies", True, ("v1",), "v1", short_names=("netpol",)),
        R("rbac.authorization.k8s.io", "Role", "roles", True, ("v1",), "v1"),
        R("rbac.authorization.k8s.io", "RoleBinding", "rolebindings", True, ("v1",), "v1"),
        R("rbac.authorization.k8s.io", "ClusterRole", "clusterroles", False, ("v1",), "v1"),
        R("rbac.authorization.k8s.io", "ClusterRoleBinding", "clusterrolebindings", False, ("v1",), "v1"),
        R("coordination.k8s.io", "Lease", "leases", True, ("v1",), "v1"),
        R("admissionregistration.k8s.io", "MutatingWebhookConfiguration", "mutatingwebhookconfigurations", False,
          ("v1",), "v1"),
        R("apiextensions.k8s.io", "CustomResourceDefinition", "customresourcedefinitions", False, ("v1",), "v1",
          True, short_names=("crd",)),
        R("authentication.k8s.io", "TokenReview", "tokenreviews", False, ("v1",), "v1", True),
        R("certificates.k8s.io", "CertificateSigningRequest", "certificatesigningrequests", False, ("v1",), "v1",
          True, short_names=("csr",)),
        R("authorization.k8s.io", "SubjectAccessReview", "subjectaccessreviews", False, ("v1",), "v1", True),
    ):
        s.register(info)


def _custom(s: Scheme) -> None:
    R = ResourceInfo
    for info in (
        # kf/config/crd/bases/kubeflow.org_notebooks.yaml: v1 storage, v1alpha1/v1beta1 served
        R("kubeflow.org", "Notebook", "notebooks", True, ("v1", "v1alpha1", "v1beta1"), "v1", True),
        R("networking.istio.io", "VirtualService", "virtualservices", True, ("v1alpha3", "v1beta1", "v1"), "v1alpha3",
          short_names=("vs",)),
        R("gateway.networking.k8s.io", "HTTPRoute", "httproutes", True, ("v1", "v1beta1"), "v1", True),
        R("gateway.networking.k8s.io", "Gateway", "gateways", True, ("v1", "v1beta1"), "v1", True),
        R("gateway.networking.k8s.io", "ReferenceGrant", "referencegrants", True, ("v1beta1",), "v1beta1"),
        R("image.openshift.io", "ImageStream", "imagestreams", True, ("v1",), "v1", True, short_names=("is",)),
        R("config.openshift.io", "Proxy", "proxies", False, ("v1",), "v1", True),
        R("route.openshift.io", "Route", "routes", True, ("v1",), "v1", True),
        R("oauth.openshift.io", "OAuthClient", "oauthclients", False, ("v1",), "v1"),
        R("datasciencepipelinesapplications.opendatahub.io", "DataSciencePipelinesApplication",
          "datasciencepipelinesapplications", True, ("v1", "v1alpha1"), "v1", True, short_names=("dspa",)),
    ):
        s.register(info)


SCHEME = Scheme()
_builtin(SCHEME)
_custom(SCHEME)

# Resources whose CRDs are not part of a vanilla Kubernetes cluster.  The fake
# apiserver serves them only when "installed" (mirrors envtest's CRDDirectoryPaths
# in odh/controllers/suite_test.go and lets tests exercise meta.IsNoMatchError paths).
OPTIONAL_CRDS = {
    "virtualservices.networking.istio.io", "httproutes.gateway.networking.k8s.io",
    "gateways.gateway.networking.k8s.io", "referencegrants.gateway.networking.k8s.io",
    "imagestreams.image.openshift.io", "proxies.config.openshift.io", "routes.route.openshift.io",
    "oauthclients.oauth.openshift.io",
    "datasciencepipelinesapplications.datasciencepipelinesapplications.opendatahub.io",
}


# ------------------------------------------------------------------ REST paths


class ParsedPath:
    __slots__ = ("info", "version", "namespace", "name", "sub")

    def __init__(self, info, version, namespace, name, sub):
        self.info, self.version, self.namespace, self.name, self.sub = info, version, namespace, name, sub


def parse_path(path: str) -> Optional[ParsedPath]:
    segs = [s for s in path.split("/") if s]
    if not segs:
        return None
    if segs[0] == "api" and len(segs) >= 3:
        group, version, rest = "", segs[1], segs[2:]
    elif segs[0] == "apis" and len(segs) >= 4:
        group, version, rest = segs[1], segs[2], segs[3:]
    else:
        return None
    ns = None
    if rest[0] == "namespaces" and len(rest) >= 3 and SCHEME.for_plural(group, rest[2]) is not None:
        ns, rest = rest[1], rest[2:]
    info = SCHEME.for_plural(group, rest[0])
    if info is None or len(rest) > 3:
        return None
    name = rest[1] if len(rest) > 1 else None
    sub = rest[2] if len(rest) > 2 else None
    return ParsedPath(info, version, ns, name, sub)
