"""Deployment manifests, generated from the code's own constants.

``python -m odh_kubeflow_amd.deploy.manifests [--out config]`` writes the kustomize tree
(the reference's ``kf/config/**`` + ``odh/config/**``):

* ``crd/`` — ``notebooks.kubeflow.org`` with v1 (storage), v1alpha1, v1beta1 served,
  ``status`` subresource and ``conversion: None`` (identical schemas);
* ``rbac/`` — ClusterRoles from the verbs each controller actually uses (the reference's
  kubebuilder markers, ``odh/controllers/notebook_controller.go:89-113``), leader-election
  Roles, user aggregation roles (``kubeflow-notebooks-{admin,edit,view}``);
* ``manager/`` — the two manager Deployments with the reference flags, probes on
  :8081, metrics on :8080, ``GOMEMLIMIT``-style limits, env from ConfigMaps;
* ``node-agent/`` — the MI355X node agent DaemonSet (``amd.com/gpu.family`` nodes):
  read-only amdgpu telemetry + pod→GPU attribution (``nodeagent/``), no apiserver access,
  no GPU device files, never ``amd.com/gpu`` itself; its enrollment containers obtain the
  node's own serving certificate through a CSR, which the ``node-agent-signer`` Deployment
  issues for the requesting pod's node only (``nodeagent/identity.py``);
* ``webhook/`` — Service + MutatingWebhookConfiguration (``failurePolicy: Fail``);
* ``webhook-certs/`` — outside OpenShift (no service-ca): the serving-cert provisioner
  (``cmd/webhook_certs.py``) as a Job + weekly renewal CronJob with the RBAC it needs
  (the reference's kind CI does this step with ``openssl`` + ``kubectl patch``);
* ``control-plane/`` — the sharded control plane: ``cmd/control_plane.py`` as a
  StatefulSet of N replicas (``--shard=ordinal``: replica k owns the namespaces labelled
  ``notebooks.amd.com/shard=k``; replica k labels the new namespaces that hash to k), one webhook Service
  and MutatingWebhookConfiguration per shard (``namespaceSelector`` on that label) plus
  one for not-yet-assigned namespaces, RBAC = kf ∪ odh roles + namespace labelling;
* ``overlays/{kubeflow,standalone,openshift,mi355x}`` — Istio on/off, OpenShift
  service-ca injection + ``ADD_FSGROUP=false``, MI355X placement + GPU-busy culling
  (ConfigMap settings merged with ``configMapGenerator behavior: merge``, as the
  reference's overlays do); ``overlays/mi355x-sharded`` — the MI355X settings with the
  sharded control plane instead of the two cluster-wide managers;
* ``samples/`` — Notebooks requesting 1 and 8 ``amd.com/gpu`` with the PyTorch-ROCm image.

The CRD is the reference's, structurally equal per version: the full expanded ``core/v1``
PodSpec schema (vendored as data, ``models/schema/podspec.json``) with
``kf/config/crd/patches/validation_patches.yaml`` applied (containers ``minItems: 1``,
required ``name``/``image``), three served versions, v1 storage, status subresource,
``conversion: None`` (``models/crd.py``).
"""

from __future__ import annotations

import argparse
import os
from typing import Dict, List, Optional

import yaml

from ..models.notebook import GPU_RESOURCE
from ..nodeagent.identity import IDENTITY_DOMAIN, SIGNER_NAME

ROCM_NOTEBOOK_IMAGE = "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0"
NAME_PREFIX = "odh-kubeflow-amd-"
WEBHOOK_CERT_SECRET = "odh-notebook-controller-webhook-cert"  # created by service-ca / the certs Job
WEBHOOK_SERVICE = "odh-notebook-controller-webhook-service"
AGENT_TOKEN_SECRET = "mi355x-node-agent-token"  # nodeagent/auth.py TOKEN_SECRET
AGENT_TOKEN_MOUNT = "/var/run/secrets/odh/node-agent"
# the node agents serve HTTPS, each node's agent with a certificate of its own node
# (nodeagent/identity.py): the key is made in the pod (memory-backed emptyDir), the
# certificate issued by the node-agent-signer for the requesting pod's node; the signer's CA
# stays in its Secret, the trust bundle is published to the culler in a ConfigMap
AGENT_NAME = "mi355x-node-agent"
AGENT_SIGNER = "mi355x-node-agent-signer"
AGENT_CA_SECRET = "mi355x-node-agent-ca"  # the signer's CA (ca.crt / ca.key): only the signer reads it
AGENT_TLS_MOUNT = "/var/run/odh/node-agent-tls"
AGENT_ENROLL_ID = 65532  # uid / gid of the enrollment containers, the pod's fsGroup
AGENT_CA_CONFIGMAP = "mi355x-node-agent-ca"
AGENT_CA_MOUNT = "/var/run/odh/node-agent-ca"
MWC_NAME = "mutating-webhook-configuration"
SHARDS = 8  # one control-plane shard per MI355X of an 8-GPU node
CULLER_LITERALS = ["ENABLE_CULLING=false", "CULL_IDLE_TIME=1440", "IDLENESS_CHECK_PERIOD=1",
                   "CULLING_ACTIVITY_SOURCE=jupyter", "CULLING_GPU_BUSY_THRESHOLD=5",
                   "CULLING_GPU_AGENT_PORT=9464", "CULLING_GPU_VRAM_ACTIVE_BYTES=0", "CULL_CHECK_STAMP_EVERY=1"]
CULLER_KEYS = [lit.split("=", 1)[0] for lit in CULLER_LITERALS]
PARAMS_ENV = "USE_ISTIO=false\nISTIO_GATEWAY=kubeflow/kubeflow-gateway\nISTIO_HOST=*\n" \
             "CLUSTER_DOMAIN=cluster.local\nADD_FSGROUP=true\nGPU_NODE_SELECTOR=false\n" \
             "GPU_SHM_SIZE_PER_GPU=\nMULTI_GPU_ENV=\nGPU_DEVICE_GROUPS=\n" \
             "GPU_STARTUP_PROBE=false\nGPU_PROBE_RCCL=false\n"
# GPU_STARTUP_PROBE: the start-up probe for every GPU notebook (else opt-in per notebook,
# amd.com/gpu-probe); GPU_PROBE_RCCL: its RCCL all-reduce for every probed multi-GPU notebook


def params_env(version: str) -> str:
    """The kf controller's ``config`` ConfigMap: the reference's settings (params.env) plus the
    MI355X ones; the start-up probe image is pinned to the release (images/probe.Dockerfile)."""
    return PARAMS_ENV + f"GPU_PROBE_IMAGE={PROBE_IMAGE_NAME}:{version}\n"
# MI355X node settings (overlays mi355x and mi355x-sharded)
# the host groups owning /dev/kfd and /dev/dri/renderD*: HOST-SPECIFIC (Ubuntu allocates the
# render gid dynamically), so the overlays ship it empty — an operator sets the nodes' own gids
# (`stat -c %g /dev/kfd /dev/dri/renderD128` on a node; docs/DEPLOY.md).  A wrong gid would only
# give every GPU pod an unrelated host group, and world-writable device nodes need none.
MI355X_DEVICE_GROUPS = ""
MI355X_PARAMS = ["GPU_NODE_SELECTOR=true", "GPU_SHM_SIZE_PER_GPU=16Gi",
                 # multi-GPU notebooks: RCCL's intra-node IPC over dmabuf (hosts whose amdgpu
                 # driver only offers dmabuf IPC fail hipIpcGetMemHandle otherwise)
                 "MULTI_GPU_ENV=HSA_ENABLE_IPC_MODE_LEGACY=0",
                 # non-root containers of GPU pods get these gids as supplementalGroups
                 f"GPU_DEVICE_GROUPS={MI355X_DEVICE_GROUPS}"]
# CULL_CHECK_STAMP_EVERY: an idle notebook's last_activity_check_timestamp is rewritten on every
# 10th check (10 min at the 1 min period) instead of every check — one Notebook write, admission
# and watch fan-out per idle notebook per 10 periods (controllers/culling.py)
MI355X_CULLER = ["CULLING_ACTIVITY_SOURCE=combined", "ENABLE_CULLING=true", "CULL_CHECK_STAMP_EVERY=10"]
# overlay mi355x: each manager runs its controllers in this many namespace-partitioned worker
# processes (runtime/workers.py; the odh webhook stays on the supervisor's own event loop) —
# one core per worker, so an 8-GPU node's notebooks are not serialised on one Python loop
MI355X_WORKERS = 4
# --webhook-replicas: at 4 streams the one webhook process (the supervisor, which also leads and
# watches cluster-wide) ran ≈75 % busy; 1 / 2 / 4 webhook processes gave 561–572 / 586 / 598–606
# notebooks/s, interleaved (pass r5_p13).  With the final tree (connections recycled, so
# every process gets its share) 3 beat 2 in every interleaved run: 751–760 vs 667–745
# notebooks/s (pass r5_f10, r5_f11)
MI355X_WEBHOOK_REPLICAS = 3
# kf --split-workers: each namespace set served by a notebook-reconciler process and a culler +
# event re-emitter process, as a shard pod does; with 2 webhook processes, against neither, at 4
# streams: 607 / 627 vs 596 / 605 notebooks/s, interleaved (pass r5_p15; split alone
# 590 / 605 vs 560 / 587, pass r5_p14)
MI355X_KF_SPLIT_WORKERS = True
# the odh manager caches ConfigMap/Secret data, as a shard does: the webhook and the reconcilers
# read them from the cache instead of confirming absences live (+12 % notebooks/s at 4 streams,
# interleaved on one box, pass r4_p16); the reference's overlays keep its uncached reads
MI355X_CACHE_CONFIGMAPS = True
# the base manifests carry the development tag; every overlay pins the release tag through
# kustomize `images` (releasing/VERSION, set by tools/release.py — the reference's
# releasing/update-manifests-images + releasing/version/VERSION)
MANAGER_IMAGE_NAME = "quay.io/opendatahub/odh-kubeflow-amd"
MANAGER_IMAGE = MANAGER_IMAGE_NAME + ":main"
PROBE_IMAGE_NAME = MANAGER_IMAGE_NAME + "-gpu-probe"  # images/probe.Dockerfile
CONFORMANCE_IMAGE_NAME = MANAGER_IMAGE_NAME + "-conformance"  # images/conformance.Dockerfile
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def release_version(root: str = REPO_ROOT) -> str:
    with open(os.path.join(root, "releasing", "VERSION")) as f:
        return f.read().strip()


KUBE_RBAC_PROXY_IMAGE = "quay.io/brancz/kube-rbac-proxy:v0.18.1"


# ------------------------------------------------------------------ CRD


def notebook_crd() -> dict:
    """``notebooks.kubeflow.org`` with the reference's full per-version schema (``models/crd.py``)."""
    from ..models.crd import notebook_crd as crd

    return crd()


# ------------------------------------------------------------------ RBAC


def _rule(groups, resources, verbs) -> dict:
    return {"apiGroups": list(groups), "resources": list(resources), "verbs": list(verbs)}


ALL = ["create", "delete", "get", "list", "patch", "update", "watch"]


def kf_role() -> dict:
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": "notebook-controller-role"},
            "rules": [
                _rule([""], ["events"], ["create", "get", "list", "patch", "watch"]),
                _rule([""], ["pods"], ["delete", "get", "list", "watch"]),
                _rule([""], ["services"], ALL),
                _rule(["apps"], ["statefulsets"], ALL),
                _rule(["kubeflow.org"], ["notebooks", "notebooks/finalizers", "notebooks/status"], ALL),
                _rule(["networking.istio.io"], ["virtualservices"], ALL),
                _rule([""], ["nodes"], ["get", "list", "watch"]),
            ]}


def odh_role() -> dict:
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": "odh-notebook-controller-manager-role"},
            "rules": [
                _rule(["authentication.k8s.io"], ["tokenreviews"], ["create"]),
                _rule(["authorization.k8s.io"], ["subjectaccessreviews"], ["create"]),
                _rule(["kubeflow.org"], ["notebooks"], ["get", "list", "watch", "patch", "update"]),
                _rule(["kubeflow.org"], ["notebooks/status"], ["get"]),
                _rule(["kubeflow.org"], ["notebooks/finalizers"], ["update", "patch"]),
                _rule(["gateway.networking.k8s.io"], ["httproutes", "referencegrants"], ALL),
                _rule(["gateway.networking.k8s.io"], ["gateways"], ["get", "list", "watch"]),
                _rule([""], ["services", "serviceaccounts", "secrets", "configmaps"],
                      ["get", "list", "watch", "create", "update", "patch"]),
                _rule(["config.openshift.io"], ["proxies"], ["get", "list", "watch"]),
                _rule(["networking.k8s.io"], ["networkpolicies"], ["get", "list", "watch", "create", "update", "patch"]),
                _rule(["networking.k8s.io"], ["networkpolicies/finalizers"], ["update", "patch"]),
                _rule(["oauth.openshift.io"], ["oauthclients"], ["get", "list", "watch", "update", "patch", "delete"]),
                _rule(["rbac.authorization.k8s.io"], ["roles"], ["get", "list", "watch", "create", "update", "patch"]),
                _rule(["rbac.authorization.k8s.io"], ["rolebindings", "clusterrolebindings"], ALL),
                _rule(["route.openshift.io"], ["routes"], ["get", "list", "watch"]),
                _rule(["image.openshift.io"], ["imagestreams"], ["list", "get", "watch"]),
                _rule(["datasciencepipelinesapplications.opendatahub.io"], ["datasciencepipelinesapplications"],
                      ["get", "list", "watch"]),
                _rule(["datasciencepipelinesapplications.opendatahub.io"], ["datasciencepipelinesapplications/api"],
                      ["get", "create", "update", "patch", "delete"]),
            ]}


def leader_election_role(name: str) -> dict:
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": name},
            "rules": [_rule(["coordination.k8s.io"], ["leases"], ALL), _rule([""], ["events"], ["create", "patch"])]}


def user_cluster_roles() -> List[dict]:
    out = []
    for name, verbs, agg in (("kubeflow-notebooks-admin", ["get", "list", "watch", "create", "delete",
                                                           "deletecollection", "patch", "update"], "admin"),
                             ("kubeflow-notebooks-edit", ["get", "list", "watch", "create", "delete",
                                                          "deletecollection", "patch", "update"], "edit"),
                             ("kubeflow-notebooks-view", ["get", "list", "watch"], "view")):
        out.append({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                    "metadata": {"name": name, "labels": {f"rbac.authorization.kubeflow.org/aggregate-to-kubeflow-{agg}":
                                                          "true"}},
                    "rules": [_rule(["kubeflow.org"], ["notebooks", "notebooks/status"], verbs)]})
    return out


def binding(kind: str, name: str, role: str, sa: str, ns: str = "system") -> dict:
    b = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": kind, "metadata": {"name": name},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": kind.replace("Binding", ""), "name": role},
         "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": ns}]}
    return b


# ------------------------------------------------------------------ workloads


def _probes(port: int = 8081) -> dict:
    return {"livenessProbe": {"httpGet": {"path": "/healthz", "port": port}, "initialDelaySeconds": 15,
                              "periodSeconds": 20},
            "readinessProbe": {"httpGet": {"path": "/readyz", "port": port}, "initialDelaySeconds": 5,
                               "periodSeconds": 10}}


AUDIT_POLICY = """# Audit policy the test apiservers use when DEBUG_WRITE_AUDITLOG=<path> is set (the
# reference's envtest debug aid).  Very verbose: every request about the `developer`
# namespace at RequestResponse level.  Analyse with jq, e.g.
#   jq 'select(.verb != "get" and .verb != "watch" and .verb != "list")' < "$DEBUG_WRITE_AUDITLOG"
apiVersion: audit.k8s.io/v1
kind: Policy
omitStages: []
rules:
  - level: RequestResponse
    namespaces: ["developer"]
"""

# restricted Pod Security profile for every controller container (the node agent is the one
# root container: the kubelet pod-resources socket is root-only; tools/lint.py allows it)
RESTRICTED = {"allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}, "runAsNonRoot": True,
              "seccompProfile": {"type": "RuntimeDefault"}}


def _culler_env() -> List[dict]:
    return [{"name": k, "valueFrom": {"configMapKeyRef": {"name": "notebook-controller-culler-config",
                                                          "key": k, "optional": True}}} for k in CULLER_KEYS] + [
        {"name": "CULLING_GPU_AGENT_TOKEN_FILE", "value": f"{AGENT_TOKEN_MOUNT}/token"},
        {"name": "CULLING_GPU_AGENT_CA_FILE", "value": f"{AGENT_CA_MOUNT}/ca.crt"},
        # an agent's certificate must name the pod's node: <spec.nodeName>.<this domain>
        {"name": "CULLING_GPU_AGENT_IDENTITY_DOMAIN", "value": IDENTITY_DOMAIN}]


def _agent_ca_volume() -> dict:
    """The node agents' trust bundle for the culler (published by the node-agent-signer).
    Optional: until it exists the culler asks no agent (no GPU data; Jupyter decides)."""
    return {"name": "node-agent-ca", "configMap": {"name": AGENT_CA_CONFIGMAP, "optional": True}}


AGENT_CA_MOUNT_SPEC = {"name": "node-agent-ca", "mountPath": AGENT_CA_MOUNT, "readOnly": True}


def _agent_token_volume() -> dict:
    """The node agent / culler shared bearer token (``nodeagent/auth.py``).  Optional: until the
    Secret exists (``cmd/webhook_certs --random-secret`` writes it in the standalone / mi355x
    overlays; an admin elsewhere) the agent refuses data requests and the culler gets no GPU
    data — never idleness.  The kubelet fills the volume once the Secret appears."""
    return {"name": "node-agent-token", "secret": {"secretName": AGENT_TOKEN_SECRET, "optional": True,
                                                   "defaultMode": 0o444}}


AGENT_TOKEN_MOUNT_SPEC = {"name": "node-agent-token", "mountPath": AGENT_TOKEN_MOUNT, "readOnly": True}


def _workers_patches(workers: int, webhook_replicas: int = 1, cache_configmaps: bool = False,
                     kf_split: bool = False) -> List[dict]:
    """``--workers`` for both managers, and the CPU to run them: one core per worker plus the
    supervisor (which leads, aggregates /metrics and, in the odh manager, serves the webhook);
    the odh manager's ``--webhook-replicas`` add a core each (webhook-only processes sharing the
    webhook port); the kf manager's ``--split-workers`` doubles its worker processes (each
    namespace set: notebook reconciler + culler / event re-emitter), the second of each pair
    lightly loaded — 1.5 cores per set."""
    ops = [{"op": "add", "path": "/spec/template/spec/containers/0/args/-", "value": f"--workers={workers}"},
           {"op": "replace", "path": "/spec/template/spec/containers/0/resources/limits/cpu", "value": str(workers + 1)},
           {"op": "replace", "path": "/spec/template/spec/containers/0/resources/requests/cpu", "value": str(workers)}]
    kf = list(ops)
    if kf_split:
        kf = [ops[0], {"op": "add", "path": "/spec/template/spec/containers/0/args/-", "value": "--split-workers"},
              {**ops[1], "value": str(2 * workers + 1)}, {**ops[2], "value": str(workers + workers // 2)}]
    out = [{"target": {"kind": "Deployment", "name": f"{NAME_PREFIX}deployment"},
            "patch": yaml.safe_dump(kf, sort_keys=False)}]
    extra = max(0, webhook_replicas - 1)
    odh = [*ops[:1], *([{"op": "add", "path": "/spec/template/spec/containers/0/args/-",
                         "value": f"--webhook-replicas={webhook_replicas}"}] if extra else []),
           *([{"op": "add", "path": "/spec/template/spec/containers/0/args/-",
               "value": "--cache-configmaps-secrets=true"}] if cache_configmaps else []),
           {**ops[1], "value": str(workers + 1 + extra)}, {**ops[2], "value": str(workers + extra)}]
    out.append({"target": {"kind": "Deployment", "name": f"{NAME_PREFIX}manager"},
                "patch": yaml.safe_dump(odh, sort_keys=False)})
    return out


def kf_deployment() -> dict:
    c = {"name": "manager", "image": MANAGER_IMAGE,
         "command": ["python", "-m", "odh_kubeflow_amd.cmd.kf_manager"],
         "args": ["--enable-leader-election", "--metrics-addr=:8080", "--probe-addr=:8081"],
         "envFrom": [{"configMapRef": {"name": "config"}}],
         "env": _culler_env(),
         "ports": [{"name": "metrics", "containerPort": 8080}, {"name": "probes", "containerPort": 8081}],
         "resources": {"requests": {"cpu": "500m", "memory": "256Mi"}, "limits": {"cpu": "2", "memory": "2Gi"}},
         "volumeMounts": [dict(AGENT_TOKEN_MOUNT_SPEC), dict(AGENT_CA_MOUNT_SPEC)],
         "securityContext": dict(RESTRICTED), **_probes()}
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": "deployment", "labels": {"app": "notebook-controller"}},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "notebook-controller"}},
                     "template": {"metadata": {"labels": {"app": "notebook-controller"}},
                                  "spec": {"serviceAccountName": "service-account", "containers": [c],
                                           "volumes": [_agent_token_volume(), _agent_ca_volume()]}}}}


def odh_deployment() -> dict:
    c = {"name": "manager", "image": MANAGER_IMAGE,
         "command": ["python", "-m", "odh_kubeflow_amd.cmd.odh_manager"],
         "args": ["--leader-elect", f"--kube-rbac-proxy-image=$(KUBE_RBAC_PROXY_IMAGE)",
                  "--webhook-cert-dir=/tmp/k8s-webhook-server/serving-certs", "--webhook-port=8443"],
         "env": [{"name": "KUBE_RBAC_PROXY_IMAGE", "value": KUBE_RBAC_PROXY_IMAGE},
                 {"name": "SET_PIPELINE_RBAC", "value": "true"}, {"name": "SET_PIPELINE_SECRET", "value": "true"},
                 {"name": "INJECT_CLUSTER_PROXY_ENV", "valueFrom": {"configMapKeyRef": {
                     "name": "notebook-controller-setting-config", "key": "INJECT_CLUSTER_PROXY_ENV",
                     "optional": True}}},
                 {"name": "K8S_NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}],
         "ports": [{"name": "webhook", "containerPort": 8443}, {"name": "metrics", "containerPort": 8080},
                   {"name": "probes", "containerPort": 8081}],
         "resources": {"requests": {"cpu": "500m", "memory": "256Mi"}, "limits": {"cpu": "2", "memory": "4Gi"}},
         "volumeMounts": [{"name": "cert", "mountPath": "/tmp/k8s-webhook-server/serving-certs", "readOnly": True}],
         "securityContext": dict(RESTRICTED), **_probes()}
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": "manager", "labels": {"app": "odh-notebook-controller"}},
            "spec": {"replicas": 1, "strategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": "100%"}},
                     "selector": {"matchLabels": {"app": "odh-notebook-controller"}},
                     "template": {"metadata": {"labels": {"app": "odh-notebook-controller"}},
                                  "spec": {"serviceAccountName": "manager", "containers": [c],
                                           "volumes": [_cert_volume()]}}}}


def node_agent_daemonset() -> dict:
    """The production node agent (``cmd/node_agent.py``): read-only amdgpu telemetry + pod→GPU
    attribution.  The agent container has no apiserver access (no token), no GPU device files;
    it reads host ``/sys`` (amdgpu + KFD), host ``/proc`` (pod cgroup of each GPU process), the
    kubelet pod-resources socket and device-plugin checkpoint.  The culler reaches it on the
    hostPort.

    Its serving identity is the node's own (``nodeagent/identity.py``): the ``enroll`` init
    container makes a key in a memory-backed volume and obtains a certificate for this node
    through a CSR (``cmd/node_agent_enroll.py --once``: the agent starts with one), the
    ``enroll-renew`` container renews it.  Only these two mount a service account token — a
    projected one, bound to the pod, which is what the signer checks the node against."""
    node_env = [{"name": "NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                {"name": "HOST_IP", "valueFrom": {"fieldRef": {"fieldPath": "status.hostIP"}}}]
    tls_rw = {"name": "tls", "mountPath": AGENT_TLS_MOUNT}
    sa_mount = {"name": "enroll-token", "mountPath": "/var/run/secrets/kubernetes.io/serviceaccount",
                "readOnly": True}

    def enroll(name: str, once: bool) -> dict:
        return {"name": name, "image": MANAGER_IMAGE,
                "command": ["python", "-m", "odh_kubeflow_amd.cmd.node_agent_enroll"],
                "args": ["--node-name=$(NODE_NAME)", "--host-ip=$(HOST_IP)", f"--cert-dir={AGENT_TLS_MOUNT}"]
                + (["--once"] if once else []),
                "env": node_env, "volumeMounts": [tls_rw, sa_mount],
                "securityContext": {**RESTRICTED, "readOnlyRootFilesystem": True, "runAsUser": AGENT_ENROLL_ID,
                                    "runAsGroup": AGENT_ENROLL_ID},
                "resources": {"requests": {"cpu": "10m", "memory": "32Mi"}, "limits": {"memory": "128Mi"}}}
    c = {"name": "agent", "image": MANAGER_IMAGE,
         "command": ["python", "-m", "odh_kubeflow_amd.cmd.node_agent"],
         "args": ["--port=9464", "--sysfs-root=/host/sys", "--proc-root=/host/proc",
                  "--pod-resources-socket=/var/lib/kubelet/pod-resources/kubelet.sock",
                  "--device-plugin-checkpoint=/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint",
                  f"--token-file={AGENT_TOKEN_MOUNT}/token", f"--tls-cert-dir={AGENT_TLS_MOUNT}"],
         "ports": [{"name": "gpu-activity", "containerPort": 9464, "hostPort": 9464}],
         "livenessProbe": {"httpGet": {"path": "/healthz", "port": 9464, "scheme": "HTTPS"}, "periodSeconds": 20},
         "volumeMounts": [{"name": "sys", "mountPath": "/host/sys", "readOnly": True},
                          {"name": "proc", "mountPath": "/host/proc", "readOnly": True},
                          {"name": "pod-resources", "mountPath": "/var/lib/kubelet/pod-resources"},
                          {"name": "device-plugins", "mountPath": "/var/lib/kubelet/device-plugins",
                           "readOnly": True}, dict(AGENT_TOKEN_MOUNT_SPEC),
                          {**tls_rw, "readOnly": True}],
         # uid 0 explicitly: the image runs as 65532, and the kubelet's pod-resources socket is
         # root-owned 0660 (no capability is needed for that: owner permissions; every
         # capability stays dropped)
         "securityContext": {"runAsUser": 0, "runAsNonRoot": False, "readOnlyRootFilesystem": True,
                             "allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}},
         "resources": {"requests": {"cpu": "50m", "memory": "128Mi"}, "limits": {"memory": "512Mi"}}}
    return {"apiVersion": "apps/v1", "kind": "DaemonSet",
            "metadata": {"name": AGENT_NAME, "labels": {"app": AGENT_NAME}},
            "spec": {"selector": {"matchLabels": {"app": AGENT_NAME}},
                     "template": {"metadata": {"labels": {"app": AGENT_NAME}},
                                  "spec": {"serviceAccountName": AGENT_NAME,
                                           "automountServiceAccountToken": False,
                                           "nodeSelector": {"amd.com/gpu.family": "AI"},
                                           "tolerations": [{"key": GPU_RESOURCE, "operator": "Exists",
                                                            "effect": "NoSchedule"}],
                                           # the enrollment containers write the pair as uid and
                                           # gid 65532, the key 0640; the agent (uid 0, every
                                           # capability dropped: no DAC override) reads it through
                                           # this group, which the kubelet adds to every container
                                           "securityContext": {"fsGroup": AGENT_ENROLL_ID},
                                           "initContainers": [enroll("enroll", once=True)],
                                           "containers": [c, enroll("enroll-renew", once=False)],
                                           "volumes": [{"name": "sys", "hostPath": {"path": "/sys"}},
                                                       {"name": "proc", "hostPath": {"path": "/proc"}},
                                                       {"name": "pod-resources", "hostPath": {
                                                           "path": "/var/lib/kubelet/pod-resources"}},
                                                       {"name": "device-plugins", "hostPath": {
                                                           "path": "/var/lib/kubelet/device-plugins"}},
                                                       _agent_token_volume(),
                                                       # the node's key: in memory, in this pod only
                                                       {"name": "tls", "emptyDir": {"medium": "Memory",
                                                                                    "sizeLimit": "1Mi"}},
                                                       # a token bound to this pod (1 h, rotated by the
                                                       # kubelet): the signer checks its pod's node
                                                       {"name": "enroll-token", "projected": {"sources": [
                                                           {"serviceAccountToken": {"path": "token",
                                                                                    "expirationSeconds": 3600}},
                                                           {"configMap": {"name": "kube-root-ca.crt", "items": [
                                                               {"key": "ca.crt", "path": "ca.crt"}]}},
                                                           {"downwardAPI": {"items": [
                                                               {"path": "namespace", "fieldRef": {
                                                                   "fieldPath": "metadata.namespace"}}]}}]}}]}}}}


def node_agent_rbac() -> List[dict]:
    """The agents' ServiceAccount may submit CSRs and read them back (to collect its
    certificate) — nothing else; the signer decides what a CSR gets."""
    return [{"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": AGENT_NAME}},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
             "metadata": {"name": f"{AGENT_NAME}-csr"},
             "rules": [_rule(["certificates.k8s.io"], ["certificatesigningrequests"], ["create", "get"])]},
            binding("ClusterRoleBinding", f"{AGENT_NAME}-csr", f"{AGENT_NAME}-csr", AGENT_NAME)]


def node_agent_signer_docs() -> List[dict]:
    """The signer (``cmd/node_agent_signer.py``): its CSRs (approve + sign, for its signerName
    only), the agent pods and their DaemonSet (get: the binding check), its CA Secret and the
    trust ConfigMap."""
    sa = "node-agent-signer"
    c = {"name": "signer", "image": MANAGER_IMAGE,
         "command": ["python", "-m", "odh_kubeflow_amd.cmd.node_agent_signer"],
         "args": ["--leader-elect", f"--service-account={AGENT_NAME}", f"--daemonset={AGENT_NAME}",
                  f"--ca-secret={AGENT_CA_SECRET}", f"--ca-configmap={AGENT_CA_CONFIGMAP}"],
         "env": [{"name": "K8S_NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}],
         "ports": [{"name": "metrics", "containerPort": 8080}, {"name": "probes", "containerPort": 8081}],
         "securityContext": dict(RESTRICTED),
         "resources": {"requests": {"cpu": "20m", "memory": "64Mi"}, "limits": {"memory": "256Mi"}},
         **_probes()}
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": sa}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": AGENT_SIGNER},
         "rules": [_rule(["certificates.k8s.io"], ["certificatesigningrequests"], ["get", "list", "watch"]),
                   _rule(["certificates.k8s.io"], ["certificatesigningrequests/approval",
                                                   "certificatesigningrequests/status"], ["update", "patch"]),
                   {**_rule(["certificates.k8s.io"], ["signers"], ["approve", "sign"]),
                    "resourceNames": [SIGNER_NAME]}]},
        binding("ClusterRoleBinding", AGENT_SIGNER, AGENT_SIGNER, sa),
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": AGENT_SIGNER},
         "rules": [_rule([""], ["pods"], ["get"]),
                   {**_rule(["apps"], ["daemonsets"], ["get"]), "resourceNames": [AGENT_NAME]},
                   {**_rule([""], ["secrets"], ["get", "update"]), "resourceNames": [AGENT_CA_SECRET]},
                   _rule([""], ["secrets"], ["create"]),
                   {**_rule([""], ["configmaps"], ["get", "update"]), "resourceNames": [AGENT_CA_CONFIGMAP]},
                   _rule([""], ["configmaps"], ["create"]),
                   _rule(["coordination.k8s.io"], ["leases"], ALL), _rule([""], ["events"], ["create", "patch"])]},
        binding("RoleBinding", AGENT_SIGNER, AGENT_SIGNER, sa),
        {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"name": AGENT_SIGNER, "labels": {"app": AGENT_SIGNER}},
         "spec": {"replicas": 1, "selector": {"matchLabels": {"app": AGENT_SIGNER}},
                  "template": {"metadata": {"labels": {"app": AGENT_SIGNER}},
                               "spec": {"serviceAccountName": sa, "containers": [c]}}}}]


CONFORMANCE_NS = "odh-kubeflow-amd-conformance"
CONFORMANCE_REPORT_DIR = "/tmp/odh-conformance"


def conformance_docs(version: str) -> Dict[str, object]:
    """In-cluster conformance run of the e2e suite (the reference's ``conformance/1.7``:
    a namespace + ServiceAccount + binding, then a test pod that leaves a report and a
    ``done`` file for ``report-pod.sh`` to copy out).  The pod runs ``pytest e2e
    --in-cluster`` with its ServiceAccount and writes a JUnit report."""
    sa = "conformance"
    ns_doc = {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": CONFORMANCE_NS}}
    sa_doc = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": sa, "namespace": CONFORMANCE_NS}}
    role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": "odh-kubeflow-amd-conformance"},
            "rules": [{"apiGroups": ["kubeflow.org"], "resources": ["notebooks"], "verbs": ["*"]},
                      {"apiGroups": ["apps"], "resources": ["statefulsets", "deployments"],
                       "verbs": ["get", "list", "watch", "patch"]},
                      {"apiGroups": [""], "resources": ["pods", "services", "serviceaccounts", "events"],
                       "verbs": ["get", "list", "watch"]},
                      {"apiGroups": [""], "resources": ["configmaps"],
                       "verbs": ["get", "list", "watch", "create", "update", "delete"]},
                      {"apiGroups": ["networking.k8s.io"], "resources": ["networkpolicies"],
                       "verbs": ["get", "list", "watch"]},
                      {"apiGroups": ["gateway.networking.k8s.io"], "resources": ["httproutes", "referencegrants"],
                       "verbs": ["get", "list", "watch"]},
                      {"apiGroups": ["rbac.authorization.k8s.io"], "resources": ["clusterrolebindings"],
                       "verbs": ["get", "list"]},
                      {"apiGroups": ["apiextensions.k8s.io"], "resources": ["customresourcedefinitions"],
                       "verbs": ["get"]},
                      {"apiGroups": ["coordination.k8s.io"], "resources": ["leases"], "verbs": ["get", "list"]}]}
    binding_doc = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                   "metadata": {"name": "odh-kubeflow-amd-conformance"},
                   "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                               "name": "odh-kubeflow-amd-conformance"},
                   "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": CONFORMANCE_NS}]}
    run = (f"mkdir -p {CONFORMANCE_REPORT_DIR}; python -m pytest e2e -v --in-cluster "
           f"--nb-namespace {CONFORMANCE_NS} --junitxml {CONFORMANCE_REPORT_DIR}/junit.xml "
           f"> {CONFORMANCE_REPORT_DIR}/e2e.log 2>&1; echo $? > {CONFORMANCE_REPORT_DIR}/exit_code; "
           f"touch {CONFORMANCE_REPORT_DIR}/done; sleep 86400")
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": "notebook-conformance", "namespace": CONFORMANCE_NS,
                        "labels": {"app": "odh-kubeflow-amd-conformance"}},
           "spec": {"serviceAccountName": sa, "restartPolicy": "Never",
                    "containers": [{"name": "e2e", "image": f"{CONFORMANCE_IMAGE_NAME}:{version}",
                                    "workingDir": "/opt/odh-kubeflow-amd",
                                    "command": ["/bin/sh", "-c", run],
                                    "env": [{"name": "HOME", "value": "/tmp"}],
                                    "securityContext": dict(RESTRICTED),
                                    "resources": {"requests": {"cpu": "200m", "memory": "256Mi"},
                                                  "limits": {"memory": "1Gi"}}}]}}
    return {"setup.yaml": [ns_doc, sa_doc, role, binding_doc], "e2e-conformance.yaml": pod}


def webhook_service() -> dict:
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": "odh-notebook-controller-webhook-service"},
            "spec": {"ports": [{"port": 443, "targetPort": 8443, "protocol": "TCP"}],
                     "selector": {"app": "odh-notebook-controller"}}}


def metrics_service(name: str, app: str) -> dict:
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "labels": {"app": app}},
            "spec": {"ports": [{"name": "metrics", "port": 8080, "targetPort": 8080}], "selector": {"app": app}}}


def mwc() -> dict:
    from ..webhook.server import mutating_webhook_configuration

    o = mutating_webhook_configuration("", service_namespace="system")
    o["webhooks"][0]["clientConfig"].pop("caBundle")
    return o


# ------------------------------------------------------------------ webhook serving cert (non-OpenShift)


def _cert_volume() -> dict:
    """The serving Secret as the webhook server's cert dir: ``tls.crt`` / ``tls.key`` only — the
    Secret also holds the provisioner's long-lived CA key (``webhook/certs.py``), which no
    serving pod needs."""
    return {"name": "cert", "secret": {"secretName": WEBHOOK_CERT_SECRET, "defaultMode": 420,
                                       "items": [{"key": "tls.crt", "path": "tls.crt"},
                                                 {"key": "tls.key", "path": "tls.key"}]}}


def webhook_certs_rbac(mwcs: List[str]) -> List[dict]:
    """Least privilege for the provisioner: get/update of exactly the Secrets it keeps and the
    MutatingWebhookConfigurations it names (``resourceNames``), create of Secrets (create cannot
    be scoped by name) — nothing else in the cluster's admission chain."""
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "webhook-certs"}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "webhook-certs-role"},
         "rules": [{**_rule([""], ["secrets"], ["get", "update"]),
                    "resourceNames": [WEBHOOK_CERT_SECRET, AGENT_TOKEN_SECRET]},
                   _rule([""], ["secrets"], ["create"])]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
         "metadata": {"name": "webhook-certs-cabundle-role"},
         "rules": [{**_rule(["admissionregistration.k8s.io"], ["mutatingwebhookconfigurations"], ["get", "update"]),
                    "resourceNames": list(mwcs)}]},
        binding("RoleBinding", "webhook-certs-rolebinding", "webhook-certs-role", "webhook-certs"),
        binding("ClusterRoleBinding", "webhook-certs-cabundle-rolebinding", "webhook-certs-cabundle-role",
                "webhook-certs")]


def webhook_certs_args(services: List[str], mwcs: List[str]) -> List[str]:
    """``cmd/webhook_certs.py`` arguments.  Names are the *rendered* (prefixed) names: they
    are plain strings to kustomize, so its name-reference fix-ups do not reach them."""
    return ([f"--secret-name={WEBHOOK_CERT_SECRET}"] + [f"--service-name={x}" for x in services]
            + [f"--mwc-name={x}" for x in mwcs] + [f"--random-secret={AGENT_TOKEN_SECRET}"])


def webhook_certs_docs(services: List[str], mwcs: List[str]) -> Dict[str, object]:
    """SA + RBAC + Job + renewal CronJob of the serving-cert provisioner: the Secret the
    webhook server mounts and the caBundle of every MutatingWebhookConfiguration
    (``.github/workflows/odh_notebook_controller_integration_test.yaml:190-216`` does the
    same by hand on kind)."""
    c = {"name": "webhook-certs", "image": MANAGER_IMAGE,
         "command": ["python", "-m", "odh_kubeflow_amd.cmd.webhook_certs"],
         "args": webhook_certs_args(services, mwcs),
         "env": [{"name": "K8S_NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}],
         "securityContext": dict(RESTRICTED),
         "resources": {"requests": {"cpu": "50m", "memory": "64Mi"}, "limits": {"memory": "256Mi"}}}
    pod = {"serviceAccountName": "webhook-certs", "restartPolicy": "OnFailure", "containers": [c]}
    job_spec = {"backoffLimit": 6, "ttlSecondsAfterFinished": 3600, "template": {
        "metadata": {"labels": {"app": "odh-webhook-certs"}}, "spec": pod}}
    return {
        "rbac.yaml": webhook_certs_rbac(mwcs),
        "job.yaml": [
            {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "webhook-certs"}, "spec": job_spec},
            # renewal: re-run weekly; the provisioner reissues within 90 days of expiry (or when a
            # shard's Service is missing from the SANs) and the webhook servers reload the files
            {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": {"name": "webhook-certs-renew"},
             "spec": {"schedule": "17 3 * * 1", "concurrencyPolicy": "Forbid", "jobTemplate": {"spec": job_spec}}}],
    }


# ------------------------------------------------------------------ sharded control plane


def control_plane_role() -> dict:
    """kf ∪ odh manager permissions, plus labelling namespaces (the shard assigner)."""
    rules = kf_role()["rules"] + odh_role()["rules"] + [_rule([""], ["namespaces"], ["get", "list", "watch", "patch"])]
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": "control-plane-role"}, "rules": rules}


def control_plane_statefulset(shards: int) -> dict:
    """One replica per shard; its pod runs ``cmd/control_plane.py`` four times, split by
    ``--controllers``: ``notebook`` (the kf notebook reconciler + event re-emitter + the
    namespace assigner), ``culler``, ``odh`` and ``webhook`` — four event loops, so an admission
    never waits behind a reconcile, the odh pipeline never behind kf (the webhook's own process:
    ``pass r4_p11``), and a new notebook's kf hops never behind the culler's periodic checks
    of every resident notebook (R=1000 checked every second: new-notebook create→Ready 1.14× the
    empty cluster's with the culler apart, 1.32× with it in the kf process; ``pass r5_p5``)."""
    common = ["--shard=ordinal", "--leader-elect", "--kube-rbac-proxy-image=$(KUBE_RBAC_PROXY_IMAGE)"]
    kf = _control_plane_container("manager-kf", common + ["--controllers=notebook", f"--shard-count={shards}",
                                                          "--assign-namespaces", "--assign-policy=balanced"],
                                  8080, 8081, role="kf")
    culler = _control_plane_container("manager-culler", common + [
        "--controllers=culler,events", "--metrics-bind-address=:8086", "--health-probe-bind-address=:8087"], 8086, 8087,
        role="culler")
    odh = _control_plane_container("manager-odh", common + [
        "--controllers=odh", "--metrics-bind-address=:8082", "--health-probe-bind-address=:8083"], 8082, 8083,
        role="odh")
    wh = _control_plane_container("manager-webhook", common + [
        "--controllers=webhook", "--metrics-bind-address=:8084", "--health-probe-bind-address=:8085",
        "--webhook-cert-dir=/tmp/k8s-webhook-server/serving-certs", "--webhook-port=8443"], 8084, 8085,
        role="webhook")
    labels = {"app": "notebook-control-plane"}
    return {"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "control-plane", "labels": labels},
            "spec": {"replicas": shards, "serviceName": "control-plane", "podManagementPolicy": "Parallel",
                     "selector": {"matchLabels": labels},
                     "template": {"metadata": {"labels": labels},
                                  "spec": {"serviceAccountName": "control-plane", "containers": [kf, culler, odh, wh],
                                           "volumes": [_cert_volume(), _agent_token_volume(),
                                                       _agent_ca_volume()]}}}}


_CP_PORT_NAMES = {"kf": ("metrics", "probes"), "culler": ("metrics-culler", "probes-culler"),
                  "odh": ("metrics-odh", "probes-odh"), "webhook": ("metrics-wh", "probes-wh")}


def _control_plane_container(name: str, args: list, metrics: int, probes: int, role: str) -> dict:
    mname, pname = _CP_PORT_NAMES[role]
    c = {"name": name, "image": MANAGER_IMAGE,
         "command": ["python", "-m", "odh_kubeflow_amd.cmd.control_plane"],
         "args": args,
         "envFrom": [{"configMapRef": {"name": "config"}}],
         "env": [{"name": "POD_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}},
                 {"name": "K8S_NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}},
                 {"name": "KUBE_RBAC_PROXY_IMAGE", "value": KUBE_RBAC_PROXY_IMAGE},
                 {"name": "SET_PIPELINE_RBAC", "value": "true"}, {"name": "SET_PIPELINE_SECRET", "value": "true"},
                 {"name": "INJECT_CLUSTER_PROXY_ENV", "valueFrom": {"configMapKeyRef": {
                     "name": "notebook-controller-setting-config", "key": "INJECT_CLUSTER_PROXY_ENV",
                     "optional": True}}}] + _culler_env(),
         "ports": ([{"name": "webhook", "containerPort": 8443}] if role == "webhook" else []) + [
             {"name": mname, "containerPort": metrics}, {"name": pname, "containerPort": probes}],
         "resources": {"requests": {"cpu": "500m", "memory": "256Mi"}, "limits": {"cpu": "2", "memory": "2Gi"}},
         # the culler container reads the node agents' token (GPU-busy culling); the webhook one serves TLS
         "volumeMounts": {"culler": [dict(AGENT_TOKEN_MOUNT_SPEC), dict(AGENT_CA_MOUNT_SPEC)], "kf": [], "odh": [],
                          "webhook": [{"name": "cert", "mountPath": "/tmp/k8s-webhook-server/serving-certs",
                                       "readOnly": True}]}[role],
         "securityContext": dict(RESTRICTED), **_probes(probes)}
    return c


def _webhook_svc(name: str, selector: dict) -> dict:
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name},
            "spec": {"ports": [{"port": 443, "targetPort": 8443, "protocol": "TCP"}], "selector": selector}}


def control_plane_docs(shards: int, prefix: str = NAME_PREFIX) -> Dict[str, object]:
    """The ``control-plane/`` base.  A shard's webhook Service selects its pod by the
    StatefulSet pod-name label, whose value is the *rendered* pod name (``prefix`` +
    ``control-plane-<k>``): label values are not renamed by kustomize."""
    from ..controllers.setup import SHARD_LABEL
    from ..webhook.server import mutating_webhook_configuration

    def mwc_for(svc: str, name: str, selector: dict) -> dict:
        o = mutating_webhook_configuration("", service_namespace="system", service_name=svc, name=name,
                                           namespace_selector=selector)
        o["webhooks"][0]["clientConfig"].pop("caBundle")
        return o

    svcs, mwcs = [], []
    for k in range(shards):
        svcs.append(_webhook_svc(f"control-plane-webhook-{k}",
                                 {"statefulset.kubernetes.io/pod-name": f"{prefix}control-plane-{k}"}))
        mwcs.append(mwc_for(f"control-plane-webhook-{k}", f"notebook-webhook-shard-{k}",
                            {"matchLabels": {SHARD_LABEL: str(k)}}))
    # namespaces the assigner has not labelled yet: any shard admits them (reads live)
    svcs.append(_webhook_svc("control-plane-webhook", {"app": "notebook-control-plane"}))
    mwcs.append(mwc_for("control-plane-webhook", "notebook-webhook-unassigned",
                        {"matchExpressions": [{"key": SHARD_LABEL, "operator": "DoesNotExist"}]}))
    return {
        "rbac.yaml": [{"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "control-plane"}},
                      control_plane_role(),
                      binding("ClusterRoleBinding", "control-plane-rolebinding", "control-plane-role", "control-plane"),
                      leader_election_role("control-plane-leader-election-role"),
                      binding("RoleBinding", "control-plane-leader-election-rolebinding",
                              "control-plane-leader-election-role", "control-plane")],
        "statefulset.yaml": control_plane_statefulset(shards),
        "services.yaml": [{"apiVersion": "v1", "kind": "Service", "metadata": {"name": "control-plane"},
                           "spec": {"clusterIP": "None", "selector": {"app": "notebook-control-plane"},
                                    "ports": [{"name": "metrics", "port": 8080, "targetPort": 8080},
                                              {"name": "metrics-odh", "port": 8082, "targetPort": 8082},
                                              {"name": "metrics-wh", "port": 8084, "targetPort": 8084}]}}] + svcs,
        "webhooks.yaml": mwcs,
    }


def sample(name: str, gpus: int, version: str = "v1", auth: bool = False) -> dict:
    ann = {"notebooks.opendatahub.io/inject-auth": "true"} if auth else {}
    c = {"name": name, "image": ROCM_NOTEBOOK_IMAGE,
         "resources": {"limits": {GPU_RESOURCE: str(gpus), "memory": f"{64 * gpus}Gi", "cpu": str(8 * gpus)},
                       "requests": {GPU_RESOURCE: str(gpus), "memory": f"{32 * gpus}Gi", "cpu": str(4 * gpus)}},
         "volumeMounts": [{"name": "dshm", "mountPath": "/dev/shm"}]}
    return {"apiVersion": f"kubeflow.org/{version}", "kind": "Notebook",
            "metadata": {"name": name, **({"annotations": ann} if ann else {})},
            "spec": {"template": {"spec": {"containers": [c], "volumes": [
                # /dev/shm sized for RCCL/xGMI collectives of a multi-GPU notebook
                {"name": "dshm", "emptyDir": {"medium": "Memory", "sizeLimit": f"{16 * gpus}Gi"}}]}}}}


def _certs_args_patches(services: List[str], mwcs: List[str]) -> List[dict]:
    """JSON6902 patches setting the provisioner's arguments in the Job and the CronJob, and the
    MutatingWebhookConfiguration names its ClusterRole may touch."""
    args = webhook_certs_args(services, mwcs)
    patches = [{"target": {"kind": kind, "name": name},
                "patch": yaml.safe_dump([{"op": "replace", "path": path, "value": args}], sort_keys=False)}
               for kind, name, path in (("Job", "webhook-certs", "/spec/template/spec/containers/0/args"),
                                        ("CronJob", "webhook-certs-renew",
                                         "/spec/jobTemplate/spec/template/spec/containers/0/args"))]
    patches.append({"target": {"kind": "ClusterRole", "name": "webhook-certs-cabundle-role"},
                    "patch": yaml.safe_dump([{"op": "replace", "path": "/rules/0/resourceNames",
                                              "value": list(mwcs)}], sort_keys=False)})
    return patches


def kustomization(resources: List[str], **extra) -> dict:
    k = {"apiVersion": "kustomize.config.k8s.io/v1beta1", "kind": "Kustomization", "resources": resources}
    k.update(extra)
    return k


def tree(version: Optional[str] = None) -> Dict[str, object]:
    """path → document (or list of documents); ``version`` = the image tag every overlay
    pins (default: ``releasing/VERSION``)."""
    version = version or release_version()
    images = [{"name": MANAGER_IMAGE_NAME, "newTag": version}]
    t: Dict[str, object] = {}
    t["crd/bases/kubeflow.org_notebooks.yaml"] = notebook_crd()
    t["crd/kustomization.yaml"] = kustomization(["bases/kubeflow.org_notebooks.yaml"])
    t["rbac/kf_role.yaml"] = kf_role()
    t["rbac/odh_role.yaml"] = odh_role()
    t["rbac/leader_election_roles.yaml"] = [leader_election_role("notebook-controller-leader-election-role"),
                                            leader_election_role("odh-notebook-controller-leader-election-role")]
    t["rbac/role_bindings.yaml"] = [
        binding("ClusterRoleBinding", "notebook-controller-role-binding", "notebook-controller-role", "service-account"),
        binding("ClusterRoleBinding", "odh-notebook-controller-manager-rolebinding",
                "odh-notebook-controller-manager-role", "manager"),
        binding("RoleBinding", "notebook-controller-leader-election-rolebinding",
                "notebook-controller-leader-election-role", "service-account"),
        binding("RoleBinding", "odh-notebook-controller-leader-election-rolebinding",
                "odh-notebook-controller-leader-election-role", "manager")]
    t["rbac/service_accounts.yaml"] = [{"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": n}}
                                       for n in ("service-account", "manager")]
    t["user-rbac/user_cluster_roles.yaml"] = user_cluster_roles()
    t["user-rbac/kustomization.yaml"] = kustomization(["user_cluster_roles.yaml"])
    t["rbac/kustomization.yaml"] = kustomization(sorted(p.split("/", 1)[1] for p in t if p.startswith("rbac/")
                                                        and not p.endswith("kustomization.yaml")) + ["../user-rbac"])
    t["manager/kf_manager.yaml"] = kf_deployment()
    t["manager/odh_manager.yaml"] = odh_deployment()
    t["manager/services.yaml"] = [metrics_service("notebook-controller-service", "notebook-controller"),
                                  metrics_service("odh-notebook-controller-service", "odh-notebook-controller")]
    generators = [{"name": "config", "envs": ["params.env"]},
                  {"name": "notebook-controller-culler-config", "literals": list(CULLER_LITERALS)}]
    t["manager/kustomization.yaml"] = kustomization(["kf_manager.yaml", "odh_manager.yaml", "services.yaml"],
                                                    configMapGenerator=generators,
                                                    generatorOptions={"disableNameSuffixHash": True})
    t["manager/params.env"] = params_env(version)
    t["node-agent/daemonset.yaml"] = node_agent_daemonset()
    t["node-agent/rbac.yaml"] = node_agent_rbac()
    t["node-agent/signer.yaml"] = node_agent_signer_docs()
    t["node-agent/kustomization.yaml"] = kustomization(["rbac.yaml", "daemonset.yaml", "signer.yaml"])
    t["webhook/service.yaml"] = webhook_service()
    t["webhook/manifests.yaml"] = mwc()
    t["webhook/kustomization.yaml"] = kustomization(["service.yaml", "manifests.yaml"])
    # serving cert for the two-manager layout (non-OpenShift overlays)
    for f, doc in webhook_certs_docs([NAME_PREFIX + WEBHOOK_SERVICE], [NAME_PREFIX + MWC_NAME]).items():
        t[f"webhook-certs/{f}"] = doc
    t["webhook-certs/kustomization.yaml"] = kustomization(["rbac.yaml", "job.yaml"])
    # sharded control plane (one cmd/control_plane.py replica per MI355X)
    cp = control_plane_docs(SHARDS)
    for f, doc in cp.items():
        t[f"control-plane/{f}"] = doc
    t["control-plane/params.env"] = params_env(version)
    t["control-plane/kustomization.yaml"] = kustomization(
        ["rbac.yaml", "statefulset.yaml", "services.yaml", "webhooks.yaml"],
        configMapGenerator=generators, generatorOptions={"disableNameSuffixHash": True})
    t["default/kustomization.yaml"] = kustomization(["../crd", "../rbac", "../manager", "../webhook", "../node-agent"],
                                                    namespace="opendatahub", namePrefix=NAME_PREFIX, images=images)
    t["overlays/standalone/kustomization.yaml"] = kustomization(["../../default", "../../webhook-certs"],
                                                                namespace="opendatahub", images=images)
    t["overlays/kubeflow/kustomization.yaml"] = kustomization(
        ["../../default", "../../webhook-certs"], namespace="kubeflow", images=images,
        configMapGenerator=[{"name": "config", "behavior": "merge", "literals": ["USE_ISTIO=true"]}])
    # OpenShift: service-ca serves the webhook; the node agents' per-node identities come from
    # the node-agent signer as everywhere (a service-ca certificate names a Service, not a node)
    t["overlays/openshift/kustomization.yaml"] = kustomization(
        ["../../default"], images=images,
        configMapGenerator=[{"name": "config", "behavior": "merge", "literals": ["ADD_FSGROUP=false"]}],
        patches=[{"target": {"kind": "Service", "name": ".*webhook-service"}, "patch":
                  "- op: add\n  path: /metadata/annotations\n  value:\n    service.beta.openshift.io/"
                  f"serving-cert-secret-name: {WEBHOOK_CERT_SECRET}\n"},
                 {"target": {"kind": "MutatingWebhookConfiguration"}, "patch":
                  "- op: add\n  path: /metadata/annotations\n  value:\n    service.beta.openshift.io/"
                  "inject-cabundle: \"true\"\n"}])
    mi355x_generators = [{"name": "config", "behavior": "merge", "literals": list(MI355X_PARAMS)},
                         {"name": "notebook-controller-culler-config", "behavior": "merge",
                          "literals": list(MI355X_CULLER)}]
    t["overlays/mi355x/kustomization.yaml"] = kustomization(["../../default", "../../webhook-certs"],
                                                            namespace="opendatahub", images=images,
                                                            configMapGenerator=mi355x_generators,
                                                            patches=_workers_patches(MI355X_WORKERS, MI355X_WEBHOOK_REPLICAS,
                                                                                     MI355X_CACHE_CONFIGMAPS,
                                                                                     MI355X_KF_SPLIT_WORKERS))
    # the serving cert covers every shard's Service; every shard's configuration gets the caBundle
    svc_names = [NAME_PREFIX + o["metadata"]["name"] for o in cp["services.yaml"][1:]]
    mwc_names = [NAME_PREFIX + o["metadata"]["name"] for o in cp["webhooks.yaml"]]
    t["overlays/mi355x-sharded/kustomization.yaml"] = kustomization(
        ["../../crd", "../../user-rbac", "../../node-agent", "../../webhook-certs", "../../control-plane"],
        namespace="opendatahub", namePrefix=NAME_PREFIX, configMapGenerator=mi355x_generators, images=images,
        patches=_certs_args_patches(svc_names, mwc_names))
    # in-cluster conformance run of the e2e suite (not part of any overlay; make conformance-run)
    for f, doc in conformance_docs(version).items():
        t[f"conformance/{f}"] = doc
    # debug aid: the test apiservers' audit policy (DEBUG_WRITE_AUDITLOG, apiserver/audit.py)
    t["debug/audit-policy.yaml"] = AUDIT_POLICY
    t["samples/notebook_v1_1gpu.yaml"] = sample("rocm-pytorch-1gpu", 1)
    t["samples/notebook_v1_8gpu_auth.yaml"] = sample("rocm-pytorch-8gpu", 8, auth=True)
    t["samples/notebook_v1alpha1.yaml"] = sample("rocm-pytorch-v1alpha1", 1, "v1alpha1")
    t["samples/notebook_v1beta1.yaml"] = sample("rocm-pytorch-v1beta1", 1, "v1beta1")
    return t


class _Dumper(yaml.SafeDumper):
    """Block style for structure, flow style (``[a, b]``) for short lists of scalars."""


def _represent_list(dumper, data):
    flow = 0 < len(data) <= 8 and all(isinstance(x, (str, int, float, bool)) or x is None for x in data) \
        and sum(len(str(x)) for x in data) <= 72
    return dumper.represent_sequence("tag:yaml.org,2002:seq", data, flow_style=flow)


_Dumper.add_representer(list, _represent_list)


def write(out: str, version: Optional[str] = None) -> List[str]:
    written = []
    for path, doc in sorted(tree(version).items()):
        full = os.path.join(out, path)
        os.makedirs(os.path.dirname(full), exist_ok=True)
        with open(full, "w") as f:
            f.write("# generated by `python -m odh_kubeflow_amd.deploy.manifests` — do not edit\n")
            if isinstance(doc, str):
                f.write(doc)
            elif isinstance(doc, list):
                yaml.dump_all(doc, f, Dumper=_Dumper, sort_keys=False)
            else:
                yaml.dump(doc, f, Dumper=_Dumper, sort_keys=False)
        written.append(full)
    return written


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), "config"))
    a = p.parse_args(argv)
    for w in write(a.out):
        print(w)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
