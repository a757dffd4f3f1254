"""Generated deployment manifests: CRD shape + schema, kustomize tree integrity, RBAC
coverage of every kind the controllers touch, samples valid against the CRD."""

import os

import pytest
import yaml

from odh_kubeflow_amd.deploy import manifests
from odh_kubeflow_amd.models import openapi
from odh_kubeflow_amd.models.notebook import notebook

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_crd_names_versions_and_status():
    crd = manifests.notebook_crd()
    spec = crd["spec"]
    assert crd["metadata"]["name"] == "notebooks.kubeflow.org"
    assert spec["names"] == {"kind": "Notebook", "listKind": "NotebookList", "plural": "notebooks",
                             "singular": "notebook"}
    assert spec["scope"] == "Namespaced" and spec["conversion"] == {"strategy": "None"}
    assert [(v["name"], v["served"], v["storage"]) for v in spec["versions"]] == [
        ("v1", True, True), ("v1alpha1", True, False), ("v1beta1", True, False)]
    assert all(v["subresources"] == {"status": {}} for v in spec["versions"])
    st = openapi.crd_version_schema(crd, "v1")["properties"]["status"]
    assert set(st["properties"]) == {"conditions", "readyReplicas", "containerState"}
    assert set(st["properties"]["conditions"]["items"]["properties"]) == {
        "type", "status", "lastProbeTime", "lastTransitionTime", "reason", "message"}


@pytest.mark.parametrize("version", ["v1", "v1alpha1", "v1beta1"])
def test_crd_schema_validation(version):
    schema = openapi.crd_version_schema(manifests.notebook_crd(), version)
    assert openapi.validate(schema, notebook("nb", "ns", gpus=8, version=version)) == []
    bad = notebook("nb", "ns")
    bad["spec"]["template"]["spec"]["containers"] = []
    assert any("at least 1 items" in e for e in openapi.validate(schema, bad))
    bad["spec"]["template"]["spec"]["containers"] = [{"name": "x"}]
    assert openapi.validate(schema, bad) == ["spec.template.spec.containers[0].image: Required value"]
    st = {"status": {"readyReplicas": 1, "conditions": [{"type": "Ready", "status": "True"}], "containerState": {}}}
    assert openapi.validate(schema, {**notebook("nb", "ns"), **st}) == []
    assert openapi.validate(schema, {**notebook("nb", "ns"), "status": {"readyReplicas": "x", "conditions": [],
                                                                         "containerState": {}}})


def test_checked_in_config_matches_generator():
    for path, doc in manifests.tree().items():
        full = os.path.join(ROOT, "config", path)
        assert os.path.exists(full), f"run `python -m odh_kubeflow_amd.deploy.manifests`: missing {path}"
        with open(full) as f:
            text = f.read()
        if isinstance(doc, str):
            assert text.endswith(doc)
        elif isinstance(doc, list):
            assert list(yaml.safe_load_all(text)) == doc
        else:
            assert yaml.safe_load(text) == doc, path


def test_kustomizations_reference_existing_files():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "config")):
        if "kustomization.yaml" not in files:
            continue
        k = yaml.safe_load(open(os.path.join(dirpath, "kustomization.yaml")))
        for r in k.get("resources", []):
            assert os.path.exists(os.path.join(dirpath, r)), (dirpath, r)
        for g in k.get("configMapGenerator", []):
            for e in g.get("envs", []):
                assert os.path.exists(os.path.join(dirpath, e))


def _allowed(role, group, resource, verb):
    for r in role["rules"]:
        if group in r["apiGroups"] and resource in r["resources"] and (verb in r["verbs"] or "*" in r["verbs"]):
            return True
    return False


def test_rbac_covers_controller_access():
    kf, odh = manifests.kf_role(), manifests.odh_role()
    for res, verb in (("statefulsets", "create"), ("statefulsets", "update"), ("services", "create"),
                      ("notebooks/status", "update"), ("virtualservices", "create")):
        group = {"statefulsets": "apps", "services": "", "notebooks/status": "kubeflow.org",
                 "virtualservices": "networking.istio.io"}[res]
        assert _allowed(kf, group, res, verb), res
    assert _allowed(kf, "", "pods", "delete") and _allowed(kf, "", "events", "create")
    for group, res, verb in (("gateway.networking.k8s.io", "httproutes", "delete"),
                             ("gateway.networking.k8s.io", "referencegrants", "create"),
                             ("rbac.authorization.k8s.io", "clusterrolebindings", "delete"),
                             ("networking.k8s.io", "networkpolicies", "update"),
                             ("kubeflow.org", "notebooks", "patch"), ("", "configmaps", "create"),
                             ("", "serviceaccounts", "create"), ("oauth.openshift.io", "oauthclients", "delete"),
                             ("image.openshift.io", "imagestreams", "list")):
        assert _allowed(odh, group, res, verb), (group, res, verb)


def test_samples_request_mi355x_and_validate():
    crd = manifests.notebook_crd()
    for name in ("notebook_v1_1gpu.yaml", "notebook_v1_8gpu_auth.yaml", "notebook_v1alpha1.yaml",
                 "notebook_v1beta1.yaml"):
        doc = yaml.safe_load(open(os.path.join(ROOT, "config", "samples", name)))
        v = doc["apiVersion"].split("/")[1]
        assert openapi.validate(openapi.crd_version_schema(crd, v), doc) == []
        res = doc["spec"]["template"]["spec"]["containers"][0]["resources"]
        assert int(res["limits"]["amd.com/gpu"]) in (1, 8)
        assert "rocm" in doc["spec"]["template"]["spec"]["containers"][0]["image"]


# ------------------------------------------------------------------ rendered overlays

OVERLAYS = ("standalone", "kubeflow", "openshift", "mi355x", "mi355x-sharded")


def _render(overlay):
    from odh_kubeflow_amd.deploy import kustomize

    return kustomize.build(os.path.join(ROOT, "config", "overlays", overlay))


def _by(objs, kind):
    return {o["metadata"]["name"]: o for o in objs if o["kind"] == kind}


def _pod_specs(objs):
    from odh_kubeflow_amd.deploy.kustomize import _pod_spec

    for o in objs:
        ps = _pod_spec(o)
        if ps is not None:
            yield o, ps


def test_overlay_configmap_settings_merge_without_touching_other_configmaps():
    """Overlay settings go through ``configMapGenerator behavior: merge`` on the ``config``
    ConfigMap (as the reference's overlays do); a ``.*config`` JSON6902 target would also hit
    ``notebook-controller-culler-config`` and fail to build."""
    def cms(overlay):
        return {n.replace("odh-kubeflow-amd-", ""): o.get("data") for n, o in _by(_render(overlay), "ConfigMap").items()}

    base = cms("standalone")
    assert base["config"]["USE_ISTIO"] == "false" and base["config"]["ADD_FSGROUP"] == "true"
    assert cms("kubeflow")["config"]["USE_ISTIO"] == "true"
    assert cms("openshift")["config"]["ADD_FSGROUP"] == "false"
    for overlay in ("mi355x", "mi355x-sharded"):
        c = cms(overlay)
        assert c["config"]["GPU_NODE_SELECTOR"] == "true" and c["config"]["GPU_SHM_SIZE_PER_GPU"] == "16Gi"
        assert c["config"]["MULTI_GPU_ENV"] == "HSA_ENABLE_IPC_MODE_LEGACY=0"
        cull = c["notebook-controller-culler-config"]
        assert cull["ENABLE_CULLING"] == "true" and cull["CULLING_ACTIVITY_SOURCE"] == "combined"
        assert cull["CULL_IDLE_TIME"] == "1440" and "USE_ISTIO" not in cull
    for overlay in OVERLAYS:  # the culler ConfigMap never receives the params keys
        assert set(cms(overlay)["notebook-controller-culler-config"]) == set(
            x.split("=")[0] for x in manifests.CULLER_LITERALS)


def test_broad_configmap_regex_patch_fails_like_kustomize(tmp_path):
    """The renderer reproduces kustomize's failure for the old ``.*config`` target."""
    from odh_kubeflow_amd.deploy import kustomize

    base = tmp_path / "base"
    base.mkdir()
    (base / "kustomization.yaml").write_text(yaml.safe_dump({
        "configMapGenerator": [{"name": "config", "literals": ["A=1"]},
                               {"name": "culler-config", "literals": ["B=2"]}],
        "generatorOptions": {"disableNameSuffixHash": True}, "namePrefix": "p-"}))
    ov = tmp_path / "ov"
    ov.mkdir()
    (ov / "kustomization.yaml").write_text(yaml.safe_dump({
        "resources": ["../base"],
        "patches": [{"target": {"kind": "ConfigMap", "name": ".*config"},
                     "patch": "- op: replace\n  path: /data/A\n  value: '3'\n"}]}))
    with pytest.raises(kustomize.KustomizeError, match="culler-config"):
        kustomize.build(str(ov))


@pytest.mark.parametrize("overlay", OVERLAYS)
def test_overlay_references_resolve(overlay):
    """Every name a rendered overlay refers to exists in it: ConfigMaps, ServiceAccounts,
    roles, webhook Services, the serving-cert Secret/Services/MWCs the certs Job manages."""
    objs = _render(overlay)
    cms, sas, svcs = _by(objs, "ConfigMap"), _by(objs, "ServiceAccount"), _by(objs, "Service")
    roles = {**_by(objs, "Role"), **_by(objs, "ClusterRole")}
    mwcs = _by(objs, "MutatingWebhookConfiguration")
    for o in objs:
        if o["kind"] not in manifests_cluster_scoped():
            assert o["metadata"].get("namespace"), (overlay, o["kind"], o["metadata"]["name"])
    ns = {o["metadata"]["namespace"] for o in objs if o["metadata"].get("namespace")}
    assert len(ns) == 1
    pod_labels = []
    cert_secret_mounts = set()
    for o, ps in _pod_specs(objs):
        assert ps["serviceAccountName"] in sas, (o["metadata"]["name"], ps["serviceAccountName"])
        pod_labels.append(((o.get("spec") or {}).get("template") or {}).get("metadata", {}).get("labels") or {})
        for c in ps["containers"]:
            for ef in c.get("envFrom") or []:
                assert ef["configMapRef"]["name"] in cms
            for e in c.get("env") or []:
                ref = (e.get("valueFrom") or {}).get("configMapKeyRef")
                if ref and not ref.get("optional"):
                    assert ref["name"] in cms
                if ref and ref["name"] in cms:
                    assert ref["key"] in cms[ref["name"]]["data"], (ref, overlay)
        for v in ps.get("volumes") or []:
            if "secret" in v and v["secret"]["secretName"] == manifests.WEBHOOK_CERT_SECRET:
                cert_secret_mounts.add(v["secret"]["secretName"])
    for b in list(_by(objs, "RoleBinding").values()) + list(_by(objs, "ClusterRoleBinding").values()):
        assert b["roleRef"]["name"] in roles, b["metadata"]["name"]
        for sub in b["subjects"]:
            assert sub["name"] in sas and sub["namespace"] in ns, (b["metadata"]["name"], sub)
    for name, w in mwcs.items():
        svc = w["webhooks"][0]["clientConfig"]["service"]
        assert svc["name"] in svcs and svc["namespace"] in ns, (name, svc)
        sel = svcs[svc["name"]]["spec"]["selector"]
        assert any(all(lb.get(k) == v for k, v in sel.items()) for lb in pod_labels) or \
            "statefulset.kubernetes.io/pod-name" in sel, (name, sel)
    assert cert_secret_mounts == {manifests.WEBHOOK_CERT_SECRET}
    jobs = _by(objs, "Job")
    if overlay == "openshift":
        assert not jobs  # service-ca provides the cert and the caBundle
        return
    for jname, path in (("webhook-certs", ("spec",)), ("webhook-certs-renew", ("spec", "jobTemplate", "spec"))):
        job = {n.replace("odh-kubeflow-amd-", ""): o for n, o in {**jobs, **_by(objs, "CronJob")}.items()}[jname]
        for p in path:
            job = job[p]
        args = job["template"]["spec"]["containers"][0]["args"]
        want_svcs = {a.split("=", 1)[1] for a in args if a.startswith("--service-name=")}
        want_mwcs = {a.split("=", 1)[1] for a in args if a.startswith("--mwc-name=")}
        assert want_svcs and want_svcs <= set(svcs) and want_mwcs == set(mwcs), (overlay, want_svcs, want_mwcs)
        assert f"--secret-name={manifests.WEBHOOK_CERT_SECRET}" in args


def manifests_cluster_scoped():
    from odh_kubeflow_amd.deploy.kustomize import CLUSTER_SCOPED

    return CLUSTER_SCOPED


def test_sharded_overlay_shape():
    """mi355x-sharded: one control-plane replica per MI355X, each shard's webhook Service
    selects exactly its replica, each shard's configuration selects its namespaces, and
    not-yet-assigned namespaces go to any shard."""
    objs = _render("mi355x-sharded")
    # the two cluster-wide managers are not deployed (the node agents' signer is)
    assert list(_by(objs, "Deployment")) == ["odh-kubeflow-amd-mi355x-node-agent-signer"]
    (sts,) = _by(objs, "StatefulSet").values()
    n = sts["spec"]["replicas"]
    assert n == manifests.SHARDS == 8
    # the shard pod: the control plane split into a kf (notebook), a culler, an odh and a webhook process
    kf, cull, odh, wh = sts["spec"]["template"]["spec"]["containers"]
    assert "--shard=ordinal" in kf["args"] and f"--shard-count={n}" in kf["args"] and "--assign-namespaces" in kf["args"]
    assert "--controllers=notebook" in kf["args"] and "--controllers=culler,events" in cull["args"]
    assert "--controllers=odh" in odh["args"] and "--controllers=webhook" in wh["args"]
    for c in (cull, odh, wh):
        assert "--shard=ordinal" in c["args"] and "--assign-namespaces" not in c["args"]
    assert [p["containerPort"] for p in kf["ports"]] == [8080, 8081]
    assert [p["containerPort"] for p in cull["ports"]] == [8086, 8087]
    assert [p["containerPort"] for p in odh["ports"]] == [8082, 8083]
    assert [p["containerPort"] for p in wh["ports"]] == [8443, 8084, 8085]
    assert len({p["name"] for c in (kf, cull, odh, wh) for p in c["ports"]}) == 9  # pod-unique port names
    assert [c["readinessProbe"]["httpGet"]["port"] for c in (kf, cull, odh, wh)] == [8081, 8087, 8083, 8085]
    assert [v["name"] for v in wh["volumeMounts"]] == ["cert"] and odh["volumeMounts"] == [] == kf["volumeMounts"]
    # the culler asks the node agents (GPU-busy culling): their token and CA
    assert {v["mountPath"] for v in cull["volumeMounts"]} == {manifests.AGENT_TOKEN_MOUNT_SPEC["mountPath"],
                                                                manifests.AGENT_CA_MOUNT_SPEC["mountPath"]}
    svcs = _by(objs, "Service")
    mwcs = _by(objs, "MutatingWebhookConfiguration")
    assert len(mwcs) == n + 1
    for k in range(n):
        w = mwcs[f"odh-kubeflow-amd-notebook-webhook-shard-{k}"]["webhooks"][0]
        assert w["namespaceSelector"] == {"matchLabels": {"notebooks.amd.com/shard": str(k)}}
        svc = svcs[w["clientConfig"]["service"]["name"]]
        assert svc["spec"]["selector"] == {"statefulset.kubernetes.io/pod-name": f"{sts['metadata']['name']}-{k}"}
    w = mwcs["odh-kubeflow-amd-notebook-webhook-unassigned"]["webhooks"][0]
    assert w["namespaceSelector"]["matchExpressions"] == [{"key": "notebooks.amd.com/shard", "operator": "DoesNotExist"}]
    role = _by(objs, "ClusterRole")["odh-kubeflow-amd-control-plane-role"]
    assert _allowed(role, "", "namespaces", "patch") and _allowed(role, "apps", "statefulsets", "create")
    assert _allowed(role, "gateway.networking.k8s.io", "httproutes", "delete")


def test_kustomize_images_transformer_and_release_tag(tmp_path):
    import shutil

    from odh_kubeflow_amd.deploy import kustomize, manifests

    assert kustomize.split_image("registry:5000/org/img:v1@sha256:ab") == ("registry:5000/org/img", "v1", "sha256:ab")
    assert kustomize.split_image("registry:5000/org/img") == ("registry:5000/org/img", None, None)
    # overlays pin the release tag; the base keeps the development tag
    tag = manifests.release_version()
    for ov in ("standalone", "kubeflow", "openshift", "mi355x", "mi355x-sharded"):
        imgs = {c["image"] for d in kustomize.build(os.path.join(ROOT, "config", "overlays", ov))
                for c in ((kustomize._pod_spec(d) or {}).get("containers") or []) if "odh-kubeflow-amd" in c["image"]}
        assert imgs == {f"{manifests.MANAGER_IMAGE_NAME}:{tag}"}, (ov, imgs)
    base = yaml.safe_load(open(os.path.join(ROOT, "config", "manager", "kf_manager.yaml")))
    assert base["spec"]["template"]["spec"]["containers"][0]["image"].endswith(":main")
    # the release tool: VERSION, __version__, regenerated overlays
    os.makedirs(tmp_path / "odh_kubeflow_amd")
    shutil.copy(os.path.join(ROOT, "odh_kubeflow_amd", "__init__.py"), tmp_path / "odh_kubeflow_amd" / "__init__.py")
    import importlib.util

    spec = importlib.util.spec_from_file_location("release_tool", os.path.join(ROOT, "tools", "release.py"))
    rel = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rel)
    changed = rel.release("v9.8.7-rc.1", str(tmp_path))
    assert "releasing/VERSION" in changed and (tmp_path / "releasing" / "VERSION").read_text().strip() == "v9.8.7-rc.1"
    assert '__version__ = "9.8.7rc1"' in (tmp_path / "odh_kubeflow_amd" / "__init__.py").read_text()
    docs = kustomize.build(str(tmp_path / "config" / "overlays" / "mi355x-sharded"))
    imgs = {c["image"] for d in docs for c in ((kustomize._pod_spec(d) or {}).get("containers") or [])
            if "odh-kubeflow-amd" in c["image"]}
    assert imgs == {f"{manifests.MANAGER_IMAGE_NAME}:v9.8.7-rc.1"}
    with pytest.raises(ValueError):
        rel.pep440("1.2")


def test_conformance_bundle_runs_the_e2e_suite_in_cluster():
    setup = list(yaml.safe_load_all(open(os.path.join(ROOT, "config", "conformance", "setup.yaml"))))
    pod = yaml.safe_load(open(os.path.join(ROOT, "config", "conformance", "e2e-conformance.yaml")))
    kinds_ = [d["kind"] for d in setup]
    assert kinds_ == ["Namespace", "ServiceAccount", "ClusterRole", "ClusterRoleBinding"]
    ns = setup[0]["metadata"]["name"]
    assert pod["metadata"]["namespace"] == ns and pod["spec"]["serviceAccountName"] == setup[1]["metadata"]["name"]
    c = pod["spec"]["containers"][0]
    assert c["image"] == f"{manifests.CONFORMANCE_IMAGE_NAME}:{manifests.release_version()}"
    cmd = c["command"][-1]
    assert "pytest e2e" in cmd and "--in-cluster" in cmd and f"--nb-namespace {ns}" in cmd and "done" in cmd
    assert c["securityContext"]["runAsNonRoot"] and c["securityContext"]["allowPrivilegeEscalation"] is False
    # the ServiceAccount may do what the suite does: notebooks, culler ConfigMap, rollouts
    rules = setup[2]["rules"]
    assert any(r["resources"] == ["notebooks"] and r["verbs"] == ["*"] for r in rules)
    assert any("deployments" in r["resources"] and "patch" in r["verbs"] for r in rules)
    assert any(r["resources"] == ["configmaps"] and "update" in r["verbs"] for r in rules)


@pytest.mark.parametrize("overlay", ["standalone", "kubeflow", "mi355x", "mi355x-sharded"])
def test_webhook_certs_rbac_is_scoped_to_its_objects(overlay):
    """The cert provisioner may get/update exactly the MutatingWebhookConfigurations it keeps
    the caBundle of (by name) and exactly its Secrets — a compromised Job pod cannot rewrite
    any other admission webhook of the cluster.  No list, patch or delete anywhere."""
    objs = _render(overlay)
    mwc_names = sorted(_by(objs, "MutatingWebhookConfiguration"))
    job = next(o for o in objs if o["kind"] == "Job" and o["metadata"]["name"].endswith("webhook-certs"))
    args = job["spec"]["template"]["spec"]["containers"][0]["args"]
    assert sorted(a.split("=", 1)[1] for a in args if a.startswith("--mwc-name=")) == mwc_names
    (cr,) = [o for n, o in _by(objs, "ClusterRole").items() if n.endswith("webhook-certs-cabundle-role")]
    (rule,) = cr["rules"]
    assert rule["resources"] == ["mutatingwebhookconfigurations"] and sorted(rule["verbs"]) == ["get", "update"]
    assert sorted(rule["resourceNames"]) == mwc_names
    (role,) = [o for n, o in _by(objs, "Role").items() if n.endswith("webhook-certs-role")]
    named = {r["resources"][0]: r for r in role["rules"] if r.get("resourceNames")}
    assert sorted(named) == ["secrets"]
    assert all(sorted(r["verbs"]) == ["get", "update"] for r in named.values())
    assert sorted(named["secrets"]["resourceNames"]) == sorted([manifests.WEBHOOK_CERT_SECRET,
                                                                manifests.AGENT_TOKEN_SECRET])
    unnamed = [r for r in role["rules"] if not r.get("resourceNames")]
    assert [sorted(r["verbs"]) for r in unnamed] == [["create"]]
    # the webhook pods get the serving pair only, never the CA key; no pod mounts the agents' CA
    # Secret (only the signer reads it, through the API)
    for o, ps in _pod_specs(objs):
        for v in ps.get("volumes") or []:
            if (v.get("secret") or {}).get("secretName") == manifests.WEBHOOK_CERT_SECRET:
                assert sorted(i["key"] for i in v["secret"]["items"]) == ["tls.crt", "tls.key"], o["metadata"]
            assert (v.get("secret") or {}).get("secretName") != manifests.AGENT_CA_SECRET


def test_mi355x_overlay_runs_manager_workers_and_webhook_replicas():
    """Overlay mi355x (the reference's two-Deployment layout): both managers with ``--workers=4``
    and a CPU request to match; the kf manager's workers split (notebook | culler,events), the odh
    manager with two webhook processes.  Other overlays run none of it."""
    deps = _by(_render("mi355x"), "Deployment")
    kf = deps["odh-kubeflow-amd-deployment"]["spec"]["template"]["spec"]["containers"][0]
    odh = deps["odh-kubeflow-amd-manager"]["spec"]["template"]["spec"]["containers"][0]
    assert "--workers=4" in kf["args"] and "--split-workers" in kf["args"]
    assert not any(a.startswith("--webhook-replicas") for a in kf["args"])
    assert kf["resources"]["requests"]["cpu"] == "6" and kf["resources"]["limits"]["cpu"] == "9"
    assert "--workers=4" in odh["args"] and "--webhook-replicas=3" in odh["args"]
    assert "--cache-configmaps-secrets=true" in odh["args"] and not any("cache-configmaps" in a for a in kf["args"])
    assert odh["resources"]["requests"]["cpu"] == "6" and odh["resources"]["limits"]["cpu"] == "7"
    plain = _by(_render("standalone"), "Deployment")
    for d in plain.values():
        assert not any(a.startswith(("--workers", "--webhook-replicas", "--cache-configmaps", "--split-workers"))
                       for a in d["spec"]["template"]["spec"]["containers"][0]["args"])


def test_node_agent_identity_plumbing():
    """each node's agent enrolls its own identity.  The DaemonSet's enroll init
    container and renewal sidecar alone mount a (projected, pod-bound) token; the agent reads the
    pair from a memory-backed volume, read-only; the agents' SA may only create/get CSRs; the
    signer may approve/sign for its own signerName only and reads the agent pods; the culler
    checks the node name."""
    from odh_kubeflow_amd.nodeagent.identity import IDENTITY_DOMAIN, SIGNER_NAME

    for overlay in ("mi355x", "mi355x-sharded", "openshift"):
        objs = _render(overlay)
        (ds,) = _by(objs, "DaemonSet").values()
        ps = ds["spec"]["template"]["spec"]
        assert ps["automountServiceAccountToken"] is False
        assert [c["name"] for c in ps["initContainers"]] == ["enroll"] and "--once" in ps["initContainers"][0]["args"]
        conts = {c["name"]: c for c in ps["containers"]}
        assert set(conts) == {"agent", "enroll-renew"}
        token_vol = next(v for v in ps["volumes"] if v["name"] == "enroll-token")
        assert token_vol["projected"]["sources"][0]["serviceAccountToken"]["expirationSeconds"] == 3600
        for c in [*ps["initContainers"], *ps["containers"]]:
            mounts = {m["name"]: m for m in c.get("volumeMounts") or []}
            assert ("enroll-token" in mounts) == (c["name"] != "agent"), c["name"]
        agent_tls = next(m for m in conts["agent"]["volumeMounts"] if m["name"] == "tls")
        assert agent_tls["readOnly"] is True
        assert next(v for v in ps["volumes"] if v["name"] == "tls")["emptyDir"]["medium"] == "Memory"
        crs = _by(objs, "ClusterRole")
        (agent_cr,) = [o for n, o in crs.items() if n.endswith("mi355x-node-agent-csr")]
        assert agent_cr["rules"] == [{"apiGroups": ["certificates.k8s.io"], "resources": ["certificatesigningrequests"],
                                      "verbs": ["create", "get"]}]
        (signer_cr,) = [o for n, o in crs.items() if n.endswith("mi355x-node-agent-signer")]
        signers = [r for r in signer_cr["rules"] if r["resources"] == ["signers"]]
        assert signers == [{"apiGroups": ["certificates.k8s.io"], "resources": ["signers"],
                            "verbs": ["approve", "sign"], "resourceNames": [SIGNER_NAME]}]
        envs = [e for o, p in _pod_specs(objs) for c in p["containers"] for e in c.get("env") or []
                if e["name"] == "CULLING_GPU_AGENT_IDENTITY_DOMAIN"]
        assert envs and all(e["value"] == IDENTITY_DOMAIN for e in envs)


def test_node_agent_can_read_the_key_its_enroll_containers_write():
    """the enrollment containers write the node key into the shared
    emptyDir as their own uid; the agent container runs as another uid with every capability
    dropped (no CAP_DAC_OVERRIDE / CAP_DAC_READ_SEARCH), so it reads the key only through
    the file's mode bits: owner (same uid), or group via the pod's fsGroup — which the kubelet
    adds to every container's supplementary groups and gives the emptyDir (setgid)."""
    from odh_kubeflow_amd.deploy.manifests import AGENT_TLS_MOUNT, node_agent_daemonset
    from odh_kubeflow_amd.nodeagent.identity import KEY_FILE_MODE

    spec = node_agent_daemonset()["spec"]["template"]["spec"]
    fs_group = spec["securityContext"]["fsGroup"]
    writers = [c for c in spec["initContainers"] + spec["containers"] if c["name"].startswith("enroll")]
    agent = next(c for c in spec["containers"] if c["name"] == "agent")
    assert writers and all(c["securityContext"]["runAsGroup"] == fs_group for c in writers)
    owner_uid = writers[0]["securityContext"]["runAsUser"]
    assert {c["securityContext"]["runAsUser"] for c in writers} == {owner_uid}
    caps = set(agent["securityContext"].get("capabilities", {}).get("drop", []))
    assert "ALL" in caps  # no DAC override: permission bits decide
    agent_uid = agent["securityContext"]["runAsUser"]
    agent_groups = {fs_group} | set(spec["securityContext"].get("supplementalGroups", []))
    readable = ((agent_uid == owner_uid and KEY_FILE_MODE & 0o400) or (fs_group in agent_groups and KEY_FILE_MODE & 0o040)
                or KEY_FILE_MODE & 0o004)
    assert readable
    assert not KEY_FILE_MODE & 0o007  # and nobody else
    # the agent mounts that same volume (read-only) where the enrollment containers write
    tls = lambda c: [vm for vm in c["volumeMounts"] if vm["mountPath"] == AGENT_TLS_MOUNT]  # noqa: E731
    assert [vm["name"] for vm in tls(agent)] == [vm["name"] for vm in tls(writers[0])] and tls(agent)[0]["readOnly"]
