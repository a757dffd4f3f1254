"""Static analysis and licence checks (the reference's code-quality CI: golangci-lint,
``semgrep.yaml``, gitleaks, ``check-license.sh``) — the repository is clean, and each
rule fires on the pattern it exists for."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import lint  # noqa: E402
import licenses  # noqa: E402


def test_repository_is_lint_clean():
    found = lint.run(native=True)
    assert found == [], "\n".join(str(f) for f in found)


def test_runtime_dependencies_have_permissive_licences():
    rows = licenses.report()
    assert rows and all(r["ok"] for r in rows), rows
    assert {"aiohttp", "prometheus_client", "yaml"} <= {r["module"] for r in rows}


@pytest.mark.parametrize("src,rule", [
    ("eval(x)\n", "python-eval-exec-injection"),
    ("import pickle\npickle.loads(b)\n", "python-pickle-unsafe-load"),
    ("import yaml\nyaml.load(s)\n", "python-yaml-unsafe-load"),
    ("import subprocess\nsubprocess.run(c, shell=True)\n", "python-shell-injection-subprocess"),
    ("import os\nos.system('x')\n", "python-os-system"),
    ("import torch\ntorch.load('p')\n", "python-torch-load-unsafe"),
    ("import requests\nrequests.get(u)\n", "http-client-no-timeout"),
    ("import aiohttp\naiohttp.ClientSession()\n", "http-client-no-timeout"),
    ("import hashlib\nhashlib.md5(b)\n", "weak-crypto"),
    ("import ssl\nc.verify_mode = ssl.CERT_NONE\n", "python-ssl-verify-disabled"),
    ("try:\n    f()\nexcept:\n    pass\n", "bare-except"),
    ("import json\n", "unused-import"),
])
def test_python_rules_fire(src, rule):
    path = os.path.join(ROOT, "odh_kubeflow_amd", "_probe_rule.py")
    assert rule in {f["rule"] for f in lint.check_python_source(path, src)}


def test_inline_allow_comment():
    path = os.path.join(ROOT, "odh_kubeflow_amd", "_probe_rule.py")
    src = "import hashlib\nhashlib.md5(b)  # lint: allow weak-crypto — cache key\n"
    assert lint.check_python_source(path, src) == []
    assert lint.check_python_source(path, "import yaml\nyaml.load(s, Loader=yaml.SafeLoader)\n") == []


def test_manifest_rules_fire():
    pod = {"serviceAccountName": "sa", "containers": [{"name": "c", "securityContext": {"privileged": True}}],
           "volumes": [{"name": "h", "hostPath": {"path": "/"}}]}
    objs = [
        {"kind": "ClusterRole", "metadata": {"name": "r"},
         "rules": [{"apiGroups": ["*"], "resources": ["*"], "verbs": ["*"]}]},
        {"kind": "ClusterRoleBinding", "metadata": {"name": "b"}, "roleRef": {"name": "cluster-admin"},
         "subjects": [{"kind": "ServiceAccount", "name": "other"}]},
        {"kind": "Deployment", "metadata": {"name": "d"}, "spec": {"template": {"spec": pod}}},
    ]
    rules = {f["rule"] for f in lint.check_manifests(objs, "x")}
    assert rules >= {"k8s-rbac-wildcard-resources", "k8s-rbac-wildcard-verbs", "k8s-rbac-cluster-admin-binding",
                     "k8s-privileged-container", "k8s-hostpath-mount", "k8s-pod-automount-token",
                     "k8s-missing-security-context-runAsNonRoot"}


def test_secret_patterns_fire(tmp_path):
    f = tmp_path / "leak.txt"
    f.write_text("-----BEGIN RSA PRIVATE" + " KEY-----\nAKIA" + "ABCDEFGHIJKLMNOP\n")
    assert {x["rule"] for x in lint.check_secrets([str(f)])} == {"generic-private-key", "generic-aws-access-key"}


def test_ci_workflows_reference_existing_targets_and_paths():
    """The CI definitions (.github/workflows) parse and only call make targets, tools and
    paths that exist in the tree."""
    import re

    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    wf_dir = os.path.join(root, ".github", "workflows")
    with open(os.path.join(root, "Makefile")) as f:
        targets = set(re.findall(r"^([a-z0-9][a-z0-9-]*):", f.read(), re.M))
    names = sorted(os.listdir(wf_dir))
    assert {"unit_test.yaml", "code_quality.yaml", "integration_test.yaml", "gpu_test.yaml", "release.yaml"} <= set(names)
    for n in names:
        with open(os.path.join(wf_dir, n)) as f:
            wf = yaml.safe_load(f)
        assert wf.get("jobs"), n
        for job in wf["jobs"].values():
            for step in job["steps"]:
                run = step.get("run") or ""
                for t in re.findall(r"\bmake ((?:[a-z0-9-]+ ?)+)", run):
                    for tgt in t.split():
                        if "=" not in tgt:
                            assert tgt in targets, (n, tgt)
                for path in re.findall(r"\b((?:tools|config|e2e|releasing|\.github)/[\w./-]+)", run):
                    assert os.path.exists(os.path.join(root, path.rstrip("/"))), (n, path)
                cfg = (step.get("with") or {}).get("config")
                if cfg:
                    assert os.path.exists(os.path.join(root, cfg)), (n, cfg)


def test_third_party_imports_are_declared():
    """Every third-party module the package imports (lazy imports included) is a declared
    dependency and installed in the controller / node-agent image; torch comes with the ROCm
    base image.  (grpcio was missing: the node agent's pod-resources source would have reported
    an import error on every node and fallen back to the checkpoint.)"""
    import ast
    import sys

    pkg = os.path.join(ROOT, "odh_kubeflow_amd")
    mods = set()
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                with open(os.path.join(root, f)) as fh:
                    tree = ast.parse(fh.read())
                for n in ast.walk(tree):
                    if isinstance(n, ast.Import):
                        mods.update(a.name.split(".")[0] for a in n.names)
                    elif isinstance(n, ast.ImportFrom) and n.level == 0 and n.module:
                        mods.add(n.module.split(".")[0])
    third = {m for m in mods if m not in sys.stdlib_module_names} - {"odh_kubeflow_amd", "bench", "torch"}
    dist = {"yaml": "pyyaml", "grpc": "grpcio"}
    with open(os.path.join(ROOT, "pyproject.toml")) as f:
        pyproject = f.read()
    with open(os.path.join(ROOT, "images", "Dockerfile")) as f:
        docker = f.read()
    for m in sorted(third):
        d = dist.get(m, m)
        assert f'"{d}"' in pyproject, f"{d} missing from pyproject dependencies"
        assert f" {d}" in docker, f"{d} not installed in images/Dockerfile"
