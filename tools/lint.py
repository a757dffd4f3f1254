#!/usr/bin/env python3
"""Static analysis for this repository: the counterpart of the reference's code-quality CI
(``.github/workflows/code-quality.yaml:17-40`` golangci-lint, ``semgrep.yaml``,
``.gitleaks.toml``, ``kf/third_party/check-license.sh``) for a Python/C++/HIP code base.

    python tools/lint.py            # all checks; exit 1 on any finding
    python tools/lint.py --json     # machine-readable findings

Checks (rule ids follow ``semgrep.yaml`` where the reference has an equivalent):

* Python (AST): ``python-eval-exec-injection``, ``python-pickle-unsafe-load``,
  ``python-yaml-unsafe-load``, ``python-shell-injection-subprocess``, ``python-os-system``,
  ``python-torch-load-unsafe``, ``python-ssl-verify-disabled``, ``http-client-no-timeout``
  (``go-http-client-no-timeout``), ``weak-crypto`` (``go-weak-crypto-md5/sha1``),
  ``bare-except``, ``unused-import`` and ``undefined-name``-free module imports (the
  pyflakes subset golangci-lint's ``unused``/``typecheck`` cover in Go);
* secrets in tracked files (``generic-private-key``, ``generic-aws-access-key``,
  ``generic-github-token``, ``generic-slack-webhook``);
* deployment manifests, rendered per overlay (``deploy/kustomize.py``):
  ``k8s-rbac-wildcard-resources``, ``k8s-rbac-wildcard-verbs``,
  ``k8s-rbac-cluster-admin-binding``, ``k8s-privileged-container``,
  ``k8s-missing-security-context-runAsNonRoot``, ``k8s-hostpath-mount``,
  ``k8s-pod-automount-token`` (pods whose service account has no RBAC must not mount a
  token), ``k8s-rbac-secrets-cluster-access``;
* native code: every C++/HIP source compiles warning-free under ``-Wall -Wextra -Werror``.

A finding that is intended is allowed in place with a comment
``# lint: allow <rule-id> — <reason>`` on the offending line (Python), or through
``MANIFEST_ALLOW`` below with its reason.
"""

from __future__ import annotations

import argparse
import ast
import json
import os
import re
import subprocess
import sys
from typing import Dict, Iterable, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY_DIRS = ("odh_kubeflow_amd", "tools", "tests", "e2e")
PY_FILES = ("bench.py", "__graft_entry__.py")

# (rule, kind, name-regex) → reason.  Manifest findings the design needs.
MANIFEST_ALLOW = {
    ("k8s-hostpath-mount", "DaemonSet", r".*mi355x-node-agent"):
        "the node agent reads amdgpu/KFD sysfs, /proc and the kubelet pod-resources socket, all read-only",
    ("k8s-missing-security-context-runAsNonRoot", "DaemonSet", r".*mi355x-node-agent"):
        "the kubelet pod-resources socket only accepts root; the agent runs with a read-only root filesystem, "
        "all capabilities dropped, no service-account token and no GPU device files",
    ("k8s-rbac-secrets-cluster-access", "ClusterRole", r".*(odh-notebook-controller-manager-role|control-plane-role)"):
        "reference parity: the odh controller reads DSPA object-storage Secrets and writes the Elyra runtime Secret "
        "in every notebook namespace (odh/controllers/notebook_controller.go:89-113)",
}


class Finding(dict):
    def __init__(self, rule: str, path: str, line: int, msg: str):
        super().__init__(rule=rule, path=os.path.relpath(path, ROOT), line=line, msg=msg)

    def __str__(self):
        return f"{self['path']}:{self['line']}: [{self['rule']}] {self['msg']}"


# ------------------------------------------------------------------ python


def _dotted(node) -> str:
    parts = []
    while isinstance(node, ast.Attribute):
        parts.append(node.attr)
        node = node.value
    if isinstance(node, ast.Name):
        parts.append(node.id)
    return ".".join(reversed(parts))


def _kw(call: ast.Call, name: str):
    for k in call.keywords:
        if k.arg == name:
            return k.value
    return None


def _const(node, value) -> bool:
    return isinstance(node, ast.Constant) and node.value == value


def _allowed(lines: List[str], lineno: int, rule: str) -> bool:
    for ln in (lineno, lineno - 1):
        if 0 < ln <= len(lines):
            m = re.search(r"#\s*lint:\s*allow\s+([\w,-]+)", lines[ln - 1])
            if m and rule in m.group(1).split(","):
                return True
    return False


def check_python_source(path: str, text: str) -> List[Finding]:
    try:
        tree = ast.parse(text, path)
    except SyntaxError as e:
        return [Finding("syntax-error", path, e.lineno or 0, str(e))]
    lines = text.splitlines()
    out: List[Finding] = []
    is_test = os.path.relpath(path, ROOT).startswith(("tests" + os.sep, "e2e" + os.sep))

    def add(rule, node, msg):
        ln = getattr(node, "lineno", 0)
        if not _allowed(lines, ln, rule):
            out.append(Finding(rule, path, ln, msg))

    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            add("bare-except", node, "bare `except:` also swallows KeyboardInterrupt/SystemExit/CancelledError")
        if isinstance(node, ast.Attribute) and _dotted(node) == "ssl.CERT_NONE" and not is_test:
            add("python-ssl-verify-disabled", node, "TLS peer verification disabled")
        if not isinstance(node, ast.Call):
            continue
        fn = _dotted(node.func)
        short = fn.rsplit(".", 1)[-1]
        if fn in ("eval", "exec"):
            add("python-eval-exec-injection", node, f"{fn}() on dynamic input")
        if fn in ("pickle.load", "pickle.loads", "cloudpickle.load", "cloudpickle.loads", "dill.load", "dill.loads",
                  "joblib.load", "pandas.read_pickle", "pd.read_pickle"):
            add("python-pickle-unsafe-load", node, f"{fn} executes code from the input")
        if fn in ("yaml.load", "yaml.load_all"):
            loader = _kw(node, "Loader") or (node.args[1] if len(node.args) > 1 else None)
            if loader is None or "Safe" not in _dotted(loader):
                add("python-yaml-unsafe-load", node, f"{fn} without SafeLoader")
        if fn in ("yaml.unsafe_load", "yaml.full_load"):
            add("python-yaml-unsafe-load", node, fn)
        if fn.startswith("subprocess.") and _const(_kw(node, "shell"), True):
            add("python-shell-injection-subprocess", node, f"{fn}(shell=True)")
        if fn in ("os.system", "os.popen"):
            add("python-os-system", node, f"{fn} runs a shell")
        if fn == "torch.load" and not _const(_kw(node, "weights_only"), True):
            add("python-torch-load-unsafe", node, "torch.load without weights_only=True")
        if short in ("get", "post", "put", "patch", "delete", "request") and fn.startswith("requests.") \
                and _kw(node, "timeout") is None:
            add("http-client-no-timeout", node, f"{fn} without timeout=")
        if fn.endswith("urlopen") and _kw(node, "timeout") is None and len(node.args) < 3:
            add("http-client-no-timeout", node, "urlopen without timeout=")
        if fn in ("aiohttp.ClientSession", "ClientSession") and _kw(node, "timeout") is None and not is_test:
            add("http-client-no-timeout", node, "aiohttp.ClientSession without a default timeout=")
        if fn in ("hashlib.md5", "hashlib.sha1") and not _const(_kw(node, "usedforsecurity"), False):
            add("weak-crypto", node, f"{fn} (pass usedforsecurity=False for non-security digests)")
        for k in ("verify", "ssl", "verify_ssl"):
            if _const(_kw(node, k), False) and not is_test:
                add("python-ssl-verify-disabled", node, f"{fn}({k}=False)")
    out.extend(_unused_imports(path, tree, lines))
    return out


def _unused_imports(path: str, tree: ast.Module, lines: List[str]) -> List[Finding]:
    if os.path.basename(path) == "__init__.py":
        return []  # package re-exports
    imported: Dict[str, ast.AST] = {}
    for node in tree.body:
        if isinstance(node, ast.Import):
            for a in node.names:
                imported[(a.asname or a.name).split(".")[0]] = node
        elif isinstance(node, ast.ImportFrom) and node.module != "__future__":
            for a in node.names:
                if a.name != "*":
                    imported[a.asname or a.name] = node
    if not imported:
        return []
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
    exported = set()
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                exported |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    text = "\n".join(lines)
    out = []
    for name, node in imported.items():
        if name in used or name in exported:
            continue
        ln = node.lineno
        if "noqa" in lines[ln - 1] or _allowed(lines, ln, "unused-import"):
            continue
        if re.search(rf"['\"]{re.escape(name)}['\"]", text):  # string-referenced (typing, getattr)
            continue
        out.append(Finding("unused-import", path, ln, f"'{name}' imported but unused"))
    return out


def python_files() -> Iterable[str]:
    for d in PY_DIRS:
        for dirpath, dirnames, files in os.walk(os.path.join(ROOT, d)):
            dirnames[:] = [x for x in dirnames if x not in ("__pycache__", "_lib", "bin")]
            for f in files:
                if f.endswith(".py"):
                    yield os.path.join(dirpath, f)
    for f in PY_FILES:
        if os.path.exists(os.path.join(ROOT, f)):
            yield os.path.join(ROOT, f)


# ------------------------------------------------------------------ secrets

SECRET_PATTERNS = {
    "generic-private-key": re.compile(r"-----BEGIN (?:RSA |EC |DSA |OPENSSH |ENCRYPTED )?PRIVATE KEY-----"),
    "generic-aws-access-key": re.compile(r"\b(?:AKIA|ASIA)[0-9A-Z]{16}\b"),
    "generic-github-token": re.compile(r"\bgh[pousr]_[A-Za-z0-9]{36,}\b"),
    "generic-slack-webhook": re.compile(r"https://hooks\.slack\.com/services/[A-Za-z0-9/]+"),
}


def tracked_files() -> List[str]:
    try:
        out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout
        return [os.path.join(ROOT, f) for f in out.splitlines()]
    except (subprocess.CalledProcessError, OSError):
        return []


def check_secrets(paths: Iterable[str]) -> List[Finding]:
    out = []
    for p in paths:
        if os.path.abspath(p) == os.path.abspath(__file__) or p.endswith((".db", ".png", ".so")):
            continue
        try:
            with open(p, errors="replace") as f:
                for i, line in enumerate(f, 1):
                    for rule, rx in SECRET_PATTERNS.items():
                        if rx.search(line) and "lint: allow" not in line:
                            out.append(Finding(rule, p, i, "possible secret"))
        except (OSError, UnicodeDecodeError):
            continue
    return out


# ------------------------------------------------------------------ manifests


def _manifest_allowed(rule: str, obj: dict) -> bool:
    name = obj["metadata"]["name"]
    return any(r == rule and k == obj["kind"] and re.fullmatch(rx, name) for (r, k, rx) in MANIFEST_ALLOW)


def check_manifests(objs: List[dict], where: str) -> List[Finding]:
    from odh_kubeflow_amd.deploy.kustomize import _pod_spec

    out = []
    path = os.path.join(ROOT, "config", "overlays", where, "kustomization.yaml")

    def add(rule, obj, msg):
        if not _manifest_allowed(rule, obj):
            out.append(Finding(rule, path, 0, f"{obj['kind']}/{obj['metadata']['name']}: {msg}"))

    bound_sas = set()
    for o in objs:
        if o["kind"] in ("RoleBinding", "ClusterRoleBinding"):
            if o["roleRef"]["name"] == "cluster-admin":
                add("k8s-rbac-cluster-admin-binding", o, "binds cluster-admin")
            bound_sas |= {s["name"] for s in o.get("subjects") or [] if s.get("kind") == "ServiceAccount"}
        if o["kind"] in ("Role", "ClusterRole"):
            for r in o.get("rules") or []:
                if "*" in (r.get("resources") or []):
                    add("k8s-rbac-wildcard-resources", o, "resources: ['*']")
                if "*" in (r.get("verbs") or []):
                    add("k8s-rbac-wildcard-verbs", o, "verbs: ['*']")
                if o["kind"] == "ClusterRole" and "secrets" in (r.get("resources") or []) and \
                        set(r.get("verbs") or []) & {"get", "list", "watch"}:
                    add("k8s-rbac-secrets-cluster-access", o, "reads Secrets cluster-wide")
    for o in objs:
        ps = _pod_spec(o)
        if ps is None:
            continue
        for v in ps.get("volumes") or []:
            if "hostPath" in v:
                add("k8s-hostpath-mount", o, f"hostPath {v['hostPath'].get('path')}")
        if ps.get("serviceAccountName") not in bound_sas and ps.get("automountServiceAccountToken") is not False:
            add("k8s-pod-automount-token", o, "service account without RBAC still mounts an API token")
        for c in ps.get("containers") or []:
            sc = c.get("securityContext") or {}
            if sc.get("privileged"):
                add("k8s-privileged-container", o, f"container {c['name']} is privileged")
            if not (sc.get("runAsNonRoot") or (ps.get("securityContext") or {}).get("runAsNonRoot")):
                add("k8s-missing-security-context-runAsNonRoot", o, f"container {c['name']} may run as root")
    return out


def manifest_findings() -> List[Finding]:
    from odh_kubeflow_amd.deploy import kustomize

    out = []
    overlays = os.path.join(ROOT, "config", "overlays")
    for ov in sorted(os.listdir(overlays)):
        out.extend(check_manifests(kustomize.build(os.path.join(overlays, ov)), ov))
    return out


# ------------------------------------------------------------------ native


NATIVE = (
    (["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-pthread"],
     "odh_kubeflow_amd/testing/native/apiserver/apiserver.cpp"),
    (["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-pthread"],
     "odh_kubeflow_amd/ops/csrc/gpu_telemetry.cpp"),
    (["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-fno-strict-aliasing", "{pyinc}"],
     "odh_kubeflow_amd/native/objcore.cpp"),
    (["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
      "-Wno-unused-command-line-argument"], "odh_kubeflow_amd/ops/csrc/gpu_probe.hip"),
    (["/opt/rocm/bin/hipcc", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
      "-Wno-unused-command-line-argument"], "odh_kubeflow_amd/ops/csrc/probe_cli.cpp"),
)


def native_findings() -> List[Finding]:
    import sysconfig

    out = []
    for cmd, src in NATIVE:
        if not os.path.exists(cmd[0]) and cmd[0].startswith("/"):
            continue
        cmd = [c.replace("{pyinc}", "-I" + sysconfig.get_paths()["include"]) for c in cmd]
        r = subprocess.run(cmd + [os.path.join(ROOT, src)], capture_output=True, text=True)
        if r.returncode != 0:
            first = next((ln for ln in r.stderr.splitlines() if "error" in ln or "warning" in ln), r.stderr[:200])
            out.append(Finding("native-warnings", os.path.join(ROOT, src), 0, first.strip()))
    return out


# ------------------------------------------------------------------ main


def run(native: bool = True) -> List[Finding]:
    sys.path.insert(0, ROOT)
    out: List[Finding] = []
    for p in python_files():
        with open(p) as f:
            out.extend(check_python_source(p, f.read()))
    out.extend(check_secrets(tracked_files()))
    out.extend(manifest_findings())
    if native:
        out.extend(native_findings())
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--no-native", action="store_true", help="skip the -Werror compiles")
    a = ap.parse_args(argv)
    found = run(native=not a.no_native)
    if a.json:
        print(json.dumps(found, indent=1))
    else:
        for f in found:
            print(f)
        print(f"{len(found)} finding(s)")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
