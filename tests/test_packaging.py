"""What ships: production entry points stay free of the test platform, torch and HIP.

* the static import closure (module- and function-level imports) of every production entry
  point reaches neither ``odh_kubeflow_amd.testing`` nor ``torch``;
* importing them in a fresh interpreter with ``torch`` blocked works, loads no HIP/HSA
  runtime library and leaves ``odh_kubeflow_amd.testing`` unimported — what the slim
  controller and node-agent images (``images/Dockerfile``) rely on;
* the wheel excludes the testing package and the test-only console script.

Reference counterpart: the manager images are ``ubi9/ubi-minimal`` plus one static Go binary
(``kf/Dockerfile:45``, ``odh/Dockerfile:43``); nothing of envtest ships in them.
"""

from __future__ import annotations

import ast
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "odh_kubeflow_amd"
ENTRY_POINTS = [f"{PKG}.cmd.control_plane", f"{PKG}.cmd.kf_manager", f"{PKG}.cmd.odh_manager",
                f"{PKG}.cmd.node_agent", f"{PKG}.cmd.webhook_certs"]


def _path_of(mod: str):
    p = os.path.join(ROOT, *mod.split("."))
    if os.path.isdir(p):
        return os.path.join(p, "__init__.py")
    return p + ".py" if os.path.exists(p + ".py") else None


def _imports(mod: str):
    p = _path_of(mod)
    tree = ast.parse(open(p).read())
    pkg = mod if p.endswith("__init__.py") else mod.rsplit(".", 1)[0]
    for n in ast.walk(tree):
        if isinstance(n, ast.Import):
            for a in n.names:
                yield a.name, n.lineno
        elif isinstance(n, ast.ImportFrom):
            if n.level:
                base = pkg.split(".")
                if n.level > 1:
                    base = base[: len(base) - (n.level - 1)]
                m = ".".join(base + ([n.module] if n.module else []))
            else:
                m = n.module or ""
            yield m, n.lineno
            for a in n.names:
                yield f"{m}.{a.name}", n.lineno


def import_closure(roots):
    """module → "importer:line" for everything reachable from ``roots`` (package modules are
    followed; names that are not modules, and third-party modules, are leaves)."""
    seen = {}
    stack = [(r, "<root>") for r in roots]
    while stack:
        mod, frm = stack.pop()
        if mod in seen:
            continue
        if mod.startswith(PKG + ".") or mod == PKG:
            if _path_of(mod) is None:
                continue  # an imported name, not a module
            seen[mod] = frm
            stack.extend((im, f"{mod}:{ln}") for im, ln in _imports(mod) if im not in seen)
        else:
            seen[mod] = frm
    return seen


def test_static_closure_has_no_testing_or_torch():
    seen = import_closure(ENTRY_POINTS)
    bad = {m: f for m, f in seen.items() if m.startswith(PKG + ".testing") or m.split(".")[0] == "torch"}
    assert not bad, f"production entry points reach the test platform / torch: {bad}"
    assert f"{PKG}.ops.telemetry" in seen  # the closure walk is real: the node agent's sampler is in it


def test_closure_detects_a_testing_import():
    # the checker itself: the benchmark shard does use the test platform
    seen = import_closure([f"{PKG}.parallel.shard"])
    assert any(m.startswith(PKG + ".testing") for m in seen)


_PROBE = r"""
import importlib, importlib.abc, json, sys
class Block(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path=None, target=None):
        if name == "torch" or name.startswith("torch."):
            raise ImportError("torch is not in the production image")
        return None
sys.meta_path.insert(0, Block())
mods = sys.argv[1:]
for m in mods:
    importlib.import_module(m)
maps = open("/proc/self/maps").read()
print(json.dumps({
    "testing": sorted(k for k in sys.modules if k.startswith("odh_kubeflow_amd.testing")),
    "torch": "torch" in sys.modules,
    "hip": [lib for lib in ("libamdhip64", "libhsa-runtime64", "libodh_gpu_probe") if lib in maps],
}))
"""


def test_entry_points_import_without_torch_or_hip():
    import json

    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env["PYTHONPATH"] = ROOT
    out = subprocess.run([sys.executable, "-c", _PROBE, *ENTRY_POINTS], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res == {"testing": [], "torch": False, "hip": []}, res


def test_wheel_excludes_test_platform():
    try:
        import tomllib  # py3.11+
    except ImportError:
        import tomli as tomllib
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as f:
        proj = tomllib.load(f)
    find = proj["tool"]["setuptools"]["packages"]["find"]
    assert f"{PKG}.testing*" in find.get("exclude", []) and f"{PKG}.testing" in find.get("exclude", [])
    scripts = proj["project"]["scripts"]
    assert not any(".testing." in v for v in scripts.values()), scripts
    data = proj["tool"]["setuptools"]["package-data"][PKG]
    assert not any(d.startswith("native/apiserver") or d.startswith("native/bin") for d in data), data
