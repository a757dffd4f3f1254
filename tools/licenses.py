#!/usr/bin/env python3
"""Third-party licence check (the reference's ``kf/third_party/check-license.sh`` +
``concatenate_license.py`` for Go modules, here for the Python distributions the package
imports at run time).

    python tools/licenses.py            # table; exit 1 if a dependency's licence is unknown
                                        # or not on the permissive allowlist
    python tools/licenses.py --json

Only the runtime package (``odh_kubeflow_amd/``) is scanned — tests and tools may use
more.  Native code links only system libraries (OpenSSL for the apiserver, libamdhip64 /
amdgpu sysfs for the GPU pieces) and the ROCm toolchain, which are not redistributed.
"""

from __future__ import annotations

import argparse
import ast
import json
import os
import sys
from importlib import metadata
from typing import Dict, List, Set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACKAGE = "odh_kubeflow_amd"

# SPDX-ish spellings seen in package metadata, all permissive
ALLOWED = ("mit", "bsd", "apache", "psf", "python software foundation", "isc", "mpl", "unlicense",
           "zlib", "hpnd", "lgpl")


def runtime_imports() -> Set[str]:
    names: Set[str] = set()
    for dirpath, dirnames, files in os.walk(os.path.join(ROOT, PACKAGE)):
        dirnames[:] = [d for d in dirnames if d != "__pycache__"]
        for f in files:
            if not f.endswith(".py"):
                continue
            with open(os.path.join(dirpath, f)) as fh:
                tree = ast.parse(fh.read())
            for node in ast.walk(tree):
                if isinstance(node, ast.Import):
                    names |= {a.name.split(".")[0] for a in node.names}
                elif isinstance(node, ast.ImportFrom) and node.level == 0 and node.module:
                    names.add(node.module.split(".")[0])
    stdlib = set(getattr(sys, "stdlib_module_names", ())) | {"__future__"}
    local = {f[:-3] for f in os.listdir(ROOT) if f.endswith(".py")}  # bench.py, __graft_entry__.py
    return {n for n in names if n not in stdlib and n != PACKAGE and n not in local}


def licence_of(dist: str) -> str:
    md = metadata.metadata(dist)
    lic = (md.get("License-Expression") or md.get("License") or "").strip()
    if lic and len(lic) < 80 and lic.upper() != "UNKNOWN":
        return lic
    classifiers = [c.split("::")[-1].strip() for c in md.get_all("Classifier") or [] if c.startswith("License ::")]
    return "; ".join(classifiers) or (lic.splitlines()[0][:80] if lic else "UNKNOWN")


def report() -> List[Dict[str, str]]:
    dists = metadata.packages_distributions()
    rows = []
    for mod in sorted(runtime_imports()):
        for dist in sorted(set(dists.get(mod, []))) or ["?"]:
            if dist == "?":
                rows.append({"module": mod, "distribution": "?", "version": "?", "license": "UNKNOWN", "ok": False})
                continue
            lic = licence_of(dist)
            ok = any(a in lic.lower() for a in ALLOWED)
            rows.append({"module": mod, "distribution": dist, "version": metadata.version(dist), "license": lic,
                         "ok": ok})
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    rows = report()
    if a.json:
        print(json.dumps(rows, indent=1))
    else:
        for r in rows:
            print(f"{'ok ' if r['ok'] else 'BAD'} {r['module']:<20} {r['distribution']:<22} {r['version']:<12} "
                  f"{r['license']}")
    return 0 if all(r["ok"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
