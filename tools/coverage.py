"""Line coverage of the package under the CPU test suite, per component flag.

    python tools/coverage.py [--flag kf=80 --flag odh=80 ...] [-- <pytest args>]

The reference uploads per-component coverage with separate flags and a 2 % threshold
(``.codecov.yml:19-32``).  No coverage package is installed here, so this is a small
tracer of its own: ``sys.settrace`` / ``threading.settrace`` with a global hook that only
returns a line tracer for frames whose code lives in ``odh_kubeflow_amd/`` (other code
runs untraced), executable lines from the compiled code objects (``co_lines``), the test
run in-process through ``pytest.main``.  Code that only runs in child processes (the
multi-process e2e tests) is not counted.

Writes ``coverage.json`` (per file and per flag) and prints a summary; ``--flag NAME=PCT``
fails the run when a component is under ``PCT`` percent.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import types
from collections import defaultdict
from typing import Dict, Set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "odh_kubeflow_amd") + os.sep

# component flags (the reference's per-component codecov flags, mapped onto this tree)
FLAGS = {
    "kf": ("controllers/notebook.py", "controllers/culling.py", "controllers/metrics.py", "utils/"),
    "odh": ("controllers/odh/", "webhook/"),
    "runtime": ("runtime/", "tracing/"),
    "apiserver": ("apiserver/", "models/"),
    "platform": ("kubelet/", "nodeagent/", "ops/", "notebook_server/"),
    "deploy": ("deploy/", "cmd/", "parallel/", "cluster.py"),
}

_hits: Dict[str, Set[int]] = defaultdict(set)


def _local(frame, event, arg):
    if event == "line":
        _hits[frame.f_code.co_filename].add(frame.f_lineno)
    return _local


def _global(frame, event, arg):
    if frame.f_code.co_filename.startswith(PKG):
        _hits[frame.f_code.co_filename].add(frame.f_lineno)
        return _local
    return None


def executable_lines(path: str) -> Set[int]:
    with open(path, "rb") as f:
        src = f.read()
    try:
        code = compile(src, path, "exec", dont_inherit=True)
    except SyntaxError:
        return set()
    lines: Set[int] = set()
    stack = [code]
    while stack:
        c = stack.pop()
        lines.update(ln for _, _, ln in c.co_lines() if ln is not None)
        stack.extend(k for k in c.co_consts if isinstance(k, types.CodeType))
    # docstring-only / module-level constant lines are executed at import: keep them
    return lines


def flag_of(rel: str) -> str:
    for flag, prefixes in FLAGS.items():
        if any(rel == p or rel.startswith(p) for p in prefixes):
            return flag
    return "other"


def report() -> dict:
    files = {}
    per_flag = defaultdict(lambda: [0, 0])
    for dirpath, _, names in os.walk(PKG):
        for n in names:
            if not n.endswith(".py"):
                continue
            path = os.path.join(dirpath, n)
            rel = os.path.relpath(path, PKG)
            ex = executable_lines(path)
            if not ex:
                continue
            hit = _hits.get(path, set()) & ex
            files[rel] = {"lines": len(ex), "hit": len(hit), "pct": round(100.0 * len(hit) / len(ex), 1)}
            f = per_flag[flag_of(rel)]
            f[0] += len(hit)
            f[1] += len(ex)
    flags = {k: {"hit": h, "lines": t, "pct": round(100.0 * h / t, 1) if t else 0.0} for k, (h, t) in per_flag.items()}
    tot_h = sum(v["hit"] for v in files.values())
    tot = sum(v["lines"] for v in files.values())
    return {"total": {"hit": tot_h, "lines": tot, "pct": round(100.0 * tot_h / tot, 1) if tot else 0.0},
            "flags": flags, "files": files}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    pytest_args = ["tests", "-q", "-m", "not gpu and not slow", "-p", "no:cacheprovider"]
    if "--" in argv:
        i = argv.index("--")
        argv, pytest_args = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--flag", action="append", default=[], help="NAME=PCT minimum for a component")
    ap.add_argument("--out", default=os.path.join(ROOT, "coverage.json"))
    a = ap.parse_args(argv)
    import pytest

    sys.path.insert(0, ROOT)
    threading.settrace(_global)
    sys.settrace(_global)
    try:
        rc = pytest.main(pytest_args)
    finally:
        sys.settrace(None)
        threading.settrace(None)
    rep = report()
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    print(f"coverage total {rep['total']['pct']}% ({rep['total']['hit']}/{rep['total']['lines']} lines)")
    for k, v in sorted(rep["flags"].items()):
        print(f"  {k:10s} {v['pct']:5.1f}%  ({v['hit']}/{v['lines']})")
    fail = []
    for spec in a.flag:
        name, _, pct = spec.partition("=")
        got = rep["flags"].get(name, {}).get("pct", 0.0)
        if got < float(pct):
            fail.append(f"{name} {got}% < {pct}%")
    if fail:
        print("coverage below threshold: " + "; ".join(fail))
        return 2
    return int(rc)


if __name__ == "__main__":
    sys.exit(main())
