"""Cut a release: set the version everywhere the deployment and the package carry it.

    python tools/release.py v0.3.0-rc.0      # then review `git diff` and commit

The reference's ``releasing/update-manifests-images <VERSION>`` rewrites the image tags of
its kustomizations and ``releasing/version/VERSION`` records the version
(``releasing/README.md``).  Here the manifests are generated (``deploy/manifests.py``), so
the release:

1. writes ``releasing/VERSION``;
2. sets ``__version__`` in ``odh_kubeflow_amd/__init__.py`` (PEP 440 form of the tag);
3. regenerates ``config/``: every overlay pins ``quay.io/opendatahub/odh-kubeflow-amd`` to
   the tag through kustomize ``images`` (the base manifests keep the ``main`` tag).
"""

from __future__ import annotations

import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = re.compile(r"^v(\d+)\.(\d+)\.(\d+)(?:-(rc|alpha|beta)\.(\d+))?$")


def pep440(tag: str) -> str:
    m = TAG.match(tag)
    if not m:
        raise ValueError(f"not a release tag (vMAJOR.MINOR.PATCH[-rc.N]): {tag!r}")
    base = ".".join(m.group(i) for i in (1, 2, 3))
    if m.group(4):
        return base + {"rc": "rc", "alpha": "a", "beta": "b"}[m.group(4)] + m.group(5)
    return base


def release(tag: str, root: str = ROOT) -> list:
    ver = pep440(tag)
    changed = []
    os.makedirs(os.path.join(root, "releasing"), exist_ok=True)
    with open(os.path.join(root, "releasing", "VERSION"), "w") as f:
        f.write(tag + "\n")
    changed.append("releasing/VERSION")
    init = os.path.join(root, "odh_kubeflow_amd", "__init__.py")
    with open(init) as f:
        src = f.read()
    new, n = re.subn(r'^__version__ = "[^"]*"', f'__version__ = "{ver}"', src, flags=re.M)
    if n != 1:
        raise RuntimeError(f"{init}: no __version__ line")
    with open(init, "w") as f:
        f.write(new)
    changed.append("odh_kubeflow_amd/__init__.py")
    sys.path.insert(0, ROOT)
    from odh_kubeflow_amd.deploy import manifests

    out = os.path.join(root, "config")
    changed += [os.path.relpath(p, root) for p in manifests.write(out, tag)]
    return changed


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("version", help="release tag, e.g. v0.3.0 or v0.3.0-rc.0")
    ap.add_argument("--root", default=ROOT, help="repository root to write into")
    a = ap.parse_args(argv)
    for p in release(a.version, a.root):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
