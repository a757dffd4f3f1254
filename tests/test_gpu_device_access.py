"""GPU device access for non-root containers.

The device plugin hands ``/dev/kfd`` and ``/dev/dri/renderD*`` to a container with the host's
owner and mode — typically ``root:render 0660``.  The injected containers run as non-root users
(the ``amd-gpu-probe`` init container as 65532, ``images/probe.Dockerfile``; notebook images as
1000), so they open the GPU only as members of the owning group: ``GPU_DEVICE_GROUPS`` makes the
kf StatefulSet generator put those gids into the pod's ``securityContext.supplementalGroups``
(which apply to every container of the pod, init containers included; a value the user set wins).

* CPU: the generator's rules (GPU pods only, user value wins, parsing);
* MI355X (``-m gpu``): stat the box's device nodes, configure ``GPU_DEVICE_GROUPS`` from their
  owning groups, and check that the generated pod spec is what lets uid 65532 open them: by the
  kernel's access rule (owner / group / other bits) for 65532 with and without the injected
  groups, and — when the test runs as root — by running ``odh-gpu-probe`` as uid 65532 with and
  without them.  Run as an ordinary user (the GPU boxes), the current user's own ``open()`` of
  each node is checked against the same rule.  ``ODH_DEVICE_ACCESS_REPORT`` names a file for the
  findings (the box's gids and modes, which setting the overlays need).

Reference counterpart: ``kf/controllers/notebook_controller.go:510-520`` (the fsGroup defaulting
this mirrors); the reference never injects groups for device access.
"""

from __future__ import annotations

import glob
import json
import os
import stat
import subprocess

import pytest

from odh_kubeflow_amd.controllers.notebook import generate_statefulset, parse_gids
from odh_kubeflow_amd.models.notebook import notebook


def _pod_spec(nb, env):
    return generate_statefulset(nb, False, env)["spec"]["template"]["spec"]


def test_device_groups_only_for_gpu_pods_and_user_value_wins():
    env = {"GPU_DEVICE_GROUPS": "video=44, render=110, junk, 110"}
    assert parse_gids(env["GPU_DEVICE_GROUPS"]) == [44, 110]
    gpu = _pod_spec(notebook("nb", "ns", gpus=1), env)
    assert gpu["securityContext"] == {"fsGroup": 100, "supplementalGroups": [44, 110]}
    assert "supplementalGroups" not in (_pod_spec(notebook("nb", "ns"), env).get("securityContext") or {})
    mine = notebook("nb", "ns", gpus=1)
    mine["spec"]["template"]["spec"]["securityContext"] = {"runAsUser": 1000, "supplementalGroups": [7]}
    assert _pod_spec(mine, env)["securityContext"] == {"runAsUser": 1000, "supplementalGroups": [7]}
    off = _pod_spec(notebook("nb", "ns", gpus=1), {"ADD_FSGROUP": "false"})
    assert "securityContext" not in off or "supplementalGroups" not in off["securityContext"]
    only = _pod_spec(notebook("nb", "ns", gpus=1), {"ADD_FSGROUP": "false", "GPU_DEVICE_GROUPS": "110"})
    assert only["securityContext"] == {"supplementalGroups": [110]}


def dac_allows_rw(st: os.stat_result, uid: int, gids) -> bool:
    """The kernel's discretionary access check for read+write by a process without
    CAP_DAC_OVERRIDE (the injected containers drop ALL capabilities)."""
    if st.st_uid == uid:
        bits = (st.st_mode >> 6) & 7
    elif st.st_gid in set(gids):
        bits = (st.st_mode >> 3) & 7
    else:
        bits = st.st_mode & 7
    return bits & 6 == 6


@pytest.mark.gpu
def test_injected_groups_let_the_non_root_probe_open_the_gpu(tmp_path):
    from odh_kubeflow_amd.ops import probe_main

    nodes = ["/dev/kfd", *sorted(glob.glob("/dev/dri/renderD*"))]
    nodes = [n for n in nodes if os.path.exists(n)]
    assert "/dev/kfd" in nodes and len(nodes) >= 2, nodes
    sts = {n: os.stat(n) for n in nodes}
    world = all(st.st_mode & 6 == 6 for st in sts.values())
    owning = sorted({st.st_gid for st in sts.values() if st.st_mode & 6 != 6})
    env = {"GPU_DEVICE_GROUPS": ",".join(str(g) for g in owning)}
    spec = _pod_spec(notebook("nb", "ns", gpus=1, annotations={"amd.com/gpu-probe": "true"}), env)
    groups = (spec.get("securityContext") or {}).get("supplementalGroups") or []
    assert set(owning) <= set(groups)
    probe_uid = 65532  # images/probe.Dockerfile: USER 65532:65532
    with_groups = {n: dac_allows_rw(st, probe_uid, {probe_uid, *groups}) for n, st in sts.items()}
    without = {n: dac_allows_rw(st, probe_uid, {probe_uid}) for n, st in sts.items()}
    assert all(with_groups.values()), with_groups
    assert world or not all(without.values())  # the groups are what makes it work (or the nodes are 0666)
    rec = {"nodes": {n: {"uid": st.st_uid, "gid": st.st_gid, "mode": oct(stat.S_IMODE(st.st_mode))}
                     for n, st in sts.items()},
           "world_rw": world, "GPU_DEVICE_GROUPS": env["GPU_DEVICE_GROUPS"],
           "uid_65532": {"with_injected_groups": all(with_groups.values()), "without": all(without.values())},
           "euid": os.geteuid(), "groups_of_this_process": sorted(os.getgroups())}
    me = {os.getegid(), *os.getgroups()}
    opened = {}
    for n, st in sts.items():  # the same rule predicts what this process may open
        try:
            os.close(os.open(n, os.O_RDWR))
            opened[n] = True
        except OSError:
            opened[n] = False
        if os.geteuid() != 0 and opened[n]:
            # (a node the rule allows can still be closed to this container by its device cgroup)
            assert dac_allows_rw(st, os.geteuid(), me), (n, rec)
    rec["this_process_opened"] = opened
    if os.geteuid() == 0:
        exe = probe_main.executable()
        os.chmod(tmp_path, 0o777)

        def probe(extra):
            out = tmp_path / f"verdict-{len(extra)}.json"
            r = subprocess.run([exe, "--json", str(out), "--quiet"], user=probe_uid, group=probe_uid,
                               extra_groups=extra, capture_output=True, text=True, timeout=120)
            return r.returncode
        rec["probe_as_65532"] = {"with_injected_groups": probe(groups), "without": probe([])}
        assert rec["probe_as_65532"]["with_injected_groups"] == 0, rec
        if not world:
            assert rec["probe_as_65532"]["without"] != 0, rec
    path = os.environ.get("ODH_DEVICE_ACCESS_REPORT")
    if path:
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
    print(json.dumps(rec))
