"""The MI355X start-up probe as a shipped init container.

* the kf StatefulSet generator injects ``odh-gpu-probe`` for ``amd.com/gpu`` notebooks when the
  Notebook (``amd.com/gpu-probe``) or the operator (``GPU_STARTUP_PROBE``) asks for it, with
  the notebook's GPU count, before any user init container — and never for CPU notebooks;
* the kubelet stand-in runs a pod's init containers before its containers: a failing one
  keeps the pod ``Initialized=False`` with the exit code and message in
  ``initContainerStatuses`` and is retried after a back-off, as a kubelet does; Ready is gated
  on nothing else;
* the native program and ``python -m odh_kubeflow_amd.ops.probe_main``: usage errors, the
  no-GPU verdict (CPU), and on an MI355X (``-m gpu``) a clean pass, injected GEMM / HBM
  faults failing with exit status 1, the added process latency, and a notebook reaching Ready
  behind the probe through the whole control plane.

Reference counterpart: none — upstream starts GPU pods unchecked (kf generateStatefulSet
copies ``resources.limits`` verbatim, ``kf/controllers/notebook_controller.go:433-523``); the
injection follows the odh sidecar injector's pattern (``odh/controllers/notebook_webhook.go:177-326``).
"""

from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import time

import pytest

from odh_kubeflow_amd.controllers.notebook import (GPU_PROBE_ANNOTATION, GPU_PROBE_CONTAINER, generate_statefulset,
                                                   gpu_probe_enabled)
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.ops import probe_main

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inits(nb, env=None):
    sts = generate_statefulset(nb, False, env or {})
    return sts["spec"]["template"]["spec"].get("initContainers") or []


# ------------------------------------------------------------------ injection (CPU)


def test_probe_injected_on_annotation_with_the_notebooks_gpu_count():
    nb = notebook("nb", "ns", gpus=2, annotations={GPU_PROBE_ANNOTATION: "true"})
    inits = _inits(nb, {"GPU_PROBE_IMAGE": "registry/odh-gpu-probe:1"})
    assert [c["name"] for c in inits] == [GPU_PROBE_CONTAINER]
    c = inits[0]
    assert c["image"] == "registry/odh-gpu-probe:1"
    assert c["command"] == ["odh-gpu-probe"] and "/dev/termination-log" in c["args"]
    assert c["resources"]["limits"]["amd.com/gpu"] == "2" and c["resources"]["requests"]["amd.com/gpu"] == "2"
    assert c["terminationMessagePolicy"] == "FallbackToLogsOnError"
    assert c["securityContext"]["allowPrivilegeEscalation"] is False


def test_probe_off_by_default_operator_switch_and_opt_out():
    nb = notebook("nb", "ns", gpus=1)
    assert _inits(nb) == []  # default deployment: no probe (opt-in)
    assert [c["name"] for c in _inits(nb, {"GPU_STARTUP_PROBE": "true"})] == [GPU_PROBE_CONTAINER]
    out = notebook("nb", "ns", gpus=1, annotations={GPU_PROBE_ANNOTATION: "false"})
    assert _inits(out, {"GPU_STARTUP_PROBE": "true"}) == []
    cpu = notebook("nb", "ns", annotations={GPU_PROBE_ANNOTATION: "true"})
    assert not gpu_probe_enabled(cpu, cpu["spec"]["template"]["spec"], {}) and _inits(cpu) == []


def test_probe_runs_before_user_init_containers_and_user_copy_wins():
    nb = notebook("nb", "ns", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"})
    nb["spec"]["template"]["spec"]["initContainers"] = [{"name": "fetch-data", "image": "busybox"}]
    assert [c["name"] for c in _inits(nb)] == [GPU_PROBE_CONTAINER, "fetch-data"]
    mine = {"name": GPU_PROBE_CONTAINER, "image": "mine", "command": ["odh-gpu-probe"], "args": ["--hbm-mib", "64"]}
    nb["spec"]["template"]["spec"]["initContainers"] = [mine]
    assert _inits(nb) == [mine]


def test_probe_rccl_mode():
    """``amd.com/gpu-probe: "rccl"`` (or ``GPU_PROBE_RCCL=true`` for every multi-GPU notebook
    that gets the probe) adds the RCCL all-reduce step."""
    nb = notebook("nb", "ns", gpus=4, annotations={GPU_PROBE_ANNOTATION: "rccl"})
    (c,) = _inits(nb)
    assert c["args"][c["args"].index("--rccl-mib") + 1] == "64"
    plain = notebook("nb", "ns", gpus=4, annotations={GPU_PROBE_ANNOTATION: "true"})
    assert "--rccl-mib" not in _inits(plain)[0]["args"]
    assert "--rccl-mib" in _inits(plain, {"GPU_PROBE_RCCL": "true"})[0]["args"]
    one = notebook("nb", "ns", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"})
    assert "--rccl-mib" not in _inits(one, {"GPU_PROBE_RCCL": "true"})[0]["args"]  # nothing to all-reduce over


def test_probe_annotation_reaches_the_pod_template():
    nb = notebook("nb", "ns", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"})
    sts = generate_statefulset(nb, False, {})
    assert sts["spec"]["template"]["metadata"]["annotations"][GPU_PROBE_ANNOTATION] == "true"


def test_probe_statefulset_is_steady(run):
    """With the probe on, the generated StatefulSet equals the defaulted stored one: no
    steady-state update loop (the 0-writes property of ``tests/test_defaulting.py``)."""
    from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster

    async def go():
        async with LocalCluster(ClusterConfig(env={"GPU_STARTUP_PROBE": "true"})) as cl:
            await cl.ensure_namespace("p")
            await cl.admin.create(notebook("nb", "p", gpus=1))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "p"), 30)
            assert await cl.settle(10)
            sts = cl.store.peek(kinds.STATEFUL_SET, "nb", "p")
            rv = sts["metadata"]["resourceVersion"]
            pod = cl.store.peek(kinds.POD, "nb-0", "p")
            assert [c["name"] for c in pod["spec"]["initContainers"]] == [GPU_PROBE_CONTAINER]
            st = pod["status"]["initContainerStatuses"][0]
            assert st["name"] == GPU_PROBE_CONTAINER and st["state"]["terminated"]["exitCode"] == 0
            # the stored (apiserver-defaulted) StatefulSet needs no update from a fresh generation
            from odh_kubeflow_amd.utils.objutil import deepcopy_json
            from odh_kubeflow_amd.utils.reconcilehelper import copy_statefulset_fields

            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "p")
            want = generate_statefulset(nb, False, {"GPU_STARTUP_PROBE": "true"})
            assert not copy_statefulset_fields(want, deepcopy_json(sts))
            assert cl.store.peek(kinds.STATEFUL_SET, "nb", "p")["metadata"]["resourceVersion"] == rv
    run(go())


# ------------------------------------------------------------------ kubelet stand-in (CPU)


class _FailingInit:
    """A container runtime whose init containers exit 1 (a GPU that fails its probe)."""

    exec_init = True
    visible_device = None

    def __init__(self):
        self.calls = 0

    async def run_init(self, pod, container, devices):
        self.calls += 1
        msg = json.dumps({"ok": False, "error": "GPU 0: 65536 GEMM mismatches"})
        return {"exitCode": 1, "message": msg, "wall_ms": 1.0, "result": json.loads(msg)}

    async def start(self, pod, devices):
        raise AssertionError("containers must not start after a failed init container")

    async def stop(self, handle):
        return None

    async def close(self):
        return None


def test_failed_init_container_keeps_pod_uninitialized(run):
    from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster

    rts = []

    def factory(d):
        rts.append(_FailingInit())
        return rts[-1]

    async def go():
        async with LocalCluster(ClusterConfig(runtime_factory=factory)) as cl:
            await cl.ensure_namespace("p")
            await cl.admin.create(notebook("nb", "p", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"}))

            def failed():
                pod = cl.store.peek(kinds.POD, "nb-0", "p")
                return bool(pod and (pod.get("status") or {}).get("initContainerStatuses"))
            assert await cl.wait_for(failed, 30)
            pod = cl.store.peek(kinds.POD, "nb-0", "p")
            st = pod["status"]
            cond = {c["type"]: c for c in st["conditions"]}
            assert cond["Initialized"]["status"] == "False" and cond["Ready"]["status"] == "False"
            assert GPU_PROBE_CONTAINER in cond["Initialized"]["message"]
            term = st["initContainerStatuses"][0]["state"]["terminated"]
            assert term["exitCode"] == 1 and "mismatches" in term["message"]
            assert st["phase"] == "Pending"
            assert not cl.notebook_ready("nb", "p")
            nb = cl.store.peek(kinds.NOTEBOOK, "nb", "p")
            assert (nb.get("status") or {}).get("readyReplicas", 0) == 0
            def backoff_events():
                return [e for e in cl.store.list_nocopy(kinds.EVENT, "p") if e.get("reason") == "BackOff"]
            assert await cl.wait_for(lambda: bool(backoff_events()), 10)  # the recorder batches its writes
            assert "amd-gpu-probe" in backoff_events()[0]["message"]
            assert sum(r.calls for r in rts) == 1  # retried only after the back-off
    run(go())


# ------------------------------------------------------------------ the program (CPU)


def _exe():
    path = probe_main.executable()
    if not os.path.exists(path):
        pytest.fail("odh-gpu-probe not built: python -m odh_kubeflow_amd.ops.build")
    return path


def test_probe_program_usage_and_no_gpu_verdict(tmp_path):
    exe = _exe()
    assert subprocess.run([exe, "--bogus"], capture_output=True).returncode == probe_main.USAGE
    assert subprocess.run([exe, "--shape", "100,100,100"], capture_output=True).returncode == probe_main.USAGE
    assert subprocess.run([exe, "--streams", "3"], capture_output=True).returncode == probe_main.USAGE
    out = tmp_path / "termination-log"
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")  # a pod without GPUs (also on the GPU box)
    r = subprocess.run([exe, "--json", str(out), "--quiet"], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == probe_main.NO_GPU
    res = json.loads(out.read_text())
    assert res["ok"] is False and res["error"].startswith("no GPU")
    assert r.stdout == ""  # --quiet: the verdict only in the termination log


def test_probe_python_module_is_torch_free():
    code = ("import sys; from odh_kubeflow_amd.ops import probe_main; rc = probe_main.run(['--json', '-']); "
            "print('TORCH' if 'torch' in sys.modules else 'NOTORCH'); sys.exit(rc)")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=ROOT, timeout=60)
    assert r.returncode == probe_main.NO_GPU, r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == "NOTORCH"
    assert probe_main.parse_result(r.stdout)["ok"] is False


def test_probe_command_prefers_the_native_program():
    assert probe_main.command(["--quiet"]) == [_exe(), "--quiet"]


# ------------------------------------------------------------------ on an MI355X


def _run_probe(*args, timeout=120):
    env = {k: v for k, v in os.environ.items() if not k.startswith(("HIP_VISIBLE", "ROCR_VISIBLE", "CUDA_VISIBLE"))}
    env["HIP_VISIBLE_DEVICES"] = "0"
    t0 = time.perf_counter()
    r = subprocess.run(["timeout", "-k", "10", str(timeout), _exe(), "--json", "-", *args], capture_output=True,
                       text=True, env=env, timeout=timeout + 20)
    return r.returncode, probe_main.parse_result(r.stdout), (time.perf_counter() - t0) * 1e3, r


@pytest.mark.gpu
def test_probe_program_passes_on_the_mi355x():
    rc, res, _wall, r = _run_probe()
    assert rc == 0, (r.stdout, r.stderr)
    assert res["ok"] and res["devices"] == 1 and res["links"] == []
    d = res["results"][0]
    assert d["gemm_errors"] == 0 and d["hbm_errors"] == 0 and d["xcds"] == 8, d
    assert d["gemm_tflops"] > 50 and d["hbm_gbps"] > 500, d  # ran on the matrix cores and HBM, not a stub
    assert res["setup_ms"]["n_streams"] == 0 and res["setup_ms"]["streams"] == 0, res


@pytest.mark.gpu
@pytest.mark.parametrize("fault", ["gemm", "hbm"])
def test_probe_program_fails_on_injected_fault(fault):
    rc, res, _wall, r = _run_probe("--inject-fault", fault)
    assert rc == probe_main.CHECK_FAILED, (r.stdout, r.stderr)
    assert res["ok"] is False and "mismatches" in res["error"]
    d = res["results"][0]
    if fault == "gemm":
        # A[0][0] corrupted: C[0][j] is wrong wherever Bt[j][0] = ((11 j) mod 7) - 3 is non-zero
        want = sum(1 for j in range(4096) if (11 * j) % 7 != 3)
        assert d["gemm_errors"] == want and d["hbm_errors"] == 0 and sum(d["err_xcd"]) == want, d
    else:
        assert d["hbm_errors"] > 0 and d["gemm_errors"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("streams", ["1", "2"])
def test_probe_program_on_created_streams(streams):
    """``--streams 1`` (one created stream) and ``--streams 2`` (the sweep overlapping the GEMM)
    check what the default null-stream run checks: a clean pass, and each injected fault found."""
    rc, res, _wall, r = _run_probe("--streams", streams)
    assert rc == 0, (r.stdout, r.stderr)
    d = res["results"][0]
    assert d["gemm_errors"] == 0 and d["hbm_errors"] == 0 and d["gemm_tflops"] > 50 and d["hbm_gbps"] > 500, d
    assert res["setup_ms"]["n_streams"] == int(streams)
    for fault, key in (("gemm", "gemm_errors"), ("hbm", "hbm_errors")):
        rc, res, _wall, r = _run_probe("--streams", streams, "--inject-fault", fault)
        assert rc == probe_main.CHECK_FAILED and res["results"][0][key] > 0, (r.stdout, r.stderr)


@pytest.mark.gpu
def test_probe_program_rccl_allreduce_on_the_mi355x():
    """``--rccl-mib``: the RCCL all-reduce over the pod's GPUs (one here: ncclCommInitAll over
    one device, the result still checked element by element on the GPU), then an injected
    wrong contribution that every element of the result must expose."""
    rc, res, _wall, r = _run_probe("--rccl-mib", "16")
    assert rc == 0, (r.stdout, r.stderr)
    rr = res["rccl"]
    assert rr["ok"] and rr["ranks"] == 1 and rr["errors"] == 0 and rr["mib"] == 16, rr
    assert rr["allreduce_ms"] > 0 and res["timings_ms"]["rccl"] >= rr["load_ms"] + rr["init_ms"] and rr["init_ms"] > 0, res
    print(f"RCCL: load {rr['load_ms']:.1f} ms, init {rr['init_ms']:.1f} ms, 16 MiB all-reduce {rr['allreduce_ms']:.3f} ms")
    rc, res, _wall, r = _run_probe("--rccl-mib", "16", "--inject-fault", "rccl")
    assert rc == probe_main.CHECK_FAILED, (r.stdout, r.stderr)
    assert res["rccl"]["errors"] == (16 << 20) // 4 and "RCCL all-reduce" in res["error"], res
    assert res["results"][0]["gemm_errors"] == 0 and res["results"][0]["hbm_errors"] == 0


@pytest.mark.gpu
def test_probe_python_module_passes_on_the_mi355x():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0", PYTHONPATH=ROOT)
    code = ("import sys; from odh_kubeflow_amd.ops import probe_main; rc = probe_main.run(['--json', '-']); "
            "assert 'torch' not in sys.modules; sys.exit(rc)")
    r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "-c", code], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=150)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert probe_main.parse_result(r.stdout)["results"][0]["gemm_errors"] == 0


@pytest.mark.gpu
def test_probe_process_latency():
    """What the init container adds to create→Ready: the whole process, HIP init included
    (target ≤ 300 ms; the in-process torch probe it replaces cost ≈1.6 s of ``import torch``)."""
    walls, totals = [], []
    for _ in range(5):
        rc, res, wall, r = _run_probe()
        assert rc == 0, r.stderr
        walls.append(wall)
        totals.append(res["timings_ms"]["total"])
    p50 = statistics.median(walls)
    print(f"odh-gpu-probe process wall p50 {p50:.1f} ms (in-process total p50 {statistics.median(totals):.1f} ms)")
    assert p50 < 1500, walls


@pytest.mark.gpu
def test_notebook_ready_behind_probe_init_container(run):
    from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster

    async def go():
        cfg = ClusterConfig(exec_gpu_probe=True, probe_visible_device=lambda d: 0)
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("p")
            await cl.admin.create(notebook("ok", "p", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"}))
            assert await cl.wait_for(lambda: cl.notebook_ready("ok", "p"), 120)
            term = cl.store.peek(kinds.POD, "ok-0", "p")["status"]["initContainerStatuses"][0]["state"]["terminated"]
            assert term["exitCode"] == 0 and probe_main.parse_result(term["message"])["ok"]
            # a user-supplied probe container with an injected fault: the pod never starts
            bad = notebook("bad", "p", gpus=1, annotations={GPU_PROBE_ANNOTATION: "true"})
            bad["spec"]["template"]["spec"]["initContainers"] = [{
                "name": GPU_PROBE_CONTAINER, "image": "probe", "command": ["odh-gpu-probe"],
                "args": ["--json", "/dev/termination-log", "--inject-fault", "gemm"],
                "resources": {"limits": {"amd.com/gpu": "1"}}}]
            await cl.admin.create(bad)

            def failed():
                pod = cl.store.peek(kinds.POD, "bad-0", "p")
                return bool(pod and (pod.get("status") or {}).get("initContainerStatuses"))
            assert await cl.wait_for(failed, 120)
            st = cl.store.peek(kinds.POD, "bad-0", "p")["status"]
            term = st["initContainerStatuses"][0]["state"]["terminated"]
            assert term["exitCode"] == 1 and "GEMM mismatches" in term["message"]
            assert not cl.notebook_ready("bad", "p")
    run(go(), timeout=300)
