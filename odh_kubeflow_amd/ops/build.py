"""In-tree build of the native libraries (``python -m odh_kubeflow_amd.ops.build``).

* ``libodh_gpu_probe.so``   — HIP kernels for gfx950 (``hipcc --offload-arch=gfx950``),
  C ABI, loaded with ctypes after ``import torch`` so it shares torch's HIP runtime
  (both resolve ``libamdhip64.so.7``).
* ``odh-gpu-probe`` — the notebook pod's start-up probe (init container), a main over
  ``odh_probe_cli`` of ``libodh_gpu_probe.so`` (``csrc/probe_cli.cpp``); needs no torch.
* ``libodh_gpu_telemetry.so`` — host C++ amdgpu sysfs sampler (g++, pthreads).

Both land in ``odh_kubeflow_amd/ops/_lib/`` so they travel with the repo snapshot to
the GPU box (no JIT cache under ``~/.cache``).  A library is rebuilt only when its
source is newer than the ``.so``.  ``--host-only`` builds the host C++ libraries (the slim
controller / node-agent image), ``--probe-only`` the probe (its ROCm image).
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from typing import Dict, List

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
NATIVE = os.path.join(os.path.dirname(HERE), "native")
TEST_NATIVE = os.path.join(os.path.dirname(HERE), "testing", "native")  # test platform: the C++ apiserver
OBJCORE = "_objcore" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")
ARCH = os.environ.get("ODH_GPU_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
PROBE_EXE = "odh-gpu-probe"


def _hipcc() -> str:
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else (shutil.which("hipcc") or p)


def targets() -> Dict[str, dict]:
    return {
        "libodh_gpu_probe.so": {
            "src": [os.path.join(CSRC, "gpu_probe.hip"), os.path.join(CSRC, "probe_cli.cpp")],
            "cmd": lambda src, out: [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
                                     *src, "-o", out],
        },
        # the init-container probe: a 5-line main over odh_probe_cli in the library next to it
        PROBE_EXE: {
            "src": [os.path.join(CSRC, "probe_main.cpp")],
            "deps": [os.path.join(LIBDIR, "libodh_gpu_probe.so")],
            "cmd": lambda src, out: [_hipcc(), "-O2", "-std=c++17", *src, f"-L{LIBDIR}", "-lodh_gpu_probe",
                                     "-Wl,-rpath,$ORIGIN", "-o", out],
        },
        OBJCORE: {
            "src": [os.path.join(NATIVE, "objcore.cpp")],
            "out": os.path.join(NATIVE, OBJCORE),
            "cmd": lambda src, out: [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall",
                                     "-fno-strict-aliasing", f"-I{sysconfig.get_paths()['include']}", *src,
                                     "-o", out],
        },
        "odh-apiserver": {
            "src": [os.path.join(TEST_NATIVE, "apiserver", "apiserver.cpp")],
            "deps": [os.path.join(TEST_NATIVE, "apiserver", "json.hpp")],
            "out": os.path.join(TEST_NATIVE, "bin", "odh-apiserver"),
            "cmd": lambda src, out: [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-pthread", "-Wall", *src,
                                     "-o", out, "-lssl", "-lcrypto"],
        },
        "libodh_gpu_telemetry.so": {
            "src": [os.path.join(CSRC, "gpu_telemetry.cpp")],
            "cmd": lambda src, out: [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-shared", "-fPIC",
                                     "-pthread", "-Wall", *src, "-o", out],
        },
    }


def lib_path(name: str) -> str:
    return os.path.join(LIBDIR, name)


def _stale(out: str, srcs: List[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


# what each image needs: the slim controller / node-agent image has no ROCm toolchain and no
# HIP runtime (host C++ only); the probe image has the HIP runtime and the probe only
HOST_TARGETS = (OBJCORE, "libodh_gpu_telemetry.so")
PROBE_TARGETS = ("libodh_gpu_probe.so", PROBE_EXE)


def build(force: bool = False, verbose: bool = True, only=None) -> Dict[str, str]:
    os.makedirs(LIBDIR, exist_ok=True)
    built = {}
    for name, spec in targets().items():
        if only is not None and name not in only:
            continue
        out = spec.get("out") or lib_path(name)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        if force or _stale(out, spec["src"] + spec.get("deps", [])):
            tmp = out + ".tmp"
            cmd = spec["cmd"](spec["src"], tmp)
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(tmp, out)
        built[name] = out
    return built


if __name__ == "__main__":
    sel = None
    if "--host-only" in sys.argv:
        sel = HOST_TARGETS
    elif "--probe-only" in sys.argv:
        sel = PROBE_TARGETS
    build(force="--force" in sys.argv, only=sel)
