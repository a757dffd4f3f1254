"""Production images are sized like the reference's (``ubi9/ubi-minimal`` + one binary,
``kf/Dockerfile:45``, ``odh/Dockerfile:43``): the controller / webhook / node-agent image is a
slim Python with host C++ only — no ROCm, no torch, no test tooling — the start-up probe
has its own ROCm-runtime image, and the conformance tooling its own image on top."""

import os
import re

from odh_kubeflow_amd.deploy import manifests

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(name):
    with open(os.path.join(ROOT, "images", name)) as f:
        return f.read()


def _froms(text):
    args = dict(re.findall(r"^ARG (\w+)=(\S+)", text, re.M))
    out = []
    for ref in re.findall(r"^FROM (\S+)", text, re.M):
        mo = re.fullmatch(r"\$\{(\w+)\}", ref)
        out.append(args.get(mo.group(1), ref) if mo else ref)
    return out


def test_controller_image_is_slim_python_without_rocm_or_tests():
    d = _read("Dockerfile")
    froms = _froms(d)
    assert froms and all(f.startswith("python:") and "slim" in f for f in froms if f != "build"), froms
    runtime = d.split("\nFROM ")[-1]
    for word in ("rocm", "torch", "pytest", "hipcc"):
        assert word not in runtime.lower(), word
    assert "ops.build --host-only" in d  # host C++ only: _objcore + the telemetry sampler
    assert "testing" in d and "rm -rf" in d  # the test platform is not shipped
    assert "openssl" in runtime  # the cert provisioner drives the CLI
    assert "USER 65532" in runtime


def test_probe_image_runs_the_native_probe_on_the_rocm_runtime():
    d = _read("probe.Dockerfile")
    froms = _froms(d)
    assert len(froms) == 2 and "rocm" in froms[0] and "rocm" in froms[1] and "complete" not in froms[1]
    assert "--offload-arch=${GPU_ARCH}" in d and "probe_cli.cpp" in d
    runtime = d.split("\nFROM ")[-1]
    assert 'ENTRYPOINT ["odh-gpu-probe"]' in runtime and "python" not in runtime.lower()


def test_conformance_image_layers_test_tooling_on_the_controller_image():
    d = _read("conformance.Dockerfile")
    assert "pytest" in d and "e2e" in d
    pod = manifests.conformance_docs("v9")["e2e-conformance.yaml"]
    assert pod["spec"]["containers"][0]["image"] == f"{manifests.CONFORMANCE_IMAGE_NAME}:v9"


def test_kf_config_pins_the_probe_image_to_the_release():
    env = manifests.params_env("v9")
    assert "GPU_STARTUP_PROBE=false" in env
    assert f"GPU_PROBE_IMAGE={manifests.PROBE_IMAGE_NAME}:v9" in env
