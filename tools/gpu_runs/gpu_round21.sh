#!/bin/bash
# GPU pass 21: BASELINE config #5 — idle culling across 8 GPU notebooks with a real MFMA
# load on the visible MI355X (amdgpu sysfs busy counters via the native sampler).
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
python - <<'PY' > gpurun_out/pci21.txt 2>&1
import torch
p = torch.cuda.get_device_properties(0)
print({k: getattr(p, k) for k in dir(p) if not k.startswith("_") and "pci" in k.lower()})
from odh_kubeflow_amd.ops.telemetry import Telemetry
t = Telemetry("/sys")
for d in t.devices():
    print(d)
PY
cat gpurun_out/pci21.txt | head -20
timeout -k 10 120 python tools/bench_culling.py > gpurun_out/cull21.log 2>&1 || { tail -30 gpurun_out/cull21.log; exit 1; }
tail -1 gpurun_out/cull21.log
