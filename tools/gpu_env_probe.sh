#!/bin/bash
# One-shot inventory of the GPU box: telemetry paths the culler can use.
set -u
out=gpurun_out/env_probe.txt
mkdir -p gpurun_out
{
echo "== whoami/nproc"; whoami; nproc
echo "== env"; env | grep -E 'HIP|ROCR|CUDA|GPU|HSA' | sort
echo "== drm sysfs"; ls /sys/class/drm/ 2>&1 | head -40
for c in /sys/class/drm/card*/device; do
  [ -e "$c/gpu_busy_percent" ] && echo "$c busy=$(cat $c/gpu_busy_percent 2>&1) vram_used=$(cat $c/mem_info_vram_used 2>&1) vram_total=$(cat $c/mem_info_vram_total 2>&1)"
done
echo "== kfd topology"; ls /sys/class/kfd/kfd/topology/nodes/ 2>&1
echo "== rocm-smi"; timeout -k 5 30 rocm-smi --showuse --showmemuse 2>&1 | head -40
echo "== amd-smi py"; timeout -k 5 60 python3 - <<'PY' 2>&1
import amdsmi
amdsmi.amdsmi_init()
hs = amdsmi.amdsmi_get_processor_handles()
print("handles", len(hs))
for h in hs[:8]:
    try:
        print("bdf", amdsmi.amdsmi_get_gpu_device_bdf(h), "busy", amdsmi.amdsmi_get_gpu_busy_percent(h), "act", amdsmi.amdsmi_get_gpu_activity(h), "vram", amdsmi.amdsmi_get_gpu_vram_usage(h))
    except Exception as e:
        print("err", repr(e))
amdsmi.amdsmi_shut_down()
PY
echo "== torch"; timeout -k 5 120 python3 -c "import torch;print(torch.cuda.is_available(), torch.cuda.device_count(), torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))" 2>&1
} > $out 2>&1
cat $out | tail -60
