# The MI355X start-up probe (init container `amd-gpu-probe`, injected by the kf StatefulSet
# generator for notebooks annotated amd.com/gpu-probe: "true" / "rccl" or with GPU_STARTUP_PROBE=true).
# odh-gpu-probe + libodh_gpu_probe.so on the ROCm runtime only: no Python, no torch — the
# probe's cost in the pod's create→Ready is process start + HIP init + ~0.2 ms of GPU work.
ARG ROCM_DEV_IMAGE=rocm/dev-ubuntu-22.04:7.0-complete
ARG ROCM_RUNTIME_IMAGE=rocm/dev-ubuntu-22.04:7.0
FROM ${ROCM_DEV_IMAGE} AS build
ARG GPU_ARCH=gfx950
WORKDIR /src
COPY odh_kubeflow_amd/ops/csrc ./csrc
RUN mkdir -p /opt/odh/bin \
 && hipcc --offload-arch=${GPU_ARCH} -O3 -std=c++17 -shared -fPIC csrc/gpu_probe.hip csrc/probe_cli.cpp \
      -o /opt/odh/bin/libodh_gpu_probe.so \
 && hipcc -O2 -std=c++17 csrc/probe_main.cpp -L/opt/odh/bin -lodh_gpu_probe -Wl,-rpath,'$ORIGIN' \
      -o /opt/odh/bin/odh-gpu-probe

FROM ${ROCM_RUNTIME_IMAGE}
COPY --from=build /opt/odh/bin /opt/odh/bin
# RCCL for the optional all-reduce step (--rccl-mib; amd.com/gpu-probe: "rccl"): dlopen'ed
# only by that step, so a plain probe never maps the 570 MB library
COPY --from=build /opt/rocm/lib/librccl.so.1* /opt/rocm/lib/
ENV PATH=/opt/odh/bin:${PATH} LD_LIBRARY_PATH=/opt/rocm/lib
USER 65532:65532
ENTRYPOINT ["odh-gpu-probe"]
CMD ["--json", "/dev/termination-log"]
