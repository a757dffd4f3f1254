# PyTorch-ROCm Jupyter workbench: ROCm-only (no CUDA compat layers), port 8888 under
# NB_PREFIX, /home/jovyan — the contract the kf controller's StatefulSet assumes
# (kf/controllers/notebook_controller.go:433-523).
ARG ROCM_IMAGE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${ROCM_IMAGE}
RUN pip install --no-cache-dir jupyterlab \
 && useradd -m -u 1000 -g 100 jovyan
ENV HOME=/home/jovyan NB_PREFIX=/ HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /home/jovyan
USER 1000:100
EXPOSE 8888
CMD ["sh", "-c", "jupyter lab --ip=0.0.0.0 --port=8888 --no-browser --ServerApp.base_url=${NB_PREFIX} --ServerApp.token='' --ServerApp.password='' --ServerApp.allow_origin='*'"]
