"""Notebook pods whose container is a real PyTorch-ROCm workbench process
(``kubelet/process_runtime.py`` + ``notebook_server/workbench.py``): BASELINE configs #2/#3
without an image registry.  The CPU tests run the process without GPU work; the GPU test
has its first cell initialise HIP on the allocated MI355X and run a bf16 matmul.  In the
default ``first-cell`` mode the server is Ready before that cell (JupyterLab's behaviour);
``before-ready`` holds readiness until the cell has run."""

import aiohttp
import pytest

from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.testing.kubelet.process_runtime import ProcessContainerRuntime
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.notebook import notebook


async def _lifecycle(matmul: int, gpus: int = 1, gpu_init: str = "first-cell"):
    rts = []

    def factory(d):
        rt = ProcessContainerRuntime(matmul=matmul, visible_device=lambda _d: 0, gpu_init=gpu_init)
        rts.append(rt)
        return rt

    cfg = ClusterConfig(odh=True, webhook=True, runtime_factory=factory,
                        env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
    async with LocalCluster(cfg) as cl:
        await cl.ensure_namespace("user")
        await cl.admin.create(notebook("wb", "user", gpus=gpus))
        assert await cl.wait_for(lambda: cl.notebook_ready("wb", "user"), 240)
        pod = cl.store.peek(kinds.POD, "wb-0", "user")
        ep = m.annotations(pod)["amd.com/notebook-endpoint"]
        (rt,) = [rt for rt in rts if "user/wb-0" in rt.reports]
        ready = rt.reports["user/wb-0"]
        assert ready["gpu_init"] == gpu_init
        if gpu_init == "first-cell":
            assert "import_torch_ms" not in ready  # Ready came before the cell imported PyTorch
        cell = await rt.first_cell("user/wb-0", 240)
        assert cell["import_torch_ms"] > 0
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=10)) as s:
            async with s.get(f"http://{ep}/notebook/user/wb/api") as r:
                info = await r.json()
            async with s.get(f"http://{ep}/notebook/user/wb/api/kernels") as r:
                assert r.status == 200 and await r.json() == []
        await cl.admin.delete(kinds.NOTEBOOK, "wb", "user")
        assert await cl.wait_for(lambda: cl.store.peek(kinds.POD, "wb-0", "user") is None, 60)
        assert await cl.wait_for(lambda: not any(rt.procs for rt in rts), 30)  # process stopped with the pod
        return info


@pytest.mark.parametrize("gpu_init", ["first-cell", "before-ready"])
def test_workbench_process_pod_becomes_ready_cpu(run, gpu_init):
    info = run(_lifecycle(matmul=0, gpu_init=gpu_init), timeout=300)
    assert info["torch"] and info["gpu"] is None and info["import_torch_ms"] > 0


@pytest.mark.gpu
def test_workbench_process_initialises_the_mi355x(run):
    info = run(_lifecycle(matmul=1024), timeout=300)
    assert info["visible_devices"] == "0" and info["first_matmul_ms"] > 0
    assert info["arch"] == "gfx950" and info["hbm_total_gib"] > 250, info  # MI355X: gfx950, 288 GB HBM3E
