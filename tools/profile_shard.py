"""cProfile of one control-plane shard (native apiserver child process) over N notebook lifecycles."""
import asyncio
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer  # noqa: E402
from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS  # noqa: E402
from odh_kubeflow_amd.models import kinds  # noqa: E402
from odh_kubeflow_amd.models.notebook import notebook  # noqa: E402
from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig  # noqa: E402
from odh_kubeflow_amd.utils import gctune  # noqa: E402


async def main(n_steps: int, sort: str):
    from odh_kubeflow_amd.parallel.platform import NodePlatform

    native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
    # as in the benchmark: the node's scheduler + StatefulSet controller and kubelet are processes
    platform = await NodePlatform(native.url).start()
    # the control plane in this process, so cProfile sees its reconcile paths
    sh = await ControlPlaneShard(ShardConfig(apiserver_url=native.url, namespace="bench-0", shard="0", bootstrap=True,
                                             env={"SET_PIPELINE_RBAC": "false",
                                                  "SET_PIPELINE_SECRET": "false"})).start()

    async def step(i):
        nm = f"nb{i}"
        await sh.admin.create(notebook(nm, "bench-0", image="img", gpus=1,
                                       annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
        await sh.wait_until(lambda: sh.notebook_ready(nm), 30)
        await sh.admin.delete(kinds.NOTEBOOK, nm, "bench-0")
        await sh.wait_until(lambda: sh.gone(nm), 30)

    for i in range(5):
        await step(i)
    await sh.settle(5)
    gctune.tune()
    pr = cProfile.Profile()
    pr.enable()
    t = time.perf_counter()
    for i in range(5, 5 + n_steps):
        await step(i)
    el = time.perf_counter() - t
    pr.disable()
    print(f"ms/step {el / n_steps * 1e3:.3f}")
    pstats.Stats(pr).sort_stats(sort).print_stats(45)
    await sh.stop()
    await platform.stop()
    await native.stop()


if __name__ == "__main__":
    asyncio.run(main(int(sys.argv[1]) if len(sys.argv) > 1 else 100, sys.argv[2] if len(sys.argv) > 2 else "tottime"))
