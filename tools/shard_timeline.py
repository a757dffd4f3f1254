"""Per-hop timeline of one notebook lifecycle through a single control-plane shard (REST calls + watch events)."""
import asyncio, os, time, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig
from odh_kubeflow_amd.apiserver.native import NativeApiServer
from odh_kubeflow_amd.cluster import OPENSHIFT_CRDS
from odh_kubeflow_amd.runtime import rest as _rest
ev = []; T = [0.0]
_orig = _rest.RestClient.request
async def _req(self, method, path, *a, **kw):
    t = time.perf_counter()
    try:
        return await _orig(self, method, path, *a, **kw)
    finally:
        ev.append((t - T[0], "REQ", method, str(path)[22:90], "%.2fms" % ((time.perf_counter()-t)*1e3)))
_rest.RestClient.request = _req

async def main():
    native = await NativeApiServer(OPENSHIFT_CRDS, gc=True).start()
    sh = await ControlPlaneShard(ShardConfig(apiserver_url=native.url, namespace="bench-0", gpu=0, bootstrap=True,
                                              env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})).start()
    def cb(kind):
        def f(et, o, old):
            ev.append((time.perf_counter() - T[0], kind.split("/")[-1], et, o["metadata"]["name"], o["metadata"].get("resourceVersion")))
        return f
    for k in (kinds.NOTEBOOK, kinds.STATEFUL_SET, kinds.POD):
        sh.cache.subscribe(k, cb(k))
    for step in range(5):
        ev.clear()
        nm = f"nb{step}"
        T[0] = time.perf_counter()
        await sh.admin.create(notebook(nm, "bench-0", image="img", gpus=1, annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
        ev.append((time.perf_counter() - T[0], "create-returned", "", "", ""))
        await sh.wait_for(lambda: sh.notebook_ready(nm), 30)
        ev.append((time.perf_counter() - T[0], "READY", "", "", ""))
        await sh.admin.delete(kinds.NOTEBOOK, nm, "bench-0")
        await sh.wait_for(lambda: sh.gone(nm), 30)
        ev.append((time.perf_counter() - T[0], "GONE", "", "", ""))
        await sh.settle(5)
        ev.append((time.perf_counter() - T[0], "SETTLED", "", "", ""))
    for e in sorted(ev):
        print("%8.2f ms %-16s %-9s %-60s %s" % ((e[0]*1e3,) + tuple(e[1:])))
    await sh.stop(); await native.stop()
asyncio.run(main())
