"""Race and memory-error detection for the native apiserver (host code).

The reference runs no ``-race`` and no sanitizers.  The native apiserver is
the multi-threaded piece of this framework — one thread per connection, a store mutex,
per-namespace watcher wake-ups, a pooled HTTPS client for admission webhooks — so it is
rebuilt here with ThreadSanitizer and with AddressSanitizer + UBSan (host-only builds:
no GPU code is involved) and driven with a concurrent workload: writers in several
namespaces (create / update / merge- and JSON-patch / delete with GC of dependents),
namespace-scoped and cluster-wide watches that come and go, and two control-plane shards
taking notebooks to Ready through the HTTPS webhook.  Any sanitizer report fails the test.
"""

import asyncio
import glob
import os
import shutil
import subprocess

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.errors import ApiError
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "odh_kubeflow_amd", "testing", "native", "apiserver", "apiserver.cpp")

# OpenSSL is not instrumented: ignore what TSAN cannot see inside it
TSAN_SUPP = "called_from_lib:libssl.so\ncalled_from_lib:libcrypto.so\n"


def _build(tmp, sanitize: str) -> str:
    if shutil.which("g++") is None:
        pytest.skip("g++ missing")
    out = os.path.join(tmp, "odh-apiserver-" + sanitize.replace(",", "-"))
    cmd = ["g++", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}", "-std=c++17", "-pthread",
           "-I", os.path.dirname(SRC), SRC, "-o", out, "-lssl", "-lcrypto"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip(f"-fsanitize={sanitize} unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    return out


async def _workload(url: str) -> None:
    c = RestClient(RestConfig(host=url))
    namespaces = [f"race-{i}" for i in range(4)]
    for ns in namespaces:
        await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})

    async def writer(ns: str, w: int):
        for i in range(25):
            name = f"cm-{w}-{i}"
            owner = await c.create({"apiVersion": "v1", "kind": "ConfigMap",
                                    "metadata": {"name": name, "namespace": ns, "labels": {"w": str(w)}},
                                    "data": {"i": str(i)}})
            await c.create({"apiVersion": "v1", "kind": "Secret",
                            "metadata": {"name": name, "namespace": ns, "ownerReferences": [
                                {"apiVersion": "v1", "kind": "ConfigMap", "name": name,
                                 "uid": owner["metadata"]["uid"]}]}})
            cur = await c.get(kinds.CONFIG_MAP, name, ns)
            cur["data"]["u"] = "1"
            await c.update(cur)
            await c.patch(kinds.CONFIG_MAP, {"data": {"m": "2"}}, name=name, namespace=ns)
            await c.patch(kinds.CONFIG_MAP, [{"op": "add", "path": "/data/j", "value": "3"}], "json", name=name,
                          namespace=ns)
            if i % 2:
                await c.delete(kinds.CONFIG_MAP, name, ns)  # GC takes the Secret with it

    async def watcher(ns, stop: asyncio.Event):
        while not stop.is_set():
            try:
                async for _et, _obj in c.watch("v1/ConfigMap", ns, "", timeout_s=1):
                    if stop.is_set():
                        break
            except ApiError:
                pass

    stop = asyncio.Event()
    watchers = [asyncio.ensure_future(watcher(ns, stop)) for ns in namespaces + [None]]
    await asyncio.gather(*(writer(ns, w) for ns in namespaces for w in range(3)))
    stop.set()
    await asyncio.gather(*watchers, return_exceptions=True)
    await c.close()


async def _two_shards(url: str) -> None:
    from odh_kubeflow_amd.models.notebook import notebook
    from odh_kubeflow_amd.parallel.platform import NodePlatform
    from odh_kubeflow_amd.parallel.shard import ControlPlaneShard, ShardConfig

    env = {"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"}
    platform = await NodePlatform(url, process=False).start()
    shards = [await ControlPlaneShard(ShardConfig(url, "bench-0", shard="0", bootstrap=True, env=env)).start()]
    shards.append(await ControlPlaneShard(ShardConfig(url, "bench-1", shard="1", env=env)).start())
    try:
        for step in range(3):
            for i, sh in enumerate(shards):
                await sh.admin.create(notebook(f"nb{step}", f"bench-{i}", image="img", gpus=1,
                                               annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
            for sh in shards:
                assert await sh.wait_until(lambda: sh.notebook_ready(f"nb{step}"), 60)
            for i, sh in enumerate(shards):
                await sh.admin.delete(kinds.NOTEBOOK, f"nb{step}", f"bench-{i}")
            for sh in shards:
                assert await sh.wait_until(lambda: sh.gone(f"nb{step}"), 60)
    finally:
        for sh in reversed(shards):
            await sh.stop()
        await platform.stop()


@pytest.mark.parametrize("sanitize", ["thread", "address,undefined"])
def test_native_apiserver_under_sanitizers(run, tmp_path, sanitize):
    from odh_kubeflow_amd.testing.apiserver.native import NativeApiServer
    from odh_kubeflow_amd.testing.cluster import OPENSHIFT_CRDS

    binary = _build(str(tmp_path), sanitize)
    logs = str(tmp_path / "san")
    supp = tmp_path / "tsan.supp"
    supp.write_text(TSAN_SUPP)
    env = {"TSAN_OPTIONS": f"halt_on_error=0 log_path={logs} suppressions={supp} second_deadlock_stack=1",
           "ASAN_OPTIONS": f"log_path={logs} detect_leaks=0", "UBSAN_OPTIONS": f"log_path={logs} print_stacktrace=1"}

    async def go():
        srv = await NativeApiServer(OPENSHIFT_CRDS, gc=True, binary=binary, env=env).start()
        try:
            await _workload(srv.url)
            await _two_shards(srv.url)
        finally:
            await srv.stop()

    run(go(), timeout=600)
    reports = []
    for f in glob.glob(logs + "*"):
        with open(f) as fh:
            text = fh.read()
        if "ThreadSanitizer" in text or "AddressSanitizer" in text or "runtime error" in text:
            reports.append(text[:4000])
    assert not reports, "\n\n".join(reports)
