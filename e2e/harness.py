"""Where the e2e suite runs: a deployed cluster, or the dev stack as local processes.

The reference's e2e suite (``odh/e2e/*.go``, driver ``odh/run-e2e-test.sh``) runs against
a cluster after ``make deploy``: it checks the controller Deployments, then walks two
notebooks through create → route / NetworkPolicies / StatefulSet 1/1 / auth sidecar →
culling (culler ConfigMap + controller rollout) → image update → deletion.  The same
suite here (``e2e/test_notebook_e2e.py``) talks to either:

* :class:`ClusterHarness` — any cluster reachable through a kubeconfig, with an overlay
  of ``config/`` deployed (``make deploy`` / ``make deploy-sharded``): Deployments or the
  sharded control-plane StatefulSet are checked for availability, culling is switched on
  through the culler ConfigMap and a rollout, exactly as the reference does;
* :class:`LocalHarness` — no cluster: the dev apiserver (+ StatefulSet controller,
  scheduler, GC), the kf and odh managers (HTTPS webhook behind a MutatingWebhookConfiguration
  with a self-signed caBundle) and the dev kubelet serving the Jupyter API, each its own
  process; culling is switched on by restarting the kf manager with the culler settings
  (the in-cluster rollout's effect).

Both expose the same operations; timeouts follow the reference (3 min / 10 s polls on a
cluster, tens of seconds / 100 ms polls locally).
"""

from __future__ import annotations

import asyncio
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time
from typing import Dict, List, Optional, Tuple

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models import meta as m
from odh_kubeflow_amd.models.errors import ApiError
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Harness:
    timeout = 180.0  # odh/e2e/notebook_controller_setup_test.go:94-95
    interval = 10.0
    cull_wait = 300.0

    def __init__(self, nb_namespace: str, controller_namespace: str):
        self.nb_ns = nb_namespace
        self.ctrl_ns = controller_namespace
        self.client: Optional[RestClient] = None
        self.loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self.loop.run_forever, name="e2e-loop", daemon=True)
        self._thread.start()

    # the suite is synchronous (pytest); every API call runs on the harness' loop
    def run(self, coro, timeout: Optional[float] = None):
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout or self.timeout + 60)

    def eventually(self, fn, timeout: Optional[float] = None, interval: Optional[float] = None, what: str = ""):
        """Poll ``fn`` (an async callable) until it returns a truthy value."""
        async def poll():
            deadline = time.monotonic() + (timeout or self.timeout)
            last = None
            while time.monotonic() < deadline:
                try:
                    last = await fn()
                    if last:
                        return last
                except ApiError as e:
                    last = e
                await asyncio.sleep(interval or self.interval)
            raise AssertionError(f"timed out waiting for {what or fn}: last={last!r}")
        return self.run(poll(), (timeout or self.timeout) + 30)

    # -------------------------------------------------------------- hooks
    def controllers(self) -> List[Tuple[str, bool, str]]:
        raise NotImplementedError

    def enable_culling(self) -> None:
        raise NotImplementedError

    def restore_culling(self) -> None:
        raise NotImplementedError

    def jupyter_kernels(self, nb: dict) -> Optional[int]:
        """HTTP status of the notebook's Jupyter ``/api/kernels`` where the runner can reach
        it directly, else ``None`` (the in-cluster check goes through the Service, as the
        reference's ``testNotebookServiceConnectivity`` does)."""
        return None

    def close(self) -> None:
        if self.client is not None:
            self.run(self.client.close(), 30)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self._thread.join(10)


class ClusterHarness(Harness):
    """A deployed overlay on a real cluster (``--kubeconfig`` / ``KUBECONFIG``)."""

    def __init__(self, nb_namespace: str, controller_namespace: str, kubeconfig: Optional[str] = None,
                 name_prefix: str = "odh-kubeflow-amd-", in_cluster: bool = False):
        super().__init__(nb_namespace, controller_namespace)
        self.client = RestClient(RestConfig.in_cluster() if in_cluster else RestConfig.load(None, kubeconfig))
        self.prefix = name_prefix
        self._culler_saved: Optional[Dict[str, str]] = None
        self._culler_created = False

        async def ensure_ns():  # the reference's run-e2e-test.sh creates it (`oc new-project`)
            try:
                await self.client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": nb_namespace}})
            except ApiError as e:
                if e.code not in (403, 409):
                    raise
        self.run(ensure_ns())

    def _workloads(self) -> List[Tuple[str, str]]:
        async def find():
            out = []
            for kind in (kinds.DEPLOYMENT, kinds.STATEFUL_SET):
                for o in await self.client.list(kind, self.ctrl_ns):
                    n = m.name(o)
                    if n in (f"{self.prefix}deployment", f"{self.prefix}manager", f"{self.prefix}control-plane"):
                        out.append((kind, n))
            return out
        return self.run(find())

    def controllers(self) -> List[Tuple[str, bool, str]]:
        workloads = self._workloads()
        if not workloads:
            return [("controller workloads", False, f"none named {self.prefix}deployment / manager / control-plane "
                                                    f"in {self.ctrl_ns}")]

        async def check():
            res = []
            cms = [m.name(c) for c in await self.client.list(kinds.CONFIG_MAP, self.ctrl_ns)]
            res.append(("notebook-controller config ConfigMap", any(n.endswith("config") and "culler" not in n
                                                                    for n in cms), ",".join(cms)))
            try:
                await self.client.get(kinds.CRD, "notebooks.kubeflow.org")
                res.append(("Notebook CRD", True, ""))
            except ApiError as e:
                res.append(("Notebook CRD", False, str(e)))
            names = {n for _, n in workloads}
            if f"{self.prefix}control-plane" not in names:  # unsharded overlays: both managers
                for n in (f"{self.prefix}deployment", f"{self.prefix}manager"):
                    if n not in names:
                        res.append((f"Deployment {n}", False, "not deployed"))
            for kind, name in workloads:
                o = await self.client.get(kind, name, self.ctrl_ns)
                st = o.get("status") or {}
                want = (o.get("spec") or {}).get("replicas", 1)
                ok = (st.get("readyReplicas") or 0) >= min(1, want) and \
                    st.get("observedGeneration", 0) >= m.meta(o).get("generation", 0)
                res.append((f"{kind.split('/')[-1]} {name}", ok, f"ready {st.get('readyReplicas')}/{want}"))
            return res
        return self.run(check())

    def _kf_workload(self) -> Tuple[str, str]:
        wl = dict((n, k) for k, n in self._workloads())
        for n in (f"{self.prefix}deployment", f"{self.prefix}control-plane"):
            if n in wl:
                return wl[n], n
        raise AssertionError("no kf controller workload deployed")

    def _rollout(self) -> None:
        kind, name = self._kf_workload()

        async def restart():
            stamp = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
            o = await self.client.patch(kind, {"spec": {"template": {"metadata": {"annotations": {
                "kubectl.kubernetes.io/restartedAt": stamp}}}}}, "merge", name=name, namespace=self.ctrl_ns)
            return m.meta(o).get("generation", 0)
        gen = self.run(restart())

        async def rolled():
            o = await self.client.get(kind, name, self.ctrl_ns)
            st = o.get("status") or {}
            want = (o.get("spec") or {}).get("replicas", 1)
            return st.get("observedGeneration", 0) >= gen and st.get("updatedReplicas", 0) >= want and \
                st.get("readyReplicas", 0) >= want
        self.eventually(rolled, what=f"rollout of {name}")

    def enable_culling(self) -> None:
        name = f"{self.prefix}notebook-controller-culler-config"
        data = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME": "2", "IDLENESS_CHECK_PERIOD": "1"}

        async def apply():
            try:
                cm = await self.client.get(kinds.CONFIG_MAP, name, self.ctrl_ns)
                self._culler_saved = dict(cm.get("data") or {})
                cm["data"] = {**self._culler_saved, **data}
                await self.client.update(cm)
            except ApiError:
                self._culler_created = True
                await self.client.create({"apiVersion": "v1", "kind": "ConfigMap",
                                          "metadata": {"name": name, "namespace": self.ctrl_ns}, "data": data})
        self.run(apply())
        self._rollout()

    def restore_culling(self) -> None:
        name = f"{self.prefix}notebook-controller-culler-config"

        async def revert():
            if self._culler_created:
                await self.client.delete(kinds.CONFIG_MAP, name, self.ctrl_ns)
            elif self._culler_saved is not None:
                cm = await self.client.get(kinds.CONFIG_MAP, name, self.ctrl_ns)
                cm["data"] = self._culler_saved
                await self.client.update(cm)
        self.run(revert())
        self._rollout()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class LocalHarness(Harness):
    """The dev stack as separate processes, no cluster needed (CI, this repository's tests)."""

    timeout = 60.0
    interval = 0.1
    cull_wait = 60.0
    CULLER = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME_SECONDS": "2.5", "IDLENESS_CHECK_PERIOD_SECONDS": "0.3",
              "CULLER_USE_POD_ENDPOINT": "true"}

    def __init__(self, nb_namespace: str, controller_namespace: str, workdir: Optional[str] = None):
        super().__init__(nb_namespace, controller_namespace)
        self.workdir = workdir or tempfile.mkdtemp(prefix="odh-e2e-")
        self.procs: Dict[str, subprocess.Popen] = {}
        self._log = open(os.path.join(self.workdir, "processes.log"), "wb")
        self.api_port, self.wh_port = _free_port(), _free_port()
        self.master = f"http://127.0.0.1:{self.api_port}"
        self.common = {"K8S_NAMESPACE": controller_namespace, "SET_PIPELINE_RBAC": "false"}
        self._start()

    def _spawn(self, key: str, args: List[str], env: Optional[dict] = None) -> None:
        e = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), **(env or {}))
        self.procs[key] = subprocess.Popen([sys.executable, "-m", *args], cwd=ROOT, env=e, stdout=self._log,
                                           stderr=subprocess.STDOUT)

    def _kf_args(self) -> List[str]:
        return ["odh_kubeflow_amd.cmd.kf_manager", "--master", self.master, "--metrics-addr", "0", "--probe-addr",
                "0", "--enable-leader-election"]

    def _start(self) -> None:
        from odh_kubeflow_amd.webhook.certs import generate
        from odh_kubeflow_amd.webhook.server import mutating_webhook_configuration

        self._spawn("apiserver", ["odh_kubeflow_amd.testing.cmd.apiserver", "--port", str(self.api_port), "--controllers",
                                  "--no-openshift-apis"])
        certs = generate(("127.0.0.1", "localhost"), os.path.join(self.workdir, "certs"))
        self._wait_http(self.master + "/healthz")
        self.client = RestClient(RestConfig(host=self.master))

        async def bootstrap():
            for ns in (self.ctrl_ns, self.nb_ns):
                await self.client.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        self.run(bootstrap())
        self._spawn("kf", self._kf_args(), self.common)
        self._spawn("odh", ["odh_kubeflow_amd.cmd.odh_manager", "--master", self.master, "--metrics-bind-address",
                            "0", "--health-probe-bind-address", "0", "--kube-rbac-proxy-image",
                            "quay.io/brancz/kube-rbac-proxy:v0.18.1", "--webhook-cert-dir", certs.cert_dir,
                            "--webhook-port", str(self.wh_port), "--webhook-host", "127.0.0.1", "--leader-elect"],
                    self.common)
        self._spawn("kubelet", ["odh_kubeflow_amd.testing.cmd.fake_kubelet", "--master", self.master, "--jupyter",
                                "--checkpoint-path", os.path.join(self.workdir, "dp", "cp")], self.common)
        self._wait_http(f"https://127.0.0.1:{self.wh_port}/healthz")
        self.run(self.client.create(mutating_webhook_configuration(
            certs.ca_bundle_b64, url=f"https://127.0.0.1:{self.wh_port}/mutate-notebook-v1")))
        self.eventually(lambda: self.client.get(kinds.NODE, "mi355x-node-0"), what="dev kubelet Node")

    def _wait_http(self, url: str, timeout: float = 60.0) -> None:
        import ssl
        import urllib.request

        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE  # lint: allow python-ssl-verify-disabled — local health probe of a self-signed dev server
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            try:
                with urllib.request.urlopen(url, timeout=2, context=ctx) as r:
                    if r.status == 200:
                        return
            except OSError:
                pass
            time.sleep(0.1)
        raise TimeoutError(url)

    def controllers(self) -> List[Tuple[str, bool, str]]:
        async def leases():
            return {m.name(x) for x in await self.client.list(kinds.LEASE, self.ctrl_ns)}
        held = self.eventually(lambda: self._leases_held(leases), what="controller leases")
        res = [(f"process {k}", p.poll() is None, f"pid {p.pid}") for k, p in self.procs.items()]
        res.append(("leases", True, ",".join(sorted(held))))
        return res

    async def _leases_held(self, leases):
        held = await leases()
        return held if {"kubeflow-notebook-controller", "odh-notebook-controller"} <= held else None

    def _restart_kf(self, env: dict) -> None:
        p = self.procs.pop("kf")
        p.terminate()
        try:
            p.wait(15)
        except subprocess.TimeoutExpired:
            p.kill()
        self._spawn("kf", self._kf_args(), env)

    def enable_culling(self) -> None:
        self._restart_kf({**self.common, **self.CULLER})

    def restore_culling(self) -> None:
        self._restart_kf(self.common)

    def jupyter_kernels(self, nb: dict) -> Optional[int]:
        import urllib.request

        pod = self.run(self.client.get(kinds.POD, f"{m.name(nb)}-0", m.namespace(nb)))
        ep = m.annotations(pod).get("amd.com/notebook-endpoint")
        if not ep:
            return None
        url = f"http://{ep}/notebook/{m.namespace(nb)}/{m.name(nb)}/api/kernels"
        deadline = time.monotonic() + self.timeout
        while True:  # the server may still be binding its port when the pod turns Ready
            try:
                with urllib.request.urlopen(url, timeout=10) as r:
                    return r.status
            except OSError:
                if time.monotonic() > deadline:
                    raise
                time.sleep(self.interval)

    def close(self) -> None:
        try:
            super().close()
        finally:
            for p in self.procs.values():
                p.terminate()
            for p in self.procs.values():
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
            self._log.close()
