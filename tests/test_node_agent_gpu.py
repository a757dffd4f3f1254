"""The production node agent (``cmd/node_agent.py``) on a real MI355X, as the DaemonSet runs it.

The agent runs as its own process against the box's real ``/sys`` (amdgpu busy counters, the
KFD topology and KFD's per-process VRAM) with a bearer token, a pod-resources socket served
by the kubelet stand-in, and a ``/proc`` view whose cgroup file puts THIS test process — which
holds ≥ 1 GiB of VRAM on the GPU — in a pod.  It checks, on hardware:

* KFD per-process VRAM: this process is listed on the KFD node whose PCI address is the one
  torch reports for ``cuda:0``, with ≥ 1 GiB (``ops/csrc/gpu_telemetry.cpp:odh_tel_kfd_procs``);
* attribution: the pod (via the pod-resources API, by namespace/name) and the pod UID (via
  KFD + cgroup) both resolve to that GPU's PCI address, with the pod's own VRAM;
* ``/gpu/activity``: busy_mean ≥ 90 while the MFMA load generator runs, ≤ 5 after it stopped;
* HTTPS with the agents' CA (a cleartext request gets nothing); auth: 401 without the token, 200
  with it; source health on ``/metrics``.

Reference signal replaced: Jupyter ``/api/kernels`` + ``/api/terminals`` last-activity
(``kf/controllers/culling_controller.go:161-196,220-241``).
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.request
import uuid

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_CTX = [None]  # the agent's CA (HTTPS, as the DaemonSet serves)


def _get(url, token=None, timeout=10):
    req = urllib.request.Request(url, headers={"Authorization": f"Bearer {token}"} if token else {})
    try:
        with urllib.request.urlopen(req, timeout=timeout, context=_CTX[0]) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


def _torch_bdf(dev: int = 0):
    p = torch.cuda.get_device_properties(dev)
    if not all(hasattr(p, a) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id")):
        return None
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def _kfd_listing() -> str:
    root = "/sys/class/kfd/kfd/proc"
    try:
        return ", ".join(f"{p}:{sorted(os.listdir(os.path.join(root, p)))}" for p in sorted(os.listdir(root))[:8])
    except OSError as e:
        return repr(e)


@pytest.fixture(scope="module")
def gpu_state():
    """This process's KFD entry, found the way a node agent must find it: KFD names processes by
    their host PID (``/sys/class/kfd/kfd/proc/<pid>``), which differs from ``os.getpid()`` inside
    a container — so the entry is the one whose VRAM grows by the 1 GiB this fixture allocates."""
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from odh_kubeflow_amd.ops.telemetry import Telemetry

    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    tel = Telemetry("/sys")
    before = {(p.pid, p.gpu_id): p.vram_bytes for p in tel.kfd_processes("/proc")}
    hold = torch.empty((1 << 30) // 4 + (64 << 20), dtype=torch.float32, device="cuda:0")  # > 1 GiB, resident
    hold.fill_(1.0)
    torch.cuda.synchronize()
    after = tel.kfd_processes("/proc")
    mine = [p for p in after if p.vram_bytes - before.get((p.pid, p.gpu_id), 0) >= (1 << 30)]
    yield {"hold": hold, "tel": tel, "mine": mine, "devs": tel.devices(), "after": after}
    tel.close()


def test_kfd_lists_this_process_on_torchs_gpu(gpu_state):
    mine, devs = gpu_state["mine"], gpu_state["devs"]
    assert devs, "no KFD GPU nodes under /sys"
    assert len(mine) == 1, f"no single KFD entry grew by the 1 GiB allocation: {gpu_state['after']} " \
                           f"(/sys/class/kfd/kfd/proc: {_kfd_listing()})"
    assert mine[0].vram_bytes >= 1 << 30
    dev = {d.gpu_id: d for d in devs}[mine[0].gpu_id]
    bdf = _torch_bdf(0)
    print(f"KFD: pid {mine[0].pid} (os.getpid() {os.getpid()}) holds {mine[0].vram_bytes >> 20} MiB on "
          f"{dev.pci_bdf} (torch cuda:0: {bdf})")
    if bdf is not None:
        assert dev.pci_bdf.lower() == bdf.lower(), (dev.pci_bdf, bdf)


def test_node_agent_process_on_the_mi355x(gpu_state, tmp_path):
    from odh_kubeflow_amd.ops.gpu import LoadGenerator
    from odh_kubeflow_amd.testing.kubelet.podresources_server import FakePodResourcesServer

    mine, devs = gpu_state["mine"], gpu_state["devs"]
    assert len(mine) == 1
    dev = {d.gpu_id: d for d in devs}[mine[0].gpu_id]
    bdf, idx = dev.pci_bdf, dev.index

    # this process in a pod: a host-/proc view whose cgroup file (for the host PID KFD uses)
    # names a pod UID (systemd driver) — what the DaemonSet's hostPath /proc mount shows
    uid = str(uuid.uuid4())
    proc = tmp_path / "proc" / str(mine[0].pid)
    proc.mkdir(parents=True)
    (proc / "cgroup").write_text(
        f"0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{uid.replace('-', '_')}.slice/"
        f"cri-containerd-{os.getpid():064x}.scope\n")
    token = "s3cret-" + uuid.uuid4().hex
    tok = tmp_path / "token"
    tok.write_text(token)
    sock = str(tmp_path / "kubelet.sock")
    srv = FakePodResourcesServer(sock).start()
    srv.assign("team", "nb-0", "nb", "amd.com/gpu", [bdf])
    port = _port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    from odh_kubeflow_amd.utils.tlsreload import client_context
    from odh_kubeflow_amd.webhook.certs import generate

    certs = generate(("127.0.0.1", "mi355x-node-agent.opendatahub.svc"), str(tmp_path / "tls"))
    _CTX[0] = client_context(os.path.join(certs.cert_dir, "ca.crt"))
    agent = subprocess.Popen([sys.executable, "-m", "odh_kubeflow_amd.cmd.node_agent", "--bind", "127.0.0.1",
                              "--port", str(port), "--sysfs-root", "/sys", "--proc-root", str(tmp_path / "proc"),
                              "--pod-resources-socket", sock, "--device-plugin-checkpoint", "",
                              "--telemetry-interval-ms", "50", "--attribution-ttl-s", "0.2",
                              "--token-file", str(tok), "--tls-cert-dir", certs.cert_dir], cwd=ROOT, env=env,
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    base = f"https://127.0.0.1:{port}"
    load = None
    try:
        deadline = time.monotonic() + 60
        while time.monotonic() < deadline:
            try:
                if _get(base + "/healthz")[0] == 200:
                    break
            except OSError:
                time.sleep(0.1)
        else:
            pytest.fail(f"node agent did not come up: {agent.stderr.read() if agent.poll() is not None else ''}")
        # HTTPS only: a cleartext request gets no answer
        with pytest.raises(Exception):
            urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5).read()
        # auth: data endpoints need the token, /healthz does not
        assert _get(base + "/gpu/pods")[0] == 401
        assert _get(base + "/gpu/activity?devices=0")[0] == 401
        assert _get(base + "/metrics", token="wrong")[0] == 401
        st, body = _get(base + "/gpu/pods", token)
        assert st == 200
        pods = json.loads(body)
        assert pods["sources"] == {"podresources": "ok", "kfd": "ok"}, pods
        assert pods["by_name"]["team/nb-0"] == [idx]
        assert pods["kfd_vram_bytes"][uid][str(idx)] >= 1 << 30
        # the pod by namespace/name (pod-resources) and by UID (KFD + cgroup): the same GPU
        st, body = _get(f"{base}/gpu/activity?namespace=team&name=nb-0&pod_uid={uid}&window=2", token)
        a = json.loads(body)
        assert st == 200 and a["attributed"] and a["devices"] == [bdf], a
        assert set(a["sources"]) == {"podresources", "kfd"} and a["pod_vram_bytes"] >= 1 << 30, a
        # busy under an MFMA load, idle after it stops
        load = LoadGenerator(device=0, duty=1.0).start()
        time.sleep(3.0)
        busy = json.loads(_get(f"{base}/gpu/activity?devices={idx}&window=2", token)[1])
        load.stop()
        load = None
        time.sleep(3.0)
        idle = json.loads(_get(f"{base}/gpu/activity?devices={idx}&window=2", token)[1])
        print(f"node agent on {bdf}: busy_mean {busy.get('busy_mean')} under load, {idle.get('busy_mean')} idle")
        assert busy["n"] > 10 and busy["busy_mean"] >= 90, busy
        assert idle["n"] > 10 and idle["busy_mean"] <= 5, idle
        st, metrics = _get(base + "/metrics", token)
        assert st == 200
        assert 'odh_node_agent_attribution_source_up{source="podresources"} 1' in metrics
        assert f'amdgpu_busy_percent{{gpu="{idx}",bdf="{bdf}"' in metrics
    finally:
        if load is not None:
            load.stop()
        agent.terminate()
        try:
            agent.wait(10)
        except subprocess.TimeoutExpired:
            agent.kill()
        srv.stop()
