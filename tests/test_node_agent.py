"""Production node agent (``nodeagent/``, ``cmd/node_agent.py``): pod→GPU attribution from the
kubelet pod-resources API, the device-plugin checkpoint and KFD per-process sysfs; its HTTP
API; GPU-busy culling through it with no ``amd.com/gpu-ids`` on any pod; and the guarantee
that the shipped agent never writes to the apiserver.

Replaces the fake-scheduler annotation lookup the round-1 culler used; the reference signal
being replaced is ``kf/controllers/culling_controller.go:161-196,243-273``."""

import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

from odh_kubeflow_amd.nodeagent import podresources as pr
from odh_kubeflow_amd.testing.kubelet.podresources_server import FakePodResourcesServer
from odh_kubeflow_amd.nodeagent.attribution import Attributor, DeviceResolver
from odh_kubeflow_amd.nodeagent.checkpoint import CheckpointWriter, read_checkpoint
from odh_kubeflow_amd.nodeagent.server import NodeTelemetryAgent
from odh_kubeflow_amd.ops.telemetry import (Telemetry, fake_bdf, fake_gpu_id, set_fake_counter, set_fake_kfd_process,
                                            write_fake_sysfs)

UID_A = "0d6f2a50-1c9e-4f0e-9a53-2b7c8d9e0f11"
UID_B = "7e1c3b2a-9d8f-4e6a-b5c4-3a2b1c0d9e8f"


@pytest.fixture
def sysfs(tmp_path):
    root = str(tmp_path / "sys")
    proc = str(tmp_path / "proc")
    os.makedirs(proc)
    minors = write_fake_sysfs(root, gpus=8)
    tel = Telemetry(root).start(interval_ms=10, capacity=1000)
    yield root, proc, minors, tel
    tel.close()


def test_podresources_codec_roundtrip():
    pods = [pr.PodResources("nb-0", "user", [pr.ContainerResources("nb", [
        pr.ContainerDevices("amd.com/gpu", ["0000:10:00.0", "0000:20:00.0"]),
        pr.ContainerDevices("example.com/nic", ["eth9"])])]), pr.PodResources("cpu-0", "user", [])]
    back = pr.decode_list_response(pr.encode_list_response(pods))
    assert back == pods
    assert back[0].device_ids("amd.com/gpu") == ["0000:10:00.0", "0000:20:00.0"]
    # unknown fields (cpu_ids as packed varints, topology) are skipped
    extra = pr._ld(1, pr._s(1, "x") + pr._s(2, "ns") + pr._ld(3, pr._s(1, "c") + pr._ld(3, b"\x01\x02")
                                                        + pr._varint(4 << 3 | 0) + pr._varint(300)))
    assert pr.decode_list_response(extra)[0].containers[0].name == "c"


def test_podresources_grpc_list(tmp_path):
    sock = str(tmp_path / "kubelet.sock")
    srv = FakePodResourcesServer(sock).start()
    try:
        srv.assign("user", "nb-0", "nb", "amd.com/gpu", [fake_bdf(3)])
        cli = pr.PodResourcesClient(sock)
        assert cli.available()
        got = asyncio.run(cli.list())
        assert [(p.namespace, p.name, p.device_ids("amd.com/gpu")) for p in got] == [("user", "nb-0", [fake_bdf(3)])]
        cli.close()
    finally:
        srv.stop()


def test_checkpoint_shapes(tmp_path):
    path = str(tmp_path / "kubelet_internal_checkpoint")
    with open(path, "w") as f:
        json.dump({"Data": {"PodDeviceEntries": [
            {"PodUID": UID_A, "ContainerName": "a", "ResourceName": "amd.com/gpu", "DeviceIDs": {"1": [fake_bdf(2)],
                                                                                                 "0": [fake_bdf(1)]}},
            {"PodUID": UID_B, "ContainerName": "b", "ResourceName": "amd.com/gpu", "DeviceIDs": [fake_bdf(5)]},
            {"PodUID": UID_B, "ContainerName": "b", "ResourceName": "nvidia.com/gpu", "DeviceIDs": ["GPU-x"]}],
            "RegisteredDevices": {}}, "Checksum": 1}, f)
    assert read_checkpoint(path) == {UID_A: [fake_bdf(1), fake_bdf(2)], UID_B: [fake_bdf(5)]}
    assert read_checkpoint(str(tmp_path / "missing")) is None
    w = CheckpointWriter(str(tmp_path / "dp" / "cp"))
    w.allocate(UID_A, "nb", [fake_bdf(0)])
    assert read_checkpoint(w.path) == {UID_A: [fake_bdf(0)]}
    w.release(UID_A)
    assert read_checkpoint(w.path) == {}


def test_device_resolver_bdf_partitions(tmp_path):
    write_fake_sysfs(str(tmp_path), gpus=2, partitions=4)  # CPX-style: 4 KFD nodes per MI355X
    tel = Telemetry(str(tmp_path))
    try:
        res = DeviceResolver(tel.devices())
        assert res.resolve(fake_bdf(1)) == [4, 5, 6, 7]
        assert res.resolve(fake_bdf(1).upper()) == [4, 5, 6, 7]
        assert res.resolve(fake_bdf(1)[5:]) == [4, 5, 6, 7]  # domain omitted
        assert res.resolve("renderD129") == [1] and res.resolve("card2") == [2] and res.resolve("3") == [3]
        assert res.resolve("0000:99:00.0") == [] and res.resolve("GPU-uuid") == []
    finally:
        tel.close()


def test_attribution_sources(run, sysfs, tmp_path):
    root, proc, _minors, tel = sysfs
    sock = str(tmp_path / "pr.sock")
    srv = FakePodResourcesServer(sock).start()
    cp = CheckpointWriter(str(tmp_path / "dp" / "kubelet_internal_checkpoint"))
    try:
        srv.assign("user", "a-0", "a", "amd.com/gpu", [fake_bdf(0)])
        cp.allocate(UID_B, "b", [fake_bdf(6), "0000:99:00.0"])
        set_fake_kfd_process(root, proc, 4242, {fake_gpu_id(3): 5 << 30}, UID_A, systemd=True)
        set_fake_kfd_process(root, proc, 4243, {fake_gpu_id(3): 1 << 30, fake_gpu_id(0): 7}, UID_A, systemd=False)
        set_fake_kfd_process(root, proc, 99, {fake_gpu_id(1): 1 << 20})  # host daemon, no pod

        async def go():
            att = Attributor(tel, pod_resources=pr.PodResourcesClient(sock), checkpoint_path=cp.path,
                             proc_root=proc, ttl_s=0.0)
            a = await att.lookup(UID_A, "user", "a-0")
            assert a.devices == [0, 3] and set(a.sources) == {"podresources", "kfd"}
            assert a.vram_bytes == {3: 6 << 30, 0: 7} and a.pod_vram_bytes == (6 << 30) + 7
            b = await att.lookup(UID_B, "user", "b-0")
            assert b.devices == [6] and b.sources == ["checkpoint"] and b.pod_vram_bytes is None
            assert await att.lookup("no-such-uid", "user", "c-0") is None
            tables = await att.all_pods()
            assert tables["sources"] == {"podresources": "ok", "checkpoint": "ok", "kfd": "ok"}
            assert tables["unresolved_device_ids"] == ["0000:99:00.0"]
            # a source that fails is reported, the others still answer
            bogus = tmp_path / "not-a-grpc.sock"
            bogus.write_text("")
            att2 = Attributor(tel, pod_resources=pr.PodResourcesClient(str(bogus), timeout_s=0.2),
                              checkpoint_path=cp.path, ttl_s=0.0)
            assert (await att2.lookup(UID_B)).devices == [6]
            assert (await att2.all_pods())["sources"]["podresources"].startswith("error")
            assert att2.source_health() == {"podresources": 0, "checkpoint": 1}
        run(go())
    finally:
        srv.stop()


def test_pod_resources_socket_that_appears_later_is_used(run, sysfs, tmp_path):
    """The kubelet socket is re-checked on every refresh: an agent started before the kubelet
    mounted it switches to the pod-resources API as soon as it appears (and reports it gone
    when it disappears), instead of losing that source for its whole lifetime."""
    _root, _proc, _minors, tel = sysfs
    sock = str(tmp_path / "late.sock")

    async def go():
        att = Attributor(tel, pod_resources=pr.PodResourcesClient(sock, timeout_s=0.5), ttl_s=0.0)
        assert await att.lookup(None, "user", "a-0") is None
        assert (await att.all_pods())["sources"] == {"podresources": "unavailable"}
        assert att.source_health() == {"podresources": 0}
        srv = FakePodResourcesServer(sock).start()
        try:
            srv.assign("user", "a-0", "a", "amd.com/gpu", [fake_bdf(2)])
            a = await att.lookup(None, "user", "a-0")
            assert a is not None and a.devices == [2] and a.sources == ["podresources"]
            assert att.source_health() == {"podresources": 1}
        finally:
            srv.stop()
        if os.path.exists(sock):
            os.unlink(sock)
        assert await att.lookup(None, "user", "a-0") is None
        assert att.source_health() == {"podresources": 0}
    run(go())


def test_concurrent_lookups_share_one_refresh(run, sysfs, tmp_path):
    """A burst of culler queries finding the tables stale triggers ONE refresh (one List on
    the kubelet socket, one checkpoint read, one KFD scan), not one per query."""
    _root, _proc, _minors, tel = sysfs
    cp = CheckpointWriter(str(tmp_path / "dp" / "kubelet_internal_checkpoint"))
    cp.allocate(UID_B, "b", [fake_bdf(1)])

    async def go():
        att = Attributor(tel, checkpoint_path=cp.path, ttl_s=30.0)
        calls = {"n": 0}
        inner = att.refresh

        async def slow_refresh():
            calls["n"] += 1
            await asyncio.sleep(0.05)
            return await inner()
        att.refresh = slow_refresh
        res = await asyncio.gather(*(att.lookup(UID_B) for _ in range(16)))
        assert calls["n"] == 1 and all(r.devices == [1] for r in res)
        await att.lookup(UID_B)  # fresh: served from the table
        assert calls["n"] == 1
    run(go())


def _get(url):
    with urllib.request.urlopen(url, timeout=5) as r:
        return r.status, r.read().decode()


def test_agent_http_api(run, sysfs, tmp_path):
    root, proc, minors, tel = sysfs
    cp = CheckpointWriter(str(tmp_path / "dp" / "cp"))
    cp.allocate(UID_A, "nb", [fake_bdf(2)])
    set_fake_kfd_process(root, proc, 777, {fake_gpu_id(2): 3 << 30}, UID_A)
    set_fake_counter(root, minors[2], busy=80, vram_used=50 << 30)

    async def go():
        agent = await NodeTelemetryAgent(tel, Attributor(tel, checkpoint_path=cp.path, proc_root=proc, ttl_s=0.0),
                                         host="127.0.0.1", port=0).start()
        try:
            await asyncio.sleep(0.1)
            base = f"http://127.0.0.1:{agent.port}"
            st, body = await asyncio.to_thread(_get, f"{base}/gpu/activity?pod_uid={UID_A}&window=0.05")
            d = json.loads(body)
            assert st == 200 and d["attributed"] and d["devices"] == [fake_bdf(2)]
            assert d["busy_mean"] == 80 and d["n"] > 0 and d["pod_vram_bytes"] == 3 << 30
            d = json.loads((await asyncio.to_thread(_get, f"{base}/gpu/activity?pod_uid={UID_B}&window=5"))[1])
            assert d == {"attributed": False, "n": 0}
            pods = json.loads((await asyncio.to_thread(_get, f"{base}/gpu/pods"))[1])
            assert pods["by_uid"] == {UID_A: [2]} and pods["kfd_vram_bytes"] == {UID_A: {"2": 3 << 30}}
            devs = json.loads((await asyncio.to_thread(_get, f"{base}/gpu/devices"))[1])
            assert [x["pci_bdf"] for x in devs] == [fake_bdf(i) for i in range(8)]
            metrics = (await asyncio.to_thread(_get, f"{base}/metrics"))[1]
            assert f'amdgpu_busy_percent{{gpu="2",bdf="{fake_bdf(2)}",render_minor="{minors[2]}"}} 80' in metrics
            with pytest.raises(urllib.error.HTTPError):
                await asyncio.to_thread(_get, f"{base}/gpu/activity?window=5")
        finally:
            await agent.stop()
    run(go())


def test_culler_kfd_attribution_only(run, sysfs):
    """No checkpoint, no pod-resources, no annotation: the agent finds each notebook's GPU from
    the processes in its pod cgroup (KFD), culls the idle GPU notebook, keeps the busy one."""
    from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
    from odh_kubeflow_amd.controllers import culling as c
    from odh_kubeflow_amd.models import kinds
    from odh_kubeflow_amd.models import meta as m
    from odh_kubeflow_amd.models.notebook import STOP_ANNOTATION, notebook
    from odh_kubeflow_amd.utils import timeutil

    root, proc, minors, tel = sysfs
    offset = [0.0]
    timeutil.set_clock(lambda: time.time() + offset[0])

    import tempfile

    ca_dir = _ca(tempfile.mkdtemp(prefix="odh-agent-ca-"))

    async def go():
        # the cluster's one node (mi355x-node-0): its agent, with that node's own identity
        agent = await NodeTelemetryAgent(tel, Attributor(tel, proc_root=proc, ttl_s=0.0), host="127.0.0.1",
                                         port=0, tls_cert_dir=_node_identity(ca_dir, "mi355x-node-0")).start()
        # production defaults: https://<pod.status.hostIP>:<CULLING_GPU_AGENT_PORT>, verified against
        # the agents' CA and the name of the pod's node (<spec.nodeName>.mi355x-node-agent.nodes)
        env = {"ENABLE_CULLING": "true", "CULL_IDLE_TIME": "60", "IDLENESS_CHECK_PERIOD_SECONDS": "0.2",
               "CULLING_ACTIVITY_SOURCE": "amdgpu", "CULLING_GPU_AGENT_PORT": str(agent.port),
               "CULLING_GPU_AGENT_CA_FILE": os.path.join(ca_dir, "ca.crt"),
               "CLUSTER_DOMAIN": "invalid.example"}
        try:
            async with LocalCluster(ClusterConfig(culler=True, env=env)) as cl:
                await cl.ensure_namespace("u")
                for i, n in enumerate(("busy", "idle")):
                    await cl.admin.create(notebook(n, "u", gpus=1))
                    assert await cl.wait_for(lambda: cl.notebook_ready(n, "u"))
                    pod = cl.store.peek(kinds.POD, f"{n}-0", "u")
                    assert pod["status"]["hostIP"] == "127.0.0.1"
                    # the notebook's python process holds VRAM on GPU 4+i (KFD), in the pod's cgroup
                    set_fake_kfd_process(root, proc, 1000 + i, {fake_gpu_id(4 + i): 8 << 30}, m.uid(pod))
                set_fake_counter(root, minors[4], busy=90)
                culler = cl.reconcilers["culler"]
                assert await cl.wait_for(lambda: c.annotations_exist(cl.store.peek(kinds.NOTEBOOK, "busy", "u")))
                await asyncio.sleep(0.4)
                # checks made before the fake KFD entries existed fell back to Jupyter (no GPU
                # sample yet — how early depends on the transport); from here on none may
                jupyter0 = culler.jupyter.requests
                offset[0] += 7200
                assert await cl.wait_for(lambda: STOP_ANNOTATION in m.annotations(
                    cl.store.peek(kinds.NOTEBOOK, "idle", "u")), 10)
                assert STOP_ANNOTATION not in m.annotations(cl.store.peek(kinds.NOTEBOOK, "busy", "u"))
                assert agent.attributed_queries >= 2 and culler.jupyter.requests == jupyter0
        finally:
            await agent.stop()
    try:
        run(go(), timeout=60)
    finally:
        timeutil.set_clock(None)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shipped_agent_never_touches_the_apiserver(run, sysfs, tmp_path):
    """``python -m odh_kubeflow_amd.cmd.node_agent`` with in-cluster env and a kubeconfig both
    pointing at a listener that records every connection: it serves attribution and
    telemetry, and never connects."""
    from odh_kubeflow_amd.cmd import node_agent

    root, proc, minors, _tel = sysfs
    args = node_agent.parse(["--insecure"])
    assert not hasattr(args, "master") and not hasattr(args, "kubeconfig")
    with pytest.raises(SystemExit):
        node_agent.parse([])  # plain HTTP only when asked for
    cp = CheckpointWriter(str(tmp_path / "dp" / "cp"))
    cp.allocate(UID_A, "nb", [fake_bdf(1)])
    set_fake_counter(root, minors[1], busy=33)

    async def go():
        seen = []

        async def record(reader, writer):
            seen.append(await reader.read(64))
            writer.close()
        api = await asyncio.start_server(record, "127.0.0.1", 0)
        aport = api.sockets[0].getsockname()[1]
        kc = tmp_path / "kubeconfig"
        kc.write_text(f"apiVersion: v1\nclusters: [{{name: c, cluster: {{server: 'http://127.0.0.1:{aport}'}}}}]\n"
                      "contexts: [{name: c, context: {cluster: c, user: u}}]\ncurrent-context: c\n"
                      "users: [{name: u, user: {token: t}}]\n")
        port = _free_port()
        env = {**os.environ, "KUBERNETES_SERVICE_HOST": "127.0.0.1", "KUBERNETES_SERVICE_PORT": str(aport),
               "KUBECONFIG": str(kc)}
        p = subprocess.Popen([sys.executable, "-m", "odh_kubeflow_amd.cmd.node_agent", "--insecure", "--bind", "127.0.0.1",
                              "--port", str(port), "--sysfs-root", root, "--proc-root", proc,
                              "--pod-resources-socket", str(tmp_path / "absent.sock"),
                              "--device-plugin-checkpoint", cp.path, "--telemetry-interval-ms", "10"],
                             env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        try:
            body = None
            for _ in range(300):
                try:
                    st, body = await asyncio.to_thread(
                        _get, f"http://127.0.0.1:{port}/gpu/activity?pod_uid={UID_A}&window=0.5")
                    if json.loads(body).get("n", 0) > 0:
                        break
                except OSError:
                    pass
                await asyncio.sleep(0.05)
            d = json.loads(body)
            assert d["attributed"] and d["devices"] == [fake_bdf(1)] and d["busy_mean"] == 33
        finally:
            p.send_signal(signal.SIGTERM)
            out = await asyncio.to_thread(p.communicate, timeout=20)
            api.close()
        assert p.returncode == 0, out[0].decode()[-2000:]
        assert seen == [], seen  # not one request, let alone a Node or pods/status write
    run(go(), timeout=90)


def test_shipped_manifests_have_no_kubelet_stand_in():
    from odh_kubeflow_amd.deploy import manifests

    t = manifests.tree()
    ds = t["node-agent/daemonset.yaml"]
    spec = ds["spec"]["template"]["spec"]
    assert spec["automountServiceAccountToken"] is False
    c = spec["containers"][0]
    assert c["command"] == ["python", "-m", "odh_kubeflow_amd.cmd.node_agent"]
    assert not any(a.startswith(("--master", "--devices", "--node-name")) for a in c["args"])
    mounts = {v["mountPath"]: v for v in c["volumeMounts"]}
    assert mounts["/host/sys"]["readOnly"] and mounts["/host/proc"]["readOnly"]
    assert "/dev/kfd" not in mounts and "/dev/dri" not in mounts
    # uid 0 (the image's user is 65532; the pod-resources socket is root-owned 0660), no capabilities
    sc = c["securityContext"]
    assert sc["runAsUser"] == 0 and sc["capabilities"] == {"drop": ["ALL"]} and not sc["allowPrivilegeEscalation"]
    assert sc["readOnlyRootFilesystem"] and not sc.get("privileged")
    assert any(a.startswith("--token-file=") for a in c["args"])
    assert any(a.startswith("--tls-cert-dir=") for a in c["args"]) and "--insecure" not in c["args"]
    assert c["livenessProbe"]["httpGet"]["scheme"] == "HTTPS"
    # no RBAC at all for the agent: it cannot write a Node or pods/status
    for path, doc in t.items():
        for d in doc if isinstance(doc, list) else [doc]:
            if not isinstance(d, dict):
                continue
            assert "mi355x-node-agent-role" not in json.dumps(d), path
            for r in d.get("rules") or []:
                assert "pods/status" not in r["resources"] or set(r["verbs"]) <= {"get", "list", "watch"}, path
                if "nodes" in r["resources"]:
                    assert set(r["verbs"]) <= {"get", "list", "watch"}, path
    # the production agent module imports nothing from the kubelet stand-in or a k8s client
    import odh_kubeflow_amd.cmd.node_agent as na
    import odh_kubeflow_amd.nodeagent.server as srv
    for mod in (na, srv):
        import ast

        tree = ast.parse(open(mod.__file__).read())
        imported = [n.module or "" for n in ast.walk(tree) if isinstance(n, ast.ImportFrom)]
        imported += [a.name for n in ast.walk(tree) if isinstance(n, ast.Import) for a in n.names]
        for name in imported:
            assert not any(x in name for x in ("kubelet", "runtime", "apiserver")), (mod.__name__, name)


def _get_auth(url, token=None):
    req = urllib.request.Request(url, headers={"Authorization": f"Bearer {token}"} if token else {})
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


def test_agent_token_required_and_rotated(run, sysfs, tmp_path):
    """With --token-file, /gpu/* and /metrics need the bearer token (401 otherwise), /healthz
    stays open; a rotated file takes effect without a restart; a missing file fails closed."""
    from odh_kubeflow_amd.nodeagent.auth import TokenFile

    root, proc, minors, tel = sysfs
    cp = CheckpointWriter(str(tmp_path / "dp" / "cp"))
    cp.allocate(UID_A, "nb", [fake_bdf(1)])
    set_fake_counter(root, minors[1], busy=40)
    tok = tmp_path / "token"
    tok.write_text("s3cret\n")

    async def go():
        agent = await NodeTelemetryAgent(tel, Attributor(tel, checkpoint_path=cp.path, ttl_s=0.0), host="127.0.0.1",
                                         port=0, token=TokenFile(str(tok), recheck_s=0.0)).start()
        try:
            base = f"http://127.0.0.1:{agent.port}"
            act = f"{base}/gpu/activity?pod_uid={UID_A}&window=0.05"
            assert (await asyncio.to_thread(_get_auth, f"{base}/healthz"))[0] == 200
            for path in (act, f"{base}/gpu/pods", f"{base}/gpu/devices", f"{base}/metrics"):
                assert (await asyncio.to_thread(_get_auth, path))[0] == 401
                assert (await asyncio.to_thread(_get_auth, path, "wrong"))[0] == 401
                assert (await asyncio.to_thread(_get_auth, path, "s3cret"))[0] == 200
            st, body = await asyncio.to_thread(_get_auth, act, "s3cret")
            assert json.loads(body)["devices"] == [fake_bdf(1)]
            # rotation (the kubelet swaps the Secret volume's files in place)
            tok.write_text("n3w-token")
            os.utime(tok, ns=(time.time_ns() + 10**9, time.time_ns() + 10**9))
            assert (await asyncio.to_thread(_get_auth, act, "s3cret"))[0] == 401
            assert (await asyncio.to_thread(_get_auth, act, "n3w-token"))[0] == 200
            # missing / empty token file: every data request refused
            tok.unlink()
            assert (await asyncio.to_thread(_get_auth, act, "n3w-token"))[0] == 401
            tok.write_text("")
            assert (await asyncio.to_thread(_get_auth, act, ""))[0] == 401
            assert agent.refused >= 10
            # a bad window is a 400, not a crash
            tok.write_text("t")
            assert (await asyncio.to_thread(_get_auth, f"{base}/gpu/activity?pod_uid={UID_A}&window=nan", "t"))[0] == 400
        finally:
            await agent.stop()
    run(go())


def _node_identity(ca_dir, node, host_ip="127.0.0.1"):
    """A node agent's own key and certificate, as the signer issues them (nodeagent/identity.py)."""
    from odh_kubeflow_amd.nodeagent.identity import LEAF_VALIDITY_S, new_key_and_csr, sign_leaf

    d = os.path.join(ca_dir, node)
    os.makedirs(d, exist_ok=True)
    key, csr = new_key_and_csr(node, host_ip)
    with open(os.path.join(ca_dir, "ca.crt")) as f, open(os.path.join(ca_dir, "ca.key")) as g:
        crt = sign_leaf(csr, f.read(), g.read(), node, host_ip, LEAF_VALIDITY_S)
    for name, pem in (("tls.key", key), ("tls.crt", crt)):
        with open(os.path.join(d, name), "w") as f:
            f.write(pem)
    return d


def _ca(path):
    from odh_kubeflow_amd.webhook.certs import generate_ca

    os.makedirs(path, exist_ok=True)
    generate_ca(str(path))
    return str(path)


def test_culler_sends_agent_token(run, sysfs, tmp_path):
    """The culler's node-agent client reads CULLING_GPU_AGENT_TOKEN_FILE: with the right token it
    gets GPU data; with none it gets no data (None: never idleness).  Over HTTPS, as deployed."""
    from odh_kubeflow_amd.controllers import culling as c
    from odh_kubeflow_amd.nodeagent.auth import TokenFile

    ca_dir = _ca(tmp_path / "ca")
    ca = os.path.join(ca_dir, "ca.crt")
    root, proc, minors, tel = sysfs
    cp = CheckpointWriter(str(tmp_path / "dp" / "cp"))
    cp.allocate(UID_A, "nb", [fake_bdf(2)])
    set_fake_counter(root, minors[2], busy=70)
    tok = tmp_path / "token"
    tok.write_text("abc")
    pod = {"metadata": {"name": "nb-0", "namespace": "u", "uid": UID_A}, "spec": {"nodeName": "gpu-a"},
           "status": {"hostIP": "127.0.0.1"}}

    async def go():
        agent = await NodeTelemetryAgent(tel, Attributor(tel, checkpoint_path=cp.path, ttl_s=0.0), host="127.0.0.1",
                                         port=0, token=TokenFile(str(tok)),
                                         tls_cert_dir=_node_identity(ca_dir, "gpu-a")).start()
        good = c.NodeAgentActivity(port=agent.port, token_file=str(tok), ca_file=ca)
        none = c.NodeAgentActivity(port=agent.port, ca_file=ca)
        try:
            await asyncio.sleep(0.1)
            got = await good.busy(pod, 0.05)
            assert got is not None and got["busy_mean"] == 70
            assert await none.busy(pod, 0.05) is None
            cfg = c.CullerConfig.from_env({"CULLING_GPU_AGENT_TOKEN_FILE": str(tok)})
            assert cfg.gpu_agent_token_file == str(tok)
        finally:
            await good.close()
            await none.close()
            await agent.stop()
    run(go())


def test_agent_serves_https_only_and_the_culler_verifies_it(run, sysfs, tmp_path):
    """the agent's answers decide culls, and its token must not cross the
    node network in cleartext.  The agent serves HTTPS with its node's own certificate; the
    culler asks only over HTTPS, verifying the certificate against the agents' CA and the name
    of the pod's node — a cleartext client, another CA's certificate, and **node B's certificate
    answering for a pod on node A** all get nothing (no GPU data: never idleness, never a cull);
    a renewed certificate is picked up without a restart."""
    import ssl as _ssl

    from odh_kubeflow_amd.controllers import culling as c
    from odh_kubeflow_amd.nodeagent.identity import IDENTITY_DOMAIN, LEAF_VALIDITY_S, new_key_and_csr, sign_leaf

    root, proc, minors, tel = sysfs
    cp = CheckpointWriter(str(tmp_path / "dp" / "cp"))
    cp.allocate(UID_A, "nb", [fake_bdf(3)])
    set_fake_counter(root, minors[3], busy=55)
    ca_dir = _ca(tmp_path / "ca")
    ca = os.path.join(ca_dir, "ca.crt")
    other_ca = os.path.join(_ca(tmp_path / "other"), "ca.crt")
    a_dir = _node_identity(ca_dir, "gpu-a")
    b_dir = _node_identity(ca_dir, "gpu-b")
    on_a = {"metadata": {"name": "nb-0", "namespace": "u", "uid": UID_A}, "spec": {"nodeName": "gpu-a"},
            "status": {"hostIP": "127.0.0.1"}}
    on_b = {**on_a, "spec": {"nodeName": "gpu-b"}}
    unscheduled = {**on_a, "spec": {}}

    async def go():
        attr = Attributor(tel, checkpoint_path=cp.path, ttl_s=0.0)
        agent = await NodeTelemetryAgent(tel, attr, host="127.0.0.1", port=0, tls_cert_dir=a_dir,
                                         cert_reload_s=0.05).start()
        # node B's agent (its own, valid certificate) answering at node A's address
        impostor = await NodeTelemetryAgent(tel, attr, host="127.0.0.1", port=0, tls_cert_dir=b_dir).start()
        ok = c.NodeAgentActivity(port=agent.port, ca_file=ca)
        cleartext = c.NodeAgentActivity(port=agent.port)  # no CA, not --insecure: refuses to ask
        insecure = c.NodeAgentActivity(port=agent.port, insecure=True)  # plain HTTP to an HTTPS agent
        wrong_ca = c.NodeAgentActivity(port=agent.port, ca_file=other_ca)
        b_for_a = c.NodeAgentActivity(port=impostor.port, ca_file=ca)
        clients = (ok, cleartext, insecure, wrong_ca, b_for_a)
        try:
            await asyncio.sleep(0.1)
            got = await ok.busy(on_a, 0.05)
            assert got is not None and got["busy_mean"] == 55
            assert await cleartext.busy(on_a, 0.05) is None and cleartext.refused_cleartext == 1
            assert await insecure.busy(on_a, 0.05) is None
            assert await wrong_ca.busy(on_a, 0.05) is None
            # the pod is on node A; B's agent holds a valid certificate of the same CA, for B
            assert await b_for_a.busy(on_a, 0.05) is None
            assert (await b_for_a.busy(on_b, 0.05) or {}).get("busy_mean") == 55  # ... good for B's pods
            assert await ok.busy(on_b, 0.05) is None  # A's agent cannot answer for a pod on B either
            assert await ok.busy(unscheduled, 0.05) is None and ok.no_node == 1
            # renewal: a new key and certificate for the same node replace the files; reloaded live
            before = agent.tls.reloads
            key, csr = new_key_and_csr("gpu-a", "127.0.0.1")
            with open(ca) as f, open(os.path.join(ca_dir, "ca.key")) as g:
                crt = sign_leaf(csr, f.read(), g.read(), "gpu-a", "127.0.0.1", LEAF_VALIDITY_S)
            for name, pem in (("tls.key", key), ("tls.crt", crt)):
                with open(os.path.join(a_dir, name), "w") as f:
                    f.write(pem)
            for _ in range(100):
                if agent.tls.reloads > before:
                    break
                await asyncio.sleep(0.05)
            assert agent.tls.reloads > before
            pem = await asyncio.to_thread(_ssl.get_server_certificate, ("127.0.0.1", agent.port))
            assert pem.split() == crt.split()  # the renewed leaf is served
            got = await ok.busy(on_a, 0.05)
            assert got is not None and got["busy_mean"] == 55
            cfg = c.CullerConfig.from_env({"CULLING_GPU_AGENT_CA_FILE": ca})
            assert cfg.gpu_agent_ca_file == ca and cfg.gpu_agent_identity_domain == IDENTITY_DOMAIN
            assert not cfg.gpu_agent_insecure
        finally:
            for x in clients:
                await x.close()
            await agent.stop()
            await impostor.stop()
    run(go())
