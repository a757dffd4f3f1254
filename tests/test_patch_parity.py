"""Property tests: the C++ apiserver's patch engines against ``utils/jsonpatch.py``.

Both test apiservers apply the JSON (RFC 6902), merge (RFC 7386) and strategic-merge
patches the controllers, the webhook and ``kubectl`` send; a divergence would make the same
scenario pass over one transport and fail over the other.  Hypothesis generates JSON
documents and patches (mostly against paths that exist, some that do not), the native
engines run through the server's ``/debug/patch`` endpoint, and the two must agree: same
result, or both refuse (HTTP 422 / ``PatchError``)."""

import http.client
import json
import os
import subprocess
import tempfile

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from odh_kubeflow_amd.testing.apiserver import native
from odh_kubeflow_amd.utils.jsonpatch import (PatchError, apply_merge_patch, apply_patch,
                                              apply_strategic_merge_patch)

pytestmark = pytest.mark.skipif(not native.available(), reason="native apiserver not built")

KEYS = st.sampled_from(["a", "b", "c", "name", "env", "containers", "x/y", "t~n", "0"])
SCALARS = st.one_of(st.none(), st.booleans(), st.integers(-5, 5), st.sampled_from(["", "v", "w", "1"]),
                    st.sampled_from([0.5, 1.0, -2.25]))
JSON = st.recursive(SCALARS, lambda kids: st.one_of(st.lists(kids, max_size=4),
                                                    st.dictionaries(KEYS, kids, max_size=4)), max_leaves=12)


@pytest.fixture(scope="module")
def server():
    fd, cfg = tempfile.mkstemp(suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(native.scheme_config((), False, None, 64), f)
    proc = subprocess.Popen([native.BINARY, "--config", cfg, "--host", "127.0.0.1", "--port", "0"],
                            stdout=subprocess.PIPE)
    line = proc.stdout.readline()
    assert line.startswith(b"LISTENING"), line
    conn = http.client.HTTPConnection("127.0.0.1", int(line.split()[1]), timeout=10)
    yield conn
    conn.close()
    proc.terminate()
    proc.wait(10)
    os.unlink(cfg)


def native_apply(conn, kind, doc, patch):
    conn.request("POST", "/debug/patch", json.dumps({"type": kind, "doc": doc, "patch": patch}),
                 {"Content-Type": "application/json"})
    r = conn.getresponse()
    body = json.loads(r.read())
    return ("error", None) if r.status == 422 else ("ok", body["result"])


def python_apply(kind, doc, patch):
    fn = {"json": apply_patch, "merge": apply_merge_patch, "strategic": apply_strategic_merge_patch}[kind]
    try:
        return "ok", fn(doc, patch)
    except PatchError:
        return "error", None


def norm(x):
    """JSON value identity as both engines see it (the wire form)."""
    return json.loads(json.dumps(x))


def _paths(doc, prefix=""):
    out = [prefix]
    if isinstance(doc, dict):
        for k, v in doc.items():
            out += _paths(v, prefix + "/" + k.replace("~", "~0").replace("/", "~1"))
    elif isinstance(doc, list):
        for i, v in enumerate(doc):
            out += _paths(v, f"{prefix}/{i}")
        out.append(prefix + "/-")
    return out


@st.composite
def doc_and_ops(draw):
    doc = draw(st.dictionaries(KEYS, JSON, max_size=4))
    paths = _paths(doc)
    path = st.one_of(st.sampled_from(paths), st.sampled_from(["/zz", "/a/0", "/0", "/a/-1", "/a/01", "/a/ 1",
                                                               "/a/1_0", "/a/+1", "x"]))
    ops = []
    for _ in range(draw(st.integers(1, 4))):
        op = draw(st.sampled_from(["add", "remove", "replace", "move", "copy", "test"]))
        o = {"op": op, "path": draw(path)}
        if op in ("add", "replace", "test"):
            o["value"] = draw(JSON)
        if op in ("move", "copy"):
            o["from"] = draw(path)
        ops.append(o)
    return doc, ops


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(doc_and_ops())
def test_json_patch_parity(server, case):
    doc, ops = case
    py, nat = python_apply("json", doc, ops), native_apply(server, "json", doc, ops)
    assert py[0] == nat[0], (doc, ops, py, nat)
    if py[0] == "ok":
        assert norm(py[1]) == nat[1], (doc, ops, py, nat)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.dictionaries(KEYS, JSON, max_size=4), st.dictionaries(KEYS, JSON, max_size=4),
       st.sampled_from(["merge", "strategic"]))
def test_merge_and_strategic_patch_parity(server, doc, patch, kind):
    py, nat = python_apply(kind, doc, patch), native_apply(server, kind, doc, patch)
    assert py[0] == nat[0] == "ok"
    assert norm(py[1]) == nat[1], (kind, doc, patch, py, nat)


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.lists(st.fixed_dictionaries({"name": st.sampled_from(["a", "b", "c"]), "v": SCALARS}), max_size=4),
       st.lists(st.fixed_dictionaries({"name": st.sampled_from(["a", "b", "d"]), "v": SCALARS},
                                      optional={"$patch": st.just("delete")}), max_size=4))
def test_strategic_merge_keyed_lists_parity(server, cur, patch):
    """Keyed lists (containers / env by ``name``): merge by key, ``$patch: delete`` removes."""
    doc, p = {"spec": {"containers": cur}}, {"spec": {"containers": patch}}
    py, nat = python_apply("strategic", doc, p), native_apply(server, "strategic", doc, p)
    assert py[0] == nat[0] == "ok"
    assert norm(py[1]) == nat[1], (doc, p, py, nat)


def _raw(port, data: bytes) -> bytes:
    import socket

    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    try:
        s.sendall(data)
        out = b""
        while True:
            try:
                chunk = s.recv(65536)
            except socket.timeout:
                break
            if not chunk:
                break
            out += chunk
            if b"\r\n\r\n" in out and (b"Content-Length: " in out or b"400" in out[:20]):
                break
        return out
    finally:
        s.close()


def test_native_server_survives_malformed_requests(server):
    """Malformed framing or parameters end that request (or connection), never the server:
    bad Content-Length, bad chunk size, bad %-escapes, a non-numeric watch resourceVersion,
    a JSON patch with a non-numeric list index over the real PATCH path."""
    port = server.port
    _raw(port, b"POST /debug/patch HTTP/1.1\r\nHost: x\r\nContent-Length: abc\r\n\r\n{}")
    _raw(port, b"POST /debug/patch HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n{}\r\n0\r\n\r\n")
    out = _raw(port, b"GET /api/v1/namespaces/%zz/pods HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 ")
    out = _raw(port, b"GET /api/v1/pods?watch=true&resourceVersion=abc HTTP/1.1\r\nHost: x\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 400"), out[:80]
    body = json.dumps({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c", "namespace": "default"},
                       "data": {"k": "v"}})
    server.request("POST", "/api/v1/namespaces/default/configmaps", body, {"Content-Type": "application/json"})
    assert server.getresponse().read() and True
    server.request("PATCH", "/api/v1/namespaces/default/configmaps/c",
                   json.dumps([{"op": "add", "path": "/metadata/finalizers", "value": []},
                               {"op": "add", "path": "/metadata/finalizers/x", "value": "f"}]),
                   {"Content-Type": "application/json-patch+json"})
    r = server.getresponse()
    r.read()
    assert r.status == 422, r.status
    server.request("GET", "/healthz")
    r = server.getresponse()
    assert r.status == 200 and r.read() == b"ok"


# ------------------------------------------------------------------ selectors

LKEYS = ["app", "tier", "gpu", "example.com/role"]
LVALS = ["a", "b", "c", ""]


@pytest.fixture(scope="module")
def labelled_pool(server):
    """30 ConfigMaps with pseudo-random labels in the native server; the same list for the
    Python matcher."""
    import random

    rnd = random.Random(7)
    pool = []
    for i in range(30):
        labels = {k: rnd.choice(LVALS) for k in LKEYS if rnd.random() < 0.6}
        cm = {"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": f"sel-{i}", "namespace": "sel", "labels": labels}, "data": {"i": str(i % 3)}}
        server.request("POST", "/api/v1/namespaces/sel/configmaps", json.dumps(cm), {"Content-Type": "application/json"})
        r = server.getresponse()
        r.read()
        assert r.status == 201, r.status
        pool.append(cm)
    return pool


@st.composite
def label_selector(draw):
    reqs = []
    for _ in range(draw(st.integers(1, 3))):
        k = draw(st.sampled_from(LKEYS))
        op = draw(st.sampled_from(["=", "==", "!=", "in", "notin", "exists", "!"]))
        if op in ("in", "notin"):
            vals = draw(st.lists(st.sampled_from(["a", "b", "c"]), min_size=1, max_size=3))
            reqs.append(f"{k} {op} ({','.join(vals)})")
        elif op == "exists":
            reqs.append(k)
        elif op == "!":
            reqs.append(f"!{k}")
        else:
            reqs.append(f"{k}{op}{draw(st.sampled_from(['a', 'b', 'c']))}")
    return ",".join(reqs)


def _native_names(server, query):
    from urllib.parse import quote

    server.request("GET", f"/api/v1/namespaces/sel/configmaps?{query[0]}={quote(query[1])}")
    r = server.getresponse()
    body = json.loads(r.read())
    assert r.status == 200, body
    return sorted(o["metadata"]["name"] for o in body["items"])


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(label_selector())
def test_label_selector_parity(server, labelled_pool, sel):
    from odh_kubeflow_amd.utils.selectors import match_labels, parse_label_selector

    reqs = parse_label_selector(sel)
    want = sorted(cm["metadata"]["name"] for cm in labelled_pool if match_labels(reqs, cm["metadata"]["labels"]))
    assert _native_names(server, ("labelSelector", sel)) == want, sel


@settings(max_examples=100, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.lists(st.tuples(st.sampled_from(["metadata.name", "data.i", "metadata.namespace"]),
                          st.sampled_from(["=", "==", "!="]),
                          st.sampled_from(["sel-1", "sel-2", "0", "1", "sel", "x"])), min_size=1, max_size=2))
def test_field_selector_parity(server, labelled_pool, reqs):
    from odh_kubeflow_amd.utils.selectors import field_matcher, parse_field_selector

    sel = ",".join(f"{k}{op}{v}" for k, op, v in reqs)
    match = field_matcher(parse_field_selector(sel))
    want = sorted(cm["metadata"]["name"] for cm in labelled_pool if match(cm))
    assert _native_names(server, ("fieldSelector", sel)) == want, sel
