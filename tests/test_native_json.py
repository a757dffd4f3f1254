"""The native JSON decoder (``native/objcore.cpp`` ``loads_shared`` / ``loads_event``): what
``json.loads`` returns, for any document; decoded against a previous version, the unchanged
subtrees are that version's objects (the informer's watch path, ``runtime/rest.py``)."""

from __future__ import annotations

import json
import random

import pytest

oc = pytest.importorskip("odh_kubeflow_amd.native._objcore")

ALPHABET = ["a", "Z", "0", " ", '"', "\\", "/", "\n", "\t", "é", "中", "\U0001F600", "\x01", " "]


def _rand(rnd: random.Random, depth: int = 0):
    r = rnd.random()
    if depth > 4 or r < 0.35:
        k = rnd.randrange(8)
        if k == 0:
            return rnd.randrange(-10**6, 10**6)
        if k == 1:
            return rnd.choice([0, -0, 2**63 - 1, -2**63, 2**64 + 7, -(10**30)])
        if k == 2:
            return rnd.choice([0.5, -1e-7, 1.5e300, 3.0, -2.25, 1e22])
        if k == 3:
            return rnd.choice([True, False, None])
        return "".join(rnd.choice(ALPHABET) for _ in range(rnd.randrange(0, 12)))
    if r < 0.65:
        return [_rand(rnd, depth + 1) for _ in range(rnd.randrange(0, 5))]
    return {"".join(rnd.choice(ALPHABET[:6]) for _ in range(rnd.randrange(1, 6))): _rand(rnd, depth + 1)
            for _ in range(rnd.randrange(0, 6))}


def _mutate(rnd: random.Random, o):
    """A copy of ``o`` with a few leaves changed, keys added or dropped."""
    if isinstance(o, dict):
        out = {k: (_mutate(rnd, v) if rnd.random() < 0.3 else v) for k, v in o.items()}
        if rnd.random() < 0.2:
            out["new" + str(rnd.randrange(3))] = _rand(rnd, 3)
        if out and rnd.random() < 0.2:
            out.pop(rnd.choice(list(out)))
        return out
    if isinstance(o, list):
        out = [(_mutate(rnd, v) if rnd.random() < 0.3 else v) for v in o]
        if rnd.random() < 0.2:
            out.append(_rand(rnd, 3))
        return out
    return _rand(rnd, 5) if rnd.random() < 0.5 else o


@pytest.mark.parametrize("seed", range(40))
def test_decodes_as_json_loads(seed):
    rnd = random.Random(seed)
    doc = _rand(rnd)
    for text in (json.dumps(doc), json.dumps(doc, ensure_ascii=False), json.dumps(doc, indent=2)):
        for data in (text, text.encode()):
            got = oc.loads_shared(data)
            want = json.loads(text)
            assert got == want and json.dumps(got) == json.dumps(want)


def _identities(new, old, path=""):
    """Every container of ``new`` equal to the corresponding one of ``old`` is that object."""
    if isinstance(new, dict) and isinstance(old, dict):
        if path and new == old:
            assert new is old, path
        for k, v in new.items():
            if k in old:
                _identities(v, old[k], f"{path}.{k}")
    elif isinstance(new, list) and isinstance(old, list):
        if path and new == old:
            assert new is old, path
        for i, (a, b) in enumerate(zip(new, old)):
            _identities(a, b, f"{path}[{i}]")


@pytest.mark.parametrize("seed", range(40))
def test_shares_the_unchanged_subtrees(seed):
    rnd = random.Random(1000 + seed)
    old = {"metadata": {"name": "x", "namespace": "n"}, "spec": _rand(rnd), "status": _rand(rnd)}
    new = _mutate(rnd, old)
    frozen = json.dumps(old, sort_keys=True)
    got = oc.loads_shared(json.dumps(new), old)
    assert got == json.loads(json.dumps(new))
    assert got is not old  # the top level is always a new object
    _identities(got, old)
    assert json.dumps(old, sort_keys=True) == frozen  # the old version is never modified


def test_event_lookup_and_fallbacks():
    old = {"metadata": {"name": "nb", "namespace": "u", "resourceVersion": "1"}, "spec": {"a": [1, {"b": "c"}]}}
    line = json.dumps({"type": "MODIFIED", "object": {"metadata": {"namespace": "u", "resourceVersion": "2",
                                                                    "name": "nb"}, "spec": {"a": [1, {"b": "c"}]}}})
    seen = []
    et, obj = oc.loads_event(line.encode(), lambda ns, name: seen.append((ns, name)) or old)
    assert et == "MODIFIED" and seen == [("u", "nb")] and obj["spec"] is old["spec"]
    # a cluster-scoped object: namespace ""; a lookup that has nothing: plain decode
    et, obj = oc.loads_event(b'{"object":{"metadata":{"name":"c"}},"type":"ADDED"}', lambda ns, name: None)
    assert et == "ADDED" and obj == {"metadata": {"name": "c"}}
    assert oc.loads_event(b'{"type":"ERROR","object":{"kind":"Status","code":410}}', None) == (
        "ERROR", {"kind": "Status", "code": 410})
    for bad in (b"{", b'{"type":}', b"[1,]", b"nul", b'"abc', b'{"a":1}x', b"NaN", b'{"a":1,}'):
        with pytest.raises(ValueError):
            oc.loads_shared(bad)
    with pytest.raises(ZeroDivisionError):  # a failing lookup surfaces, nothing is half-built
        oc.loads_event(line.encode(), lambda ns, name: 1 / 0)


@pytest.mark.parametrize("new_text, old", [
    # the old string verbatim, but the new JSON string ends earlier: an escaped quote inside
    ('{"s": "a\\"b", "t": 1}', {"s": 'a"b', "t": 1}),
    ('{"s": "a\\\\", "t": "x"}', {"s": "a\\", "t": "x"}),
    ('{"s": "ab", "t": "x"}', {"s": 'ab"', "t": "x"}),  # old longer than the new string
    ('{"s": "a\\u0062", "t": 2}', {"s": "ab", "t": 2}),  # an escape spelling the same text
    ('{"s": "\\/x"}', {"s": "/x"}),
    ('{"b": 1, "a": 2}', {"a": 2, "b": 1}),  # the keys in another order
    ('{"a": 1, "c": 3, "b": 2}', {"a": 1, "b": 2}),  # a key added in the middle
    ('{"a": 1}', {"a": 1, "b": 2}),  # a key removed
    ('{"a": {"x": "y"}, "b": [1, -0, 123456789012345678, 1234567890123456789012]}',
     {"a": {"x": "y"}, "b": [1, 0, 123456789012345678, 1234567890123456789012]}),
])
def test_fast_paths_against_the_old_version(new_text, old):
    """The decoder's shortcuts against the old version (a string compared verbatim, the keys
    walked in the old dict's order) give json.loads's answer whatever the old version holds."""
    got = oc.loads_shared(new_text, old)
    assert got == json.loads(new_text) and list(got) == list(json.loads(new_text))
    _identities(got, old)


@pytest.mark.parametrize("seed", range(40))
def test_dumps_is_compact_json_dumps(seed):
    """``dumps`` writes what json.dumps(separators=(",", ":"), ensure_ascii=False) writes."""
    rnd = random.Random(5000 + seed)
    doc = {"metadata": {"name": "x"}, "spec": _rand(rnd), "list": [_rand(rnd) for _ in range(3)]}
    assert oc.dumps(doc) == json.dumps(doc, separators=(",", ":"), ensure_ascii=False).encode("utf-8", "surrogatepass")


def test_dumps_declines_what_is_not_a_json_tree():
    from odh_kubeflow_amd.runtime.rest import dumps_json

    for bad in ({1: "int key"}, {"a": object()}, {"a": {1, 2}}):
        with pytest.raises(TypeError):
            oc.dumps(bad)
    assert dumps_json({1: "a"}) == b'{"1":"a"}'  # json.dumps's answer
    assert dumps_json((1, "é")) == '[1,"é"]'.encode()


def test_a_duplicated_key_never_stands_in_for_a_missing_one():
    """decoding against an old object, ``{"x":1,"x":1}`` is not ``{"x":1,"y":2}``
    (json.loads keeps the last duplicate: ``{"x":1}``)."""
    old = {"a": {"x": 1, "y": 2}}
    for text in ('{"a":{"x":1,"x":1}}', '{"a":{"y":2,"y":2}}'):
        got = oc.loads_shared(text.encode(), old)
        assert got == json.loads(text) and got["a"] is not old["a"]
    # out of order but complete: still the old subtree
    got = oc.loads_shared(b'{"a":{"y":2,"x":1}}', old)
    assert got == {"a": {"x": 1, "y": 2}} and got["a"] is old["a"]
    got = oc.loads_shared(b'{"a":{"x":1,"y":2}}', old)
    assert got["a"] is old["a"]
