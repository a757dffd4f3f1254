"""``runtime/http1.py``: the watch stream's chunked-body line reader, fed byte splits that
cut chunk headers, chunk bodies and lines anywhere (the apiserver writes one chunk per
batch of watch events; TCP delivers them in arbitrary pieces)."""

from __future__ import annotations

import asyncio
import random

import pytest

from odh_kubeflow_amd.runtime.http1 import _Conn, _Stream, _dechunk


class _T:
    def close(self):
        pass

    def write(self, _data):
        pass


def _chunked(chunks):
    out = b""
    for c in chunks:
        out += b"%x\r\n" % len(c) + c + b"\r\n"
    return out + b"0\r\n\r\n"


async def _read(pieces, chunked=True):
    conn = _Conn()
    conn.connection_made(_T())
    head = b"HTTP/1.1 200 OK\r\n" + (b"Transfer-Encoding: chunked\r\n" if chunked else b"") + b"\r\n"
    opened = asyncio.ensure_future(conn.open_stream(b"GET / HTTP/1.1\r\n\r\n"))
    await asyncio.sleep(0)
    conn.data_received(head)
    assert (await opened)[0] == 200
    s = _Stream(conn)

    async def feed():
        for p in pieces:
            conn.data_received(p)
            await asyncio.sleep(0)
        conn.connection_lost(None)

    t = asyncio.ensure_future(feed())
    got = [line async for line in s.lines()]
    await t
    return got


@pytest.mark.parametrize("seed", range(20))
def test_chunked_lines_survive_any_split(seed):
    rnd = random.Random(seed)
    lines = [b'{"type":"ADDED","object":{"n":%d,"pad":"%s"}}' % (i, b"x" * rnd.randrange(0, 300)) for i in range(40)]
    text = b"".join(x + b"\n" for x in lines)
    chunks, i = [], 0
    while i < len(text):  # chunk boundaries anywhere, lines split across chunks
        n = rnd.randrange(1, 700)
        chunks.append(text[i:i + n])
        i += n
    wire = _chunked(chunks)
    pieces, j = [], 0
    while j < len(wire):  # and the wire split anywhere, chunk headers included
        n = rnd.randrange(1, 97)
        pieces.append(wire[j:j + n])
        j += n
    assert asyncio.run(_read(pieces)) == lines


def test_chunk_extension_and_early_eof():
    wire = b"5;ext=1\r\nab\ncd\r\n3\r\nef\n\r\n"  # no terminal chunk: the connection just ends
    assert asyncio.run(_read([wire])) == [b"ab", b"cdef"]
    assert asyncio.run(_read([b"a\nb\n"], chunked=False)) == [b"a", b"b"]


async def _roundtrips(responses, seed):
    """Responses back to back on one keep-alive connection, the wire split anywhere."""
    rnd = random.Random(seed)
    conn = _Conn()
    conn.connection_made(_T())
    out = []
    for wire in responses:
        fut = asyncio.ensure_future(conn.roundtrip(b"GET / HTTP/1.1\r\n\r\n"))
        await asyncio.sleep(0)
        j = 0
        while j < len(wire):
            n = rnd.randrange(1, 23)
            conn.data_received(wire[j:j + n])
            j += n
        out.append(await fut)
    return out


@pytest.mark.parametrize("seed", range(10))
def test_keepalive_responses_parse_across_any_split(seed):
    body = b'{"kind":"ConfigMap","data":{"k":"' + b"v" * 300 + b'"}}'
    cl = b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body
    ch = b"HTTP/1.1 201 Created\r\nTransfer-Encoding: chunked\r\n\r\n" + _chunked([body[:100], body[100:]])
    empty = b"HTTP/1.1 404 Not Found\r\nContent-Length: 0\r\nConnection: close\r\n\r\n"
    got = asyncio.run(_roundtrips([cl, ch, cl, empty], seed))
    assert got == [(200, body, False), (201, body, False), (200, body, False), (404, b"", True)]


@pytest.mark.parametrize("seed", range(4))
def test_bodyless_responses_complete_without_waiting_for_close(seed):
    """1xx-less bodyless answers — 204 and 304, or a keep-alive response with neither
    Content-Length nor chunked encoding — complete at their head, and the next response on the
    connection parses; only ``Connection: close`` delimits a body by end of stream."""
    body = b'{"a":1}'
    ok = b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body
    no_content = b"HTTP/1.1 204 No Content\r\n\r\n"
    not_modified = b"HTTP/1.1 304 Not Modified\r\nContent-Type: application/json\r\n\r\n"
    bare = b"HTTP/1.1 200 OK\r\nContent-Type: text/plain\r\n\r\n"
    got = asyncio.run(asyncio.wait_for(_roundtrips([no_content, ok, not_modified, bare, ok], seed), 5))
    assert got == [(204, b"", False), (200, body, False), (304, b"", False), (200, b"", False), (200, body, False)]

    async def until_close():
        conn = _Conn()
        conn.connection_made(_T())
        fut = asyncio.ensure_future(conn.roundtrip(b"GET / HTTP/1.1\r\n\r\n"))
        await asyncio.sleep(0)
        conn.data_received(b"HTTP/1.1 200 OK\r\nConnection: close\r\n\r\nall of ")
        conn.data_received(b"it")
        conn.connection_lost(None)
        return await fut
    assert asyncio.run(until_close()) == (200, b"all of it", True)

    async def head():
        conn = _Conn()
        conn.connection_made(_T())
        fut = asyncio.ensure_future(conn.roundtrip(b"HEAD / HTTP/1.1\r\n\r\n"))
        await asyncio.sleep(0)
        conn.data_received(b"HTTP/1.1 200 OK\r\nContent-Length: 42\r\n\r\n")
        return await asyncio.wait_for(fut, 5)
    assert asyncio.run(head()) == (200, b"", False)


def test_dechunk_waits_for_the_final_crlf():
    raw, body = bytearray(b"3\r\nabc\r\n0\r\n"), bytearray()
    assert not _dechunk(raw, body) and body == b"abc"
    raw += b"\r\nHTTP/1.1"
    assert _dechunk(raw, body) and raw == b"HTTP/1.1"


def test_connection_lost_mid_response_fails_the_request():
    async def go():
        conn = _Conn()
        conn.connection_made(_T())
        fut = asyncio.ensure_future(conn.roundtrip(b"GET / HTTP/1.1\r\n\r\n"))
        await asyncio.sleep(0)
        conn.data_received(b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\nabc")
        conn.connection_lost(None)
        with pytest.raises(ConnectionResetError):
            await fut
        with pytest.raises(ConnectionResetError):
            await conn.roundtrip(b"GET / HTTP/1.1\r\n\r\n")  # closed: the pool skips it
    asyncio.run(go())


def test_server_closes_a_connection_after_max_requests():
    """``max_requests_per_conn``: the webhook replicas sharing a port (SO_REUSEPORT) make the
    apiserver re-connect now and then, so its pooled connections spread over them again."""
    from odh_kubeflow_amd.runtime.http1 import Http1Server

    async def handler(method, path, headers, body):
        return 200, "text/plain", b"ok"

    async def go():
        srv = await Http1Server(handler, max_requests_per_conn=3).start()
        r, w = await asyncio.open_connection("127.0.0.1", srv.port)
        answers = []
        for _ in range(3):
            w.write(b"POST /x HTTP/1.1\r\nContent-Length: 0\r\n\r\n")
            head = await r.readuntil(b"\r\n\r\n")
            answers.append(head)
            await r.readexactly(2)
        assert b"Connection: close" not in answers[0] and b"Connection: close" not in answers[1]
        assert b"Connection: close" in answers[2]
        assert await r.read() == b""  # the server hung up
        w.close()
        await srv.stop()
    asyncio.run(go())


def test_pool_keeps_spare_connections_open_ahead_of_demand():
    """``spare``: the REST client's pool opens connections before a request needs one, so a
    burst does not wait for new connections to be accepted (profiles/r6_g38: 80-170 ms in the
    apiserver's listen queue on the GPU boxes).  Concurrent requests beyond the pool's idle
    connections still open their own."""
    from odh_kubeflow_amd.runtime.http1 import Http1Pool, Http1Server

    async def handler(method, path, headers, body):
        await asyncio.sleep(0.01)
        return 200, "text/plain", b"ok"

    async def go():
        srv = await Http1Server(handler).start()
        pool = Http1Pool(f"http://127.0.0.1:{srv.port}", spare=2)
        assert await pool.request("GET", "/a") == (200, b"ok")
        for _ in range(100):
            if len(pool._idle) >= 3:
                break
            await asyncio.sleep(0.01)
        assert len(pool._idle) == 3 and pool.opened == 3  # the request's own + 2 spares
        got = await asyncio.gather(*(pool.request("GET", f"/b{i}") for i in range(5)))
        assert got == [(200, b"ok")] * 5
        await asyncio.sleep(0.1)
        assert len(pool._idle) >= 5 and pool.opened <= 5 + 2 + 2
        await pool.close()
        assert pool._idle == [] and pool.spare == 0
        await srv.stop()
    asyncio.run(asyncio.wait_for(go(), 20))
