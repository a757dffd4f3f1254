"""``runtime/http1.py``: the watch stream's chunked-body line reader, fed byte splits that
cut chunk headers, chunk bodies and lines anywhere (the apiserver writes one chunk per
batch of watch events; TCP delivers them in arbitrary pieces)."""

from __future__ import annotations

import asyncio
import random

import pytest

from odh_kubeflow_amd.runtime.http1 import _Conn, _Stream


class _W:
    def close(self):
        pass


def _chunked(chunks):
    out = b""
    for c in chunks:
        out += b"%x\r\n" % len(c) + c + b"\r\n"
    return out + b"0\r\n\r\n"


async def _read(pieces, chunked=True):
    r = asyncio.StreamReader()
    s = _Stream(_Conn(r, _W()), {"transfer-encoding": "chunked"} if chunked else {})

    async def feed():
        for p in pieces:
            r.feed_data(p)
            await asyncio.sleep(0)
        r.feed_eof()

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
    assert asyncio.run(_read([b"a\nb\n"], chunked=False)) == [b"a\n", b"b\n"]
