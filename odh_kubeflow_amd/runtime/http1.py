"""Lean HTTP/1.1 client for the apiserver REST path (asyncio streams, keep-alive pool).

A control-plane process spends most of its CPU time talking to the apiserver; a generic
client (aiohttp) costs ~4× the raw socket round trip per request on this path (measured
0.14 ms vs 0.03 ms for a GET on loopback).  This client does only what the Kubernetes
REST API needs: persistent connections, ``Content-Length`` or ``chunked`` bodies,
optional TLS, and a streaming mode for watches.  Stale pooled connections (closed by the
server while idle) are retried once for requests other than POST.
"""

from __future__ import annotations

import asyncio
import ssl as _ssl
from typing import AsyncIterator, Dict, List, Optional, Tuple
from urllib.parse import urlsplit


class HttpError(Exception):
    pass


class _Conn:
    __slots__ = ("reader", "writer")

    def __init__(self, reader, writer):
        self.reader = reader
        self.writer = writer

    def close(self) -> None:
        try:
            self.writer.close()
        except Exception:
            pass


async def _read_head(reader) -> Tuple[int, Dict[str, str]]:
    raw = await reader.readuntil(b"\r\n\r\n")
    lines = raw.decode("latin-1").split("\r\n")
    parts = lines[0].split(" ", 2)
    if len(parts) < 2 or not parts[0].startswith("HTTP/"):
        raise HttpError(f"bad status line {lines[0]!r}")
    headers = {}
    for line in lines[1:]:
        if ":" in line:
            k, v = line.split(":", 1)
            headers[k.strip().lower()] = v.strip()
    return int(parts[1]), headers


async def _read_chunked(reader) -> bytes:
    out = bytearray()
    while True:
        line = await reader.readuntil(b"\r\n")
        size = int(line.split(b";", 1)[0].strip(), 16)
        if size == 0:
            await reader.readuntil(b"\r\n")
            return bytes(out)
        out += await reader.readexactly(size)
        await reader.readexactly(2)


class Http1Pool:
    def __init__(self, base_url: str, ssl_context: Optional[_ssl.SSLContext] = None,
                 headers: Optional[Dict[str, str]] = None, size: int = 64):
        u = urlsplit(base_url)
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.ssl = ssl_context if u.scheme == "https" else None
        hdr = {"Host": f"{self.host}:{self.port}", "Accept": "application/json"}
        hdr.update(headers or {})
        self._static = "".join(f"{k}: {v}\r\n" for k, v in hdr.items())
        self._idle: List[_Conn] = []
        self.size = size
        self.opened = 0

    async def _connect(self) -> _Conn:
        reader, writer = await asyncio.open_connection(self.host, self.port, ssl=self.ssl,
                                                       limit=1 << 24)
        sock = writer.get_extra_info("socket")
        if sock is not None:
            import socket

            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        self.opened += 1
        return _Conn(reader, writer)

    def _head(self, method: str, target: str, body: Optional[bytes], content_type: Optional[str]) -> bytes:
        h = f"{method} {target} HTTP/1.1\r\n{self._static}"
        if body is not None:
            h += f"Content-Type: {content_type or 'application/json'}\r\nContent-Length: {len(body)}\r\n"
        return (h + "\r\n").encode("latin-1") + (body or b"")

    async def request(self, method: str, target: str, body: Optional[bytes] = None,
                      content_type: Optional[str] = None) -> Tuple[int, bytes]:
        payload = self._head(method, target, body, content_type)
        for attempt in (0, 1):
            reused = bool(self._idle)
            conn = self._idle.pop() if reused else await self._connect()
            try:
                conn.writer.write(payload)
                status, headers = await _read_head(conn.reader)
                if headers.get("transfer-encoding", "").lower() == "chunked":
                    data = await _read_chunked(conn.reader)
                else:
                    n = int(headers.get("content-length", "0"))
                    data = await conn.reader.readexactly(n) if n else b""
            except (asyncio.IncompleteReadError, ConnectionError, OSError) as e:
                conn.close()
                if reused and attempt == 0 and method != "POST":
                    continue
                raise HttpError(f"{method} {target}: {e!r}") from e
            except BaseException:
                conn.close()
                raise
            if headers.get("connection", "").lower() == "close" or len(self._idle) >= self.size:
                conn.close()
            else:
                self._idle.append(conn)
            return status, data
        raise HttpError("unreachable")

    async def stream(self, method: str, target: str) -> Tuple[int, Dict[str, str], "_Stream"]:
        conn = await self._connect()
        conn.writer.write(self._head(method, target, None, None))
        status, headers = await _read_head(conn.reader)
        return status, headers, _Stream(conn, headers)

    async def close(self) -> None:
        for c in self._idle:
            c.close()
        self._idle.clear()


class _Stream:
    """Body of a streaming (watch) response; iterate lines, then close."""

    def __init__(self, conn: _Conn, headers: Dict[str, str]):
        self.conn = conn
        self.chunked = headers.get("transfer-encoding", "").lower() == "chunked"

    async def read_all(self) -> bytes:
        try:
            if self.chunked:
                return await _read_chunked(self.conn.reader)
            return await self.conn.reader.read()
        finally:
            self.close()

    async def lines(self) -> AsyncIterator[bytes]:
        """The body's lines (without their newline).  Chunked bodies are read as whatever has
        arrived — one await per arrival, however many chunks and events it holds — and
        de-chunked here, rather than three stream reads per chunk."""
        r = self.conn.reader
        try:
            if not self.chunked:
                async for line in r:
                    yield line
                return
            raw = bytearray()  # chunked framing not yet parsed
            body = bytearray()  # de-chunked bytes not yet split into lines
            while True:
                data = await r.read(1 << 16)
                if not data:
                    return
                raw += data
                pos, done = 0, False
                while True:
                    crlf = raw.find(b"\r\n", pos)
                    if crlf < 0:
                        break
                    size = int(bytes(raw[pos:crlf]).split(b";", 1)[0].strip(), 16)
                    if size == 0:
                        done = True
                        break
                    end = crlf + 2 + size
                    if len(raw) < end + 2:
                        break
                    body += raw[crlf + 2:end]
                    pos = end + 2
                del raw[:pos]
                start = 0
                while True:
                    nl = body.find(b"\n", start)
                    if nl < 0:
                        break
                    yield bytes(body[start:nl])
                    start = nl + 1
                del body[:start]
                if done:
                    return
        except (asyncio.IncompleteReadError, ConnectionError, OSError):
            return
        finally:
            self.close()

    def close(self) -> None:
        self.conn.close()


# --------------------------------------------------------------------------- server

_REASONS = {200: "OK", 400: "Bad Request", 404: "Not Found", 405: "Method Not Allowed", 413: "Payload Too Large",
            500: "Internal Server Error"}
Handler = "Callable[[str, str, Dict[str, str], bytes], Awaitable[Tuple[int, str, bytes]]]"


class Http1Server:
    """Minimal keep-alive HTTP/1.1 server (optionally TLS) for the admission webhook.

    The apiserver keeps a pooled TLS connection to the webhook and posts one
    AdmissionReview at a time on it; this server reads ``Content-Length`` bodies, calls
    ``handler(method, path, headers, body) -> (status, content_type, body)`` and writes
    the response — no routing tables, middlewares or access logs on the admission path.
    """

    def __init__(self, handler, host: str = "127.0.0.1", port: int = 0,
                 ssl_context: Optional[_ssl.SSLContext] = None, max_body: int = 16 << 20, reuse_port: bool = False):
        self.handler = handler
        self.reuse_port = reuse_port  # SO_REUSEPORT: several processes accept on one port
        self.host = host
        self.port = port
        self.ssl = ssl_context
        self.max_body = max_body
        self._server = None
        self._conns: set = set()

    async def start(self) -> "Http1Server":
        self._server = await asyncio.start_server(self._serve, self.host, self.port, ssl=self.ssl, limit=1 << 24,
                                                  reuse_port=self.reuse_port or None)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def _serve(self, reader, writer) -> None:
        task = asyncio.current_task()
        self._conns.add(task)
        sock = writer.get_extra_info("socket")
        if sock is not None:
            import socket

            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        try:
            while True:
                try:
                    raw = await reader.readuntil(b"\r\n\r\n")
                except (asyncio.IncompleteReadError, ConnectionError, OSError, _ssl.SSLError):
                    return
                lines = raw.decode("latin-1").split("\r\n")
                parts = lines[0].split(" ")
                if len(parts) < 3:
                    return
                method, target = parts[0], parts[1]
                headers = {}
                for line in lines[1:]:
                    if ":" in line:
                        k, v = line.split(":", 1)
                        headers[k.strip().lower()] = v.strip()
                n = int(headers.get("content-length", "0") or 0)
                if n > self.max_body:
                    status, ctype, body = 413, "text/plain", b"request body too large"
                else:
                    data = await reader.readexactly(n) if n else b""
                    try:
                        status, ctype, body = await self.handler(method, target.split("?", 1)[0], headers, data)
                    except Exception as e:  # the handler's bug must not kill the connection loop
                        status, ctype, body = 500, "text/plain", repr(e).encode()
                close = headers.get("connection", "").lower() == "close"
                head = (f"HTTP/1.1 {status} {_REASONS.get(status, 'OK')}\r\nContent-Type: {ctype}\r\n"
                        f"Content-Length: {len(body)}\r\n{'Connection: close' + chr(13) + chr(10) if close else ''}\r\n")
                writer.write(head.encode("latin-1") + body)
                await writer.drain()
                if close:
                    return
        except (ConnectionError, OSError, asyncio.IncompleteReadError):
            return
        finally:
            self._conns.discard(task)
            try:
                writer.close()
            except Exception:
                pass

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            for t in list(self._conns):
                t.cancel()
            try:
                await asyncio.wait_for(self._server.wait_closed(), 2.0)
            except (asyncio.TimeoutError, Exception):
                pass
            self._server = None
