"""Lean HTTP/1.1 client for the apiserver REST path (asyncio protocol, keep-alive pool).

A control-plane process spends most of its CPU time talking to the apiserver; a generic
client (aiohttp) costs ~4× the raw socket round trip per request on this path (measured
0.14 ms vs 0.03 ms for a GET on loopback).  This client does only what the Kubernetes
REST API needs: persistent connections, ``Content-Length`` or ``chunked`` bodies,
optional TLS, and a streaming mode for watches.  Responses are parsed in the protocol's
``data_received`` (one future per response; a watch wakes its consumer once per arrival with
all the events it holds), not through StreamReader waits.  A pooled connection the server
closed while idle is skipped; a request that met such a close is retried once unless it is
a POST.
"""

from __future__ import annotations

import asyncio
import os
import ssl as _ssl
import sys
import time
from typing import AsyncIterator, Dict, List, Optional, Tuple
from urllib.parse import urlsplit


class HttpError(Exception):
    pass


def _parse_head(raw: bytes) -> Tuple[int, Dict[str, str]]:
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


def _dechunk(raw: bytearray, body: bytearray) -> bool:
    """Move the complete chunks at the front of ``raw`` into ``body``; True once the last chunk
    and its (empty) trailer are in — the connection may carry the next response after it."""
    pos = 0
    done = False
    while True:
        crlf = raw.find(b"\r\n", pos)
        if crlf < 0:
            break
        size = int(bytes(raw[pos:crlf]).split(b";", 1)[0].strip(), 16)
        if size == 0:
            end = raw.find(b"\r\n\r\n", crlf)
            if end >= 0:
                done = True
                pos = end + 4
            break
        end = crlf + 2 + size
        if len(raw) < end + 2:
            break
        body += raw[crlf + 2:end]
        pos = end + 2
    del raw[:pos]
    return done


# ODH_STALL_WATCHDOG_MS (diagnostics): every request that took at least this long is reported to
# stderr with its wall-clock end and whether it rode a pooled or a new connection
_STALL_MS = float(os.environ.get("ODH_STALL_WATCHDOG_MS") or 0)


def _stall_report(what: str) -> None:
    print(f"stall-watchdog: pid {os.getpid()} {what} ending at {time.time():.6f}", file=sys.stderr, flush=True)


_LAG_LOOPS: set = set()


def _ensure_loop_watchdog() -> None:
    """With ODH_STALL_WATCHDOG_MS: one task per event loop that sleeps 2 ms at a time and
    reports every wake-up that came at least the threshold late (the loop was stopped: a
    long callback, a collection, a blocking call)."""
    loop = asyncio.get_running_loop()
    if id(loop) in _LAG_LOOPS:
        return
    _LAG_LOOPS.add(id(loop))

    async def watch() -> None:
        while True:
            t0 = time.perf_counter()
            await asyncio.sleep(0.002)
            late = (time.perf_counter() - t0 - 0.002) * 1e3
            if late >= _STALL_MS:
                _stall_report(f"event loop {late:.1f} ms late")

    loop.create_task(watch())


class _Conn(asyncio.Protocol):
    """One keep-alive connection whose responses are parsed in ``data_received``.

    A request is one future, resolved when its response is complete however many reads that
    took — not a StreamReader wait per head / chunk / body part, each its own event-loop
    wake-up and task step.  A streaming (watch) response is de-chunked and split into lines
    as bytes arrive, and its consumer is woken once per arrival with every complete line."""

    def __init__(self):
        self.transport = None
        self.buf = bytearray()
        self.closed = False
        self._waiter: Optional[asyncio.Future] = None
        self._head: Optional[Tuple[int, Dict[str, str]]] = None
        self._body = bytearray()
        self._want = -1  # Content-Length body size; -2: chunked; -3: until EOF
        self._streaming = False
        self._lines: List[bytes] = []
        self._got = 0
        self._eof = False
        self._no_body = False  # the request in flight is a HEAD

    # ---------------------------------------------------------------- asyncio.Protocol

    def connection_made(self, transport) -> None:
        self.transport = transport

    def data_received(self, data: bytes) -> None:
        self.buf += data
        if self._waiter is not None or self._streaming:
            self._advance()

    def eof_received(self):
        return False  # close the transport: connection_lost follows

    def connection_lost(self, exc) -> None:
        self.closed = True
        self._eof = True
        w, self._waiter = self._waiter, None
        if w is None or w.done():
            return
        if self._streaming:
            w.set_result(None)  # stream(): no head (None) / next_lines(): the body ended
        elif self._want == -3 and self._head is not None:
            self._body += self.buf
            self.buf.clear()
            w.set_result((self._head[0], bytes(self._body), True))
        else:
            w.set_exception(ConnectionResetError(f"connection lost mid-response: {exc!r}"))

    # ---------------------------------------------------------------- parsing

    def _advance(self) -> None:
        w = self._waiter
        try:
            if self._head is None:
                i = self.buf.find(b"\r\n\r\n")
                if i < 0:
                    return
                self._head = _parse_head(bytes(self.buf[:i]))
                del self.buf[:i + 4]
                status, h = self._head
                if self._no_body or status < 200 or status in (204, 304):
                    self._want = 0  # RFC 9112 §6.3: no body, whatever the headers say
                elif h.get("transfer-encoding", "").lower() == "chunked":
                    self._want = -2
                elif "content-length" in h:
                    self._want = int(h["content-length"])
                elif h.get("connection", "").lower() == "close" or self._streaming:
                    self._want = -3  # delimited by the server closing the connection
                else:
                    self._want = 0  # a keep-alive response without a length has no body
                if self._streaming:  # stream() waits for the head alone
                    self._waiter = None
                    if w is not None and not w.done():
                        w.set_result(self._head)
            if self._streaming:
                self._stream_advance()
                return
            if self._want >= 0:
                if len(self.buf) < self._want:
                    return
                data = bytes(self.buf[:self._want])
                del self.buf[:self._want]
            elif self._want == -2:
                if not _dechunk(self.buf, self._body):
                    return
                data = bytes(self._body)
                self._body.clear()
            else:
                return  # delimited by EOF: connection_lost completes it
            status, headers = self._head
            self._head = None
            self._waiter = None
            if w is not None and not w.done():
                w.set_result((status, data, headers.get("connection", "").lower() == "close"))
        except Exception as e:  # noqa: BLE001 — a malformed response fails its request, not the loop
            self._waiter = None
            self.close()
            if w is not None and not w.done():
                w.set_exception(HttpError(f"bad response: {e!r}"))

    def _stream_advance(self) -> None:
        if self._want == -2:
            done = _dechunk(self.buf, self._body)
        else:
            self._got += len(self.buf)
            self._body += self.buf
            self.buf.clear()
            done = 0 <= self._want <= self._got  # a Content-Length body (an error Status)
        body = self._body
        start = 0
        while True:
            nl = body.find(b"\n", start)
            if nl < 0:
                break
            self._lines.append(bytes(body[start:nl]))
            start = nl + 1
        if start:
            del body[:start]
        if done:
            self._eof = True
            self.close()
        w = self._waiter
        if (self._lines or self._eof) and w is not None and not w.done():
            self._waiter = None
            w.set_result(None)

    # ---------------------------------------------------------------- client side

    async def roundtrip(self, payload: bytes) -> Tuple[int, bytes, bool]:
        if self.closed:
            raise ConnectionResetError("connection closed")
        self._waiter = w = asyncio.get_running_loop().create_future()
        self._no_body = payload.startswith(b"HEAD ")
        self.transport.write(payload)
        if self.buf:  # bytes that arrived before the request (a server error, an early close)
            self._advance()
        return await w

    async def open_stream(self, payload: bytes) -> Tuple[int, Dict[str, str]]:
        if self.closed:
            raise ConnectionResetError("connection closed")
        self._streaming = True
        self._waiter = w = asyncio.get_running_loop().create_future()
        self.transport.write(payload)
        got = await w
        if got is None:
            raise ConnectionResetError("connection lost before the response head")
        return got

    async def next_lines(self) -> List[bytes]:
        """The complete lines received since the last call; [] once the body ended."""
        while not self._lines:
            if self._eof or self.closed:
                return []
            self._waiter = w = asyncio.get_running_loop().create_future()
            try:
                await w
            finally:
                if self._waiter is w:
                    self._waiter = None
        out, self._lines = self._lines, []
        return out

    def close(self) -> None:
        self.closed = True
        if self.transport is not None:
            self.transport.close()


class Http1Pool:
    def __init__(self, base_url: str, ssl_context: Optional[_ssl.SSLContext] = None,
                 headers: Optional[Dict[str, str]] = None, size: int = 64, spare: int = 0):
        u = urlsplit(base_url)
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.ssl = ssl_context if u.scheme == "https" else None
        self._hdr = {"Host": f"{self.host}:{self.port}", "Accept": "application/json"}
        self._hdr.update(headers or {})
        self._static = "".join(f"{k}: {v}\r\n" for k, v in self._hdr.items())
        self._idle: List[_Conn] = []
        self.size = size
        self.opened = 0
        # idle connections kept open ahead of demand: a request that finds the pool empty
        # does not wait for a connection to be accepted (on the GPU boxes a burst's new
        # connections sat 80-170 ms in the apiserver's listen queue, profiles/r6_g38)
        self.spare = max(0, int(spare))
        self._warming = 0

    def set_header(self, name: str, value: Optional[str]) -> None:
        """Set (``None``: drop) a header every later request carries — e.g. a rotated bearer
        token.  Requests already written keep the one they were sent with."""
        if value is None:
            self._hdr.pop(name, None)
        else:
            self._hdr[name] = value
        self._static = "".join(f"{k}: {v}\r\n" for k, v in self._hdr.items())

    async def _connect(self) -> _Conn:
        loop = asyncio.get_running_loop()
        transport, conn = await loop.create_connection(_Conn, self.host, self.port, ssl=self.ssl)
        sock = transport.get_extra_info("socket")
        if sock is not None:
            import socket

            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        self.opened += 1
        return conn

    def _head(self, method: str, target: str, body: Optional[bytes], content_type: Optional[str]) -> bytes:
        h = f"{method} {target} HTTP/1.1\r\n{self._static}"
        if body is not None:
            h += f"Content-Type: {content_type or 'application/json'}\r\nContent-Length: {len(body)}\r\n"
        return (h + "\r\n").encode("latin-1") + (body or b"")

    def _take_idle(self) -> Optional[_Conn]:
        c = None
        while self._idle:
            c = self._idle.pop()
            if not c.closed:
                break
            c = None
        while self.spare and len(self._idle) + self._warming < self.spare:
            self._warming += 1
            asyncio.get_running_loop().create_task(self._warm())
        return c

    async def _warm(self) -> None:
        try:
            conn = await self._connect()
        except (ConnectionError, OSError):
            return
        finally:
            self._warming -= 1
        if self.spare and len(self._idle) < self.size:
            self._idle.append(conn)
        else:
            conn.close()

    async def request(self, method: str, target: str, body: Optional[bytes] = None,
                      content_type: Optional[str] = None) -> Tuple[int, bytes]:
        payload = self._head(method, target, body, content_type)
        if _STALL_MS:
            _ensure_loop_watchdog()
        for attempt in (0, 1):
            conn = self._take_idle()
            reused = conn is not None
            try:
                t0 = time.perf_counter() if _STALL_MS else 0.0
                if conn is None:
                    conn = await self._connect()
                t1 = time.perf_counter() if _STALL_MS else 0.0
                status, data, close = await conn.roundtrip(payload)
                if _STALL_MS and (time.perf_counter() - t0) * 1e3 >= _STALL_MS:
                    _stall_report(f"{method} {target[:96]}: {(time.perf_counter() - t0) * 1e3:.1f} ms "
                                  f"({'pooled' if reused else f'new connection, connect {(t1 - t0) * 1e3:.1f} ms'})")
            except (ConnectionError, OSError) as e:
                if conn is not None:
                    conn.close()
                # a pooled connection the server closed while idle: once more on a fresh one
                if reused and attempt == 0 and method != "POST":
                    continue
                raise HttpError(f"{method} {target}: {e!r}") from e
            except BaseException:
                if conn is not None:
                    conn.close()
                raise
            if close or len(self._idle) >= self.size:
                conn.close()
            else:
                self._idle.append(conn)
            return status, data
        raise HttpError("unreachable")

    async def stream(self, method: str, target: str) -> Tuple[int, Dict[str, str], "_Stream"]:
        conn = await self._connect()
        try:
            status, headers = await conn.open_stream(self._head(method, target, None, None))
        except BaseException:
            conn.close()
            raise
        return status, headers, _Stream(conn)

    async def close(self) -> None:
        self.spare = 0  # no more warming; one in flight closes its connection below
        for c in self._idle:
            c.close()
        self._idle.clear()


class _Stream:
    """Body of a streaming (watch) response: iterate batches of lines, then close."""

    def __init__(self, conn: _Conn):
        self.conn = conn

    async def read_all(self) -> bytes:
        try:
            out = []
            while True:
                got = await self.conn.next_lines()
                if not got:
                    break
                out += [x + b"\n" for x in got]
            return b"".join(out) + bytes(self.conn._body)
        finally:
            self.close()

    async def batches(self) -> AsyncIterator[List[bytes]]:
        """The complete lines (without their newline) of each arrival, until the body or the
        connection ends."""
        try:
            while True:
                got = await self.conn.next_lines()
                if not got:
                    return
                yield got
        finally:
            self.close()

    async def lines(self) -> AsyncIterator[bytes]:
        async for batch in self.batches():
            for line in batch:
                yield line

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
                 ssl_context: Optional[_ssl.SSLContext] = None, max_body: int = 16 << 20, reuse_port: bool = False,
                 max_requests_per_conn: int = 0):
        self.handler = handler
        self.reuse_port = reuse_port  # SO_REUSEPORT: several processes accept on one port
        # close a keep-alive connection after this many requests (0: never).  SO_REUSEPORT
        # spreads connections, not requests: a client holding a few long-lived connections (the
        # apiserver's webhook pool) can leave a listener idle for good; making it reconnect
        # now and then lets the kernel spread its connections again
        self.max_requests_per_conn = max_requests_per_conn
        self.host = host
        self.port = port
        self.ssl = ssl_context
        self.max_body = max_body
        self._server = None
        self._conns: set = set()

    async def start(self) -> "Http1Server":
        if _STALL_MS:
            _ensure_loop_watchdog()
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
        served = 0
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
                served += 1
                close = headers.get("connection", "").lower() == "close" or (
                    self.max_requests_per_conn > 0 and served >= self.max_requests_per_conn)
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
