"""Minimal asyncio HTTP/1.1 keep-alive client (load generation, gateway -> worker hops).

aiohttp builds a ClientRequest/ClientResponse pair, a timer context, trace hooks, a
multidict header set and a payload writer per call; in a closed-loop load generator that
shares one event loop with the server under test that is host time charged to the server
(``benchmarks/http_overhead.py --profile``: aiohttp ``_request`` was the largest single item).
This client keeps one ``asyncio.Protocol`` per pooled connection and does per request
exactly: write one pre-formatted request, parse the status line and headers, read the body
by ``Content-Length`` or ``chunked``. It speaks real HTTP/1.1 over TCP to any server.

    pool = Http1Pool("127.0.0.1", 8000, headers={"authorization": "Bearer k"})
    status, headers, body = await pool.request("POST", "/v1/chat/completions", json_bytes)
    await pool.close()
"""
from __future__ import annotations

import asyncio
import collections
from typing import Optional


class HttpError(Exception):
    pass


class _Conn(asyncio.Protocol):
    def __init__(self, loop):
        self.loop = loop
        self.transport = None
        self.buf = bytearray()
        self.fut: Optional[asyncio.Future] = None
        self.closed = False
        self.head_end = -1
        self.status = 0
        self.headers: dict = {}
        self.length = -1
        self.chunked = False
        self.keep_alive = True
        self.head_only = False

    def connection_made(self, transport):
        self.transport = transport

    def connection_lost(self, exc):
        self.closed = True
        f = self.fut
        if f is not None and not f.done():
            if self.head_end >= 0 and self.length < 0 and not self.chunked:
                self._finish(bytes(self.buf[self.head_end:]))  # body delimited by close
            else:
                f.set_exception(HttpError(f"connection closed: {exc!r}"))

    def start(self, data: bytes, head_only: bool = False) -> asyncio.Future:
        self.fut = self.loop.create_future()
        self.head_end = -1
        self.length = -1
        self.chunked = False
        self.head_only = head_only
        self.transport.write(data)
        return self.fut

    def data_received(self, data: bytes):
        self.buf += data
        if self.fut is None or self.fut.done():
            return
        buf = self.buf
        if self.head_end < 0:
            end = buf.find(b"\r\n\r\n")
            if end < 0:
                return
            lines = bytes(buf[:end]).split(b"\r\n")
            parts = lines[0].split(b" ", 2)
            try:
                self.status = int(parts[1])
            except (IndexError, ValueError):
                self.fut.set_exception(HttpError(f"bad status line {lines[0][:80]!r}"))
                return
            hdrs = {}
            for line in lines[1:]:
                i = line.find(b":")
                if i > 0:
                    hdrs[line[:i].strip().lower().decode("latin-1")] = line[i + 1:].strip().decode("latin-1")
            self.headers = hdrs
            self.keep_alive = hdrs.get("connection", "").lower() != "close" and parts[0] == b"HTTP/1.1"
            if "content-length" in hdrs:
                self.length = int(hdrs["content-length"])
            elif "chunked" in hdrs.get("transfer-encoding", "").lower():
                self.chunked = True
            elif self.status in (204, 304) or 100 <= self.status < 200:
                self.length = 0
            self.head_end = end + 4
            if 100 <= self.status < 200:  # interim response (100 Continue): wait for the real one
                del buf[:self.head_end]
                self.head_end = -1
                return self.data_received(b"")
            if self.head_only:
                self.length = 0
        start = self.head_end
        if self.length >= 0:
            if len(buf) - start >= self.length:
                body = bytes(buf[start:start + self.length])
                del buf[:start + self.length]
                self._finish(body)
        elif self.chunked:
            pos, parts = start, []
            while True:
                eol = buf.find(b"\r\n", pos)
                if eol < 0:
                    return
                n = int(bytes(buf[pos:eol]).split(b";", 1)[0], 16)
                if n == 0:
                    fin = buf.find(b"\r\n\r\n", eol)
                    if fin < 0:
                        return
                    del buf[:fin + 4]
                    self._finish(b"".join(parts))
                    return
                if len(buf) < eol + 2 + n + 2:
                    return
                parts.append(bytes(buf[eol + 2:eol + 2 + n]))
                pos = eol + 2 + n + 2

    def _finish(self, body: bytes):
        f = self.fut
        self.fut = None
        if f is not None and not f.done():
            f.set_result((self.status, self.headers, body))


def _expire(fut: asyncio.Future) -> None:
    if not fut.done():
        fut.set_exception(HttpError("request timed out"))


class Http1Pool:
    """Keep-alive connections to one ``host:port``; ``request()`` borrows an idle one (or dials)."""

    def __init__(self, host: str, port: int, headers: Optional[dict] = None, timeout: float = 300.0):
        self.host, self.port, self.timeout = host, port, timeout
        extra = "".join(f"{k}: {v}\r\n" for k, v in (headers or {}).items())
        self._fixed = (f"host: {host}:{port}\r\n" + extra).encode("latin-1")
        self._idle: collections.deque = collections.deque()
        self._all: set = set()

    async def _dial(self) -> _Conn:
        loop = asyncio.get_running_loop()
        _, conn = await loop.create_connection(lambda: _Conn(loop), self.host, self.port)
        import socket
        sock = conn.transport.get_extra_info("socket")
        if sock is not None:
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._all.add(conn)
        return conn

    async def request(self, method: str, path: str, body: bytes = b"",
                      content_type: str = "application/json") -> tuple[int, dict, bytes]:
        head = b"%s %s HTTP/1.1\r\n%scontent-type: %s\r\ncontent-length: %d\r\n\r\n" % (
            method.encode(), path.encode(), self._fixed, content_type.encode(), len(body))
        while True:
            conn = None
            while self._idle:
                c = self._idle.pop()
                if not c.closed:
                    conn = c
                    break
            reused = conn is not None
            if conn is None:
                conn = await self._dial()
            fut = conn.start(head + body, head_only=method == "HEAD")
            timer = conn.loop.call_later(self.timeout, _expire, fut) if self.timeout else None
            try:
                status, headers, data = await fut
            except HttpError:
                conn.transport.close()
                self._all.discard(conn)
                if reused and conn.closed and not conn.buf:
                    # the server closed this idle keep-alive connection (its idle timeout) as the
                    # request went out: nothing was answered, so nothing ran. Retry on a new one
                    continue
                raise
            except BaseException:
                conn.transport.close()
                self._all.discard(conn)
                raise
            finally:
                if timer is not None:
                    timer.cancel()
            break
        if conn.keep_alive and not conn.closed:
            self._idle.append(conn)
        else:
            conn.transport.close()
            self._all.discard(conn)
        return status, headers, data

    async def close(self) -> None:
        for c in list(self._all):
            if not c.closed:
                c.transport.close()
        self._all.clear()
        self._idle.clear()
        await asyncio.sleep(0)
