"""Lean HTTP/1.1 server for ASGI apps (the serving front end of ``python main.py`` and bench.py).

Why not uvicorn: without ``httptools``/``uvloop`` (neither is in the image) uvicorn parses
HTTP through ``h11``, a pure-Python state machine that validates every header with regexes.
On the headline load (concurrency 8, closed loop) every wave of requests crosses the server
one request at a time on the event loop while the engine sits idle, so the per-request
host cost is engine idle time (h11 ``handle_events`` was the largest
single item of the request path). ``uvicorn main:app`` keeps working: the app is plain ASGI.

This is an ``asyncio.Protocol`` per connection:

* request head parsed with ``bytes.find``/``split`` (request line + ``name: value`` lines,
  names lower-cased as ASGI wants), bodies by ``Content-Length`` or ``chunked``,
  ``Expect: 100-continue`` answered, head/body size limits (431 / 413), 400 on garbage;
* strict framing (request smuggling): duplicate ``Content-Length``, a non-digit length,
  ``Content-Length`` together with ``Transfer-Encoding``, whitespace before a header colon and
  obsolete line folding are 400; a transfer coding other than ``chunked`` is 501;
* keep-alive and pipelining (requests of one connection run one after another),
  ``Connection: close`` honoured both ways, HTTP/1.0 closes after the response unless it asked
  for keep-alive (echoed back);
* timeouts and limits (what ``uvicorn main:app``, the reference's deployment, gives): an idle
  keep-alive connection is closed after ``timeout_keep_alive`` seconds (5); a request whose head
  and body are not complete ``timeout_request`` seconds after its first byte gets 408 and the
  connection closes (slow / partial heads and bodies, half-closed clients); above
  ``max_connections`` open connections a new connection's first request gets 503 +
  ``Retry-After`` and is closed. One server-wide sweeper task checks the deadlines, so the
  per-request cost is a timestamp;
* responses: the app's headers are written as given; without ``content-length`` the body is
  sent ``Transfer-Encoding: chunked`` (SSE streams) to HTTP/1.1 clients, unframed + close to
  HTTP/1.0 clients; HEAD sends no body;
* ``receive()`` returns the whole body once, then blocks until the client disconnects or the
  response is complete (``http.disconnect``) — what Starlette's streaming responses listen
  for; writes pause on transport back-pressure;
* lifespan ``startup``/``shutdown`` (with ``state``), graceful stop: ``should_exit`` (or
  SIGINT/SIGTERM when ``install_signal_handlers``) closes the listener, lets running
  requests finish (``timeout_graceful_shutdown``), then closes idle connections.

The interface mirrors the parts of ``uvicorn.Server`` the repo uses (``started``,
``should_exit``, ``serve()``), so bench.py and main.py can pick either.
"""
from __future__ import annotations

import asyncio
import logging
import signal
import socket
import threading
from typing import Any, Callable, Optional
from urllib.parse import unquote

logger = logging.getLogger("vgate.server")

_REASONS = {100: b"Continue", 200: b"OK", 201: b"Created", 204: b"No Content", 301: b"Moved Permanently",
            302: b"Found", 304: b"Not Modified", 307: b"Temporary Redirect", 400: b"Bad Request",
            401: b"Unauthorized", 403: b"Forbidden", 404: b"Not Found", 405: b"Method Not Allowed",
            408: b"Request Timeout", 409: b"Conflict", 413: b"Payload Too Large", 415: b"Unsupported Media Type",
            422: b"Unprocessable Entity", 429: b"Too Many Requests", 431: b"Request Header Fields Too Large",
            500: b"Internal Server Error", 501: b"Not Implemented", 502: b"Bad Gateway",
            503: b"Service Unavailable", 504: b"Gateway Timeout"}
_STATUS_LINES: dict[int, bytes] = {}


def _status_line(code: int) -> bytes:
    line = _STATUS_LINES.get(code)
    if line is None:
        line = b"HTTP/1.1 %d %s\r\n" % (code, _REASONS.get(code, b"Unknown"))
        _STATUS_LINES[code] = line
    return line


def _plain(code: int, text: bytes, close: bool = True, extra: bytes = b"") -> bytes:
    return (_status_line(code) + b"content-type: text/plain; charset=utf-8\r\ncontent-length: %d\r\n%s%s\r\n"
            % (len(text), extra, b"connection: close\r\n" if close else b"") + text)


_WS = b" \t"


class _BadRequest(Exception):
    def __init__(self, code: int, text: bytes):
        super().__init__(text)
        self.code, self.text = code, text


class _Cycle:
    """One request/response exchange on a connection."""

    __slots__ = ("proto", "scope", "body", "body_sent", "started", "complete", "chunked", "head",
                 "keep_alive", "disconnect_waiter", "http10")

    def __init__(self, proto: "HttpProtocol", scope: dict, body: bytes, keep_alive: bool):
        self.proto = proto
        self.scope = scope
        self.body = body
        self.body_sent = False
        self.started = False
        self.complete = False
        self.chunked = False
        self.head = scope["method"] == "HEAD"
        self.keep_alive = keep_alive
        self.disconnect_waiter: Optional[asyncio.Future] = None
        self.http10 = scope["http_version"] == "1.0"

    async def receive(self) -> dict:
        if not self.body_sent:
            self.body_sent = True
            return {"type": "http.request", "body": self.body, "more_body": False}
        if not self.complete and not self.proto.closed:
            fut = self.disconnect_waiter
            if fut is None:
                fut = self.disconnect_waiter = self.proto.loop.create_future()
            await fut
        return {"type": "http.disconnect"}

    async def send(self, msg: dict) -> None:
        t = msg["type"]
        proto = self.proto
        if t == "http.response.start":
            if self.started:
                raise RuntimeError("response already started")
            self.started = True
            status = msg["status"]
            parts = [_status_line(status)]
            has_len = False
            for name, value in msg.get("headers", ()):
                ln = name.lower()
                if ln == b"content-length":
                    has_len = True
                elif ln == b"connection" and value.lower() == b"close":
                    self.keep_alive = False
                elif ln == b"transfer-encoding":
                    continue  # the framing is ours
                parts.append(name + b": " + value + b"\r\n")
            if not has_len and not self.head and status >= 200 and status not in (204, 304):
                if self.http10:
                    self.keep_alive = False  # no chunked coding for 1.0: the close ends the body
                else:
                    self.chunked = True
                    parts.append(b"transfer-encoding: chunked\r\n")
            if not self.keep_alive:
                parts.append(b"connection: close\r\n")
            elif self.http10:
                parts.append(b"connection: keep-alive\r\n")
            parts.append(b"\r\n")
            if proto.closed:
                return
            proto.transport.write(b"".join(parts))
        elif t == "http.response.body":
            if not self.started:
                raise RuntimeError("http.response.body before http.response.start")
            if self.complete:
                return
            body = msg.get("body", b"")
            more = msg.get("more_body", False)
            if proto.closed:
                if not more:
                    self.complete = True
                return
            if self.head:
                pass
            elif self.chunked:
                if body:
                    proto.transport.write(b"%x\r\n%s\r\n" % (len(body), body))
                if not more:
                    proto.transport.write(b"0\r\n\r\n")
            elif body:
                proto.transport.write(body)
            if proto.write_paused:
                await proto.drain()
            if not more:
                self.complete = True
                w = self.disconnect_waiter
                if w is not None and not w.done():
                    w.set_result(None)
        # other message types (http.response.trailers, pathsend, ...) are not advertised


class HttpProtocol(asyncio.Protocol):
    MAX_HEAD = 64 * 1024

    def __init__(self, server: "Server"):
        self.server = server
        self.app = server.app
        self.loop = server.loop
        self.transport: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.closed = False
        self.write_paused = False
        self._drain_waiters: list = []
        self.cycle: Optional[_Cycle] = None
        self.task: Optional[asyncio.Task] = None
        self.client = None
        self.sockname = None
        self._continued = False
        self.eof = False
        self.read_paused = False
        self.reject = False
        self.since = 0.0  # when the connection last became idle, or its pending request began

    # ------------------------------------------------------------------ transport events
    def connection_made(self, transport):
        self.transport = transport
        srv = self.server
        srv.connections.add(self)
        self.since = self.loop.time()
        if srv.max_connections and len(srv.connections) > srv.max_connections:
            self.reject = True  # answered 503 once its first head is in (a reply before the
            # request risks a reset that discards it at the client)
        sock = transport.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        peer = transport.get_extra_info("peername")
        self.client = tuple(peer[:2]) if isinstance(peer, tuple) else None
        sn = transport.get_extra_info("sockname")
        self.sockname = tuple(sn[:2]) if isinstance(sn, tuple) else None

    def connection_lost(self, exc):
        self.closed = True
        self.server.connections.discard(self)
        c = self.cycle
        if c is not None and c.disconnect_waiter is not None and not c.disconnect_waiter.done():
            c.disconnect_waiter.set_result(None)
        for w in self._drain_waiters:
            if not w.done():
                w.set_result(None)
        self._drain_waiters.clear()

    def pause_writing(self):
        self.write_paused = True

    def resume_writing(self):
        self.write_paused = False
        for w in self._drain_waiters:
            if not w.done():
                w.set_result(None)
        self._drain_waiters.clear()

    async def drain(self):
        if self.write_paused and not self.closed:
            w = self.loop.create_future()
            self._drain_waiters.append(w)
            await w

    def data_received(self, data: bytes):
        if self.task is None:
            if not self.buf:
                self.since = self.loop.time()  # a new request's first bytes: its read deadline
            self.buf += data
            self._next()
        else:
            self.buf += data
            if len(self.buf) > self.server.max_pending and not self.read_paused:
                self.read_paused = True  # a pipelining client ran far ahead: wait for the app
                self.transport.pause_reading()

    def eof_received(self):
        # the client half-closed: answer what is in flight, then close. A partial request with
        # no task can never complete now: close at once
        self.eof = True
        if self.task is None:
            return False
        return True

    # ------------------------------------------------------------------ parsing
    def _next(self) -> None:
        """Start the next complete request in the buffer, if any (no task running)."""
        if self.closed:
            return
        buf = self.buf
        end = buf.find(b"\r\n\r\n")
        if end < 0:
            if len(buf) > self.MAX_HEAD:
                self._fail(431, b"Request Header Fields Too Large")
            return
        try:
            scope, length, chunked, keep_alive, expect = self._parse_head(bytes(buf[:end]))
        except _BadRequest as e:
            self._fail(e.code, e.text)
            return
        if self.reject:
            self.transport.write(_plain(503, b"Too many connections", extra=b"retry-after: 1\r\n"))
            self.transport.close()
            self.closed = True
            return
        start = end + 4
        if chunked:
            got = self._dechunk(start)
            if got is None:
                if expect and not self._continued and not self.closed:
                    self._continued = True
                    self.transport.write(b"HTTP/1.1 100 Continue\r\n\r\n")
                return
            body, consumed = got
        else:
            if length > self.server.max_body:
                self._fail(413, b"Payload Too Large")
                return
            if len(buf) - start < length:
                if expect and not self._continued:
                    self._continued = True
                    self.transport.write(b"HTTP/1.1 100 Continue\r\n\r\n")
                return
            body = bytes(buf[start:start + length])
            consumed = start + length
        self._continued = False
        del buf[:consumed]
        cycle = _Cycle(self, scope, body, keep_alive)
        self.cycle = cycle
        self.task = self.loop.create_task(self._run(cycle))

    def _dechunk(self, pos: int):
        buf = self.buf
        parts = []
        total = 0
        while True:
            eol = buf.find(b"\r\n", pos)
            if eol < 0:
                return None
            try:
                n = int(bytes(buf[pos:eol]).split(b";", 1)[0].strip(), 16)
            except ValueError:
                self._fail(400, b"Invalid chunk size")
                return None
            total += n
            if total > self.server.max_body:
                self._fail(413, b"Payload Too Large")
                return None
            if n == 0:
                # trailers (ignored) end with an empty line
                fin = buf.find(b"\r\n\r\n", eol)
                if fin == eol:
                    return b"".join(parts), eol + 4
                if fin < 0:
                    if buf[eol:eol + 4] == b"\r\n\r\n":
                        return b"".join(parts), eol + 4
                    return None
                return b"".join(parts), fin + 4
            if len(buf) < eol + 2 + n + 2:
                return None
            parts.append(bytes(buf[eol + 2:eol + 2 + n]))
            pos = eol + 2 + n + 2

    def _parse_head(self, head: bytes):
        lines = head.split(b"\r\n")
        try:
            method, target, version = lines[0].split(b" ")
        except ValueError:
            raise _BadRequest(400, b"Invalid request line") from None
        if version == b"HTTP/1.1":
            http_version, keep_alive = "1.1", True
        elif version == b"HTTP/1.0":
            http_version, keep_alive = "1.0", False
        else:
            raise _BadRequest(400, b"Unsupported HTTP version")
        headers = []
        length = -1
        chunked = False
        expect = False
        for line in lines[1:]:
            i = line.find(b":")
            if i <= 0 or line[0] in _WS or line[i - 1] in _WS:
                # no name, obsolete line folding, or whitespace before the colon (RFC 9112 5.1:
                # a proxy in front may read such a line differently -> request smuggling)
                raise _BadRequest(400, b"Invalid header line")
            name = line[:i].lower()
            value = line[i + 1:].strip()
            headers.append((name, value))
            if name == b"content-length":
                if length >= 0:
                    raise _BadRequest(400, b"Duplicate Content-Length")
                if not value.isdigit():
                    raise _BadRequest(400, b"Invalid Content-Length")
                length = int(value)
            elif name == b"transfer-encoding":
                if chunked or value.lower() != b"chunked":
                    raise _BadRequest(501, b"Unsupported Transfer-Encoding")
                chunked = True
            elif name == b"connection":
                v = value.lower()
                if b"close" in v:
                    keep_alive = False
                elif b"keep-alive" in v:
                    keep_alive = True
            elif name == b"expect":
                expect = value.lower() == b"100-continue"
        q = target.find(b"?")
        if q >= 0:
            raw_path, query = target[:q], target[q + 1:]
        else:
            raw_path, query = target, b""
        path = raw_path.decode("latin-1")
        if "%" in path:
            path = unquote(path)
        scope = {"type": "http", "asgi": _ASGI, "http_version": http_version, "server": self.sockname,
                 "client": self.client, "scheme": "http", "method": method.decode("latin-1"), "root_path": "",
                 "path": path, "raw_path": raw_path, "query_string": query, "headers": headers,
                 "state": self.server.state.copy()}
        if chunked and length >= 0:
            raise _BadRequest(400, b"Content-Length with Transfer-Encoding")
        return scope, max(length, 0), chunked, keep_alive, expect

    def _fail(self, code: int, text: bytes) -> None:
        if not self.closed:
            self.transport.write(_plain(code, text))
            self.transport.close()
        self.closed = True

    # ------------------------------------------------------------------ app
    async def _run(self, cycle: _Cycle) -> None:
        try:
            await self.app(cycle.scope, cycle.receive, cycle.send)
        except BaseException as e:  # noqa: BLE001
            if isinstance(e, (KeyboardInterrupt, SystemExit)):
                raise
            logger.exception("unhandled error in the ASGI app")
            if not cycle.started and not self.closed:
                self.transport.write(_plain(500, b"Internal Server Error"))
            if not self.closed:
                self.transport.close()
            self.closed = True
        else:
            if not cycle.started and not self.closed:
                self.transport.write(_plain(500, b"Internal Server Error"))
                cycle.keep_alive = False
            elif not cycle.complete and not self.closed:
                cycle.keep_alive = False  # a body the client cannot delimit: close
        finally:
            w = cycle.disconnect_waiter
            if w is not None and not w.done():
                w.set_result(None)
            self.task = None
            self.cycle = None
            self.server.on_request_done()
        if self.closed:
            return
        if not cycle.keep_alive or self.server.should_exit or (self.eof and not self.buf):
            self.transport.close()
            self.closed = True
            return
        self.since = self.loop.time()
        if self.read_paused:
            # always resume: a request bigger than max_pending may be half-read in the buffer,
            # and _next can only start it once the rest arrives (re-paused below if another
            # request starts while the buffer is still over the bound)
            self.read_paused = False
            self.transport.resume_reading()
        if self.buf:
            self._next()
            if self.task is not None and len(self.buf) > self.server.max_pending:
                self.read_paused = True
                self.transport.pause_reading()
        if self.eof and self.task is None and not self.closed:
            self.transport.close()  # half-closed: a partial request can never complete
            self.closed = True

    def check_deadline(self, now: float, keep_alive: float, request: float) -> None:
        """Called by the server's sweeper: close an idle keep-alive connection, or answer 408 to
        a request that has not arrived in full ``request`` seconds after its first byte."""
        if self.task is not None or self.closed:
            return
        if not self.buf:
            if keep_alive and now - self.since > keep_alive:
                self.transport.close()
                self.closed = True
        elif request and now - self.since > request:
            self._fail(408, b"Request Timeout")

    def shutdown_idle(self) -> None:
        if self.task is None and not self.closed:
            self.transport.close()
            self.closed = True


_ASGI = {"version": "3.0", "spec_version": "2.3"}


class Server:
    """``Server(app, host, port).serve()`` — see the module docstring."""

    def __init__(self, app: Callable, host: str = "127.0.0.1", port: int = 8000, lifespan: str = "on",
                 install_signal_handlers: bool = False, timeout_graceful_shutdown: float = 30.0,
                 backlog: int = 2048, max_body: int = 64 * 2**20, timeout_keep_alive: float = 5.0,
                 timeout_request: float = 30.0, max_connections: int = 4096):
        self.app = app
        self.timeout_keep_alive = timeout_keep_alive
        self.timeout_request = timeout_request
        self.max_connections = max_connections
        self._sweeper: Optional[asyncio.Task] = None
        self.host = host
        self.port = port
        self.lifespan = lifespan
        self.install_signal_handlers = install_signal_handlers
        self.timeout_graceful_shutdown = timeout_graceful_shutdown
        self.backlog = backlog
        self.max_body = max_body
        self.max_pending = 1 << 20
        self.started = False
        self.should_exit = False
        self.state: dict = {}
        self.connections: set = set()
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self._server = None
        self._exit_event: Optional[asyncio.Event] = None
        self._lifespan_task = None
        self._lifespan_queue: Optional[asyncio.Queue] = None
        self._lifespan_events: dict[str, asyncio.Future] = {}
        self.sockets: list = []

    # ------------------------------------------------------------------ lifespan
    async def _lifespan_start(self) -> None:
        if self.lifespan == "off":
            return
        loop = self.loop
        q: asyncio.Queue = asyncio.Queue()
        self._lifespan_queue = q
        ev = {k: loop.create_future() for k in ("startup", "shutdown")}
        self._lifespan_events = ev
        await q.put({"type": "lifespan.startup"})

        async def send(msg):
            t = msg["type"]
            for k in ("startup", "shutdown"):
                if t.startswith(f"lifespan.{k}.") and not ev[k].done():
                    if t.endswith(".failed"):
                        ev[k].set_exception(RuntimeError(msg.get("message", f"lifespan {k} failed")))
                    else:
                        ev[k].set_result(None)

        async def run():
            scope = {"type": "lifespan", "asgi": _ASGI, "state": self.state}
            try:
                await self.app(scope, q.get, send)
            except BaseException as e:  # noqa: BLE001
                for f in ev.values():
                    if not f.done():
                        f.set_exception(e if isinstance(e, Exception) else RuntimeError(repr(e)))

        self._lifespan_task = loop.create_task(run())
        await ev["startup"]

    async def _lifespan_stop(self) -> None:
        if self._lifespan_queue is None:
            return
        await self._lifespan_queue.put({"type": "lifespan.shutdown"})
        try:
            await self._lifespan_events["shutdown"]
        except Exception:  # noqa: BLE001
            logger.exception("lifespan shutdown failed")

    # ------------------------------------------------------------------ serve
    def on_request_done(self) -> None:
        if self.should_exit and self._exit_event is not None:
            self._exit_event.set()

    async def startup(self) -> None:
        self.loop = asyncio.get_running_loop()
        await self._lifespan_start()
        self._server = await self.loop.create_server(lambda: HttpProtocol(self), self.host, self.port,
                                                     backlog=self.backlog, reuse_address=True)
        self.sockets = list(self._server.sockets or [])
        if self.port == 0 and self.sockets:
            self.port = self.sockets[0].getsockname()[1]
        if self.timeout_keep_alive or self.timeout_request:
            self._sweeper = self.loop.create_task(self._sweep())
        self.started = True

    async def _sweep(self) -> None:
        ts = [t for t in (self.timeout_keep_alive, self.timeout_request) if t]
        period = min(1.0, max(0.02, min(ts) / 4))
        ka, rq = self.timeout_keep_alive, self.timeout_request
        while True:
            await asyncio.sleep(period)
            now = self.loop.time()
            for c in list(self.connections):
                c.check_deadline(now, ka, rq)

    async def serve(self) -> None:
        restore = self._install_signals()
        try:
            await self.startup()
            self._exit_event = asyncio.Event()
            while not self.should_exit:
                try:
                    await asyncio.wait_for(self._exit_event.wait(), timeout=0.1)
                except asyncio.TimeoutError:
                    pass
            await self.shutdown()
        finally:
            restore()

    async def shutdown(self) -> None:
        if self._sweeper is not None:
            self._sweeper.cancel()
        if self._server is not None:
            self._server.close()
        for c in list(self.connections):
            c.shutdown_idle()
        t_end = self.loop.time() + self.timeout_graceful_shutdown
        while any(c.task is not None for c in self.connections) and self.loop.time() < t_end:
            await asyncio.sleep(0.02)
        for c in list(self.connections):
            if not c.closed:
                c.transport.close()
                c.closed = True
        if self._server is not None:
            await self._server.wait_closed()
        await self._lifespan_stop()

    def _install_signals(self) -> Callable[[], None]:
        if not self.install_signal_handlers or threading.current_thread() is not threading.main_thread():
            return lambda: None
        prev = {}

        def handler(sig, frame):
            self.should_exit = True
            if self._exit_event is not None and self.loop is not None:
                self.loop.call_soon_threadsafe(self._exit_event.set)

        for s in (signal.SIGINT, signal.SIGTERM):
            try:
                prev[s] = signal.signal(s, handler)
            except (ValueError, OSError):
                pass

        def restore():
            for s, h in prev.items():
                try:
                    signal.signal(s, h)
                except (ValueError, OSError):
                    pass
        return restore


def run(app: Any, host: str = "0.0.0.0", port: int = 8000, **kw) -> None:
    """Blocking entry (``python main.py``): serve until SIGINT/SIGTERM."""
    asyncio.run(Server(app, host, port, install_signal_handlers=True, **kw).serve())


def make_server(app: Any, host: str, port: int, kind: str = "vgate", log_level: str = "warning"):
    """An in-process server object with ``started`` / ``should_exit`` / ``serve()`` for an embedding
    script (bench.py, tools): ``kind`` "vgate" (this module) or "uvicorn". Neither installs signal
    handlers: the embedding script stops it by setting ``should_exit``."""
    if kind == "uvicorn":
        import contextlib

        import uvicorn
        srv = uvicorn.Server(uvicorn.Config(app, host=host, port=port, log_level=log_level, access_log=False,
                                            lifespan="on"))
        srv.capture_signals = contextlib.nullcontext
        return srv
    if kind != "vgate":
        raise ValueError(f"server kind must be vgate or uvicorn, got {kind!r}")
    return Server(app, host, port)
