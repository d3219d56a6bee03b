"""vgate.api.server (lean HTTP/1.1 ASGI server), vgate.utils.http1 (keep-alive client) and the
chat fast lane (vgate.api.app.ChatFastLane): protocol behaviour over real sockets, and the fast
lane's responses byte-identical to the FastAPI route's for valid and invalid bodies."""
import asyncio
import json
import socket

import aiohttp
import httpx
import pytest

from vgate.api.app import create_app
from vgate.api.server import Server
from vgate.backends.base import DryRunBackend
from vgate.config import VGateConfig
from vgate.engine import VGateEngine
from vgate.utils.http1 import Http1Pool
from vgate.worker_registry import NoHealthyWorkersError


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Streamer(DryRunBackend):
    def __init__(self, n=5, delay=0.0):
        self.n, self.delay, self.closed = n, delay, False

    async def stream_generate(self, prompt, sp):
        try:
            for i in range(self.n):
                await asyncio.sleep(self.delay)
                yield {"delta": f"t{i} ", "num_tokens": i + 1}
        finally:
            self.closed = True


class Failing(DryRunBackend):
    def __init__(self, exc):
        self.exc = exc

    async def agenerate(self, prompt, sp):
        raise self.exc


def make(backend=None, fast_lane=True, **cfg):
    c = VGateConfig(**cfg)
    eng = VGateEngine(model_config=c.model, worker_config=c.worker, backend=backend or DryRunBackend(), dry_run=True)
    return create_app(c, engine=eng, fast_lane=fast_lane)


async def _serve(app, fn):
    srv = Server(app, "127.0.0.1", _free_port())
    task = asyncio.create_task(srv.serve())
    while not srv.started:
        assert not task.done(), task
        await asyncio.sleep(0.01)
    try:
        return await fn(srv.port)
    finally:
        srv.should_exit = True
        await asyncio.wait_for(task, 10)


BODY = {"model": "m", "messages": [{"role": "user", "content": "hi there"}], "max_tokens": 4}


async def test_health_keepalive_and_headers():
    async def go(port):
        pool = Http1Pool("127.0.0.1", port)
        for _ in range(5):
            st, hdr, body = await pool.request("GET", "/health")
            assert st == 200 and json.loads(body)["status"] == "ok"
            assert len(hdr["x-request-id"]) == 8 and hdr["content-type"] == "application/json"
        assert len(pool._all) == 1  # one keep-alive connection served all five
        await pool.close()
        async with aiohttp.ClientSession() as s:  # a third-party client agrees
            async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions", json=BODY) as r:
                assert r.status == 200
                d = await r.json()
                assert d["object"] == "chat.completion" and d["choices"][0]["message"]["content"].startswith("[dry-run]")
            async with s.get(f"http://127.0.0.1:{port}/nope") as r:
                assert r.status == 404
    await _serve(make(), go)


async def test_pipelining_chunked_body_and_close():
    async def go(port):
        r, w = await asyncio.open_connection("127.0.0.1", port)
        body = json.dumps(BODY).encode()
        chunked = b"%x\r\n%s\r\n%x\r\n%s\r\n0\r\n\r\n" % (5, body[:5], len(body) - 5, body[5:])
        w.write(b"GET /health HTTP/1.1\r\nhost: x\r\n\r\n"
                b"POST /v1/chat/completions HTTP/1.1\r\nhost: x\r\ncontent-type: application/json\r\n"
                b"transfer-encoding: chunked\r\n\r\n" + chunked +
                b"GET /health HTTP/1.1\r\nhost: x\r\nconnection: close\r\n\r\n")
        await w.drain()
        data = await asyncio.wait_for(r.read(), 10)  # the server closes after the third response
        w.close()
        assert data.count(b"HTTP/1.1 200 OK") == 3
        assert b"chat.completion" in data and data.rstrip().endswith(b"}")
        assert b"connection: close" in data.split(b"HTTP/1.1 200 OK")[-1]
    await _serve(make(), go)


async def test_http10_and_garbage():
    async def go(port):
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(b"GET /health HTTP/1.0\r\n\r\n")
        data = await asyncio.wait_for(r.read(), 10)
        assert data.startswith(b"HTTP/1.1 200 OK") and b'"status":"ok"' in data
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(b"NONSENSE\r\n\r\n")
        data = await asyncio.wait_for(r.read(), 10)
        assert data.startswith(b"HTTP/1.1 400")
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(b"POST /v1/chat/completions HTTP/1.1\r\ncontent-length: 99999999999\r\n\r\n")
        data = await asyncio.wait_for(r.read(), 10)
        assert data.startswith(b"HTTP/1.1 413")
    await _serve(make(), go)


async def test_sse_stream_over_socket_and_disconnect_aborts():
    be = Streamer(n=5)

    async def go(port):
        async with aiohttp.ClientSession() as s:
            async with s.post(f"http://127.0.0.1:{port}/v1/chat/completions", json=dict(BODY, stream=True)) as r:
                assert r.status == 200 and r.headers["content-type"].startswith("text/event-stream")
                assert r.headers.get("transfer-encoding") == "chunked"
                text = (await r.read()).decode()
        events = [ln[6:] for ln in text.split("\n") if ln.startswith("data: ")]
        assert events[-1] == "[DONE]"
        deltas = [json.loads(e)["choices"][0]["delta"] for e in events[:-1]]
        assert deltas[0] == {"role": "assistant"} and "".join(d.get("content", "") for d in deltas) == "t0 t1 t2 t3 t4 "
        # a client that goes away mid-stream: the generator is closed (the engine would abort)
        slow = Streamer(n=1000, delay=0.01)
        app2 = make(backend=slow)

        async def go2(port2):
            r, w = await asyncio.open_connection("127.0.0.1", port2)
            b = json.dumps(dict(BODY, stream=True)).encode()
            w.write(b"POST /v1/chat/completions HTTP/1.1\r\nhost: x\r\ncontent-type: application/json\r\n"
                    b"content-length: %d\r\n\r\n%s" % (len(b), b))
            await w.drain()
            await r.readuntil(b"t2 ")
            w.close()
            for _ in range(200):
                if slow.closed:
                    break
                await asyncio.sleep(0.02)
            assert slow.closed
        await _serve(app2, go2)
    await _serve(make(backend=be), go)


async def test_http1_client_against_uvicorn_chunked():
    import uvicorn
    app = make(backend=Streamer(n=3))
    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    task = asyncio.create_task(srv.serve())
    while not srv.started:
        await asyncio.sleep(0.01)
    try:
        pool = Http1Pool("127.0.0.1", port)
        st, hdr, body = await pool.request("POST", "/v1/chat/completions", json.dumps(dict(BODY, stream=True)).encode())
        assert st == 200 and hdr.get("transfer-encoding") == "chunked" and body.endswith(b"data: [DONE]\n\n")
        st, _, body = await pool.request("POST", "/v1/chat/completions", json.dumps(BODY).encode())
        assert st == 200 and json.loads(body)["usage"]["completion_tokens"] == 8
        await pool.close()
    finally:
        srv.should_exit = True
        await task


def _norm(body: bytes):
    try:
        d = json.loads(body)
    except ValueError:
        return body
    if isinstance(d, dict):
        d.pop("id", None)
        d.pop("created", None)
    return d


BODIES = [
    (json.dumps(BODY).encode(), "application/json"),
    (json.dumps(dict(BODY, temperature=0.0, top_p=1.0)).encode(), "application/json"),
    (json.dumps(dict(BODY, extra_field=1)).encode(), "application/json"),
    (json.dumps(dict(BODY, max_tokens="3")).encode(), "application/json"),  # lax coercion
    (b'{"model": "m"}', "application/json"),
    (b'{"model": "m", "messages": [{"role": "u"}]}', "application/json"),
    (json.dumps(dict(BODY, temperature=-1)).encode(), "application/json"),
    (json.dumps(dict(BODY, max_tokens=0)).encode(), "application/json"),
    (json.dumps(dict(BODY, top_p=0)).encode(), "application/json"),
    (b'{"model": "m", "messages": [', "application/json"),  # invalid JSON
    (b"", "application/json"),
    (b"[1, 2]", "application/json"),
    (json.dumps(BODY).encode(), "text/plain"),
    (json.dumps(BODY).encode(), "application/json; charset=utf-8"),
    (json.dumps(BODY).encode(), None),
]


@pytest.mark.parametrize("backend", ["ok", "nohealthy", "boom"])
async def test_fast_lane_matches_fastapi_route(backend):
    def be():
        return {"ok": DryRunBackend(), "nohealthy": Failing(NoHealthyWorkersError("no healthy workers")),
                "boom": Failing(ValueError("kaput"))}[backend]
    out = {}
    for fast in (True, False):
        app = make(backend=be(), fast_lane=fast, cache={"enabled": False})
        res = []
        async with app.router.lifespan_context(app):
            async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
                for body, ctype in BODIES:
                    h = {"content-type": ctype} if ctype else {}
                    r = await c.post("/v1/chat/completions", content=body, headers=h)
                    hdrs = [(k, v) for k, v in r.headers.raw if k.lower() != b"x-request-id"
                            and k.lower() != b"content-length"]
                    res.append((r.status_code, hdrs, _norm(r.content)))
        out[fast] = res
    for i, (a, b) in enumerate(zip(out[True], out[False])):
        assert a == b, (i, BODIES[i], a, b)
    statuses = [r[0] for r in out[True]]
    if backend == "ok":
        assert statuses.count(200) >= 5 and 422 in statuses
    elif backend == "nohealthy":
        assert 503 in statuses and any((b"retry-after", b"5") in r[1] for r in out[True])
    else:
        assert 500 in statuses


async def test_fast_lane_is_used():
    """The fast lane serves a valid request without FastAPI's dependency solving."""
    import fastapi.dependencies.utils as fdu
    calls = []
    orig = fdu.solve_dependencies

    async def spy(*a, **k):
        calls.append(1)
        return await orig(*a, **k)
    fdu.solve_dependencies = spy
    import fastapi.routing as fr
    fr.solve_dependencies = spy
    try:
        app = make()
        async with app.router.lifespan_context(app):
            async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
                r = await c.post("/v1/chat/completions", json=BODY)
                assert r.status_code == 200 and not calls
                r = await c.post("/v1/chat/completions", json={"model": "m"})
                assert r.status_code == 422 and calls  # replayed into FastAPI
    finally:
        fdu.solve_dependencies = orig
        fr.solve_dependencies = orig
