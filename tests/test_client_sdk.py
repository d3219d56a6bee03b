"""vgate-client SDK tests (parity with reference vgate-client/tests/*: init, chat/embeddings/
health/stats, error mapping, retry policy, SSE streaming incl. early close / missing [DONE] /
in-band errors), driven through httpx.MockTransport — plus one end-to-end pass of the async
client against this repo's own FastAPI gateway (dry-run backend) over httpx.ASGITransport."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import httpx
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "vgate-client"))

import vgate_client  # noqa: E402
from vgate_client import (AsyncVGate, AuthenticationError, ChatCompletion, ChatCompletionChunk,  # noqa: E402
                          ConnectionError, EmbeddingResponse, HealthResponse, RateLimitError, ServerError,
                          VGate, VGateError)
from vgate_client.client import STREAM_DONE, parse_sse_line  # noqa: E402

MSG = [{"role": "user", "content": "hi"}]
CHAT = {"id": "chatcmpl-1", "object": "chat.completion", "created": 1, "model": "m",
        "choices": [{"index": 0, "message": {"role": "assistant", "content": "hello"}, "finish_reason": "stop"}],
        "usage": {"prompt_tokens": 3, "completion_tokens": 1, "total_tokens": 4}}
EMB = {"object": "list", "data": [{"object": "embedding", "embedding": [0.1, 0.2], "index": 0}], "model": "m",
       "usage": {"prompt_tokens": 1, "completion_tokens": 0, "total_tokens": 1}}


def chunk(delta: dict, finish=None) -> str:
    return "data: " + json.dumps({"id": "c", "object": "chat.completion.chunk", "created": 1, "model": "m",
                                  "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}) + "\n\n"


SSE_OK = chunk({"role": "assistant"}) + chunk({"content": "he"}) + chunk({"content": "llo"}) + \
    chunk({}, "stop") + "data: [DONE]\n\n"


class Recorder:
    """Route table + call log for httpx.MockTransport."""

    def __init__(self, responder):
        self.responder = responder
        self.calls: list[httpx.Request] = []

    def __call__(self, request: httpx.Request) -> httpx.Response:
        self.calls.append(request)
        return self.responder(request, len(self.calls))


def sync_client(responder, **kw):
    rec = Recorder(responder)
    return VGate(transport=httpx.MockTransport(rec), **kw), rec


def async_client(responder, **kw):
    rec = Recorder(responder)
    return AsyncVGate(transport=httpx.MockTransport(rec), **kw), rec


def sse(body: str, status=200, ctype="text/event-stream"):
    return httpx.Response(status, content=body.encode(), headers={"content-type": ctype})


@pytest.fixture(autouse=True)
def no_sleep(monkeypatch):
    slept = []
    monkeypatch.setattr("vgate_client.client._sleep", lambda s: slept.append(s))

    async def asleep(s):
        slept.append(s)
    monkeypatch.setattr("vgate_client.client._asleep", asleep)
    return slept


# ------------------------------------------------------------------ init/basics
def test_version_and_exports():
    assert vgate_client.__version__ == "0.1.0"
    for name in vgate_client.__all__:
        assert hasattr(vgate_client, name)


def test_init_defaults_and_headers():
    c = VGate()
    assert c.base_url == "http://localhost:8000"
    assert "Authorization" not in c._http.headers
    c.close()
    with VGate(base_url="http://h:9000/", api_key="sk-1") as c2:
        assert c2.base_url == "http://h:9000"
        assert c2._http.headers["Authorization"] == "Bearer sk-1"


def test_chat_create_sends_body_and_parses():
    c, rec = sync_client(lambda r, n: httpx.Response(200, json=CHAT))
    out = c.chat.create(model="m", messages=MSG, temperature=0.1, top_p=0.5, max_tokens=7)
    assert isinstance(out, ChatCompletion) and out.choices[0].message.content == "hello"
    body = json.loads(rec.calls[0].content)
    assert body == {"model": "m", "messages": MSG, "temperature": 0.1, "top_p": 0.5, "max_tokens": 7,
                    "stream": False}
    assert rec.calls[0].url.path == "/v1/chat/completions"


def test_embeddings_health_stats():
    def resp(r, n):
        return {"/v1/embeddings": httpx.Response(200, json=EMB),
                "/health": httpx.Response(200, json={"status": "ok", "version": "0.1.0"}),
                "/stats": httpx.Response(200, json={"cache": {"hits": 1}})}[r.url.path]
    c, _ = sync_client(resp)
    assert isinstance(c.embeddings.create(model="m", input="x"), EmbeddingResponse)
    h = c.health()
    assert isinstance(h, HealthResponse) and h.status == "ok"
    assert c.stats() == {"cache": {"hits": 1}}


def test_rate_limit_info_from_headers():
    c, _ = sync_client(lambda r, n: httpx.Response(200, json=CHAT, headers={
        "X-RateLimit-Limit": "60", "X-RateLimit-Remaining": "59", "X-RateLimit-Reset": "12.5"}))
    c.chat.create(model="m", messages=MSG)
    info = c.rate_limit_info()
    assert (info.limit, info.remaining, info.reset, info.retry_after) == (60, 59, 12.5, None)


# ---------------------------------------------------------------- error mapping
@pytest.mark.parametrize("status,exc", [(401, AuthenticationError), (429, RateLimitError), (500, ServerError),
                                        (503, ServerError), (422, VGateError), (404, VGateError)])
def test_error_mapping(status, exc):
    c, _ = sync_client(lambda r, n: httpx.Response(status, json={"detail": "nope"}, headers={"Retry-After": "3"}),
                       max_retries=0)
    with pytest.raises(exc) as ei:
        c.chat.create(model="m", messages=MSG)
    assert ei.value.status_code == status
    assert "nope" in str(ei.value)
    if status == 429:
        assert ei.value.retry_after == 3.0


def test_connection_error():
    def boom(r, n):
        raise httpx.ConnectError("refused", request=r)
    c, _ = sync_client(boom)
    with pytest.raises(ConnectionError):
        c.health()
    with pytest.raises(ConnectionError):
        list(c.chat.stream(model="m", messages=MSG))


def test_exception_hierarchy():
    for e in (AuthenticationError("a"), RateLimitError("b"), ServerError("c"), ConnectionError("d")):
        assert isinstance(e, VGateError)
    assert RateLimitError("x", retry_after=2.0).retry_after == 2.0


# ---------------------------------------------------------------- retry policy
def test_retry_429_uses_retry_after_then_succeeds(no_sleep):
    c, rec = sync_client(lambda r, n: httpx.Response(429, json={"detail": "slow"}, headers={"Retry-After": "1.5"})
                         if n == 1 else httpx.Response(200, json=CHAT), max_retries=2)
    assert c.chat.create(model="m", messages=MSG).id == "chatcmpl-1"
    assert len(rec.calls) == 2 and no_sleep == [1.5]


def test_retry_5xx_exponential_then_exhausted(no_sleep):
    c, rec = sync_client(lambda r, n: httpx.Response(502, json={"detail": "bad"}), max_retries=2)
    with pytest.raises(ServerError):
        c.chat.create(model="m", messages=MSG)
    assert len(rec.calls) == 3 and no_sleep == [1.0, 2.0]


def test_no_retry_on_4xx(no_sleep):
    c, rec = sync_client(lambda r, n: httpx.Response(400, json={"detail": "bad"}), max_retries=5)
    with pytest.raises(VGateError):
        c.chat.create(model="m", messages=MSG)
    assert len(rec.calls) == 1 and no_sleep == []


def test_streams_are_never_retried(no_sleep):
    c, rec = sync_client(lambda r, n: httpx.Response(503, json={"detail": "down"}), max_retries=3)
    with pytest.raises(ServerError):
        list(c.chat.stream(model="m", messages=MSG))
    assert len(rec.calls) == 1


# -------------------------------------------------------------------- SSE parse
def test_parse_sse_line_variants():
    assert parse_sse_line("") is None
    assert parse_sse_line(": keep-alive comment") is None
    assert parse_sse_line("event: message") is None
    assert parse_sse_line("data: [DONE]") is STREAM_DONE
    assert parse_sse_line("data:[DONE]") is STREAM_DONE
    c = parse_sse_line(chunk({"content": "x"}).strip())
    assert isinstance(c, ChatCompletionChunk) and c.choices[0].delta.content == "x"
    nospace = "data:" + chunk({"content": "y"}).strip()[6:]
    assert parse_sse_line(nospace).choices[0].delta.content == "y"
    with pytest.raises(ServerError, match="engine exploded"):
        parse_sse_line('data: {"error": {"message": "engine exploded"}}')


# ------------------------------------------------------------------ sync stream
def test_sync_stream_chunks_and_body():
    c, rec = sync_client(lambda r, n: sse(": ping\n\n" + SSE_OK))
    chunks = list(c.chat.stream(model="m", messages=MSG))
    assert [ch.choices[0].delta.content for ch in chunks] == [None, "he", "llo", None]
    assert chunks[0].choices[0].delta.role == "assistant" and chunks[-1].choices[0].finish_reason == "stop"
    assert json.loads(rec.calls[0].content)["stream"] is True


def test_sync_stream_missing_done_and_error_event():
    c, _ = sync_client(lambda r, n: sse(chunk({"content": "a"})))
    with pytest.raises(ServerError, match="DONE"):
        list(c.chat.stream(model="m", messages=MSG))
    c2, _ = sync_client(lambda r, n: sse(chunk({"content": "a"}) + 'data: {"error": {"message": "oom"}}\n\n'))
    got = []
    with pytest.raises(ServerError, match="oom"):
        for ch in c2.chat.stream(model="m", messages=MSG):
            got.append(ch)
    assert len(got) == 1


def test_sync_stream_wrong_content_type():
    c, _ = sync_client(lambda r, n: sse("{}", ctype="application/json"))
    with pytest.raises(VGateError, match="text/event-stream"):
        list(c.chat.stream(model="m", messages=MSG))


class TrackingStream(httpx.SyncByteStream):
    def __init__(self, body: bytes):
        self.body, self.closed = body, False

    def __iter__(self):
        for line in self.body.split(b"\n\n"):
            yield line + b"\n\n"

    def close(self):
        self.closed = True


def test_sync_stream_early_break_closes_connection():
    streams = []

    def resp(r, n):
        s = TrackingStream(SSE_OK.encode())
        streams.append(s)
        return httpx.Response(200, stream=s, headers={"content-type": "text/event-stream"})
    c, _ = sync_client(resp)
    with c.chat.stream(model="m", messages=MSG) as st:
        next(st)
    assert streams[-1].closed
    st2 = c.chat.stream(model="m", messages=MSG)
    next(st2)
    st2.close()
    assert streams[-1].closed


# ----------------------------------------------------------------- async client
async def test_async_chat_embeddings_health_errors():
    def resp(r, n):
        p = r.url.path
        if p == "/v1/chat/completions":
            return httpx.Response(200, json=CHAT)
        if p == "/v1/embeddings":
            return httpx.Response(200, json=EMB)
        if p == "/health":
            return httpx.Response(200, json={"status": "ok", "version": "0.1.0"})
        return httpx.Response(401, json={"detail": "bad key"})
    async with AsyncVGate(transport=httpx.MockTransport(Recorder(resp)), api_key="k") as c:
        assert (await c.chat.create(model="m", messages=MSG)).choices[0].message.content == "hello"
        assert (await c.embeddings.create(model="m", input="x")).data[0].embedding == [0.1, 0.2]
        assert (await c.health()).status == "ok"
        with pytest.raises(AuthenticationError):
            await c.stats()


async def test_async_retry_and_connection_error(no_sleep):
    c, rec = async_client(lambda r, n: httpx.Response(429, json={}) if n == 1 else httpx.Response(200, json=CHAT))
    await c.chat.create(model="m", messages=MSG)
    assert len(rec.calls) == 2 and no_sleep == [1.0]  # no Retry-After -> 2**0

    def boom(r, n):
        raise httpx.ConnectError("refused", request=r)
    c2, _ = async_client(boom)
    with pytest.raises(ConnectionError):
        await c2.health()


async def test_async_stream_paths():
    c, _ = async_client(lambda r, n: sse(SSE_OK))
    got = [ch async for ch in c.chat.stream(model="m", messages=MSG)]
    assert "".join(ch.choices[0].delta.content or "" for ch in got) == "hello"
    c2, _ = async_client(lambda r, n: sse(chunk({"content": "a"})))
    with pytest.raises(ServerError):
        async for _ in c2.chat.stream(model="m", messages=MSG):
            pass
    c3, _ = async_client(lambda r, n: httpx.Response(429, json={"detail": "x"}))
    with pytest.raises(RateLimitError):
        async for _ in c3.chat.stream(model="m", messages=MSG):
            pass
    c4, _ = async_client(lambda r, n: sse(SSE_OK))
    async with c4.chat.stream(model="m", messages=MSG) as st:
        first = await st.__anext__()
        assert first.choices[0].delta.role == "assistant"


# ------------------------------------------------- end-to-end against our gateway
async def test_async_client_against_own_gateway(clean_env):
    from vgate.api.app import create_app
    from vgate.backends.base import DryRunBackend
    from vgate.config import get_config
    from vgate.engine import VGateEngine
    c = get_config()
    eng = VGateEngine(model_config=c.model, worker_config=c.worker, backend=DryRunBackend(), dry_run=True)
    app = create_app(c, engine=eng)
    transport = httpx.ASGITransport(app=app)
    async with app.router.lifespan_context(app), AsyncVGate(base_url="http://gw", transport=transport) as c:
        h = await c.health()
        assert h.status in ("ok", "healthy")
        r = await c.chat.create(model="m", messages=MSG, max_tokens=8)
        assert r.choices[0].message.role == "assistant"
        chunks = [ch async for ch in c.chat.stream(model="m", messages=MSG, max_tokens=8)]
        assert chunks and chunks[-1].choices[0].finish_reason is not None
