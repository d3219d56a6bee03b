"""vgate-client SDK behaviour matrix, one assertion per behaviour and every stream behaviour for
BOTH clients (sync VGate and AsyncVGate): init, request bodies, error mapping, retry policy,
exceptions, response models and SSE streaming (role/content/finish, stream flag, context-manager
exit, mid-stream error event, HTTP error before data, wrong content type, connection error,
missing [DONE], early break / explicit close releasing the connection).

Parity target: reference vgate-client/tests (test_client.py, test_exceptions.py,
test_models.py, test_streaming.py); driven through httpx.MockTransport, no network.
"""
from __future__ import annotations

import asyncio
import json
import sys
from pathlib import Path

import httpx
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "vgate-client"))

from vgate_client import (AsyncVGate, AuthenticationError, ChatCompletion, ChatCompletionChunk,  # noqa: E402
                          ConnectionError, EmbeddingResponse, HealthResponse, RateLimitError, ServerError,
                          VGate, VGateError)
from vgate_client.models import (ChatCompletionRequest, ChatMessage, EmbeddingRequest, RateLimitInfo,  # noqa: E402
                                 Usage)

MSG = [{"role": "user", "content": "hi"}]
CHAT = {"id": "chatcmpl-9", "object": "chat.completion", "created": 7, "model": "m",
        "choices": [{"index": 0, "message": {"role": "assistant", "content": "hey"}, "finish_reason": "stop"}],
        "usage": {"prompt_tokens": 2, "completion_tokens": 1, "total_tokens": 3}}


def _chunk(delta, finish=None):
    return "data: " + json.dumps({"id": "c", "object": "chat.completion.chunk", "created": 1, "model": "m",
                                  "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}) + "\n\n"


SSE = _chunk({"role": "assistant"}) + _chunk({"content": "a"}) + _chunk({"content": "b"}) + _chunk({}, "stop") + \
    "data: [DONE]\n\n"


@pytest.fixture(autouse=True)
def _no_sleep(monkeypatch):
    monkeypatch.setattr("vgate_client.client._sleep", lambda s: None)

    async def asleep(s):
        return None
    monkeypatch.setattr("vgate_client.client._asleep", asleep)


def _mk(kind, responder, **kw):
    calls = []

    def handler(request):
        calls.append(request)
        return responder(request, len(calls))
    cls = VGate if kind == "sync" else AsyncVGate
    return cls(transport=httpx.MockTransport(handler), **kw), calls


async def _run(kind, fn):
    r = fn()
    if kind == "async":
        r = await r
    return r


async def _drain(kind, stream):
    if kind == "sync":
        return list(stream)
    return [c async for c in stream]


KINDS = ["sync", "async"]


# ------------------------------------------------------------------------- init
@pytest.mark.parametrize("kind", KINDS)
def test_default_and_custom_base_url(kind):
    cls = VGate if kind == "sync" else AsyncVGate
    assert cls().base_url == "http://localhost:8000"
    assert cls(base_url="http://gw:1234/").base_url == "http://gw:1234"


@pytest.mark.parametrize("kind", KINDS)
def test_api_key_header_present_or_absent(kind):
    cls = VGate if kind == "sync" else AsyncVGate
    assert cls(api_key="sk-9")._http.headers["Authorization"] == "Bearer sk-9"
    assert "Authorization" not in cls()._http.headers


@pytest.mark.parametrize("kind", KINDS)
async def test_api_key_sent_on_the_wire(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(200, json=CHAT), api_key="sk-w")
    await _run(kind, lambda: c.chat.create(model="m", messages=MSG))
    assert calls[0].headers["authorization"] == "Bearer sk-w"


def test_sync_context_manager_closes():
    with VGate() as c:
        assert not c._http.is_closed
    assert c._http.is_closed


async def test_async_context_manager_closes():
    async with AsyncVGate() as c:
        assert not c._http.is_closed
    assert c._http.is_closed


# ------------------------------------------------------------------------- calls
@pytest.mark.parametrize("kind", KINDS)
async def test_chat_success_and_default_params(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(200, json=CHAT))
    out = await _run(kind, lambda: c.chat.create(model="m", messages=MSG))
    assert isinstance(out, ChatCompletion) and out.usage.total_tokens == 3
    body = json.loads(calls[0].content)
    assert (body["temperature"], body["top_p"], body["max_tokens"], body["stream"]) == (0.7, 0.9, 256, False)


@pytest.mark.parametrize("kind", KINDS)
async def test_chat_custom_params(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(200, json=CHAT))
    await _run(kind, lambda: c.chat.create(model="x", messages=MSG, temperature=0.0, top_p=1.0, max_tokens=3))
    body = json.loads(calls[0].content)
    assert (body["model"], body["temperature"], body["top_p"], body["max_tokens"]) == ("x", 0.0, 1.0, 3)


@pytest.mark.parametrize("kind", KINDS)
async def test_embeddings_health_stats_success(kind):
    def resp(r, n):
        return {"/v1/embeddings": httpx.Response(200, json={"object": "list", "model": "m", "data": [
            {"object": "embedding", "embedding": [1.0], "index": 0}]}),
            "/health": httpx.Response(200, json={"status": "ok", "version": "v"}),
            "/stats": httpx.Response(200, json={"k": 1})}[r.url.path]
    c, _ = _mk(kind, resp)
    assert isinstance(await _run(kind, lambda: c.embeddings.create(model="m", input="t")), EmbeddingResponse)
    assert isinstance(await _run(kind, c.health), HealthResponse)
    assert await _run(kind, c.stats) == {"k": 1}


# ----------------------------------------------------------------------- errors
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("status,exc", [(401, AuthenticationError), (429, RateLimitError), (500, ServerError),
                                        (422, VGateError)])
async def test_status_maps_to_exception(kind, status, exc):
    c, _ = _mk(kind, lambda r, n: httpx.Response(status, json={"detail": "x"}), max_retries=0)
    with pytest.raises(exc) as ei:
        await _run(kind, lambda: c.chat.create(model="m", messages=MSG))
    assert ei.value.status_code == status


@pytest.mark.parametrize("kind", KINDS)
async def test_connection_error_on_chat_and_health(kind):
    def boom(r, n):
        raise httpx.ConnectError("refused", request=r)
    c, _ = _mk(kind, boom)
    with pytest.raises(ConnectionError):
        await _run(kind, lambda: c.chat.create(model="m", messages=MSG))
    with pytest.raises(ConnectionError):
        await _run(kind, c.health)


@pytest.mark.parametrize("kind", KINDS)
async def test_retry_on_429_then_success(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(429, json={}) if n == 1 else httpx.Response(200, json=CHAT),
                   max_retries=1)
    assert (await _run(kind, lambda: c.chat.create(model="m", messages=MSG))).id == "chatcmpl-9"
    assert len(calls) == 2


@pytest.mark.parametrize("kind", KINDS)
async def test_retry_on_500_then_success(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(500, json={}) if n < 3 else httpx.Response(200, json=CHAT),
                   max_retries=3)
    await _run(kind, lambda: c.chat.create(model="m", messages=MSG))
    assert len(calls) == 3


@pytest.mark.parametrize("kind", KINDS)
async def test_exhausted_retries_raise(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(429, json={"detail": "busy"}), max_retries=2)
    with pytest.raises(RateLimitError):
        await _run(kind, lambda: c.chat.create(model="m", messages=MSG))
    assert len(calls) == 3


# ------------------------------------------------------------------- exceptions
def test_base_error_message_and_body():
    e = VGateError("boom", status_code=418, body={"detail": "teapot"})
    assert "boom" in str(e) and e.status_code == 418 and e.body == {"detail": "teapot"}
    assert VGateError("plain").status_code is None


@pytest.mark.parametrize("cls", [AuthenticationError, RateLimitError, ServerError, ConnectionError])
def test_every_error_is_catchable_as_base(cls):
    with pytest.raises(VGateError):
        raise cls("x")


def test_rate_limit_error_retry_after_optional():
    assert RateLimitError("x").retry_after is None
    assert RateLimitError("x", retry_after=4.0).retry_after == 4.0


def test_connection_error_is_not_builtin_connection_error_subclass_requirement():
    # the SDK's ConnectionError is its own class in the VGateError tree
    assert issubclass(ConnectionError, VGateError)


# ------------------------------------------------------------------------ models
def test_request_models_minimal_custom_and_serialised():
    r = ChatCompletionRequest(model="m", messages=[ChatMessage(role="user", content="x")])
    assert (r.temperature, r.top_p, r.max_tokens, r.stream) == (0.7, 0.9, 256, False)
    r2 = ChatCompletionRequest(model="m", messages=[{"role": "user", "content": "x"}], temperature=0.1, stream=True)
    d = r2.model_dump()
    assert d["temperature"] == 0.1 and d["stream"] is True and d["messages"][0]["content"] == "x"
    assert EmbeddingRequest(model="m", input="y").input == "y"


def test_response_models_parse():
    cc = ChatCompletion.model_validate(CHAT)
    assert cc.choices[0].finish_reason == "stop" and cc.object == "chat.completion"
    assert Usage().total_tokens == 0
    role = ChatCompletionChunk.model_validate(json.loads(_chunk({"role": "assistant"})[6:]))
    assert role.choices[0].delta.role == "assistant" and role.choices[0].delta.content is None
    fin = ChatCompletionChunk.model_validate(json.loads(_chunk({}, "length")[6:]))
    assert fin.choices[0].finish_reason == "length"
    assert HealthResponse.model_validate({"status": "ok", "version": "1"}).version == "1"
    assert RateLimitInfo().limit is None
    assert RateLimitInfo(limit=5, remaining=4, reset=1.0).remaining == 4


# --------------------------------------------------------------------- streaming
@pytest.mark.parametrize("kind", KINDS)
async def test_stream_yields_role_content_finish(kind):
    c, _ = _mk(kind, lambda r, n: httpx.Response(200, content=SSE.encode(),
                                                 headers={"content-type": "text/event-stream"}))
    got = await _drain(kind, c.chat.stream(model="m", messages=MSG))
    assert got[0].choices[0].delta.role == "assistant"
    assert "".join(ch.choices[0].delta.content or "" for ch in got) == "ab"
    assert got[-1].choices[0].finish_reason == "stop"


@pytest.mark.parametrize("kind", KINDS)
async def test_stream_request_body_sets_stream_true(kind):
    c, calls = _mk(kind, lambda r, n: httpx.Response(200, content=SSE.encode(),
                                                     headers={"content-type": "text/event-stream"}))
    await _drain(kind, c.chat.stream(model="m", messages=MSG))
    assert json.loads(calls[0].content)["stream"] is True


@pytest.mark.parametrize("kind", KINDS)
async def test_stream_mid_stream_error_event(kind):
    body = _chunk({"content": "a"}) + 'data: {"error": {"message": "device lost"}}\n\n'
    c, _ = _mk(kind, lambda r, n: httpx.Response(200, content=body.encode(),
                                                 headers={"content-type": "text/event-stream"}))
    with pytest.raises(ServerError, match="device lost"):
        await _drain(kind, c.chat.stream(model="m", messages=MSG))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("status,exc", [(401, AuthenticationError), (503, ServerError)])
async def test_stream_http_error_before_data(kind, status, exc):
    c, _ = _mk(kind, lambda r, n: httpx.Response(status, json={"detail": "no"}), max_retries=3)
    with pytest.raises(exc):
        await _drain(kind, c.chat.stream(model="m", messages=MSG))


@pytest.mark.parametrize("kind", KINDS)
async def test_stream_unexpected_content_type(kind):
    c, _ = _mk(kind, lambda r, n: httpx.Response(200, json=CHAT))
    with pytest.raises(VGateError):
        await _drain(kind, c.chat.stream(model="m", messages=MSG))


@pytest.mark.parametrize("kind", KINDS)
async def test_stream_connection_error(kind):
    def boom(r, n):
        raise httpx.ConnectError("refused", request=r)
    c, _ = _mk(kind, boom)
    with pytest.raises(ConnectionError):
        await _drain(kind, c.chat.stream(model="m", messages=MSG))


@pytest.mark.parametrize("kind", KINDS)
async def test_stream_missing_done_is_an_error(kind):
    c, _ = _mk(kind, lambda r, n: httpx.Response(200, content=_chunk({"content": "x"}).encode(),
                                                 headers={"content-type": "text/event-stream"}))
    with pytest.raises(ServerError):
        await _drain(kind, c.chat.stream(model="m", messages=MSG))


class _SyncTrack(httpx.SyncByteStream):
    def __init__(self):
        self.closed = False

    def __iter__(self):
        for part in SSE.split("\n\n"):
            yield (part + "\n\n").encode()

    def close(self):
        self.closed = True


class _AsyncTrack(httpx.AsyncByteStream):
    def __init__(self):
        self.closed = False

    async def __aiter__(self):
        for part in SSE.split("\n\n"):
            yield (part + "\n\n").encode()

    async def aclose(self):
        self.closed = True


def test_sync_stream_context_exit_and_explicit_close_release_connection():
    streams = []

    def resp(r, n):
        s = _SyncTrack()
        streams.append(s)
        return httpx.Response(200, stream=s, headers={"content-type": "text/event-stream"})
    c, _ = _mk("sync", resp)
    with c.chat.stream(model="m", messages=MSG) as st:
        list(st)
    assert streams[-1].closed  # normal completion
    st = c.chat.stream(model="m", messages=MSG)
    next(st)
    st.close()
    assert streams[-1].closed  # explicit close after an early stop


async def test_async_stream_early_break_and_explicit_close_release_connection():
    streams = []

    def resp(r, n):
        s = _AsyncTrack()
        streams.append(s)
        return httpx.Response(200, stream=s, headers={"content-type": "text/event-stream"})
    c, _ = _mk("async", resp)
    async with c.chat.stream(model="m", messages=MSG) as st:
        async for _ in st:
            break
    assert streams[-1].closed
    st2 = c.chat.stream(model="m", messages=MSG)
    await st2.__anext__()
    await st2.aclose()
    assert streams[-1].closed


async def test_async_stream_context_exits_on_normal_completion():
    c, _ = _mk("async", lambda r, n: httpx.Response(200, content=SSE.encode(),
                                                    headers={"content-type": "text/event-stream"}))
    async with c.chat.stream(model="m", messages=MSG) as st:
        got = [ch async for ch in st]
    assert len(got) == 4
    await asyncio.sleep(0)
