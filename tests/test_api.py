"""HTTP surface (in-process ASGI): routes, SSE framing, status mapping, /stats, /metrics, /v1/benchmark."""
import asyncio
import json

import httpx
import pytest
from prometheus_client import REGISTRY

from vgate.api.app import create_app, messages_to_prompt, ChatMessage
from vgate.backends.base import DryRunBackend
from vgate.config import VGateConfig
from vgate.engine import VGateEngine
from vgate.worker_registry import NoHealthyWorkersError


def _metric(name, labels=None):
    v = REGISTRY.get_sample_value(name, labels or {})
    return v or 0.0


class FakeStreamBackend(DryRunBackend):
    def __init__(self, pieces=("Hel", "lo", " world"), fail_after=None, delay=0.0):
        self.pieces = pieces
        self.fail_after = fail_after
        self.delay = delay
        self.closed = False

    async def stream_generate(self, prompt, sp):
        try:
            for i, p in enumerate(self.pieces):
                if self.fail_after is not None and i == self.fail_after:
                    raise RuntimeError("stream broke")
                await asyncio.sleep(self.delay)
                yield {"delta": p, "num_tokens": i + 1}
        finally:
            self.closed = True


class NoStream(DryRunBackend):
    supports_streaming = False


class Unhealthy(DryRunBackend):
    async def agenerate(self, prompt, sp):
        raise NoHealthyWorkersError("none")


def make(backend=None, **cfg):
    c = VGateConfig(**cfg)
    eng = VGateEngine(model_config=c.model, worker_config=c.worker, backend=backend or DryRunBackend(), dry_run=True)
    return create_app(c, engine=eng)


async def _run(app, fn):
    async with app.router.lifespan_context(app):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            return await fn(c)


BODY = {"model": "m", "messages": [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hi"}]}


def test_messages_to_prompt_format():
    p = messages_to_prompt([ChatMessage(role="system", content="a"), ChatMessage(role="user", content="b")])
    assert p == "System: a\nUser: b\nAssistant:"


async def test_chat_completion_shape_and_headers():
    async def go(c):
        r = await c.post("/v1/chat/completions", json=BODY)
        assert r.status_code == 200 and len(r.headers["x-request-id"]) >= 8
        d = r.json()
        assert d["id"].startswith("chatcmpl-") and d["object"] == "chat.completion" and d["model"] == "m"
        assert d["choices"][0]["message"]["role"] == "assistant"
        assert d["choices"][0]["message"]["content"].startswith("[dry-run] echo: System: be brief")
        assert d["usage"]["completion_tokens"] == 8
        assert d["choices"][0]["finish_reason"] == "stop"
    await _run(make(), go)


@pytest.mark.parametrize("bad", [{"model": "m"}, {"messages": []}, {"model": "m", "messages": [{"role": "u"}]},
                                 {"model": "m", "messages": [], "temperature": -1},
                                 {"model": "m", "messages": [], "max_tokens": 0}])
async def test_validation_422(bad):
    async def go(c):
        assert (await c.post("/v1/chat/completions", json=bad)).status_code == 422
    await _run(make(), go)


async def test_streaming_framing_and_metrics():
    before_tok = _metric("vgate_stream_tokens_total")
    before_ok = _metric("vgate_stream_requests_total", {"status": "completed"})

    async def go(c):
        r = await c.post("/v1/chat/completions", json={**BODY, "stream": True})
        assert r.status_code == 200 and r.headers["content-type"].startswith("text/event-stream")
        lines = [ln for ln in r.text.split("\n\n") if ln]
        assert lines[-1] == "data: [DONE]"
        chunks = [json.loads(ln[6:]) for ln in lines[:-1]]
        assert chunks[0]["choices"][0]["delta"] == {"role": "assistant"}
        assert "".join(ch["choices"][0]["delta"].get("content", "") for ch in chunks) == "Hello world"
        assert chunks[-1]["choices"][0]["delta"] == {} and chunks[-1]["choices"][0]["finish_reason"] == "stop"
        assert len({ch["id"] for ch in chunks}) == 1 and all(ch["object"] == "chat.completion.chunk" for ch in chunks)
    await _run(make(FakeStreamBackend()), go)
    assert _metric("vgate_stream_tokens_total") - before_tok == 3
    assert _metric("vgate_stream_requests_total", {"status": "completed"}) - before_ok == 1


async def test_stream_error_in_band_then_done():
    before = _metric("vgate_stream_requests_total", {"status": "error"})

    async def go(c):
        r = await c.post("/v1/chat/completions", json={**BODY, "stream": True})
        parts = [p for p in r.text.split("\n\n") if p]
        err = json.loads(parts[-2][6:])
        assert err["error"]["type"] == "RuntimeError" and parts[-1] == "data: [DONE]"
    await _run(make(FakeStreamBackend(fail_after=1)), go)
    assert _metric("vgate_stream_requests_total", {"status": "error"}) - before == 1


async def test_stream_cancelled_closes_backend_generator():
    be = FakeStreamBackend(pieces=tuple("abcdefghij"), delay=0.02)
    app = make(be)
    from vgate.api.app import _stream_chat, ChatCompletionRequest

    async def go(c):
        st = app.state.vgate
        gen = _stream_chat(st, "p", ChatCompletionRequest(**{**BODY, "stream": True}))
        await gen.__anext__()
        await gen.__anext__()
        await gen.aclose()  # client disconnect
        await asyncio.sleep(0.01)
        assert be.closed
    before = _metric("vgate_stream_requests_total", {"status": "cancelled"})
    await _run(app, go)
    assert _metric("vgate_stream_requests_total", {"status": "cancelled"}) - before == 1


async def test_501_when_backend_cannot_stream():
    async def go(c):
        assert (await c.post("/v1/chat/completions", json={**BODY, "stream": True})).status_code == 501
    await _run(make(NoStream()), go)


async def test_503_retry_after_on_no_workers():
    async def go(c):
        r = await c.post("/v1/chat/completions", json=BODY)
        assert r.status_code == 503 and r.headers["retry-after"] == "5"
    await _run(make(Unhealthy()), go)


async def test_health_stats_metrics_models_ready():
    async def go(c):
        assert (await c.get("/health")).json() == {"status": "ok", "version": "0.3.2", "role": "gateway"}
        assert (await c.get("/ready")).status_code == 200
        await c.post("/v1/chat/completions", json=BODY)
        await c.post("/v1/chat/completions", json=BODY)  # cache hit
        s = (await c.get("/stats")).json()
        assert set(s["batcher"]) == {"total_requests", "total_batches", "average_batch_size", "pending_requests",
                                     "total_deduplicated", "avg_queue_time_s", "avg_ttft_s", "avg_tpot_s"}
        assert s["cache"]["hits"] == 1 and s["batcher"]["total_requests"] == 1
        assert s["config"]["batch"]["max_batch_size"] == 8 and s["version"] == "0.3.2"
        m = await c.get("/metrics")
        assert "vgate_requests_total" in m.text and "vgate_cache_hits_total" in m.text
        om = await c.get("/metrics", headers={"accept": "application/openmetrics-text"})
        assert om.headers["content-type"].startswith("application/openmetrics-text")
        assert (await c.get("/v1/models")).json()["data"][0]["id"]
    await _run(make(), go)


async def test_benchmark_endpoint_shape():
    async def go(c):
        r = await c.post("/v1/benchmark", json={"prompts": ["a", "b"], "rounds": 2, "max_tokens": 8})
        d = r.json()
        assert d["rounds"] == 2 and d["prompts_per_round"] == 2
        for k in ("latency", "ttft", "tpot", "batching", "cache", "throughput"):
            assert k in d
        assert d["cache"]["hits"] == 2  # second round fully cached
        assert d["throughput"]["total_tokens"] == 32
    await _run(make(), go)


async def test_embeddings_mock_shape():
    async def go(c):
        d = (await c.post("/v1/embeddings", json={"model": "e", "input": "hello"})).json()
        assert d["object"] == "list" and len(d["data"][0]["embedding"]) == 1536
        assert d["usage"] == {"prompt_tokens": 5, "total_tokens": 5} and d["model"] == "e"
    await _run(make(), go)


async def test_worker_role_hides_client_routes_and_serves_internal():
    async def go(c):
        assert (await c.post("/v1/chat/completions", json=BODY)).status_code == 404
        assert (await c.get("/stats")).status_code == 404
        assert (await c.get("/health")).json()["role"] == "worker"
        r = await c.post("/internal/generate", json={"prompts": ["x", "y"], "sampling_params": {"max_tokens": 4}})
        assert r.status_code == 200 and len(r.json()["results"]) == 2
        assert (await c.post("/internal/generate", json={"prompts": []})).status_code == 422
        r = await c.post("/internal/generate_stream", json={"prompt": "one two", "sampling_params": {"max_tokens": 8}})
        assert r.text.rstrip().endswith("data: [DONE]")
    await _run(make(role="worker"), go)


async def test_security_on_app():
    app = make(security={"enabled": True, "api_keys": [{"key": "k", "name": "n", "rate_limit": 1}]})

    async def go(c):
        assert (await c.get("/health")).status_code == 200  # exempt
        assert (await c.post("/v1/chat/completions", json=BODY)).status_code == 401
        h = {"Authorization": "Bearer k"}
        r = await c.post("/v1/chat/completions", json=BODY, headers=h)
        assert r.status_code == 200 and r.headers["X-RateLimit-Limit"] == "1" and "x-request-id" in r.headers
        assert (await c.post("/v1/chat/completions", json=BODY, headers=h)).status_code == 429
    await _run(app, go)
