"""Gateway behaviour contracts, expressed against this code base: configuration precedence and
validation, request fan-out (dedup / cache / admission / abandonment), SSE streaming outcomes
and metrics, structured logging + trace correlation, the dry-run capacity knobs and request
validation.

Behavioural parity targets (reference files, not copied): tests/test_config.py,
test_fanout.py, test_batcher.py, test_streaming.py, test_observability.py, test_tracing.py,
test_dryrun_knobs.py, test_chat_completions.py, test_cache_log.py.
"""
import asyncio
import io
import json
import logging
import time

import httpx
import pytest

from vgate import tracing
from vgate.api.app import create_app
from vgate.backends.base import DryRunBackend
from vgate.batcher import RequestBatcher
from vgate.cache import ResultCache
from vgate.config import (BatchConfig, CacheConfig, InferenceConfig, LoggingConfig, MetricsConfig, ModelConfig,
                          ServerConfig, TracingConfig, VGateConfig, env_overrides, get_config, load_config,
                          load_yaml_config, reset_config, set_config)
from vgate.logging_config import ConsoleFormatter, JSONFormatter, LogContext, get_logger, setup_logging
from vgate.metrics import STREAM_REQUESTS, STREAM_TOKENS


# ------------------------------------------------------------------------------- config
def test_config_defaults():
    c = VGateConfig(_env={})
    assert (c.server.host, c.server.port) == ("0.0.0.0", 8000)
    assert c.batch.max_batch_size == 8 and c.batch.max_wait_time_ms == 50.0
    assert c.cache.enabled and c.cache.maxsize == 1000
    assert (c.inference.temperature, c.inference.top_p, c.inference.max_tokens) == (0.7, 0.9, 256)
    assert c.logging.level == "INFO" and c.logging.json_format
    assert c.metrics.enabled and c.role == "gateway"
    assert c.model.engine_type == "native" and c.model.max_model_len == 2048


def test_yaml_loading_and_missing_file(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("server:\n  port: 9001\nbatch:\n  max_batch_size: 3\nmodel:\n  model_id: foo/bar\n")
    assert load_yaml_config(p)["server"]["port"] == 9001
    c = load_config(p)
    assert c.server.port == 9001 and c.batch.max_batch_size == 3 and c.model.model_id == "foo/bar"
    assert c.server.host == "0.0.0.0"  # unspecified keys keep defaults
    with pytest.raises(FileNotFoundError):
        load_yaml_config(tmp_path / "missing.yaml")
    (tmp_path / "empty.yaml").write_text("")
    assert load_yaml_config(tmp_path / "empty.yaml") == {}


@pytest.mark.parametrize("var,value,path,expect", [
    ("VGATE_SERVER__PORT", "9100", ("server", "port"), 9100),
    ("VGATE_MODEL__MODEL_ID", "org/model", ("model", "model_id"), "org/model"),
    ("VGATE_BATCH__MAX_BATCH_SIZE", "32", ("batch", "max_batch_size"), 32),
    ("VGATE_CACHE__MAXSIZE", "7", ("cache", "maxsize"), 7),
    ("VGATE_LOGGING__LEVEL", "DEBUG", ("logging", "level"), "DEBUG"),
    ("VGATE_LOGGING__JSON_FORMAT", "false", ("logging", "json_format"), False),
    ("VGATE_MODEL__GPU_MEMORY_UTILIZATION", "0.5", ("model", "gpu_memory_utilization"), 0.5),
    ("VGATE_WORKER__ENDPOINTS", '["http://w:1"]', ("worker", "endpoints"), ["http://w:1"]),
])
def test_env_overrides(var, value, path, expect):
    c = VGateConfig(_env=env_overrides({var: value}))
    assert getattr(getattr(c, path[0]), path[1]) == expect


def test_env_beats_yaml_beats_defaults(tmp_path, monkeypatch):
    p = tmp_path / "c.yaml"
    p.write_text("server:\n  port: 9001\n  host: 127.0.0.9\n")
    monkeypatch.setenv("VGATE_SERVER__PORT", "9555")
    c = load_config(p)
    assert c.server.port == 9555 and c.server.host == "127.0.0.9"


def test_non_schema_env_vars_are_ignored():
    assert env_overrides({"VGATE_DRY_RUN": "true", "VGATE_CONFIG_PATH": "/x", "OTHER": "1"}) == {}


def test_config_singleton_and_reset(tmp_path, monkeypatch):
    prev = get_config()
    try:
        p = tmp_path / "c.yaml"
        p.write_text("server:\n  port: 9333\n")
        monkeypatch.setenv("VGATE_CONFIG_PATH", str(p))
        reset_config()
        a = get_config()
        assert a is get_config() and a.server.port == 9333
        reset_config()
        assert get_config() is not a
    finally:
        set_config(prev)


@pytest.mark.parametrize("kw", [{"server": {"port": "not-a-port"}}, {"batch": {"max_batch_size": "many"}},
                                {"model": {"gpu_memory_utilization": "lots"}}, {"role": "router"},
                                {"model": {"kv_block_size": 32}}])
def test_invalid_values_are_rejected(kw):
    with pytest.raises(Exception):
        VGateConfig(_env={}, **kw)


def test_section_models_construct_standalone():
    assert ServerConfig(port=1).port == 1
    assert ModelConfig(max_model_len=4096).max_model_len == 4096
    assert BatchConfig(max_batch_size=2).max_batch_size == 2
    assert CacheConfig(maxsize=3).maxsize == 3
    assert InferenceConfig(max_tokens=5).max_tokens == 5
    assert LoggingConfig(level="WARNING").level == "WARNING"
    assert MetricsConfig(enabled=False).enabled is False
    assert TracingConfig().enabled is False


# ------------------------------------------------------------------------------ fan-out
class _CountingBackend(DryRunBackend):
    """Counts backend calls; each takes `delay` seconds; optional failure."""

    def __init__(self, delay=0.05, fail=False):
        self.calls = 0
        self.delay = delay
        self.fail = fail
        self.active = 0
        self.peak = 0

    async def agenerate(self, prompt, sp):
        self.calls += 1
        self.active += 1
        self.peak = max(self.peak, self.active)
        try:
            await asyncio.sleep(self.delay)
            if self.fail:
                raise RuntimeError("backend exploded")
            return {"text": f"out:{prompt}", "token_ids": [1, 2], "num_tokens": 2, "metrics": {}}
        finally:
            self.active -= 1


class _Eng:
    def __init__(self, backend):
        self.backend = backend


def _batcher(backend, max_batch=8, cache=False):
    b = RequestBatcher(_Eng(backend), max_batch_size=max_batch)
    b.cache = ResultCache(maxsize=100, enabled=cache)
    return b


async def test_each_distinct_request_is_its_own_backend_call():
    be = _CountingBackend()
    b = _batcher(be)
    rs = await asyncio.gather(*(b.submit(f"p{i}", 4, 0.7, 0.9) for i in range(5)))
    assert be.calls == 5 and [r["text"] for r in rs] == [f"out:p{i}" for i in range(5)]


async def test_differing_sampling_params_stay_separate():
    be = _CountingBackend()
    b = _batcher(be)
    await asyncio.gather(b.submit("p", 4, 0.7, 0.9), b.submit("p", 4, 0.8, 0.9), b.submit("p", 5, 0.7, 0.9))
    assert be.calls == 3


async def test_identical_concurrent_requests_share_one_inference():
    be = _CountingBackend(delay=0.1)
    b = _batcher(be)
    rs = await asyncio.gather(*(b.submit("same", 4, 0.7, 0.9) for _ in range(6)))
    assert be.calls == 1 and len({r["text"] for r in rs}) == 1
    assert b.total_deduplicated == 5
    assert b._inflight == {}


async def test_dedup_has_no_time_window():
    be = _CountingBackend(delay=0.3)
    b = _batcher(be)
    first = asyncio.create_task(b.submit("slow", 4, 0.7, 0.9))
    await asyncio.sleep(0.2)  # far past any batching window
    second = await b.submit("slow", 4, 0.7, 0.9)
    assert (await first)["text"] == second["text"] and be.calls == 1


async def test_sequential_identical_requests_hit_cache_not_dedup():
    be = _CountingBackend(delay=0.01)
    b = _batcher(be, cache=True)
    await b.submit("c", 4, 0.7, 0.9)
    await b.submit("c", 4, 0.7, 0.9)
    assert be.calls == 1 and b.total_deduplicated == 0 and b.cache.get_stats()["hits"] == 1


async def test_failure_propagates_to_all_waiters_and_is_not_cached():
    be = _CountingBackend(delay=0.05, fail=True)
    b = _batcher(be, cache=True)
    rs = await asyncio.gather(*(b.submit("bad", 4, 0.7, 0.9) for _ in range(3)), return_exceptions=True)
    assert all(isinstance(r, RuntimeError) for r in rs) and be.calls == 1
    assert len(b.cache) == 0 and b._inflight == {}
    be.fail = False
    assert (await b.submit("bad", 4, 0.7, 0.9))["text"] == "out:bad"  # retried, not a cached failure


async def test_admission_limit_caps_concurrency():
    be = _CountingBackend(delay=0.05)
    b = _batcher(be, max_batch=3)
    await asyncio.gather(*(b.submit(f"a{i}", 4, 0.7, 0.9) for i in range(10)))
    assert be.peak == 3 and be.calls == 10


async def test_deduplicated_waiters_do_not_consume_permits():
    be = _CountingBackend(delay=0.1)
    b = _batcher(be, max_batch=2)
    same = [b.submit("dup", 4, 0.7, 0.9) for _ in range(5)]
    other = b.submit("other", 4, 0.7, 0.9)
    t0 = time.perf_counter()
    await asyncio.gather(*same, other)
    assert be.calls == 2 and time.perf_counter() - t0 < 0.19  # both ran concurrently: one permit each


async def test_abandoned_request_is_cancelled_before_admission():
    be = _CountingBackend(delay=0.2)
    b = _batcher(be, max_batch=1)
    blocker = asyncio.create_task(b.submit("first", 4, 0.7, 0.9))
    await asyncio.sleep(0.02)
    with pytest.raises(asyncio.TimeoutError):
        await b.submit("queued", 4, 0.7, 0.9, timeout=0.05)
    await blocker
    await asyncio.sleep(0.05)
    assert be.calls == 1 and b._inflight == {}  # the abandoned one never reached the backend


async def test_started_inference_survives_abandonment_and_one_waiter_leaving():
    be = _CountingBackend(delay=0.15)
    b = _batcher(be, cache=True)
    t1 = asyncio.create_task(b.submit("shared", 4, 0.7, 0.9))
    t2 = asyncio.create_task(b.submit("shared", 4, 0.7, 0.9))
    await asyncio.sleep(0.05)
    t1.cancel()
    r2 = await t2
    assert r2["text"] == "out:shared" and be.calls == 1
    # the completed work landed in the cache even though a waiter left
    assert await b.cache.get(ResultCache.make_key("shared", 0.7, 0.9, 4)) is not None


async def test_queue_time_uses_monotonic_clock(monkeypatch):
    be = _CountingBackend(delay=0.01)
    b = _batcher(be)
    real = time.time
    monkeypatch.setattr(time, "time", lambda: real() - 3600)  # a wall-clock jump backwards
    await b.submit("t", 4, 0.7, 0.9)
    assert 0 <= b.total_queue_time < 1.0


async def test_serialized_backend_runs_one_inference_at_a_time():
    class SyncBackend:
        supports_concurrent_calls = False
        active = 0
        peak = 0

        def create_sampling_params(self, temperature, top_p, max_tokens):
            return {"max_tokens": max_tokens}

        def generate(self, prompts, sp):
            SyncBackend.active += 1
            SyncBackend.peak = max(SyncBackend.peak, SyncBackend.active)
            time.sleep(0.02)
            SyncBackend.active -= 1
            return [{"text": p, "num_tokens": 1} for p in prompts]
    b = _batcher(SyncBackend(), max_batch=8)
    assert b.max_concurrent_inferences == 1
    await asyncio.gather(*(b.submit(f"s{i}", 4, 0.7, 0.9) for i in range(4)))
    assert SyncBackend.peak == 1


def test_dry_run_backend_declares_concurrency_and_streaming():
    assert DryRunBackend.supports_concurrent_calls and DryRunBackend.supports_streaming


# ------------------------------------------------------------------------------ streaming
def _app(backend=None):
    cfg = VGateConfig(_env={}, cache={"enabled": False})
    from vgate.engine import VGateEngine
    eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=backend or DryRunBackend(),
                      dry_run=True)
    return create_app(cfg, engine=eng)


def _sse_events(text):
    return [ln[len("data: "):] for ln in text.splitlines() if ln.startswith("data: ")]


async def test_stream_true_returns_role_content_and_done():
    app = _app()
    async with app.router.lifespan_context(app):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            r = await c.post("/v1/chat/completions", json={
                "model": "m", "stream": True, "messages": [{"role": "user", "content": "alpha beta"}]})
            assert r.status_code == 200 and r.headers["content-type"].startswith("text/event-stream")
            ev = _sse_events(r.text)
            assert ev[-1] == "[DONE]"
            chunks = [json.loads(e) for e in ev[:-1]]
            assert chunks[0]["choices"][0]["delta"].get("role") == "assistant"
            assert chunks[0]["object"] == "chat.completion.chunk"
            content = "".join(ch["choices"][0]["delta"].get("content", "") for ch in chunks)
            assert "alpha beta" in content
            assert chunks[-1]["choices"][0]["finish_reason"] is not None
            assert len({ch["id"] for ch in chunks}) == 1


async def test_stream_false_is_a_plain_completion():
    app = _app()
    async with app.router.lifespan_context(app):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            r = await c.post("/v1/chat/completions", json={
                "model": "m", "stream": False, "messages": [{"role": "user", "content": "plain"}]})
            body = r.json()
            assert r.status_code == 200 and body["object"] == "chat.completion"
            assert body["choices"][0]["message"]["role"] == "assistant"


async def test_successful_stream_records_metrics():
    app = _app()
    ok0 = STREAM_REQUESTS.labels(status="completed")._value.get()
    tok0 = STREAM_TOKENS._value.get()
    async with app.router.lifespan_context(app):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            await c.post("/v1/chat/completions", json={
                "model": "m", "stream": True, "messages": [{"role": "user", "content": "one two three"}]})
    assert STREAM_REQUESTS.labels(status="completed")._value.get() == ok0 + 1
    assert STREAM_TOKENS._value.get() > tok0


async def test_backend_error_mid_stream_is_an_error_event():
    class Boom(DryRunBackend):
        async def stream_generate(self, prompt, sp):
            yield {"delta": "partial ", "num_tokens": 1}
            raise RuntimeError("mid-stream fault")
    app = _app(Boom())
    err0 = STREAM_REQUESTS.labels(status="error")._value.get()
    async with app.router.lifespan_context(app):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            r = await c.post("/v1/chat/completions", json={
                "model": "m", "stream": True, "messages": [{"role": "user", "content": "x"}]})
            events = _sse_events(r.text)
            assert any("error" in e for e in events if e != "[DONE]")
    assert STREAM_REQUESTS.labels(status="error")._value.get() == err0 + 1


# ----------------------------------------------------------------- validation / errors
@pytest.mark.parametrize("messages,status", [
    ([{"role": "user", "content": "ok"}], 200),
    ([{"role": "user"}], 422),
    (["not an object"], 422),
])
async def test_chat_message_validation(messages, status):
    app = _app()
    async with app.router.lifespan_context(app):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            r = await c.post("/v1/chat/completions", json={"model": "m", "messages": messages})
            assert r.status_code == status


# ------------------------------------------------------------------------- logging
def _record(msg="hello", **attrs):
    rec = logging.LogRecord("vgate.t", logging.INFO, __file__, 1, msg, None, None)
    for k, v in attrs.items():
        setattr(rec, k, v)
    return rec


def test_json_formatter_fields_extra_and_request_id():
    out = json.loads(JSONFormatter().format(_record(extra_data={"k": 1}, request_id="r-9")))
    assert out["message"] == "hello" and out["level"] == "INFO" and out["logger"] == "vgate.t"
    assert out["k"] == 1 and out["request_id"] == "r-9" and "timestamp" in out


def test_console_formatter_includes_extra():
    s = ConsoleFormatter().format(_record(extra_data={"worker": "w1"}))
    assert "hello" in s and "worker=w1" in s and "INFO" in s


def test_setup_logging_json_and_console():
    lg = setup_logging("DEBUG", json_format=True, logger_name="vgate.tsetup")
    assert lg.level == logging.DEBUG and isinstance(lg.handlers[0].formatter, JSONFormatter)
    assert lg.propagate is False
    lg = setup_logging("WARNING", json_format=False, logger_name="vgate.tsetup")
    assert lg.level == logging.WARNING and isinstance(lg.handlers[0].formatter, ConsoleFormatter)
    assert get_logger("vgate.tsetup") is lg


def test_log_context_adds_fields():
    lg = logging.getLogger("vgate.tctx")
    buf = io.StringIO()
    h = logging.StreamHandler(buf)
    h.setFormatter(JSONFormatter())
    lg.handlers = [h]
    lg.setLevel(logging.INFO)
    lg.propagate = False
    with LogContext(lg, request_id="abc", tenant="t1"):
        lg.info("inside")
    lg.info("outside")
    lines = [json.loads(x) for x in buf.getvalue().splitlines()]
    assert lines[0]["tenant"] == "t1" and "tenant" not in lines[1]


# ------------------------------------------------------------------------- tracing
def test_tracing_disabled_by_default_and_idempotent_shutdown():
    assert tracing.init_tracing(VGateConfig(_env={})) is False
    assert tracing.get_current_trace_id() == ""
    tracing.shutdown_tracing()
    tracing.shutdown_tracing()


def test_tracing_enabled_spans_and_log_correlation():
    cfg = VGateConfig(_env={}, tracing={"enabled": True})
    try:
        assert tracing.init_tracing(cfg) is True
        tr = tracing.get_tracer("t")
        with tr.start_as_current_span("outer"):
            tid = tracing.get_current_trace_id()
            assert len(tid) == 32
            out = json.loads(JSONFormatter().format(_record()))
            assert out["trace_id"] == tid and len(out["span_id"]) == 16
            hdr = tracing.inject_traceparent({})
            assert hdr["traceparent"].split("-")[1] == tid
        assert tracing.get_current_trace_id() == ""
    finally:
        tracing.shutdown_tracing()


# ---------------------------------------------------------------------- dry-run knobs
def test_dryrun_knobs_off_by_default_and_capacity(monkeypatch):
    from vgate.backends import base
    assert base._simulated_seconds({"max_tokens": 64}) >= 0.0
    monkeypatch.setattr(base, "_DRYRUN_LATENCY_MS", 0.0)
    t0 = time.perf_counter()
    DryRunBackend().generate(["x"] * 4, {"max_tokens": 16})
    assert time.perf_counter() - t0 < 0.05  # free without the latency knob


async def test_dryrun_capacity_bounds_concurrent_generations(monkeypatch):
    from vgate.backends import base
    monkeypatch.setattr(base, "_DRYRUN_LATENCY_MS", 40.0)
    monkeypatch.setattr(base, "_DRYRUN_MAX_CONCURRENCY", 2)
    base._dryrun_async_capacity.clear()
    be = DryRunBackend()
    t0 = time.perf_counter()
    await asyncio.gather(*(be.agenerate(f"p{i}", {"max_tokens": 1}) for i in range(4)))
    took = time.perf_counter() - t0
    assert took >= 0.08  # 4 calls through 2 slots: two rounds of ~42 ms
    monkeypatch.setattr(base, "_DRYRUN_MAX_CONCURRENCY", 0)
    t0 = time.perf_counter()
    await asyncio.gather(*(be.agenerate(f"q{i}", {"max_tokens": 1}) for i in range(4)))
    # without the capacity knob calls do not queue: one ~40 ms round fewer (relative, so a loaded
    # host or the asyncio debug pass does not flake it)
    assert time.perf_counter() - t0 < took - 0.02


# ------------------------------------------------------------------------- cache log
async def test_cache_hit_emits_debug_log():
    lg = logging.getLogger("vgate.cache")
    buf = io.StringIO()
    h = logging.StreamHandler(buf)
    h.setFormatter(JSONFormatter())
    old = (lg.handlers[:], lg.level, lg.propagate)
    lg.handlers = [h]
    lg.setLevel(logging.DEBUG)
    lg.propagate = False
    try:
        c = ResultCache(maxsize=4, enabled=True)
        await c.put("key123456", {"text": "x"})
        await c.get("key123456")
        assert any("hit" in json.loads(x)["message"].lower() for x in buf.getvalue().splitlines())
    finally:
        lg.handlers, lg.level, lg.propagate = old[0], old[1], old[2]
