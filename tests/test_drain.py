"""Worker drain on shutdown (reference ROADMAP.md:399-403; round-2 verdict item 6): a terminating
worker fails its own /health (503 "draining") and refuses new generate calls with 503 (which the
gateway retries on another worker) while the requests it already accepted finish normally."""
from __future__ import annotations

import asyncio
import os
import signal
import socket
import threading
import time

import httpx
import pytest

from vgate import worker_api
from vgate.api.app import _install_drain_on_sigterm, create_app
from vgate.backends.base import DryRunBackend
from vgate.backends.remote import RemoteBackend
from vgate.config import VGateConfig, WorkerConfig
from vgate.engine import VGateEngine
from vgate.health_checker import WorkerHealthChecker
from vgate.worker_registry import NoHealthyWorkersError, WorkerRegistry


class _SlowBackend(DryRunBackend):
    supports_concurrent_calls = True

    async def agenerate(self, prompt, sp):
        await asyncio.sleep(1.0)
        return {"text": "slow:" + prompt, "token_ids": [1, 2], "num_tokens": 2, "metrics": {}}


def _free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


async def test_draining_worker_fails_health_refuses_new_work_and_finishes_accepted():
    import uvicorn
    cfg = VGateConfig(role="worker")
    eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=_SlowBackend(), dry_run=True)
    app = create_app(cfg, engine=eng)
    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = time.time()
    while not srv.started and time.time() - t0 < 20:
        await asyncio.sleep(0.05)
    base = f"http://127.0.0.1:{port}"
    try:
        async with httpx.AsyncClient(base_url=base, timeout=10) as c:
            assert (await c.get("/health")).status_code == 200
            accepted = asyncio.create_task(c.post("/internal/generate", json={"prompts": ["a"]}))
            await asyncio.sleep(0.3)
            assert worker_api.inflight() == 1
            worker_api.begin_drain()  # what SIGTERM does first
            h = await c.get("/health")
            assert h.status_code == 503 and h.json()["status"] == "draining"
            assert (await c.get("/ready")).status_code == 503
            assert (await c.post("/internal/generate", json={"prompts": ["b"]})).status_code == 503
            assert (await c.post("/internal/generate_stream", json={"prompt": "b"})).status_code == 503
            r = await accepted  # the accepted request still completes
            assert r.status_code == 200 and r.json()["results"][0]["text"] == "slow:a"
            assert await worker_api.wait_drained(0.0, 5.0)
        # the gateway's probes demote the draining worker; a request to it is retried elsewhere
        reg = WorkerRegistry([base], failure_threshold=2)
        hc = WorkerHealthChecker(registry=reg, interval_seconds=0.05, timeout_seconds=2.0)
        async with httpx.AsyncClient() as pc:
            await hc.probe_once(pc)
            await hc.probe_once(pc)
        assert reg.healthy_endpoints() == []
        be = RemoteBackend(WorkerConfig(endpoints=[base]), registry=WorkerRegistry([base]))
        with pytest.raises(NoHealthyWorkersError):  # 503 = refused, not a mid-request failure
            await be.agenerate("c", {"max_tokens": 2})
        await be.aclose()
    finally:
        srv.should_exit = True
        th.join(timeout=10)
        worker_api.reset_drain()  # after the server's own shutdown drained


async def test_gateway_retries_a_503_refusal_on_another_worker():
    W1, W2 = "http://w1:8000", "http://w2:8000"
    calls = []

    def handler(request: httpx.Request):
        ep = f"{request.url.scheme}://{request.url.host}:{request.url.port}"
        calls.append(ep)
        if ep == W1:
            return httpx.Response(503, json={"detail": "Worker draining"})
        body = __import__("json").loads(request.content)
        return httpx.Response(200, json={"results": [{"text": "ok:" + p, "num_tokens": 1} for p in body["prompts"]]})

    be = RemoteBackend(WorkerConfig(endpoints=[W1, W2], routing="round_robin"), transport=httpx.MockTransport(handler))
    r = await be.agenerate("x", {"max_tokens": 1})
    assert r["text"] == "ok:x" and calls == [W1, W2]
    await be.aclose()


async def test_sigterm_drains_then_hands_over_to_the_server_handler():
    """The SIGTERM handler flips to draining at once and calls the server's own handler (uvicorn's
    should_exit) only after the accepted requests finished and drain_seconds passed."""
    seen = []
    old = signal.signal(signal.SIGTERM, lambda s, f: seen.append(time.monotonic()))
    cfg = VGateConfig(role="worker", worker={"drain_seconds": 0.3, "drain_timeout_seconds": 5})
    restore = _install_drain_on_sigterm(cfg)
    try:
        t0 = time.monotonic()
        with worker_api._Accepted():
            os.kill(os.getpid(), signal.SIGTERM)
            await asyncio.sleep(0.5)
            assert worker_api.is_draining() and not seen  # still one request in flight
        for _ in range(100):
            if seen:
                break
            await asyncio.sleep(0.02)
        assert seen and seen[0] - t0 >= 0.3
    finally:
        restore()
        signal.signal(signal.SIGTERM, old)
        worker_api.reset_drain()


async def test_stream_counts_from_acceptance_and_releases_a_body_that_never_ran():
    """An accepted stream counts for the drain from the endpoint's return, before the server first
    iterates its body (a drain in that window finished early), and is released exactly
    once: at the body's end, or — when the body never runs — when the response is dropped."""
    import gc

    from vgate.worker_api import StreamRequest
    cfg = VGateConfig(role="worker")
    eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=DryRunBackend(), dry_run=True)
    worker_api.reset_drain()
    prev = worker_api.get_engine()
    worker_api.set_engine(eng)
    try:
        resp = await worker_api.internal_generate_stream(StreamRequest(prompt="a b c"), request=None)
        assert worker_api.inflight() == 1
        chunks = [c async for c in resp.body_iterator]
        assert chunks[-1] == "data: [DONE]\n\n"
        assert worker_api.inflight() == 0
        dropped = await worker_api.internal_generate_stream(StreamRequest(prompt="x"), request=None)
        assert worker_api.inflight() == 1
        del dropped
        gc.collect()
        assert worker_api.inflight() == 0
    finally:
        if prev is not None:
            worker_api.set_engine(prev)
        else:
            worker_api._engine = None
        worker_api.reset_drain()
