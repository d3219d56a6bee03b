"""Worker-role internal API (mounted only when ``role == "worker"``).

``POST /internal/generate`` keeps the reference wire contract
(``{prompts: [str] (>=1), sampling_params: {temperature, top_p, max_tokens}}`` ->
``{results: [backend result dicts]}``; 503 before the engine is bound; 500
``Inference failed: <Type>``). Async backends are awaited concurrently on the
loop (each prompt is its own engine request, so they batch continuously);
sync backends run in the executor, serialised by a lock if not concurrency-safe.

``POST /internal/generate_stream`` (new) streams one prompt's deltas as SSE so
the gateway can proxy ``stream: true`` through remote workers.

Drain (reference ROADMAP.md:399-403: "a terminating worker has to fail its own /health while
still finishing the requests it already accepted"): :func:`begin_drain` (SIGTERM, or the
lifespan shutdown) flips the worker to draining — ``/health`` answers 503
``{"status": "draining"}``, new generate calls get 503 (nothing ran, so the gateway retries
them on another worker) — and :func:`wait_drained` returns once every accepted request has
finished (and the minimum drain time has passed, so the gateways' probes saw the 503).
"""
from __future__ import annotations

import asyncio
import json
import weakref
from typing import Optional

from fastapi import APIRouter, HTTPException, Request
from fastapi.responses import StreamingResponse
from pydantic import BaseModel, Field

from vgate.logging_config import get_logger
from vgate.metrics import INFERENCE_ERRORS
from vgate.tracing import attach_traceparent, get_tracer

logger = get_logger("vgate.worker_api")
tracer = get_tracer(__name__)
router = APIRouter()

_engine = None
_guard: Optional[asyncio.Lock] = None
_draining = False
_drain_started = 0.0
_inflight = 0


def begin_drain() -> None:
    """Enter the draining state (idempotent)."""
    global _draining, _drain_started
    if not _draining:
        import time
        _draining = True
        _drain_started = time.monotonic()
        logger.info("Worker draining", extra={"extra_data": {"inflight": _inflight}})


def is_draining() -> bool:
    return _draining


def inflight() -> int:
    return _inflight


async def wait_drained(min_seconds: float = 0.0, timeout: float = 120.0) -> bool:
    """Wait until no accepted request is in flight and ``min_seconds`` have passed since
    :func:`begin_drain`; False if ``timeout`` expired first."""
    import time
    t_end = time.monotonic() + timeout
    while time.monotonic() < t_end:
        if _inflight == 0 and time.monotonic() - _drain_started >= min_seconds:
            return True
        await asyncio.sleep(0.05)
    return _inflight == 0


def reset_drain() -> None:
    """Back to serving (tests)."""
    global _draining, _inflight
    _draining, _inflight = False, 0


class _Accepted:
    """Counts a request from acceptance to its last byte (the drain waits for these)."""

    def __enter__(self):
        global _inflight
        _inflight += 1
        return self

    def __exit__(self, *exc):
        global _inflight
        _inflight -= 1
        return False


class WorkerSamplingParams(BaseModel):
    temperature: float = 0.7
    top_p: float = 0.9
    max_tokens: int = 256


class GenerateRequest(BaseModel):
    prompts: list[str] = Field(min_length=1)
    sampling_params: WorkerSamplingParams = Field(default_factory=WorkerSamplingParams)


class StreamRequest(BaseModel):
    prompt: str
    sampling_params: WorkerSamplingParams = Field(default_factory=WorkerSamplingParams)


def set_engine(engine) -> None:
    global _engine, _guard
    _engine = engine
    _guard = None if getattr(engine.backend, "supports_concurrent_calls", False) else asyncio.Lock()


def get_engine():
    return _engine


def _refuse_if_draining() -> None:
    if _draining:
        raise HTTPException(status_code=503, detail="Worker draining")


@router.post("/internal/generate")
async def internal_generate(body: GenerateRequest, request: Request):
    if _engine is None:
        raise HTTPException(status_code=503, detail="Worker engine not ready")
    _refuse_if_draining()
    with _Accepted():
        return await _generate(body, request)


async def _generate(body: GenerateRequest, request: Request):
    backend = _engine.backend
    with attach_traceparent(request.headers.get("traceparent")):
        with tracer.start_as_current_span("worker.generate") as span:
            span.set_attribute("num_prompts", len(body.prompts))
            sp_in = body.sampling_params
            sp = backend.create_sampling_params(temperature=sp_in.temperature, top_p=sp_in.top_p,
                                                max_tokens=sp_in.max_tokens)
            try:
                if hasattr(backend, "agenerate"):
                    results = list(await asyncio.gather(*(backend.agenerate(p, sp) for p in body.prompts)))
                else:
                    loop = asyncio.get_running_loop()
                    if _guard is not None:
                        async with _guard:
                            results = await loop.run_in_executor(None, backend.generate, body.prompts, sp)
                    else:
                        results = await loop.run_in_executor(None, backend.generate, body.prompts, sp)
            except Exception as e:  # noqa: BLE001
                INFERENCE_ERRORS.labels(error_type=type(e).__name__).inc()
                logger.error("Worker inference failed", extra={"extra_data": {
                    "error": str(e), "error_type": type(e).__name__}})
                raise HTTPException(status_code=500, detail=f"Inference failed: {type(e).__name__}")
    return {"results": results}


@router.post("/internal/generate_stream")
async def internal_generate_stream(body: StreamRequest, request: Request):
    if _engine is None:
        raise HTTPException(status_code=503, detail="Worker engine not ready")
    _refuse_if_draining()
    backend = _engine.backend
    if not getattr(backend, "supports_streaming", False):
        raise HTTPException(status_code=501, detail="worker backend cannot stream")
    sp_in = body.sampling_params
    sp = backend.create_sampling_params(temperature=sp_in.temperature, top_p=sp_in.top_p, max_tokens=sp_in.max_tokens)

    # the stream counts from ACCEPTANCE (here, before the response object exists) to its last byte:
    # a drain that starts between this point and the server's first iteration of the body still
    # waits for it. Released once, by the body's finally or — when the body never starts (client
    # gone, response dropped) — by the generator object's finaliser.
    _Accepted().__enter__()
    released = [False]

    def release():
        global _inflight
        if not released[0]:
            released[0] = True
            _inflight -= 1

    async def gen():
        try:
            try:
                async for piece in backend.stream_generate(body.prompt, sp):
                    yield f"data: {json.dumps(piece)}\n\n"
            except (asyncio.CancelledError, GeneratorExit):
                raise
            except Exception as e:  # noqa: BLE001
                INFERENCE_ERRORS.labels(error_type=type(e).__name__).inc()
                yield f"data: {json.dumps({'error': {'message': str(e), 'type': type(e).__name__}})}\n\n"
            yield "data: [DONE]\n\n"
        finally:
            release()

    body_gen = gen()
    weakref.finalize(body_gen, release)
    return StreamingResponse(body_gen, media_type="text/event-stream")
