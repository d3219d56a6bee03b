"""Worker-role internal API (mounted only when ``role == "worker"``).

``POST /internal/generate`` keeps the reference wire contract
(``{prompts: [str] (>=1), sampling_params: {temperature, top_p, max_tokens}}`` ->
``{results: [backend result dicts]}``; 503 before the engine is bound; 500
``Inference failed: <Type>``). Async backends are awaited concurrently on the
loop (each prompt is its own engine request, so they batch continuously);
sync backends run in the executor, serialised by a lock if not concurrency-safe.

``POST /internal/generate_stream`` (new) streams one prompt's deltas as SSE so
the gateway can proxy ``stream: true`` through remote workers.
"""
from __future__ import annotations

import asyncio
import json
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


@router.post("/internal/generate")
async def internal_generate(body: GenerateRequest, request: Request):
    if _engine is None:
        raise HTTPException(status_code=503, detail="Worker engine not ready")
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
    backend = _engine.backend
    if not getattr(backend, "supports_streaming", False):
        raise HTTPException(status_code=501, detail="worker backend cannot stream")
    sp_in = body.sampling_params
    sp = backend.create_sampling_params(temperature=sp_in.temperature, top_p=sp_in.top_p, max_tokens=sp_in.max_tokens)

    async def gen():
        try:
            async for piece in backend.stream_generate(body.prompt, sp):
                yield f"data: {json.dumps(piece)}\n\n"
        except (asyncio.CancelledError, GeneratorExit):
            raise
        except Exception as e:  # noqa: BLE001
            INFERENCE_ERRORS.labels(error_type=type(e).__name__).inc()
            yield f"data: {json.dumps({'error': {'message': str(e), 'type': type(e).__name__}})}\n\n"
        yield "data: [DONE]\n\n"

    return StreamingResponse(gen(), media_type="text/event-stream")
