"""Request pipeline: result cache -> in-flight dedup -> admission -> per-request fan-out.

Contract kept from the reference (``vgate/batcher.py``):
* cache lookup first (hits do not count in ``total_requests``); failures are
  never cached;
* identical concurrent requests coalesce onto ONE inference; followers hold no
  admission permit;
* ``batch.max_batch_size`` bounds concurrent inferences (forced to 1 when the
  backend lacks ``supports_concurrent_calls``); ``max_wait_time_ms`` is accepted
  and ignored;
* each waiter is shielded (optional timeout); when every waiter of a QUEUED
  inference gives up it is cancelled (``vgate_abandoned_inferences_total``), a
  STARTED one runs on and fills the cache; ``stop()`` drains.

MI355X-engine differences: a backend exposing ``agenerate`` is awaited directly
on the event loop (no executor thread per request — the engine batches
continuously underneath); sync backends still run in the default executor with
the tracing context re-attached. Results also carry ``prompt_tokens`` and
``finish_reason`` when the backend reports them.
"""
from __future__ import annotations

import asyncio
import contextlib
import contextvars
import functools
import time
from dataclasses import dataclass
from typing import Any, Dict, Optional

from vgate.cache import ResultCache
from vgate.config import get_config
from vgate.logging_config import get_logger
from vgate.metrics import (ABANDONED_INFERENCES, BATCH_PROCESSING_TIME, BATCH_QUEUE_TIME, BATCH_SIZE,
                           DEDUP_RATIO, DEDUPLICATED_REQUESTS, INFERENCE_ERRORS, INFLIGHT_INFERENCES,
                           PENDING_REQUESTS, TOKENS_GENERATED, TOTAL_BATCHES, TPOT, TTFT, UNIQUE_PROMPTS_PER_BATCH)
from vgate.tracing import _NOOP, get_current_trace_id, get_tracer, is_tracing_enabled

logger = get_logger("vgate.batcher")
tracer = get_tracer(__name__)
_NO_SPAN = contextlib.nullcontext(_NOOP)  # reusable: yields the no-op span


@dataclass
class _Inflight:
    task: Optional[asyncio.Task] = None
    waiters: int = 0
    started: bool = False


class RequestBatcher:
    def __init__(self, engine, max_batch_size: Optional[int] = None, max_wait_time_ms: Optional[float] = None):
        cfg = get_config()
        self.engine = engine
        self.max_batch_size = max_batch_size if max_batch_size is not None else cfg.batch.max_batch_size
        self.max_wait_time_ms = max_wait_time_ms if max_wait_time_ms is not None else cfg.batch.max_wait_time_ms
        self.cache = ResultCache()
        backend = getattr(engine, "backend", None)
        self._serialize_inference = not getattr(backend, "supports_concurrent_calls", False)
        self.max_concurrent_inferences = 1 if self._serialize_inference else self.max_batch_size
        self._semaphore = asyncio.Semaphore(self.max_concurrent_inferences)
        self._inflight: Dict[str, _Inflight] = {}
        self._running = False
        self.total_requests = 0
        self.total_batches = 0
        self.total_batch_size = 0
        self.total_deduplicated = 0
        self.total_queue_time = 0.0
        self.total_queue_samples = 0
        self.total_ttft = 0.0
        self.total_tpot = 0.0
        self.total_inference_samples = 0
        self._waiting = 0

    async def start(self):
        if self._running:
            return
        self._running = True
        logger.info("Batcher started", extra={"extra_data": {
            "max_concurrent_inferences": self.max_concurrent_inferences,
            "serialized_backend": self._serialize_inference, "mode": "dedup+admission+fanout",
            "max_wait_time_ms_ignored": self.max_wait_time_ms}})

    async def stop(self):
        self._running = False
        pending = [e.task for e in self._inflight.values() if e.task is not None]
        if pending:
            await asyncio.gather(*pending, return_exceptions=True)
        logger.info("Batcher stopped")

    # ------------------------------------------------------------------ submit
    async def submit(self, prompt: str, max_tokens: Optional[int] = None, temperature: Optional[float] = None,
                     top_p: Optional[float] = None, timeout: Optional[float] = None) -> Dict[str, Any]:
        # no span objects at all while tracing is off (the serving default): this runs once per request
        cm = tracer.start_as_current_span("batcher.submit") if is_tracing_enabled() else _NO_SPAN
        with cm as span:
            cfg = get_config()
            max_tokens = cfg.inference.max_tokens if max_tokens is None else max_tokens
            temperature = cfg.inference.temperature if temperature is None else temperature
            top_p = cfg.inference.top_p if top_p is None else top_p
            span.set_attribute("prompt_length", len(prompt))
            key = ResultCache.make_key(prompt, temperature, top_p, max_tokens)
            cached = self.cache.get_nowait(key)
            if cached:
                span.set_attribute("cache_hit", True)
                return cached
            span.set_attribute("cache_hit", False)
            self.total_requests += 1
            # no await between the lookup and the registration: atomic on the event loop
            entry = self._inflight.get(key)
            coalesced = entry is not None
            if entry is None:
                entry = _Inflight()
                self._inflight[key] = entry
                entry.task = asyncio.create_task(self._execute(entry, key, prompt, temperature, top_p, max_tokens))
                entry.task.add_done_callback(functools.partial(self._retire, key))
            entry.waiters += 1
            span.set_attribute("deduplicated", coalesced)
            if coalesced:
                self.total_deduplicated += 1
                DEDUPLICATED_REQUESTS.inc()
                DEDUP_RATIO.set(self.total_deduplicated / self.total_requests if self.total_requests else 0)
            try:
                if timeout is not None:
                    return await asyncio.wait_for(asyncio.shield(entry.task), timeout=timeout)
                return await asyncio.shield(entry.task)
            finally:
                self._release_waiter(entry, key)

    def _release_waiter(self, entry: _Inflight, key: str) -> None:
        entry.waiters -= 1
        if entry.waiters > 0 or entry.started or entry.task.done():
            return
        entry.task.cancel()
        ABANDONED_INFERENCES.inc()
        logger.info("Cancelled abandoned request before admission", extra={"extra_data": {"cache_key": key[:8]}})

    def _retire(self, key: str, task: asyncio.Task) -> None:
        cur = self._inflight.get(key)
        if cur is not None and cur.task is task:
            self._inflight.pop(key, None)

    async def _execute(self, entry: _Inflight, key: str, prompt: str, temperature: float, top_p: float,
                       max_tokens: int) -> Dict[str, Any]:
        queued_at = time.monotonic()
        self._waiting += 1
        PENDING_REQUESTS.set(self._waiting)
        waiting = True
        try:
            async with self._semaphore:
                entry.started = True
                self._waiting -= 1
                waiting = False
                PENDING_REQUESTS.set(self._waiting)
                qt = time.monotonic() - queued_at
                BATCH_QUEUE_TIME.observe(qt)
                self.total_queue_time += qt
                self.total_queue_samples += 1
                INFLIGHT_INFERENCES.inc()
                try:
                    result = await self._run_inference(prompt, max_tokens, temperature, top_p)
                finally:
                    INFLIGHT_INFERENCES.dec()
        finally:
            if waiting:
                self._waiting -= 1
                PENDING_REQUESTS.set(self._waiting)
        self.cache.put_nowait(key, result)
        return result

    # --------------------------------------------------------------- inference
    async def _run_inference(self, prompt: str, max_tokens: int, temperature: float = 0.7,
                             top_p: float = 0.9) -> Dict[str, Any]:
        backend = self.engine.backend
        t0 = time.perf_counter()
        try:
            if hasattr(backend, "agenerate"):
                cm = tracer.start_as_current_span("batcher.inference") if is_tracing_enabled() else _NO_SPAN
                with cm as span:
                    span.set_attribute("num_prompts", 1)
                    sp = backend.create_sampling_params(temperature=temperature, top_p=top_p, max_tokens=max_tokens)
                    br = await backend.agenerate(prompt, sp)
                    result = self._shape(br, time.perf_counter() - t0)
                    span.set_attribute("total_tokens_generated", result["total_tokens"])
            else:
                loop = asyncio.get_running_loop()
                ctx = contextvars.copy_context()
                result = await loop.run_in_executor(
                    None, lambda: ctx.run(self._sync_inference_traced, prompt, max_tokens, temperature, top_p))
        except Exception as e:
            INFERENCE_ERRORS.labels(error_type=type(e).__name__).inc()
            logger.error("Inference error", extra={"extra_data": {"error": str(e), "error_type": type(e).__name__}})
            raise
        dur = time.perf_counter() - t0
        tid = get_current_trace_id()
        BATCH_PROCESSING_TIME.observe(dur, exemplar={"trace_id": tid} if tid else None)
        self.total_batches += 1
        self.total_batch_size += 1
        TOTAL_BATCHES.inc()
        BATCH_SIZE.observe(1)
        UNIQUE_PROMPTS_PER_BATCH.observe(1)
        if result.get("ttft", 0) > 0:
            TTFT.observe(result["ttft"])
            self.total_ttft += result["ttft"]
        if result.get("tpot", 0) > 0:
            TPOT.observe(result["tpot"])
            self.total_tpot += result["tpot"]
            self.total_inference_samples += 1
        TOKENS_GENERATED.inc(result.get("total_tokens", 0))
        return result

    def _sync_inference_traced(self, prompt, max_tokens, temperature, top_p):
        with tracer.start_as_current_span("batcher.inference") as span:
            span.set_attribute("num_prompts", 1)
            r = self._sync_inference(prompt, max_tokens, temperature, top_p)
            span.set_attribute("total_tokens_generated", r.get("total_tokens", 0))
            return r

    def _sync_inference(self, prompt: str, max_tokens: int, temperature: float = 0.7,
                        top_p: float = 0.9) -> Dict[str, Any]:
        backend = self.engine.backend
        sp = backend.create_sampling_params(temperature=temperature, top_p=top_p, max_tokens=max_tokens)
        t0 = time.perf_counter()
        br = backend.generate([prompt], sp)[0]
        return self._shape(br, time.perf_counter() - t0)

    @staticmethod
    def _shape(br: Dict[str, Any], total_time: float) -> Dict[str, Any]:
        n = br["num_tokens"]
        m = br.get("metrics", {}) or {}
        ttft = m.get("ttft", 0.0)
        gen = m.get("gen_time", total_time)
        out = {"text": br["text"], "ttft": ttft, "tpot": (gen / n) if n > 0 else 0, "total_tokens": n}
        if "prompt_tokens" in br:
            out["prompt_tokens"] = br["prompt_tokens"]
        if "finish_reason" in br:
            out["finish_reason"] = br["finish_reason"]
        return out

    def get_metrics(self) -> Dict[str, Any]:
        nb = self.total_batches
        ns = self.total_inference_samples
        return {
            "total_requests": self.total_requests, "total_batches": nb,
            "average_batch_size": round(self.total_batch_size / nb, 2) if nb else 0,
            "pending_requests": self._waiting, "inflight_inferences": len(self._inflight),
            "total_deduplicated": self.total_deduplicated,
            "avg_queue_time_s": round(self.total_queue_time / self.total_queue_samples, 4) if self.total_queue_samples else 0,
            "avg_ttft_s": round(self.total_ttft / ns, 4) if ns else 0,
            "avg_tpot_s": round(self.total_tpot / ns, 4) if ns else 0,
            "cache": self.cache.get_stats(),
        }
