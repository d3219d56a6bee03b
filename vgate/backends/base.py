"""Inference backend protocol and the dry-run backend.

Protocol (reference ``vgate/backends/base.py:65-91``) plus two async-first
additions used by the gateway when present:

* ``async agenerate(prompt, sampling_params) -> dict`` — one request, no thread
  held while it runs (the batcher prefers it over ``generate``);
* ``supports_streaming`` — capability flag checked before any SSE bytes.

Result dicts: ``{"text", "token_ids", "num_tokens", "metrics": {"ttft"?, "gen_time"?,
"wall_time"?}}`` and, from the native engine, ``"prompt_tokens"`` and
``"finish_reason"``.

Dry-run knobs (import-time env, same names/semantics as the reference):
``VGATE_DRYRUN_SIMULATED_LATENCY_MS`` adds ``latency + 2 ms x max_tokens`` per
call; ``VGATE_DRYRUN_MAX_CONCURRENCY`` bounds concurrent generations.
"""
from __future__ import annotations

import asyncio
import os
import threading
import time
from typing import Any, AsyncIterator, Dict, List, Protocol, runtime_checkable

from vgate.config import ModelConfig

_DRYRUN_LATENCY_MS = float(os.getenv("VGATE_DRYRUN_SIMULATED_LATENCY_MS", "0"))
_DRYRUN_MAX_CONCURRENCY = int(os.getenv("VGATE_DRYRUN_MAX_CONCURRENCY", "0"))
_dryrun_capacity = threading.Semaphore(_DRYRUN_MAX_CONCURRENCY) if _DRYRUN_MAX_CONCURRENCY > 0 else None
_dryrun_async_capacity: dict = {}


def _simulated_seconds(sampling_params: Any) -> float:
    if _DRYRUN_LATENCY_MS <= 0:
        return 0.0
    mt = sampling_params.get("max_tokens", 0) if isinstance(sampling_params, dict) else 0
    return (_DRYRUN_LATENCY_MS + mt * 2) / 1000.0


def _simulate_batch_compute(sampling_params: Any) -> None:
    d = _simulated_seconds(sampling_params)
    if d <= 0:
        return
    if _dryrun_capacity is None:
        time.sleep(d)
        return
    with _dryrun_capacity:
        time.sleep(d)


@runtime_checkable
class InferenceBackend(Protocol):
    def load_model(self, model_config: ModelConfig) -> None: ...

    def create_sampling_params(self, temperature: float, top_p: float, max_tokens: int) -> Any: ...

    def generate(self, prompts: List[str], sampling_params: Any) -> List[Dict[str, Any]]: ...

    def stream_generate(self, prompt: str, sampling_params: Any) -> AsyncIterator[Dict[str, Any]]:
        """Yield ``{"delta": str, "num_tokens": cumulative}`` chunks."""
        ...

    def shutdown(self) -> None: ...


def _echo(prompt: str) -> str:
    return f"[dry-run] echo: {prompt[:80]}"


class DryRunBackend:
    """Placeholder generations without a GPU (CI, gateway/scaling benchmarks)."""

    supports_concurrent_calls = True
    supports_streaming = True

    def load_model(self, model_config: ModelConfig) -> None:
        pass

    def create_sampling_params(self, temperature: float, top_p: float, max_tokens: int) -> Any:
        return {"temperature": temperature, "top_p": top_p, "max_tokens": max_tokens}

    @staticmethod
    def _result(prompt: str) -> Dict[str, Any]:
        return {"text": _echo(prompt), "token_ids": list(range(8)), "num_tokens": 8, "metrics": {}}

    def generate(self, prompts: List[str], sampling_params: Any) -> List[Dict[str, Any]]:
        _simulate_batch_compute(sampling_params)
        return [self._result(p) for p in prompts]

    async def agenerate(self, prompt: str, sampling_params: Any) -> Dict[str, Any]:
        d = _simulated_seconds(sampling_params)
        if d > 0:
            if _DRYRUN_MAX_CONCURRENCY > 0:
                loop = asyncio.get_running_loop()
                sem = _dryrun_async_capacity.get(loop)
                if sem is None:
                    sem = _dryrun_async_capacity[loop] = asyncio.Semaphore(_DRYRUN_MAX_CONCURRENCY)
                async with sem:
                    await asyncio.sleep(d)
            else:
                await asyncio.sleep(d)
        return self._result(prompt)

    async def stream_generate(self, prompt: str, sampling_params: Any) -> AsyncIterator[Dict[str, Any]]:
        mt = sampling_params.get("max_tokens", 8) if isinstance(sampling_params, dict) else 8
        words = _echo(prompt).split()
        n = min(len(words), mt) or 1
        for i in range(n):
            await asyncio.sleep(0.02)
            yield {"delta": words[i] + (" " if i < n - 1 else ""), "num_tokens": i + 1}

    def shutdown(self) -> None:
        pass
