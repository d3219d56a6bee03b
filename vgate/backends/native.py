"""Backend over the first-party MI355X engine (:mod:`vgate.runtime.engine`).

Replaces the reference's vLLM/SGLang adapters (``engine_type: vllm|sglang`` are
accepted as aliases). Properties that differ from those adapters, by design:

* ``supports_concurrent_calls = True`` and ``agenerate`` is a native coroutine:
  each request is a future completed from the engine thread via
  ``loop.call_soon_threadsafe`` — no executor thread is held per request;
* ``stream_generate`` works (incremental detokenised deltas), and closing the
  stream early (client disconnect) aborts the sequence in the engine and frees
  its KV blocks;
* results carry real ``prompt_tokens`` and ``finish_reason`` ("stop"/"length").
"""
from __future__ import annotations

import asyncio
import itertools
import os
import threading
import time
import weakref
from typing import Any, AsyncIterator, Dict, List

from vgate.config import ModelConfig
from vgate.logging_config import get_logger

logger = get_logger("vgate.backends.native")
_req_ids = itertools.count()


def engine_config_from(model_config: ModelConfig):
    from vgate.runtime.engine import EngineConfig
    weights = model_config.weights_path
    if weights is None and not model_config.random_init and os.path.isdir(os.path.expanduser(model_config.model_id)):
        weights = model_config.model_id
    return EngineConfig(
        model=model_config.model_id, weights_path=weights, tokenizer=model_config.tokenizer,
        quantization=model_config.quantization, dtype=model_config.dtype, device=model_config.device,
        tensor_parallel_size=model_config.tensor_parallel_size, max_model_len=model_config.max_model_len,
        max_num_seqs=model_config.max_num_seqs, max_num_batched_tokens=model_config.max_num_batched_tokens,
        gpu_memory_utilization=model_config.gpu_memory_utilization, num_kv_blocks=model_config.num_kv_blocks,
        enforce_eager=model_config.enforce_eager, enable_prefix_caching=model_config.enable_prefix_caching,
        seed=model_config.seed, block_size=model_config.kv_block_size,
        part_size=model_config.attention_partition_size,
        graph_token_buckets=model_config.hip_graph_token_buckets,
        warmup_max_tokens=model_config.graph_warmup_max_tokens, warmup_max_seqs=model_config.graph_warmup_max_seqs,
        idle_batch_window_ms=model_config.idle_batch_window_ms, idle_batch_gap_ms=model_config.idle_batch_gap_ms,
        idle_batch_recent_ms=model_config.idle_batch_recent_ms, prefill_autotune=model_config.prefill_autotune,
        plan_cache=model_config.plan_cache or "", tp_timeout_seconds=model_config.tp_timeout_seconds,
        tp_custom_allreduce=model_config.tp_custom_allreduce, tp_fused_allreduce=model_config.tp_fused_allreduce,
        tp_collective_self_check=model_config.tp_collective_self_check,
        tp_consistency_interval=model_config.tp_consistency_interval)


def freeze_heap() -> None:
    """Move every object alive after model load + graph warm-up (torch, transformers, the model's
    Python objects: millions) into the permanent GC generation. A full collection otherwise
    walks them all while holding the GIL: the serving event loop stalled 94 ms mid-benchmark,
    delaying one whole batch of responses (p99 0.185 s vs p50 0.091 s; bench.py
    loop_lag_max_ms / gc forensics). Later allocations are collected as usual."""
    import gc
    gc.collect()
    gc.freeze()


class NativeBackend:
    supports_concurrent_calls = True
    supports_streaming = True

    def __init__(self, engine=None, watchdog_seconds: float = 60.0):
        self.engine = engine
        self.watchdog_seconds = float(watchdog_seconds)

    # ------------------------------------------------------------------ setup
    def load_model(self, model_config: ModelConfig) -> None:
        from vgate.runtime.engine import LLMEngine
        self.watchdog_seconds = float(getattr(model_config, "watchdog_seconds", self.watchdog_seconds))
        cfg = engine_config_from(model_config)
        if getattr(model_config, "engine_process", False) and cfg.tensor_parallel_size == 1:
            from vgate.runtime.engine_process import EngineProcessClient
            self.engine = EngineProcessClient(cfg)
            return
        self.engine = LLMEngine(cfg)
        freeze_heap()
        if self.engine.tp.size > 1 and not self.engine.tp.is_first:
            # TP followers never serve HTTP: they execute rank 0's steps until shutdown
            self.engine.follower_loop()
            return
        self.engine.start()

    def create_sampling_params(self, temperature: float, top_p: float, max_tokens: int) -> Any:
        return {"temperature": temperature, "top_p": top_p, "max_tokens": max_tokens}

    @staticmethod
    def _params(sp: Any):
        from vgate.runtime.sampling_params import SamplingParams
        if isinstance(sp, SamplingParams):
            return sp
        sp = dict(sp or {})
        return SamplingParams(temperature=float(sp.get("temperature", 0.7)), top_p=float(sp.get("top_p", 0.9)),
                              top_k=int(sp.get("top_k", -1)), max_tokens=int(sp.get("max_tokens", 256)),
                              seed=sp.get("seed"), stop=list(sp.get("stop") or []),
                              ignore_eos=bool(sp.get("ignore_eos", False)))

    @staticmethod
    def _result(seq) -> Dict[str, Any]:
        ttft = (seq.first_token_time - seq.arrival) if seq.first_token_time else 0.0
        gen = (seq.finish_time - seq.first_token_time) if (seq.first_token_time and seq.finish_time) else 0.0
        wall = (seq.finish_time - seq.arrival) if seq.finish_time else 0.0
        return {"text": seq.text, "token_ids": list(seq.output_ids), "num_tokens": len(seq.output_ids),
                "prompt_tokens": len(seq.prompt_ids), "finish_reason": seq.finish_reason or "stop",
                "metrics": {"ttft": ttft, "gen_time": gen, "wall_time": wall}}

    # --------------------------------------------------------------- generate
    async def agenerate(self, prompt: str, sampling_params: Any) -> Dict[str, Any]:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        rid = f"n{next(_req_ids)}"
        done = _completions(loop)

        def cb(kind, seq, payload):
            if kind == "token":
                return
            if kind == "error":
                res = RuntimeError(f"engine error: {payload}")
            else:
                res = self._result(seq)
            done.push(fut, res)

        self.engine.add_request(rid, prompt, self._params(sampling_params), cb)
        try:
            return await fut
        except asyncio.CancelledError:
            self.engine.abort(rid)
            raise

    def generate(self, prompts: List[str], sampling_params: Any) -> List[Dict[str, Any]]:
        """Synchronous batch API (compatibility with the reference protocol)."""
        sp = self._params(sampling_params)
        done = threading.Event()
        results: list = [None] * len(prompts)
        left = [len(prompts)]
        lock = threading.Lock()

        def make_cb(i):
            def cb(kind, seq, payload):
                if kind == "token":
                    return
                results[i] = RuntimeError(payload) if kind == "error" else self._result(seq)
                with lock:
                    left[0] -= 1
                    if left[0] == 0:
                        done.set()
            return cb

        for i, p in enumerate(prompts):
            self.engine.add_request(f"g{next(_req_ids)}", p, sp, make_cb(i))
        if not self.engine._running:  # offline use without the engine thread
            self.engine.run_until_idle()
        done.wait()
        for r in results:
            if isinstance(r, Exception):
                raise r
        return results

    async def stream_generate(self, prompt: str, sampling_params: Any) -> AsyncIterator[Dict[str, Any]]:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        rid = f"s{next(_req_ids)}"
        count = [0]

        def cb(kind, seq, payload):
            if kind == "token":
                count[0] = len(seq.output_ids)
                loop.call_soon_threadsafe(q.put_nowait, ("delta", payload, len(seq.output_ids)))
            elif kind == "error":
                loop.call_soon_threadsafe(q.put_nowait, ("error", payload, 0))
            else:
                loop.call_soon_threadsafe(q.put_nowait, ("end", seq.finish_reason, len(seq.output_ids)))

        self.engine.add_request(rid, prompt, self._params(sampling_params), cb, stream=True)
        finished = False
        try:
            while True:
                kind, payload, n = await q.get()
                if kind == "delta":
                    yield {"delta": payload, "num_tokens": n}
                elif kind == "error":
                    finished = True
                    raise RuntimeError(f"engine error: {payload}")
                else:
                    finished = True
                    yield {"delta": "", "num_tokens": n, "finish_reason": payload}
                    return
        finally:
            if not finished:
                self.engine.abort(rid)

    # ------------------------------------------------------------- embeddings
    def stats(self) -> dict:
        return self.engine.snapshot() if self.engine is not None else {}

    def healthy(self) -> bool:
        if self.engine is None:
            return False
        if not self.engine.healthy:
            return False
        # watchdog: work pending but no step completed for watchdog_seconds => hung HIP queue
        if self.engine.has_unfinished() and time.monotonic() - self.engine.last_step_wall > self.watchdog_seconds:
            return False
        return True

    def shutdown(self) -> None:
        if self.engine is not None:
            self.engine.stop()
            self.engine.shutdown_followers()


class _LoopCompletions:
    """Results handed from the engine thread to one event loop, one wake-up per burst.

    A wave of requests finishes inside one engine step; ``call_soon_threadsafe`` per request
    writes the loop's self-pipe and schedules a handle each time. Here the first result of a
    burst schedules one flush and later ones only append, so the loop wakes once per step."""

    def __init__(self, loop: asyncio.AbstractEventLoop):
        self.loop = loop
        self.items: list = []
        self.lock = threading.Lock()

    def push(self, fut: asyncio.Future, res) -> None:
        with self.lock:
            first = not self.items
            self.items.append((fut, res))
        if first:
            try:
                self.loop.call_soon_threadsafe(self._flush)
            except RuntimeError:  # loop closed (shutdown): nobody is waiting any more
                pass

    def _flush(self) -> None:
        with self.lock:
            items, self.items = self.items, []
        for fut, res in items:
            _resolve(fut, res)


_loop_completions: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _completions(loop: asyncio.AbstractEventLoop) -> _LoopCompletions:
    c = _loop_completions.get(loop)
    if c is None:
        c = _loop_completions[loop] = _LoopCompletions(loop)
    return c


def _resolve(fut: asyncio.Future, res):
    if fut.done():
        return
    if isinstance(res, Exception):
        fut.set_exception(res)
    else:
        fut.set_result(res)
