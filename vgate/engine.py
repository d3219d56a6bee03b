"""Engine facade + backend factory (reference ``vgate/engine.py``).

Backend precedence is unchanged: remote (``worker.endpoints`` or
``worker.discovery.dns_name`` set) > ``VGATE_DRY_RUN`` > local engine. The local
engine is always the first-party MI355X engine; ``engine_type: vllm|sglang`` in
old configs select it too (there is no vLLM/SGLang dependency).

Embeddings: with the native engine loaded they are real (L2-normalised mean of
the model's final hidden states, dim = hidden size — 1536 for Qwen2.5-1.5B, the
same width the reference's mock used); in dry-run / remote mode the reference's
mock vector is returned for compatibility.
"""
from __future__ import annotations

import os
import time
from typing import Optional

from vgate.backends.base import DryRunBackend, InferenceBackend
from vgate.config import ModelConfig, WorkerConfig, get_config
from vgate.logging_config import get_logger
from vgate.tracing import get_tracer

tracer = get_tracer("vgate.engine")
logger = get_logger("vgate.engine")

DRY_RUN = os.getenv("VGATE_DRY_RUN", "false").lower() in ("true", "1", "yes")


def _is_remote(worker_config: WorkerConfig) -> bool:
    return bool(worker_config.endpoints) or bool(worker_config.discovery.dns_name)


def _create_backend(engine_type: str, worker_config: Optional[WorkerConfig] = None,
                    dry_run: Optional[bool] = None) -> InferenceBackend:
    if worker_config is not None and _is_remote(worker_config):
        from vgate.backends.remote import RemoteBackend
        return RemoteBackend(worker_config)
    if DRY_RUN if dry_run is None else dry_run:
        return DryRunBackend()
    if engine_type in ("native", "vllm", "sglang"):
        from vgate.backends.native import NativeBackend
        return NativeBackend()
    raise ValueError(f"Unknown engine_type: {engine_type!r}")


class VGateEngine:
    def __init__(self, model_config: Optional[ModelConfig] = None, worker_config: Optional[WorkerConfig] = None,
                 backend: Optional[InferenceBackend] = None, dry_run: Optional[bool] = None):
        cfg = get_config()
        self.model_config = model_config or cfg.model
        worker_config = worker_config or cfg.worker
        self.is_remote = _is_remote(worker_config)
        self.dry_run = DRY_RUN if dry_run is None else dry_run
        if backend is not None:
            self.backend = backend
        else:
            self.backend = _create_backend(self.model_config.engine_type, worker_config, self.dry_run)
            if self.is_remote:
                logger.info("gateway forwarding inference to %s",
                            worker_config.discovery.dns_name or worker_config.endpoints)
            elif self.dry_run:
                logger.info("V-Gate starting in DRY-RUN mode (no GPU required)")
            else:
                self.backend.load_model(self.model_config)

    def chat_completions(self, prompt: str, max_tokens: int = 256):
        """Synchronous helper (benchmarks): one generation with the default sampling."""
        with tracer.start_as_current_span("engine.chat_completions") as span:
            span.set_attribute("prompt_length", len(prompt))
            span.set_attribute("max_tokens", max_tokens)
            sp = self.backend.create_sampling_params(temperature=0.7, top_p=0.9, max_tokens=max_tokens)
            t0 = time.perf_counter()
            r = self.backend.generate([prompt], sp)[0]
            t1 = time.perf_counter()
            n = r["num_tokens"]
            m = r.get("metrics", {}) or {}
            ttft = m.get("ttft", 0.0)
            gen = m.get("gen_time", t1 - t0)
            span.set_attribute("tokens_generated", n)
            return {"text": r["text"], "ttft": ttft, "tpot": (gen / n) if n > 0 else 0, "total_tokens": n}

    def embeddings(self, input_text: str):
        eng = getattr(self.backend, "engine", None)
        if eng is not None and hasattr(eng, "embed"):
            vec, ntok = eng.embed(input_text)
            return {"object": "list", "data": [{"object": "embedding", "embedding": vec, "index": 0}],
                    "model": self.model_config.model_id,
                    "usage": {"prompt_tokens": ntok, "total_tokens": ntok}}
        return {"object": "list",
                "data": [{"object": "embedding", "embedding": [i * 0.01 for i in range(1536)], "index": 0}],
                "model": "mock-embedding-model",
                "usage": {"prompt_tokens": len(input_text), "total_tokens": len(input_text)}}
