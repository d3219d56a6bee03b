"""Prometheus metric catalog.

Names, label sets and buckets of the reference catalog are kept
byte-for-byte so dashboards and the benchmark scrapers (``vgate_stream_tokens_total``,
``vgate_worker_requests_total{outcome,worker}``) keep working; the native engine
adds ``vgate_engine_*`` series (step latency, KV usage, hipGraph replays, ...).
"""
from __future__ import annotations

from prometheus_client import REGISTRY, Counter, Gauge, Histogram, Info


def _metric(cls, name, doc, labelnames=None, buckets=None):
    """Create a collector, or return the already-registered one (module reloads in tests)."""
    kw = {}
    if labelnames:
        kw["labelnames"] = labelnames
    if buckets is not None and cls is Histogram:
        kw["buckets"] = buckets
    try:
        return cls(name, doc, **kw)
    except ValueError:
        base = name[:-6] if name.endswith("_total") else name
        for key in (name, base, base + "_info"):
            col = REGISTRY._names_to_collectors.get(key)  # noqa: SLF001
            if col is not None:
                return col
        raise


APP_INFO = _metric(Info, "vgate", "V-Gate application information")

# ---- HTTP
REQUEST_COUNT = _metric(Counter, "vgate_requests_total", "Total HTTP requests",
                        ["endpoint", "method", "status"])
REQUEST_LATENCY = _metric(Histogram, "vgate_request_latency_seconds", "HTTP request latency",
                          ["endpoint", "method"],
                          [0.001, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0])
REQUEST_IN_PROGRESS = _metric(Gauge, "vgate_requests_in_progress", "HTTP requests in progress", ["endpoint"])

# ---- batcher / admission
BATCH_SIZE = _metric(Histogram, "vgate_batch_size", "Requests per backend call",
                     buckets=[1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 24, 32])
BATCH_PROCESSING_TIME = _metric(Histogram, "vgate_batch_processing_seconds", "Backend call duration",
                                buckets=[0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0])
BATCH_QUEUE_TIME = _metric(Histogram, "vgate_batch_queue_time_seconds", "Time waiting for an admission permit",
                           buckets=[0.001, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5])
PENDING_REQUESTS = _metric(Gauge, "vgate_pending_requests", "Requests waiting for an admission permit")
INFLIGHT_INFERENCES = _metric(Gauge, "vgate_inflight_inferences", "Inferences currently running")
ABANDONED_INFERENCES = _metric(Counter, "vgate_abandoned_inferences_total",
                               "Queued inferences cancelled because every waiter gave up")
TOTAL_BATCHES = _metric(Counter, "vgate_batches_total", "Backend calls issued")

# ---- inference
TTFT = _metric(Histogram, "vgate_ttft_seconds", "Time to first token (engine)",
               buckets=[0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.0, 5.0])
TPOT = _metric(Histogram, "vgate_tpot_seconds", "Time per output token (engine)",
               buckets=[0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1])
TOKENS_GENERATED = _metric(Counter, "vgate_tokens_generated_total", "Generated tokens")
INFERENCE_ERRORS = _metric(Counter, "vgate_inference_errors_total", "Inference errors", ["error_type"])
UNIQUE_PROMPTS_PER_BATCH = _metric(Histogram, "vgate_unique_prompts_per_batch", "Unique prompts per batch",
                                   buckets=[1, 2, 3, 4, 5, 6, 7, 8, 12, 16])

# ---- streaming
STREAM_TTFT = _metric(Histogram, "vgate_stream_ttft_seconds", "Streaming time to first token (gateway clock)",
                      buckets=[0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.0, 5.0])
STREAM_TPOT = _metric(Histogram, "vgate_stream_tpot_seconds", "Streaming time per output token",
                      buckets=[0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1])
STREAM_DURATION = _metric(Histogram, "vgate_stream_duration_seconds", "Streaming request duration",
                          buckets=[0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0])
STREAM_TOKENS = _metric(Counter, "vgate_stream_tokens_total", "Tokens streamed")
STREAM_REQUESTS = _metric(Counter, "vgate_stream_requests_total", "Streaming requests by outcome", ["status"])

# ---- result cache / dedup
CACHE_HITS = _metric(Counter, "vgate_cache_hits_total", "Result cache hits")
CACHE_MISSES = _metric(Counter, "vgate_cache_misses_total", "Result cache misses")
CACHE_SIZE = _metric(Gauge, "vgate_cache_size", "Result cache entries")
CACHE_EVICTIONS = _metric(Counter, "vgate_cache_evictions_total", "Result cache evictions")
DEDUPLICATED_REQUESTS = _metric(Counter, "vgate_deduplicated_requests_total", "Requests coalesced onto in-flight work")
DEDUP_RATIO = _metric(Gauge, "vgate_dedup_ratio", "Deduplicated / total requests")

# ---- remote workers
WORKER_HEALTHY = _metric(Gauge, "vgate_worker_healthy", "1 if the worker is in rotation", ["worker"])
WORKER_STATE_CHANGES = _metric(Counter, "vgate_worker_state_changes_total", "Worker membership transitions",
                               ["worker", "transition"])
WORKER_REQUESTS = _metric(Counter, "vgate_worker_requests_total", "Requests sent to workers by outcome",
                          ["worker", "outcome"])
WORKER_RETRIES = _metric(Counter, "vgate_worker_retries_total", "Retries moved to another worker", ["worker"])
WORKER_LATENCY = _metric(Histogram, "vgate_worker_latency_seconds", "Worker request latency", ["worker"])

# ---- native engine (MI355X)
ENGINE_STEP_SECONDS = _metric(Histogram, "vgate_engine_step_seconds", "Engine step (forward+sample) latency",
                              buckets=[0.0005, 0.001, 0.002, 0.004, 0.008, 0.016, 0.032, 0.064, 0.128, 0.5])
ENGINE_RUNNING = _metric(Gauge, "vgate_engine_running_sequences", "Sequences in the running batch")
ENGINE_WAITING = _metric(Gauge, "vgate_engine_waiting_sequences", "Sequences waiting for admission")
ENGINE_KV_USAGE = _metric(Gauge, "vgate_engine_kv_cache_usage_ratio", "Fraction of KV blocks in use")
ENGINE_PREFILL_TOKENS = _metric(Counter, "vgate_engine_prefill_tokens_total", "Prompt tokens computed")
ENGINE_DECODE_TOKENS = _metric(Counter, "vgate_engine_decode_tokens_total", "Decode tokens computed")
ENGINE_GRAPH_REPLAYS = _metric(Counter, "vgate_engine_hipgraph_replays_total", "Steps replayed from a hipGraph")
ENGINE_PREEMPTIONS = _metric(Counter, "vgate_engine_preemptions_total", "Sequences preempted for KV memory")
ENGINE_PREFIX_HITS = _metric(Counter, "vgate_engine_prefix_cache_hit_blocks_total", "KV blocks reused from the prefix cache")
ENGINE_EAGER_STEPS = _metric(Counter, "vgate_engine_eager_steps_total",
                             "Steps run without a captured hipGraph (first sight of a token/sequence bucket)")
ENGINE_GRAPH_HIT_RATIO = _metric(Gauge, "vgate_engine_hipgraph_hit_ratio", "hipGraph replays / all steps (lifetime)")
ENGINE_HEALTHY = _metric(Gauge, "vgate_engine_healthy", "1 while the engine passes its fault and watchdog checks")
ENGINE_TP_CUSTOM_COLLECTIVES = _metric(Gauge, "vgate_engine_tp_custom_collectives",
                                       "1 while the TP group runs its custom IPC collectives (0: RCCL only, e.g. "
                                       "after a failed start-up self-check)")
ENGINE_ALLREDUCE_SECONDS = _metric(Histogram, "vgate_engine_allreduce_seconds",
                                   "Tensor-parallel all-reduce time per decode step (probed on the engine's own "
                                   "comm path: every layer's two collectives at the decode message size)",
                                   buckets=[1e-5, 2.5e-5, 5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2])


def init_app_info(version: str, model: str) -> None:
    APP_INFO.info({"version": version, "model": model})
