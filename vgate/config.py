"""V-Gate configuration: YAML + ``VGATE_*`` environment overrides (drop-in schema).

Priority (highest first): explicit init kwargs > environment > YAML > defaults —
the same contract as the reference (``vgate/config.py:278-298``), implemented on
plain pydantic v2 because pydantic-settings is not available here:

* env vars use the ``VGATE_`` prefix and ``__`` for nesting
  (``VGATE_MODEL__MODEL_ID``, ``VGATE_WORKER__ENDPOINTS='["http://w1:8000"]'``);
* values that parse as JSON (lists, objects, numbers, booleans) are decoded;
* a nested env var replaces only its own key, other YAML keys survive (deep merge).

Every key of the reference schema is kept; the ``model``
section gains the native engine's knobs (TP degree, KV sizing, graph buckets...).
``engine_type`` accepts ``native`` and, for drop-in configs, ``vllm``/``sglang``
which both select the first-party engine.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Any, Optional

import yaml
from pydantic import BaseModel, ConfigDict, Field, field_validator

ENV_PREFIX = "VGATE_"


class _Section(BaseModel):
    model_config = ConfigDict(extra="ignore", protected_namespaces=())


class ServerConfig(_Section):
    host: str = "0.0.0.0"
    port: int = 8000
    # HTTP front end of ``python main.py``: "vgate" (vgate.api.server, lean HTTP/1.1) or
    # "uvicorn" (h11). ``uvicorn main:app`` works either way: the app is plain ASGI.
    http: str = "vgate"
    # front-end limits (both servers): idle keep-alive connections close after this many seconds
    # (uvicorn's default, what the reference deploys); a request whose head + body are not in
    # ``timeout_request`` s after its first byte gets 408; above ``max_connections`` open
    # connections a request gets 503 + Retry-After (uvicorn: limit_concurrency). 0 = off.
    timeout_keep_alive: float = 5.0
    timeout_request: float = 30.0
    max_connections: int = 4096


class WorkerDiscoveryConfig(_Section):
    dns_name: Optional[str] = None
    port: int = 8000
    scheme: str = "http"

    @field_validator("scheme")
    @classmethod
    def _scheme(cls, v: str) -> str:
        if v not in ("http", "https"):
            raise ValueError(f"worker discovery scheme must be http or https, got {v!r}")
        return v


class WorkerConfig(_Section):
    endpoints: list[str] = Field(default_factory=list)
    discovery: WorkerDiscoveryConfig = Field(default_factory=WorkerDiscoveryConfig)
    timeout_seconds: float = 120.0
    connect_timeout_seconds: float = 5.0
    health_check_interval_seconds: float = 5.0
    health_check_timeout_seconds: float = 2.0
    failure_threshold: int = 2
    success_threshold: int = 2
    api_key: Optional[str] = None
    routing: str = "round_robin"  # round_robin | least_inflight
    max_connections: int = 512
    # worker role, SIGTERM: stay up failing /health (503 "draining") and refusing new
    # /internal/generate calls (503: the gateway retries them elsewhere) for at least
    # drain_seconds (>= failure_threshold x health_check_interval_seconds, so every gateway has
    # demoted this worker), finishing the requests already accepted, at most drain_timeout_seconds
    drain_seconds: float = 12.0
    drain_timeout_seconds: float = 120.0

    @field_validator("endpoints")
    @classmethod
    def _endpoints(cls, v: list[str]) -> list[str]:
        for e in v:
            if not e.startswith(("http://", "https://")):
                raise ValueError(f"worker endpoint must start with http:// or https://, got {e!r}")
        return [e.rstrip("/") for e in v]

    @field_validator("routing")
    @classmethod
    def _routing(cls, v: str) -> str:
        if v not in ("round_robin", "least_inflight"):
            raise ValueError("routing must be round_robin or least_inflight")
        return v


class ModelConfig(_Section):
    model_id: str = "Qwen/Qwen2.5-1.5B-Instruct-AWQ"
    quantization: Optional[str] = "awq"
    gpu_memory_utilization: float = 0.7
    max_model_len: int = 2048
    trust_remote_code: bool = True
    enforce_eager: bool = False
    engine_type: str = "native"
    # ---- native engine (MI355X) ----
    tensor_parallel_size: int = 1
    dtype: str = "bfloat16"
    device: str = "auto"
    random_init: bool = True
    # run the engine core in its own process (no GIL shared with the HTTP event loop); TP=1 only
    engine_process: bool = False
    weights_path: Optional[str] = None
    tokenizer: Optional[str] = None
    seed: int = 0
    kv_block_size: int = 16
    num_kv_blocks: Optional[int] = None
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 2048
    enable_prefix_caching: bool = True
    hip_graph_token_buckets: Optional[list[int]] = None
    attention_partition_size: int = 0  # 0 = auto
    # step watchdog: with work pending and no step completed for this long, /health fails (503)
    watchdog_seconds: float = 60.0
    # hipGraphs captured at start-up: token buckets <= graph_warmup_max_tokens x sequence buckets
    # <= graph_warmup_max_seqs (others are captured the first time the engine is idle)
    graph_warmup_max_tokens: int = 512
    graph_warmup_max_seqs: int = 16
    # admission window of an IDLE engine: a closed-loop client's next wave is prefilled in one step
    # (the first arrival waits up to idle_batch_gap_ms for the next, idle_batch_window_ms in all, and
    # only when >= 2 requests finished within idle_batch_recent_ms; vgate/runtime/engine.py)
    idle_batch_window_ms: float = 3.0
    idle_batch_gap_ms: float = 0.6
    idle_batch_recent_ms: float = 20.0
    # start-up timing of the prefill GEMM decompositions per shape and token bucket, and the JSON file
    # the measured plans persist in per (device, native build, shapes) ("" / null = no file)
    prefill_autotune: bool = True
    plan_cache: Optional[str] = "~/.cache/vgate/gemm_plans.json"
    # tensor parallel (tensor_parallel_size > 1): collective / step-ring timeout, the custom IPC
    # all-reduce kernels (false: RCCL for every collective), the all-reduce fused into the decode
    # row-parallel GEMM epilogue, and the start-up self-check of the custom collectives against
    # torch.distributed (a mismatch turns the custom paths off group-wide)
    tp_timeout_seconds: float = 120.0
    tp_custom_allreduce: bool = True
    tp_fused_allreduce: bool = True
    tp_collective_self_check: bool = True
    # run-time TP divergence guard: every N-th step every rank checksums its logits and sampled ids
    # (replicated after the collectives, bit-identical by the fixed-rank-order reductions) and the
    # group compares them; a mismatch turns the custom collectives off group-wide and marks the
    # engine unhealthy. 0 = off
    tp_consistency_interval: int = 256

    @field_validator("engine_type")
    @classmethod
    def _engine_type(cls, v: str) -> str:
        allowed = ("native", "vllm", "sglang")
        if v not in allowed:
            raise ValueError(f"engine_type must be one of {allowed}, got '{v}'")
        return v

    @field_validator("quantization")
    @classmethod
    def _quant(cls, v):
        if v in (None, "", "none", "None"):
            return None
        v = str(v).lower()
        if v not in ("awq",):
            raise ValueError(f"unsupported quantization {v!r} (supported: awq)")
        return v

    @field_validator("kv_block_size")
    @classmethod
    def _bs(cls, v):
        if v != 16:
            raise ValueError("kv_block_size must be 16 (paged attention kernels)")
        return v


class BatchConfig(_Section):
    max_batch_size: int = 8
    max_wait_time_ms: float = 50.0  # accepted for compatibility; admission has no window


class CacheConfig(_Section):
    enabled: bool = True
    maxsize: int = 1000
    # "python": OrderedDict LRU (reference semantics); "native": C++ sharded LRU of JSON bytes
    # (vgate._C.ShardedLRU, per-shard locks, GIL released) — LRU order is per shard
    backend: str = "python"
    shards: int = 16


class InferenceConfig(_Section):
    temperature: float = 0.7
    top_p: float = 0.9
    max_tokens: int = 256


class LoggingConfig(_Section):
    level: str = "INFO"
    json_format: bool = True


class MetricsConfig(_Section):
    enabled: bool = True


class TracingConfig(_Section):
    enabled: bool = False
    service_name: str = "vgate"
    otlp_endpoint: str = "http://localhost:4317"
    otlp_insecure: bool = True
    sample_rate: float = 1.0
    log_correlation: bool = True


class APIKeyConfig(_Section):
    key: str
    name: str
    rate_limit: int = 60


class RateLimitConfig(_Section):
    enabled: bool = True
    default_limit: int = 60
    window_seconds: int = 60


class SecurityConfig(_Section):
    enabled: bool = False
    api_keys: list[APIKeyConfig] = Field(default_factory=list)
    rate_limiting: RateLimitConfig = Field(default_factory=RateLimitConfig)
    exempt_paths: list[str] = Field(default_factory=lambda: ["/health", "/metrics"])


class BenchmarkConfig(_Section):
    warmup_rounds: int = 1
    test_rounds: int = 3
    max_tokens: int = 128
    prompts: list[str] = Field(default_factory=lambda: [
        "Explain the concept of machine learning in one paragraph.",
        "Write a Python function that computes the Fibonacci sequence.",
        "What are the benefits of using a load balancer?",
    ])


class VGateConfig(_Section):
    version: str = "0.3.2"
    role: str = "gateway"
    server: ServerConfig = Field(default_factory=ServerConfig)
    worker: WorkerConfig = Field(default_factory=WorkerConfig)
    model: ModelConfig = Field(default_factory=ModelConfig)
    batch: BatchConfig = Field(default_factory=BatchConfig)
    cache: CacheConfig = Field(default_factory=CacheConfig)
    inference: InferenceConfig = Field(default_factory=InferenceConfig)
    logging: LoggingConfig = Field(default_factory=LoggingConfig)
    metrics: MetricsConfig = Field(default_factory=MetricsConfig)
    security: SecurityConfig = Field(default_factory=SecurityConfig)
    tracing: TracingConfig = Field(default_factory=TracingConfig)
    benchmark: BenchmarkConfig = Field(default_factory=BenchmarkConfig)

    @field_validator("role")
    @classmethod
    def _role(cls, v: str) -> str:
        if v not in ("gateway", "worker"):
            raise ValueError(f"role must be one of ('gateway', 'worker'), got '{v}'")
        return v

    def __init__(self, _yaml: dict | None = None, _env: dict | None = None, **init: Any):
        data = _deep_merge(_yaml or {}, _env if _env is not None else env_overrides())
        data = _deep_merge(data, init)
        super().__init__(**data)


# ----------------------------------------------------------------------------- loading
def _decode(value: str) -> Any:
    s = value.strip()
    if s and (s[0] in "[{\"" or s in ("true", "false", "null") or _is_number(s)):
        try:
            return json.loads(s)
        except json.JSONDecodeError:
            return value
    return value


def _is_number(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def env_overrides(environ: dict | None = None) -> dict:
    """Collect ``VGATE_A__B=...`` variables into a nested dict (keys lower-cased)."""
    env = os.environ if environ is None else environ
    out: dict = {}
    fields = set(VGateConfig.model_fields)
    for k, v in env.items():
        if not k.startswith(ENV_PREFIX):
            continue
        path = [p.lower() for p in k[len(ENV_PREFIX):].split("__") if p]
        if not path or path[0] not in fields:
            continue  # e.g. VGATE_DRY_RUN, VGATE_CONFIG_PATH: not schema keys
        node = out
        for p in path[:-1]:
            nxt = node.get(p)
            if not isinstance(nxt, dict):
                nxt = {}
                node[p] = nxt
            node = nxt
        node[path[-1]] = _decode(v)
    return out


def _deep_merge(base: dict, over: dict) -> dict:
    out = dict(base)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _deep_merge(out[k], v)
        else:
            out[k] = v
    return out


def load_yaml_config(path: str | Path) -> dict:
    p = Path(path)
    if not p.exists():
        raise FileNotFoundError(f"Configuration file not found: {p}")
    with open(p, "r", encoding="utf-8") as f:
        data = yaml.safe_load(f)
    return data or {}


def load_config(path: Optional[str | Path] = None) -> VGateConfig:
    """YAML (if given) < env < nothing else. Missing file -> FileNotFoundError."""
    data = load_yaml_config(path) if path else {}
    return VGateConfig(_yaml=data)


_config: Optional[VGateConfig] = None


def get_config() -> VGateConfig:
    """Process singleton: $VGATE_CONFIG_PATH, else ./config.yaml, else defaults (+env)."""
    global _config
    if _config is None:
        p = os.getenv("VGATE_CONFIG_PATH")
        if p:
            _config = load_config(p)
        elif Path("config.yaml").exists():
            _config = load_config("config.yaml")
        else:
            _config = VGateConfig()
    return _config


def set_config(cfg: VGateConfig) -> None:
    global _config
    _config = cfg


def reset_config() -> None:
    global _config
    _config = None
