"""LRU result cache for completed generations (reference ``vgate/cache.py:28-108`` behavior).

Key = first 16 hex chars of sha256 over the sorted-key JSON of
``{prompt, temperature, top_p, max_tokens}`` — identical to the reference so
keys stay stable across the swap. Differences (fixes of SURVEY.md §2.9): hits
return a *copy* of the stored dict, so callers cannot mutate the cache.
"""
from __future__ import annotations

import contextlib
import copy
import hashlib
import json
from collections import OrderedDict
from typing import Any, Optional

from vgate.config import get_config
from vgate.logging_config import get_logger
from vgate.metrics import CACHE_EVICTIONS, CACHE_HITS, CACHE_MISSES, CACHE_SIZE
from vgate.tracing import _NOOP, get_tracer, is_tracing_enabled

logger = get_logger("vgate.cache")
tracer = get_tracer(__name__)
_NO_SPAN = contextlib.nullcontext(_NOOP)
_SCALARS = (str, int, float, bool, type(None), bytes)


def _copy(d: dict) -> dict:
    """Copy of a result dict: shallow where every value is immutable (the common case: text,
    counts, timings), a deepcopy otherwise."""
    for v in d.values():
        if type(v) not in _SCALARS:
            return copy.deepcopy(d)
    return dict(d)


class ResultCache:
    def __init__(self, maxsize: Optional[int] = None, enabled: Optional[bool] = None,
                 backend: Optional[str] = None):
        cfg = get_config()
        self.maxsize = maxsize if maxsize is not None else cfg.cache.maxsize
        self.enabled = enabled if enabled is not None else cfg.cache.enabled
        self.backend = (backend or getattr(cfg.cache, "backend", "python")).lower()
        self._native = None
        if self.backend == "native":
            # C++ sharded LRU (csrc/runtime/lru_cache.h): values stored as JSON bytes, so a
            # hit is a fresh object by construction (no deepcopy)
            from vgate import ops
            self._native = ops.native().ShardedLRU(max(0, self.maxsize), int(getattr(cfg.cache, "shards", 16)))
        elif self.backend != "python":
            raise ValueError(f"cache.backend must be python or native, got {self.backend!r}")
        self._data: OrderedDict[str, dict] = OrderedDict()
        self.hits = 0
        self.misses = 0
        self.evictions = 0

    @staticmethod
    def make_key(prompt: str, temperature: float, top_p: float, max_tokens: int) -> str:
        blob = json.dumps({"prompt": prompt, "temperature": temperature, "top_p": top_p,
                           "max_tokens": max_tokens}, sort_keys=True)
        return hashlib.sha256(blob.encode("utf-8")).hexdigest()[:16]

    async def get(self, key: str) -> Optional[dict[str, Any]]:
        return self.get_nowait(key)

    async def put(self, key: str, value: dict[str, Any]) -> None:
        self.put_nowait(key, value)

    def get_nowait(self, key: str) -> Optional[dict[str, Any]]:
        """Lookup (a fresh copy on a hit). Synchronous: the whole operation runs without yielding
        to the event loop, which is what the reference's asyncio.Lock guaranteed."""
        if not self.enabled:
            return None
        with (tracer.start_as_current_span("cache.get") if is_tracing_enabled() else _NO_SPAN) as span:
            if self._native is not None:
                raw = self._native.get(key)
                hit = raw is not None
                span.set_attribute("hit", hit)
                if not hit:
                    self.misses += 1
                    CACHE_MISSES.inc()
                    return None
                self.hits += 1
                CACHE_HITS.inc()
                if logger.isEnabledFor(10):
                    logger.debug("Cache hit", extra={"extra_data": {"cache_key": key[:8]}})
                return json.loads(raw)
            val = self._data.get(key)
            if val is None:
                self.misses += 1
                CACHE_MISSES.inc()
                span.set_attribute("hit", False)
                return None
            self._data.move_to_end(key)
            self.hits += 1
            CACHE_HITS.inc()
            span.set_attribute("hit", True)
            if logger.isEnabledFor(10):  # DEBUG; the check keeps the hot path free of record building
                logger.debug("Cache hit", extra={"extra_data": {"cache_key": key[:8]}})
            return _copy(val)

    def put_nowait(self, key: str, value: dict[str, Any]) -> None:
        if not self.enabled or self.maxsize <= 0:
            return
        with (tracer.start_as_current_span("cache.put") if is_tracing_enabled() else _NO_SPAN):
            if self._native is not None:
                ev = self._native.put(key, json.dumps(value, separators=(",", ":")).encode())
                if ev:
                    self.evictions += ev
                    CACHE_EVICTIONS.inc(ev)
                CACHE_SIZE.set(len(self._native))
                return
            if key in self._data:
                self._data.move_to_end(key)
            self._data[key] = _copy(value)
            while len(self._data) > self.maxsize:
                old, _ = self._data.popitem(last=False)
                self.evictions += 1
                CACHE_EVICTIONS.inc()
                logger.debug("Cache eviction", extra={"extra_data": {"cache_key": old[:8]}})
            CACHE_SIZE.set(len(self._data))

    async def clear(self) -> None:
        if self._native is not None:
            self._native.clear()
        self._data.clear()
        CACHE_SIZE.set(0)

    def __len__(self) -> int:
        return len(self._native) if self._native is not None else len(self._data)

    def get_stats(self) -> dict[str, Any]:
        total = self.hits + self.misses
        return {"size": len(self), "maxsize": self.maxsize, "hits": self.hits, "misses": self.misses,
                "evictions": self.evictions, "hit_rate": round(self.hits / total, 4) if total else 0.0}
