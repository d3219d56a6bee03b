"""Result-cache backend micro-benchmark (host only): the reference-semantics Python
OrderedDict LRU vs the native C++ sharded LRU (csrc/runtime/lru_cache.h), per-op cost of
get (hit / miss) + put through ResultCache, single event loop — the gateway's real path.

    python benchmarks/cache_bench.py [--n 20000]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from vgate.cache import ResultCache  # noqa: E402

VALUE = {"text": "the quick brown fox " * 12, "token_ids": list(range(64)), "num_tokens": 64,
         "metrics": {"ttft": 0.01, "gen_time": 0.09, "wall_time": 0.1}}


async def bench(backend: str, n: int, maxsize: int) -> dict:
    c = ResultCache(maxsize=maxsize, enabled=True, backend=backend)
    keys = [ResultCache.make_key(f"prompt {i}", 0.7, 0.9, 64) for i in range(n)]
    t0 = time.perf_counter()
    for k in keys:
        await c.put(k, VALUE)
    t_put = time.perf_counter() - t0
    t0 = time.perf_counter()
    for k in keys[-maxsize:]:
        await c.get(k)
    t_hit = time.perf_counter() - t0
    t0 = time.perf_counter()
    for k in keys[: n - maxsize]:
        await c.get(k)
    t_miss = time.perf_counter() - t0
    return {"backend": backend, "put_us": round(1e6 * t_put / n, 2), "hit_us": round(1e6 * t_hit / maxsize, 2),
            "miss_us": round(1e6 * t_miss / max(1, n - maxsize), 2), "stats": c.get_stats()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--maxsize", type=int, default=1000)
    a = ap.parse_args()
    for b in ("python", "native"):
        print(json.dumps(asyncio.run(bench(b, a.n, a.maxsize))), flush=True)


if __name__ == "__main__":
    main()
