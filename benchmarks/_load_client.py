#!/usr/bin/env python3
"""One load-generating client PROCESS for multi-process saturation runs
(benchmarks/bench_scaling.py --client-procs K).

Waits for a shared wall-clock start barrier (``--start-at`` epoch seconds) so K
clients begin together, runs a closed loop of ``--requests`` at ``--concurrency``,
and prints one JSON line with its CLOCK_MONOTONIC-free window endpoints (wall clock,
comparable across processes on one host) and per-request latencies.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import time


async def run(url: str, n: int, conc: int, max_tokens: int, tag: str) -> dict:
    import aiohttp
    sem = asyncio.Semaphore(conc)
    lat, fails = [], 0
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=600)) as s:
        async def one(i):
            nonlocal fails
            body = {"model": "default", "messages": [{"role": "user", "content": f"[{tag}-{i}] measure me"}],
                    "max_tokens": max_tokens}
            async with sem:
                t0 = time.perf_counter()
                try:
                    async with s.post(f"{url}/v1/chat/completions", json=body) as r:
                        await r.read()
                        if r.status != 200:
                            fails += 1
                            return
                except Exception:  # noqa: BLE001
                    fails += 1
                    return
                lat.append(time.perf_counter() - t0)
        t_start = time.time()
        await asyncio.gather(*(one(i) for i in range(n)))
        t_end = time.time()
    return {"tag": tag, "requests": n, "failures": fails, "t_start": t_start, "t_end": t_end, "latencies": lat}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--requests", type=int, default=100)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=1)
    ap.add_argument("--start-at", type=float, default=0.0)
    ap.add_argument("--tag", default="0")
    a = ap.parse_args()
    delay = a.start_at - time.time()
    if delay > 0:
        time.sleep(delay)
    print(json.dumps(asyncio.run(run(a.url.rstrip("/"), a.requests, a.concurrency, a.max_tokens, a.tag))))


if __name__ == "__main__":
    main()
