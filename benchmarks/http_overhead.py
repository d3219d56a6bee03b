"""Host cost of one /v1/chat/completions round trip on the serving path, without a GPU.

The headline load (bench.py: concurrency 8, equal-length requests that start together) runs in
waves: every request of a wave finishes in the same engine step, and the engine then idles until
the next wave's requests have come through HTTP -> security -> cache -> admission (bench.py's
``timed_engine_idle_ms``: ~5.9 ms per wave of 8 on the MI355X box, ~6.6 % of the bench). This
tool runs the same server (uvicorn + FastAPI app) and the same in-process aiohttp client loop as
bench.py against the dry-run backend with zero simulated latency, so the measured time per
request IS the host path, and optionally profiles it (cProfile, top functions by own time).

    VGATE_DRY_RUN=true python benchmarks/http_overhead.py [--requests 2000] [--profile]
"""
from __future__ import annotations

import argparse
import asyncio
import cProfile
import json
import os
import pstats
import sys
import time
from pathlib import Path

os.environ["VGATE_DRY_RUN"] = "true"
os.environ.setdefault("VGATE_LOGGING__LEVEL", "WARNING")
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402


async def main_async(a):
    from vgate.api.app import create_app
    from vgate.api.server import make_server
    from vgate.config import VGateConfig

    cfg = VGateConfig(role="gateway", batch={"max_batch_size": a.concurrency}, cache={"enabled": True, "maxsize": 1000},
                      logging={"level": "WARNING", "json_format": True},
                      security={"enabled": bool(a.security),
                                "api_keys": [{"key": bench.BENCH_KEY, "name": "bench", "rate_limit": 10_000_000}],
                                "rate_limiting": {"enabled": True, "window_seconds": 60}})
    app = create_app(cfg)
    server = make_server(app, "127.0.0.1", a.port, a.server)
    task = asyncio.create_task(server.serve())
    while not server.started:
        await asyncio.sleep(0.05)
    key = bench.BENCH_KEY if a.security else None
    bench.t_run = time.perf_counter()
    await bench.run_load(a.port, 200, a.concurrency, 64, 0, 0, api_key=key, client=a.client)  # warm-up
    prof = cProfile.Profile() if a.profile else None
    bench.t_run = time.perf_counter()
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    lat, fails, _, _ = (await bench.run_load(a.port, a.requests, a.concurrency, 64, 0, 10_000_000, api_key=key,
                                                client=a.client))[:4]
    if prof:
        prof.disable()
    wall = time.perf_counter() - t0
    server.should_exit = True
    await task
    print(json.dumps({"requests": a.requests, "concurrency": a.concurrency, "security": bool(a.security),
                      "server": a.server, "client": a.client,
                      "req_per_s": round(a.requests / wall, 1), "us_per_request": round(1e6 * wall / a.requests, 1),
                      "p50_ms": round(1e3 * bench.pct(lat, 50), 3), "fails": fails}), flush=True)
    if prof:
        st = pstats.Stats(prof)
        st.sort_stats("tottime").print_stats(a.top)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=2000)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--port", type=int, default=18300)
    ap.add_argument("--security", action="store_true")
    ap.add_argument("--server", default="vgate", choices=["vgate", "uvicorn"])
    ap.add_argument("--client", default="lean", choices=["lean", "aiohttp"])
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--top", type=int, default=35)
    a = ap.parse_args()
    asyncio.run(main_async(a))


if __name__ == "__main__":
    main()
