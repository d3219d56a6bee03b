"""Host cost of one /v1/chat/completions round trip on the serving path, without a GPU.

The headline load (bench.py: concurrency 8, equal-length requests that start together) runs in
waves: every request of a wave finishes in the same engine step, and the engine then idles until
the next wave's requests have come through HTTP -> security -> cache -> admission (bench.py's
``timed_engine_idle_ms``: ~5.9 ms per wave of 8 on the MI355X box, ~6.6 % of the bench). This
tool runs the same server (uvicorn + FastAPI app) and the same in-process aiohttp client loop as
bench.py against the dry-run backend with zero simulated latency, so the measured time per
request IS the host path, and optionally profiles it (cProfile, top functions by own time).

    VGATE_DRY_RUN=true python benchmarks/http_overhead.py [--requests 2000] [--profile]
    python benchmarks/http_overhead.py --waves    # the wave-boundary gap itself (see main_waves)
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


class _WaveBackend:
    """Dry-run backend that answers every request after the same fixed delay: a closed-loop client at
    concurrency c then runs in waves of c, exactly like the headline load on the engine."""
    supports_concurrent_calls = True
    supports_streaming = False

    def __init__(self, delay_s: float):
        self.delay = delay_s
        self.arr: list = []
        self.fin: list = []

    def create_sampling_params(self, temperature, top_p, max_tokens):
        return {"temperature": temperature, "top_p": top_p, "max_tokens": max_tokens}

    async def agenerate(self, prompt, sp):
        self.arr.append(time.perf_counter())
        await asyncio.sleep(self.delay)
        self.fin.append(time.perf_counter())
        return {"text": "x" * 256, "num_tokens": sp["max_tokens"], "prompt_tokens": 30, "finish_reason": "length",
                "metrics": {}}

    def shutdown(self):
        pass


async def main_waves(a):
    """Wave-boundary gap: from the last response of wave k leaving the backend to the first (and the
    last) request of wave k+1 reaching it — the engine's idle time per wave in bench.py
    (timed_engine_idle_ms / timed_waves), without a GPU."""
    from vgate.api.app import create_app
    from vgate.api.server import make_server
    from vgate.config import VGateConfig
    from vgate.engine import VGateEngine

    cfg = VGateConfig(role="gateway", batch={"max_batch_size": a.concurrency}, cache={"enabled": True, "maxsize": 1000},
                      logging={"level": "WARNING", "json_format": True})
    be = _WaveBackend(0.02)
    eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=be, dry_run=True)
    app = create_app(cfg, engine=eng)
    server = make_server(app, "127.0.0.1", a.port, a.server)
    task = asyncio.create_task(server.serve())
    while not server.started:
        await asyncio.sleep(0.05)
    bench.t_run = time.perf_counter()
    c = a.concurrency
    await bench.run_load(a.port, 10 * c, c, 64, 0, 0, client=a.client)
    be.arr.clear()
    be.fin.clear()
    nw = max(10, a.requests // c)
    await bench.run_load(a.port, nw * c, c, 64, 0, 10_000_000, client=a.client)
    server.should_exit = True
    await task
    first, last = [], []
    for w in range(1, nw):
        arr = sorted(be.arr[w * c:(w + 1) * c])
        fin = sorted(be.fin[(w - 1) * c:w * c])
        first.append(arr[0] - fin[-1])
        last.append(arr[-1] - fin[-1])
    print(json.dumps({"waves": nw, "concurrency": c, "server": a.server, "client": a.client,
                      "gap_first_arrival_ms_p50": round(1e3 * bench.pct(first, 50), 3),
                      "gap_last_arrival_ms_p50": round(1e3 * bench.pct(last, 50), 3)}), flush=True)


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
    ap.add_argument("--waves", action="store_true", help="measure the wave-boundary gap instead")
    a = ap.parse_args()
    asyncio.run(main_waves(a) if a.waves else main_async(a))


if __name__ == "__main__":
    main()
