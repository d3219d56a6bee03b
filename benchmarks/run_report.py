#!/usr/bin/env python3
"""Benchmark report orchestrator: one FRESH server process per scenario, then a markdown
report (reference benchmarks/run_report.py:73-115, :191-208 — same scenario set).

Scenarios (all against ``/v1/chat/completions`` through the full gateway pipeline):
  * baseline        — admission window (max_batch_size) 8, unique prompts;
  * sweep           — max_batch_size in {1, 4, 16, 32}, unique prompts;
  * cache_impact    — 3 repeated prompts (result cache + request coalescing on).

Each server runs in its own process group and is torn down as a group, so no engine
process outlives its scenario. ``--engine native`` serves the MI355X engine (random-init
weights of ``--model``); ``--engine dry-run`` uses the synthetic backend with a fixed
latency (default 15 ms) for a CPU-only smoke of the harness itself.

    python benchmarks/run_report.py --engine native --requests 40 --concurrency 8
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

from bench_load import DEFAULT_PROMPTS, format_markdown, run_load_test  # noqa: E402
from bench_scaling import Proc, base_env, wait_http, wait_ports_free  # noqa: E402


def scenarios(a):
    out = [("baseline", 8, False)]
    if not a.quick:
        out += [(f"sweep_mbs{m}", m, False) for m in (1, 4, 16, 32)]
    out.append(("cache_impact", 8, True))
    return out


def start_server(a, mbs: int, cache: bool, logdir: Path) -> Proc:
    wait_ports_free([a.port])
    env = dict(VGATE_ROLE="gateway", VGATE_SERVER__HOST="127.0.0.1", VGATE_SERVER__PORT=a.port,
               VGATE_BATCH__MAX_BATCH_SIZE=mbs, VGATE_CACHE__ENABLED="true" if cache else "false",
               VGATE_MODEL__MODEL_ID=a.model)
    if a.engine == "dry-run":
        env.update(VGATE_DRY_RUN="true", VGATE_DRYRUN_SIMULATED_LATENCY_MS=a.dry_latency_ms)
    else:
        env.update(VGATE_DRY_RUN="false", VGATE_MODEL__ENGINE_TYPE="native")
    p = Proc(base_env(**env), logdir / f"server_mbs{mbs}_{int(cache)}.log")
    wait_http(f"http://127.0.0.1:{a.port}/ready", a.boot_timeout)
    return p


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--engine", default="native", choices=["native", "dry-run"])
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--requests", type=int, default=40)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--port", type=int, default=8120)
    ap.add_argument("--dry-latency-ms", type=float, default=15.0)
    ap.add_argument("--boot-timeout", type=float, default=600.0)
    ap.add_argument("--quick", action="store_true", help="baseline + cache scenarios only")
    ap.add_argument("--out", default=str(Path(__file__).resolve().parent / "results" / "report"))
    a = ap.parse_args()
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    logdir = out.parent / "logs"
    logdir.mkdir(exist_ok=True)
    results = {}
    for name, mbs, cache in scenarios(a):
        srv = start_server(a, mbs, cache, logdir)
        try:
            url = f"http://127.0.0.1:{a.port}"
            # warm graphs / caches outside the measurement
            asyncio.run(run_load_test(url, a.concurrency, a.concurrency, DEFAULT_PROMPTS, 8, unique=True))
            prompts = DEFAULT_PROMPTS[:3] if cache else DEFAULT_PROMPTS
            t0 = time.time()
            r = asyncio.run(run_load_test(url, a.concurrency, a.requests, prompts, a.max_tokens, unique=not cache))
            r["scenario"] = {"name": name, "max_batch_size": mbs, "cache": cache, "started": t0}
            results[name] = r
            print(json.dumps({"scenario": name, "req_s": r["throughput"]["requests_per_second"],
                              "p50_s": r["latency"]["p50_s"], "p99_s": r["latency"]["p99_s"]}), flush=True)
        finally:
            srv.stop()
    out.with_suffix(".json").write_text(json.dumps(results, indent=2))
    md = [f"# V-Gate benchmark report ({a.engine}, {a.model})", ""]
    for name, r in results.items():
        md.append(format_markdown(r, title=name))
        md.append("")
    out.with_suffix(".md").write_text("\n".join(md))
    print(f"wrote {out.with_suffix('.md')}")


if __name__ == "__main__":
    main()
