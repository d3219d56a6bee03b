#!/usr/bin/env python3
"""Run ONE report scenario in a fresh server process and write its JSON — long GPU runs
split into short invocations (reference benchmarks/_run_scenario_cli.py), merged later by
``benchmarks/aggregate_results.py``.

    python benchmarks/run_scenario_cli.py baseline --out-dir benchmarks/results/scenarios
    python benchmarks/run_scenario_cli.py --list
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

from bench_load import DEFAULT_PROMPTS, run_load_test  # noqa: E402
from run_report import scenarios, start_server  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("scenario", nargs="?")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--engine", default="native", choices=["native", "dry-run"])
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--requests", type=int, default=40)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--port", type=int, default=8120)
    ap.add_argument("--dry-latency-ms", type=float, default=15.0)
    ap.add_argument("--boot-timeout", type=float, default=600.0)
    ap.add_argument("--out-dir", default=str(Path(__file__).resolve().parent / "results" / "scenarios"))
    a = ap.parse_args()
    a.quick = False
    table = {name: (mbs, cache) for name, mbs, cache in scenarios(a)}
    if a.list or not a.scenario:
        print("\n".join(table))
        return
    if a.scenario not in table:
        ap.error(f"unknown scenario {a.scenario!r}; one of {sorted(table)}")
    mbs, cache = table[a.scenario]
    out_dir = Path(a.out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    srv = start_server(a, mbs, cache, out_dir)
    try:
        url = f"http://127.0.0.1:{a.port}"
        asyncio.run(run_load_test(url, a.concurrency, a.concurrency, DEFAULT_PROMPTS, 8, unique=True))
        prompts = DEFAULT_PROMPTS[:3] if cache else DEFAULT_PROMPTS
        t0 = time.time()
        r = asyncio.run(run_load_test(url, a.concurrency, a.requests, prompts, a.max_tokens, unique=not cache))
    finally:
        srv.stop()
    r["scenario"] = {"name": a.scenario, "max_batch_size": mbs, "cache": cache, "started": t0,
                     "engine": a.engine, "model": a.model}
    path = out_dir / f"{a.scenario}.json"
    path.write_text(json.dumps(r, indent=2))
    print(json.dumps({"scenario": a.scenario, "req_s": r["throughput"]["requests_per_second"],
                      "p50_s": r["latency"]["p50_s"], "p99_s": r["latency"]["p99_s"], "file": str(path)}))


if __name__ == "__main__":
    main()
