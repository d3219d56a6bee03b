#!/usr/bin/env python3
"""In-process backend comparison: drive ``VGateEngine.chat_completions`` directly (no
HTTP) for each selected backend and print a table or JSON (reference
benchmarks/bench_compare.py:42-178).

Backends: ``native`` (the MI355X engine), ``dry-run`` (synthetic), and ``vllm`` /
``sglang`` — those names select the native engine in this framework (drop-in config
values), so comparing them measures the same engine.

    python benchmarks/bench_compare.py --backends native dry-run --prompts 16 --rounds 3
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def run_backend(name: str, a) -> dict:
    from vgate.backends.base import DryRunBackend
    from vgate.config import get_config, reset_config
    from vgate.engine import VGateEngine

    reset_config()
    cfg = get_config()
    if name == "dry-run":
        eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=DryRunBackend(), dry_run=True)
    else:
        cfg.model.engine_type = "native" if name in ("native", "vllm", "sglang") else name
        eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, dry_run=False)
    from concurrent.futures import ThreadPoolExecutor
    prompts = [f"[{i}] Explain the concept of machine learning in one paragraph." for i in range(a.prompts)]
    eng.chat_completions(prompts[0], max_tokens=4)  # warm-up
    lat, toks = [], 0
    t_all = time.perf_counter()
    with ThreadPoolExecutor(max_workers=a.prompts) as ex:  # one round = all prompts concurrently
        for _ in range(a.rounds):
            t0 = time.perf_counter()
            outs = list(ex.map(lambda p: eng.chat_completions(p, max_tokens=a.max_tokens), prompts))
            lat.append(time.perf_counter() - t0)
            toks += sum(o.get("total_tokens", 0) for o in outs)
    wall = time.perf_counter() - t_all
    return {"backend": name, "rounds": a.rounds, "prompts_per_round": a.prompts,
            "round_latency_mean_s": round(statistics.mean(lat), 4), "round_latency_min_s": round(min(lat), 4),
            "tokens": toks, "tokens_per_second": round(toks / wall, 1),
            "requests_per_second": round(a.rounds * a.prompts / wall, 2)}


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--backends", nargs="+", default=["native", "dry-run"])
    ap.add_argument("--prompts", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--output", choices=["table", "json"], default="table")
    a = ap.parse_args()
    os.environ.setdefault("VGATE_LOGGING__LEVEL", "WARNING")
    rows = [run_backend(b, a) for b in a.backends]
    if a.output == "json":
        print(json.dumps(rows, indent=2))
        return
    cols = ["backend", "requests_per_second", "tokens_per_second", "round_latency_mean_s", "round_latency_min_s"]
    print(" | ".join(cols))
    print(" | ".join("---" for _ in cols))
    for r in rows:
        print(" | ".join(str(r[c]) for c in cols))


if __name__ == "__main__":
    main()
