"""Engine-level throughput/latency microbenchmark (no HTTP): closed-loop concurrency
against the native engine, plus a pure decode-step timing.

    python benchmarks/bench_engine.py --model Qwen/Qwen2.5-1.5B-Instruct --concurrency 8 --requests 40
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(int(len(xs) * p / 100), len(xs) - 1)] if xs else 0.0


def closed_loop(eng, concurrency, n_requests, max_tokens, prompt_len=24):
    lat, sem = [], threading.Semaphore(concurrency)
    lock = threading.Lock()
    done_all = threading.Event()
    state = {"done": 0, "issued": 0}
    t_start = {}

    def cb(kind, seq, payload):
        if kind == "token":
            return
        with lock:
            lat.append(time.perf_counter() - t_start[seq.request_id])
            state["done"] += 1
            if state["done"] == n_requests:
                done_all.set()
        sem.release()

    t0 = time.perf_counter()
    for i in range(n_requests):
        sem.acquire()
        rid = f"b{i}"
        prompt = [100 + (i * 7919 + j * 104729) % 150000 for j in range(prompt_len)]
        t_start[rid] = time.perf_counter()
        eng.add_request(rid, params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=max_tokens,
                                                   ignore_eos=True), callback=cb, prompt_ids=prompt)
    done_all.wait()
    wall = time.perf_counter() - t0
    return {"req_s": n_requests / wall, "p50": pct(lat, 50), "p99": pct(lat, 99), "wall": wall,
            "tok_s": n_requests * max_tokens / wall}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--requests", type=int, default=40)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--decode-batch", type=int, default=8)
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, max_model_len=2048, max_num_seqs=256, enforce_eager=a.eager,
                                 quantization=a.quantization, num_kv_blocks=8192))
    eng.start()
    closed_loop(eng, a.concurrency, 2 * a.concurrency, 16)  # warm graphs
    r = closed_loop(eng, a.concurrency, a.requests, a.max_tokens)
    snap = eng.snapshot()
    eng.stop()
    r.update({"avg_step_ms": snap["avg_step_ms"], "graphs": snap["graphs_captured"],
              "avg_cycle_ms": snap["avg_cycle_ms"], "avg_gpu_ms": snap["avg_gpu_ms"], "avg_host_ms": snap["avg_host_ms"],
              "weights_gb": eng.model.weight_bytes() / 1e9})
    # pure decode step timing at a fixed batch
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
