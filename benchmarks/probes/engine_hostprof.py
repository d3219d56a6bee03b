"""Host-side profile of the engine loop (no HTTP): the engine is stepped on the MAIN thread
in a closed loop (a finished request immediately submits the next one), under cProfile,
so the per-step Python cost (schedule / launch / collect / post-process) is attributed
to functions. Prints the top entries by cumulative and by own time, plus the un-profiled
step time of the same loop for comparison.

    python benchmarks/engine_hostprof.py [--concurrency 8 --requests 40 --max-tokens 64]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402


def run(eng, concurrency, n_requests, max_tokens, tag):
    state = {"issued": 0, "done": 0}

    def submit():
        i = state["issued"]
        state["issued"] += 1
        prompt = [100 + (i * 7919 + j * 104729) % 150000 for j in range(24)]
        eng.add_request(f"{tag}{i}", params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=max_tokens,
                                                          ignore_eos=True), callback=cb, prompt_ids=prompt)

    def cb(kind, seq, payload):
        if kind == "token":
            return
        state["done"] += 1
        if state["issued"] < n_requests:
            submit()

    for _ in range(min(concurrency, n_requests)):
        submit()
    steps = 0
    t0 = time.perf_counter()
    while state["done"] < n_requests:
        eng._drain_inbox()
        eng.step()
        steps += 1
    eng._drain_inflight()
    return time.perf_counter() - t0, steps


def run_threaded(eng, concurrency, n_requests, max_tokens, tag, external):
    """engine on its own thread (eng.start()); completions re-submit from the engine thread
    (external=False) or from this (main) thread woken per completion (external=True, the
    pattern of a server thread handing results back)."""
    import threading
    state = {"issued": 0, "done": 0, "steps0": eng.stats.steps}
    done_all, wake = threading.Event(), threading.Semaphore(0)

    def submit():
        i = state["issued"]
        state["issued"] += 1
        prompt = [100 + (i * 7919 + j * 104729) % 150000 for j in range(24)]
        eng.add_request(f"{tag}{i}", params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=max_tokens,
                                                          ignore_eos=True), callback=cb, prompt_ids=prompt)

    def cb(kind, seq, payload):
        if kind == "token":
            return
        state["done"] += 1
        if state["done"] == n_requests:
            done_all.set()
        if external:
            wake.release()
        elif state["issued"] < n_requests:
            submit()

    t0 = time.perf_counter()
    for _ in range(min(concurrency, n_requests)):
        submit()
    if external:
        while state["issued"] < n_requests:
            wake.acquire()
            submit()
    done_all.wait()
    return time.perf_counter() - t0, eng.stats.steps - state["steps0"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--requests", type=int, default=40)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--threaded", action="store_true")
    ap.add_argument("--switch-us", type=float, default=0, help="sys.setswitchinterval (0 = leave)")
    a = ap.parse_args()
    if a.switch_us:
        sys.setswitchinterval(a.switch_us * 1e-6)
    eng = LLMEngine(EngineConfig(model=a.model, max_model_len=2048, max_num_seqs=256, num_kv_blocks=8192))
    run(eng, a.concurrency, 2 * a.concurrency, 16, "w")  # graphs
    eng.runner.capture_pending()
    wall, steps = run(eng, a.concurrency, a.requests, a.max_tokens, "a")
    print(json.dumps({"unprofiled_ms_per_step": round(1e3 * wall / steps, 3), "steps": steps,
                      "req_s": round(a.requests / wall, 2)}), flush=True)
    if a.threaded:
        eng.cfg.warmup = False  # graphs already captured by the main-thread runs
        eng.start()
        for ext in (False, True):
            wall, steps = run_threaded(eng, a.concurrency, a.requests, a.max_tokens, f"t{int(ext)}", ext)
            print(json.dumps({"threaded": True, "external_submit": ext, "ms_per_step": round(1e3 * wall / steps, 3),
                              "steps": steps, "req_s": round(a.requests / wall, 2),
                              "switchinterval": sys.getswitchinterval()}), flush=True)
        eng.stop()
        return
    pr = cProfile.Profile()
    pr.enable()
    wall, steps = run(eng, a.concurrency, a.requests, a.max_tokens, "p")
    pr.disable()
    print(json.dumps({"profiled_ms_per_step": round(1e3 * wall / steps, 3), "steps": steps}), flush=True)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
