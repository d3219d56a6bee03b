"""Device time of a MIXED step (decode rows + one prompt chunk) against a pure decode step (MI355X).

The headline bench (bench.py: concurrency 8, 64 new tokens per request) runs one prompt prefill per
request alongside the other requests' decode rows, so roughly one step in eight carries a prompt
chunk of ~40-50 tokens. This tool builds the engine (random init), brings ``--batch - 1`` sequences
into decode at ``--ctx`` tokens of context, then for every prompt length P adds one request and
times back-to-back hipGraph replays of the step that prefills it together with the decode rows
(and the pure decode step for reference). Prints one JSON line per case.

    python benchmarks/mixed_step.py [--batch 8] [--ctx 100] [--prompts 16,32,48,64,128]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402


def _lins(model):
    return [lin for L in model.layers for lin in (L.qkv, L.o, L.gate_up, L.down)]


def time_graph(eng, iters):
    """Capture the engine's next step (one bucket) and time ``iters`` replays of it."""
    r = eng.runner
    before = set(r.graphs)
    eng.step()
    eng._drain_inflight()
    torch.cuda.synchronize()
    new = [k for k in r.graphs if k not in before]
    key = new[0] if new else None
    if key is None:
        return None, None
    g = r.graphs[key]
    for _ in range(3):
        g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    e.synchronize()
    return key, 1e3 * s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=100)
    ap.add_argument("--prompts", default="16,32,48,64,128")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--burst", type=int, default=0, help="instead: time ONE step prefilling this many prompts "
                    "of --prompts[0] tokens together (a closed-loop wave's arrival), beside the decode rows")
    ap.add_argument("--medium", default="tuned", choices=["tuned", "mid", "default", "wide"],
                    help="medium-bucket GEMM plans (16 < M < 128): the start-up tuner's, the medium-M kernel "
                         "(its heuristic decomposition) everywhere, or the default path everywhere")
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda:0", max_model_len=2048, max_num_seqs=64,
                                 max_num_batched_tokens=2048, num_kv_blocks=4096, warmup=False,
                                 quantization=a.quantization))
    from vgate import ops
    meds = sorted({m for lin in _lins(eng.model) for m in lin.prefill_plan if m < 128})
    if a.medium == "wide":  # the wide medium kernel for gate_up (N >= CUs tiles), the tuner's plans elsewhere
        for L in eng.model.layers:
            for m in meds:
                if m <= 64:
                    L.gate_up.prefill_plan[m] = (ops.MID_BASE - 8, 0)
    elif a.medium != "tuned":
        for lin in _lins(eng.model):
            for m in meds:
                lin.prefill_plan[m] = (ops.MID_BASE - 4, 0) if a.medium == "mid" and m <= 64 else ops.MEDIUM_DEFAULT
    print(json.dumps({"medium": a.medium, "plans": {f"{n}x{k}": {m: p[m] for m in meds if m in p}
                                                    for (n, k), p in eng.prefill_plans.items()}}), flush=True)
    eng.runner.defer_capture = False
    eng.async_sched = False
    sp = SamplingParams(temperature=0.7, top_p=0.9, max_tokens=100000, ignore_eos=True)
    for i in range(a.batch - 1):
        ids = [100 + (i * 131 + j * 17) % 5000 for j in range(a.ctx)]
        eng.add_request(f"r{i}", prompt_ids=ids, params=sp)
    eng._drain_inbox()
    for _ in range(3):
        eng.step()
    for k in list(eng.runner.graphs):
        del eng.runner.graphs[k]
    key, us = time_graph(eng, a.iters)
    if us is not None:
        print(json.dumps({"case": "decode", "rows": a.batch - 1, "bucket": key, "step_us": round(us, 1)}), flush=True)
    if a.burst:
        P = int(a.prompts.split(",")[0])
        for n in range(a.burst):
            ids = [300 + (n * 97 + j * 13) % 5000 for j in range(P)]
            eng.add_request(f"b{n}", prompt_ids=ids, params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=1))
        eng._drain_inbox()
        for k in list(eng.runner.graphs):
            del eng.runner.graphs[k]
        key, us = time_graph(eng, a.iters)
        print(json.dumps({"case": "burst", "prompts": a.burst, "prompt_len": P, "decode_rows": a.batch - 1,
                          "bucket": key, "step_us": None if us is None else round(us, 1)}), flush=True)
        return
    for n, P in enumerate(int(x) for x in a.prompts.split(",")):
        ids = [200 + (n * 71 + j * 13) % 5000 for j in range(P)]
        eng.add_request(f"p{n}", prompt_ids=ids, params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=1))
        eng._drain_inbox()
        for k in list(eng.runner.graphs):
            del eng.runner.graphs[k]
        key, us = time_graph(eng, a.iters)
        print(json.dumps({"case": "mixed", "prompt": P, "decode_rows": a.batch - 1, "bucket": key,
                          "step_us": None if us is None else round(us, 1)}), flush=True)
        for _ in range(2):
            eng.step()


if __name__ == "__main__":
    main()
