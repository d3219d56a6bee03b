"""In-graph launch timeline of one engine decode step on the MI355X.

Every kernel of a freshly captured decode hipGraph stamps its blocks' [start, end] with the
100 MHz s_memrealtime clock (TLScope, csrc/kernels/common.h), so one replay shows, per
launch: the block span (first block start -> last block end) and the gap to the next
launch's first block — i.e. how much of the step is kernel bodies and how much is launch
boundaries / dispatch / drain, which rocprof's per-kernel durations cannot separate.

    python benchmarks/timeline.py [--batch 8] [--steps 4] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402
from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402

TICKS_PER_US = 100.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=40, help="prompt tokens per sequence")
    ap.add_argument("--kv-blocks", type=int, default=0, help="KV pool size in blocks (0 = engine sizing)")
    ap.add_argument("--max-seqs", type=int, default=64)
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--mixed", type=int, default=0, help="time a MIXED step: one prompt of this many tokens "
                    "beside the decode rows (benchmarks/mixed_step.py)")
    ap.add_argument("--wide-gate-up", action="store_true", help="medium buckets: the wide medium kernel for gate_up")
    ap.add_argument("--prefill", action="store_true", help="time the PREFILL step of the batch (its prompts as one "
                    "multi-prompt step) instead of a decode step")
    ap.add_argument("--replays", type=int, default=0,
                    help="after the measured step, replay its graph N times back to back (no host sync between) "
                         "and report the last replay too: a hole that only the first replay shows is the host's "
                         "graph launch, not the GPU")
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda:0", max_model_len=2048, max_num_seqs=a.max_seqs,
                                 max_num_batched_tokens=2048, num_kv_blocks=a.kv_blocks or None, warmup=False,
                                 quantization=a.quantization))
    eng.runner.defer_capture = False  # capture each bucket on first sight: the measured step replays a graph
    for i in range(a.batch):
        ids = [100 + (i * 131 + j * 17) % 5000 for j in range(a.ctx)]
        eng.add_request(f"r{i}", prompt_ids=ids,
                        params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=400, ignore_eos=True))
    eng._drain_inbox()
    for _ in range(0 if a.prefill else 4):  # prefill + a few decode steps (graphs of the decode bucket captured)
        eng.step()
    if a.wide_gate_up:
        for L in eng.model.layers:
            for m in list(L.gate_up.prefill_plan):
                if 16 < m <= 64:
                    L.gate_up.prefill_plan[m] = (ops.MID_BASE - 8, 0)
    if a.mixed:
        eng.add_request("mixed", prompt_ids=[200 + (j * 13) % 5000 for j in range(a.mixed)],
                        params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=1))
        eng._drain_inbox()
    summary, live, cap, t = measure(eng, a.replays)
    summary.update(batch=a.batch, ctx=a.ctx, replays=a.replays)
    print(json.dumps(summary), flush=True)
    for x in live[:14]:
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in x.items() if k not in ("t0", "t1")}))
    if a.json:
        Path(a.json).write_text(json.dumps({"summary": summary, "launches": live}, indent=1))


def measure(eng, replays: int = 0):
    """Re-capture the engine's decode bucket(s) with timeline slots, run one step, and return
    (summary, launches in start order, captured launch entries, raw stamps). replays > 0: then
    replay the newest graph that many times back to back and keep the last replay's stamps."""
    C = ops.native()
    r = eng.runner
    torch.cuda.synchronize()
    keys = list(r.graphs.keys())
    buf = torch.zeros(1 << 22, dtype=torch.int64, device="cuda")
    C.timeline_start(buf)
    for k in keys:  # re-capture the decode buckets with timeline slots
        del r.graphs[k]
    eng.step()
    used = C.timeline_stop()
    ents = C.timeline_entries()
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    if replays > 0:
        g = r.graphs[max(r.graphs.keys())]
        for _ in range(replays):
            g.replay()
        torch.cuda.synchronize()
    t = buf[:used].view(-1, 2).cpu()
    # the capture runs the forward twice (eager warm-up, then capture): keep the captured half
    n = len(ents)
    cap = ents[n // 2:] if n % 2 == 0 and [e[0] for e in ents[: n // 2]] == [e[0] for e in ents[n // 2:]] else ents
    rows = []
    for name, off, nb in cap:
        blk = t[off // 2: off // 2 + nb]
        ok = blk[:, 0] > 0
        if not ok.any():
            rows.append({"kernel": name, "blocks": nb, "ran": 0})
            continue
        st, en = blk[ok, 0], blk[ok, 1]
        d = ((en - st).float() / TICKS_PER_US).sort().values
        s0 = ((st - st.min()).float() / TICKS_PER_US).sort().values
        e0 = ((en - st.min()).float() / TICKS_PER_US).sort().values
        q = lambda v, f: float(v[min(len(v) - 1, int(f * len(v)))])  # noqa: E731
        rows.append({"kernel": name, "blocks": nb, "ran": int(ok.sum()), "t0": int(st.min()), "t1": int(en.max()),
                     "dur_med": q(d, 0.5), "dur_p10": q(d, 0.1), "dur_p90": q(d, 0.9), "dur_max": q(d, 1.0),
                     "start_p90": q(s0, 0.9), "start_max": q(s0, 1.0), "end_p10": q(e0, 0.1), "end_p50": q(e0, 0.5),
                     "end_p90": q(e0, 0.9)})
    live = [x for x in rows if x.get("ran")]
    live.sort(key=lambda x: x["t0"])
    T0 = live[0]["t0"]
    agg = defaultdict(lambda: {"n": 0, "span_us": 0.0, "gap_after_us": 0.0})
    for i, x in enumerate(live):
        x["start_us"] = (x["t0"] - T0) / TICKS_PER_US
        x["span_us"] = (x["t1"] - x["t0"]) / TICKS_PER_US
        x["gap_after_us"] = ((live[i + 1]["t0"] - x["t1"]) / TICKS_PER_US) if i + 1 < len(live) else 0.0
        g = agg[(x["kernel"], x["blocks"])]
        for k in ("dur_med", "dur_p10", "dur_p90", "dur_max", "start_p90", "start_max", "end_p10", "end_p50", "end_p90"):
            g[k] = g.get(k, 0.0) + x[k]
        g["n"] += 1
        g["span_us"] += x["span_us"]
        g["gap_after_us"] += x["gap_after_us"]
    total = (live[-1]["t1"] - T0) / TICKS_PER_US
    spans = sum(x["span_us"] for x in live)
    summary = {"kv_blocks": eng.num_blocks, "launches": len(live), "step_us": round(total, 1), "sum_span_us": round(spans, 1),
               "sum_gap_us": round(total - spans, 1),
               "per_kernel": {f"{k[0]}[{k[1]}]": {"n": v["n"], "avg_span_us": round(v["span_us"] / v["n"], 2),
                                                  "avg_gap_after_us": round(v["gap_after_us"] / v["n"], 2),
                                                  **{k: round(v[k] / v["n"], 2) for k in ("dur_p10", "dur_med", "dur_p90",
                                                     "dur_max", "start_p90", "start_max", "end_p10", "end_p50", "end_p90")}}
                              for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["span_us"])}}
    return summary, live, cap, t


if __name__ == "__main__":
    main()
