"""Stall hunt for the segmented sampler (MI355X): many back-to-back launches on engine-shaped
logits, timed in groups, reporting the median and the worst group. A row whose blocks wait
for each other in-kernel (row_meet) must never stall: before the atomic-RMW poll the driver
bench saw 60-470 ms sampler launches (profiles/r2_sampler_stall.txt).

    python benchmarks/sampler_stress.py [--groups 200] [--per-group 100]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=200)
    ap.add_argument("--per-group", type=int, default=100)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--nseg", default="16,32,64,128", help="caps on segments per row to sweep")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {}
    caps = [int(c) for c in a.nseg.split(",")]
    for cap, B in [(c, b) for c in caps for b in (1, 8, 32)]:
        ops.native().set_sample_nseg(cap)
        torch.manual_seed(B)
        logits = torch.randn(B, a.vocab, device=dev) * 0.8
        temp = torch.full((B,), 0.7, device=dev)
        topp = torch.full((B,), 0.9, device=dev)
        topk = torch.full((B,), -1, dtype=torch.int32, device=dev)
        seeds = torch.arange(B, dtype=torch.int64, device=dev)
        offs = torch.zeros(B, dtype=torch.int64, device=dev)
        out = torch.empty(B, dtype=torch.int32, device=dev)
        for _ in range(10):
            ops.sample(logits, temp, topp, topk, seeds, offs, out=out)
        torch.cuda.synchronize()
        times = []
        for g in range(a.groups):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.per_group):
                offs.fill_(g * a.per_group + i)
                ops.sample(logits, temp, topp, topk, seeds, offs, out=out)
            e.record()
            e.synchronize()
            times.append(1e3 * s.elapsed_time(e) / a.per_group)
        times.sort()
        res[f"cap{cap}_B{B}"] = {"median_us": round(times[len(times) // 2], 2),
                                 "max_group_avg_us": round(times[-1], 2),
                                 "nseg": ops.native().sample_segments(B, a.vocab)}
        print(json.dumps({"cap": cap, "B": B, **res[f"cap{cap}_B{B}"]}), flush=True)
    print(json.dumps({"sampler_stress": res}), flush=True)


if __name__ == "__main__":
    main()
