"""Sampler launch time by sampling mode (MI355X): greedy / temperature only / temperature + top-p /
temperature + top-k, engine-shaped logits [B, V] (Qwen2.5-1.5B vocabulary), back-to-back launches
timed with events — which part of the single-launch sampler costs the time (sweeps and their
Philox + log work, or the rejection rounds).

    python benchmarks/sampler_modes.py [--batch 8] [--vocab 151936]
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
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--scale", type=float, default=0.8, help="logit std (random-init LM heads give ~0.5-1)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, V = a.batch, a.vocab
    torch.manual_seed(0)
    logits = torch.randn(B, V, device=dev) * a.scale
    seeds = torch.arange(B, device=dev, dtype=torch.int64) * 7919 + 1
    out = torch.empty(B, dtype=torch.int32, device=dev)
    modes = {"greedy": (0.0, 1.0, -1), "temp0.7": (0.7, 1.0, -1), "temp0.7_topp0.9": (0.7, 0.9, -1),
             "temp0.7_topk50": (0.7, 1.0, 50), "temp1.0_topp0.5": (1.0, 0.5, -1)}
    for name, (t, p, k) in modes.items():
        temp = torch.full((B,), t, device=dev)
        topp = torch.full((B,), p, device=dev)
        topk = torch.full((B,), k, dtype=torch.int32, device=dev)
        for nseg_cap in (64, 1):
            ops.native().set_sample_nseg(nseg_cap)
            offs = torch.zeros(B, dtype=torch.int64, device=dev)
            for _ in range(10):
                ops.sample(logits, temp, topp, topk, seeds, offs, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.iters):
                offs.fill_(i)
                ops.sample(logits, temp, topp, topk, seeds, offs, out=out)
            e1.record()
            torch.cuda.synchronize()
            fill = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fill[0].record()
            for i in range(a.iters):
                offs.fill_(i)
            fill[1].record()
            torch.cuda.synchronize()
            us = 1e3 * (e0.elapsed_time(e1) - fill[0].elapsed_time(fill[1])) / a.iters
            print(json.dumps({"mode": name, "B": B, "V": V, "nseg": ops.native().sample_segments(B, V),
                              "us_per_launch": round(us, 2)}), flush=True)
    ops.native().set_sample_nseg(64)
    print(json.dumps({"fault": int(ops.fault_word(dev)[0].item())}))


if __name__ == "__main__":
    main()
