"""Prefill attention throughput on the MI355X: the flash kernel (K / V through LDS by DMA, shared by
the G heads of a KV head) vs the 16-query tile kernel, causal, one sequence of S tokens, Llama-3-8B
(32 / 8 heads), Qwen2.5-1.5B (12 / 2) and Llama-3-70B TP=8 per-rank (8 / 1) layouts. Reports us per
layer and TFLOP/s (4 S^2 D Hq / 2 causal FLOPs).

    python benchmarks/attn_prefill_bench.py [--lens 2048,4096]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="2048,4096")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = ops.native()
    dev = "cuda"
    D, BS = 128, 16
    for name, Hq, Hkv in (("llama3_8b", 32, 8), ("qwen2.5_1.5b", 12, 2), ("llama3_70b_tp8", 8, 1)):
        for S in [int(x) for x in a.lens.split(",")]:
            nb = S // BS + 1
            kc = (torch.randn(nb, Hkv, BS, D, device=dev) * 0.5).bfloat16()
            vc = torch.randn(nb, Hkv, BS, D, device=dev).bfloat16()
            bt = torch.randperm(nb, device=dev)[: nb].int().reshape(1, nb)
            qs = torch.tensor([0, S], dtype=torch.int32, device=dev)
            cl = torch.tensor([S], dtype=torch.int32, device=dev)
            stride = (Hq + 2 * Hkv) * D
            qkv = torch.randn(S, stride, device=dev).bfloat16()
            ts, tq = ops.prefill_tiles([S], ops.flash_lead(Hq, Hkv))  # the engine's tile order
            ts = torch.tensor(ts, dtype=torch.int32, device=dev)
            tq = torch.tensor(tq, dtype=torch.int32, device=dev)
            out = torch.empty(S, Hq * D, device=dev).bfloat16()
            flops = 2 * S * S * D * Hq  # causal: half of 4 S^2 D per head
            row = {"layout": name, "S": S}
            for mode in (1, 0):
                C.set_flash_prefill(mode)
                fn = lambda: ops.attention_prefill(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out, Hq, Hkv,
                                                   1 / math.sqrt(D))
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
                us = 1e3 * e0.elapsed_time(e1) / a.iters
                key = "flash" if mode else "tile16"
                row[key + "_us"] = round(us, 1)
                row[key + "_tflops"] = round(flops / us / 1e6, 1)
            C.set_flash_prefill(-1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
