"""Prefill GEMMs: hipBLASLt (torch.matmul on plain [N, K] weights) vs the fragment-packed
MFMA tile kernel (ops.linear) vs unpack-then-hipBLASLt, Qwen2.5-1.5B and Llama-3-8B shapes,
M = 64..2048, in-graph timing (20 launches per graph, weights cycled so they stream).

    python benchmarks/prefill_blas_probe.py
"""
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402

SHAPES = [("qwen_qkv", 2048, 1536), ("qwen_o", 1536, 1536), ("qwen_gate_up", 17920, 1536), ("qwen_down", 1536, 8960),
          ("l8b_gate_up", 28672, 4096), ("l8b_down", 4096, 14336)]


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(reps):
            fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main():
    dev = torch.device("cuda")
    for name, N, K in SHAPES:
        ncopy = max(2, math.ceil(300e6 / (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16() for _ in range(ncopy)]
        lins = [ops.Linear(w) for w in ws]
        row = {"shape": name, "N": N, "K": K}
        for M in (64, 128, 256, 512, 1024, 2048):
            x = torch.randn(M, K, device=dev).bfloat16()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t_blas = graph_us(lambda i: torch.matmul(x, ws[i % ncopy].t(), out=out))
            t_tile = graph_us(lambda i: ops.linear(x, lins[i % ncopy], out=out))
            flop = 2 * M * N * K
            row[f"M{M}"] = {"blas_us": round(t_blas, 1), "vgate_us": round(t_tile, 1),
                            "blas_TF": round(flop / t_blas / 1e6, 0), "vgate_TF": round(flop / t_tile / 1e6, 0)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
