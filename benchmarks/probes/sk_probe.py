"""Stream-K decode GEMM vs the tile-per-block decode kernels, per projection shape, MI355X.

Each case is a hipGraph of 28 launches over 28 distinct weight copies (every launch streams cold
weights, as in a decode step), replayed back to back; per-launch time = graph time / 28 (the
launch boundaries included, as in the engine). Stream-K variants: (waves, blocks per CU,
k-steps per register group).

    python benchmarks/probes/sk_probe.py [--model qwen] [--m 8]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402

SHAPES = {
    "qwen": [("qkv", 2048, 1536, "qkv"), ("o", 1536, 1536, "res"), ("gate_up", 17920, 1536, "silu"),
             ("down", 1536, 8960, "res")],
    "llama8b": [("qkv", 6144, 4096, "qkv"), ("o", 4096, 4096, "res"), ("gate_up", 28672, 4096, "silu"),
                ("down", 4096, 14336, "res")],
    "llama70b_tp8": [("qkv", 1280, 8192, "qkv"), ("o", 8192, 1024, "res"), ("gate_up", 7168, 8192, "silu"),
                     ("down", 8192, 3584, "res")],
}
VARIANTS = [None, True, (4, 2, 8), (8, 1, 4), (8, 2, 8), (4, 1, 8)]
COPIES = 28


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen")
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M = a.m
    hq, hkv, D, BS = 12, 2, 128, 16
    for name, N, K, kind in SHAPES[a.model]:
        torch.manual_seed(N + K)
        if kind == "qkv":
            hkv = 2 if a.model == "qwen" else (8 if a.model == "llama8b" else 1)
            hq = N // D - 2 * hkv
        lins = []
        for c in range(COPIES):
            w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
            lin = ops.Linear(w, layout="silu" if kind == "silu" else ("qkv" if kind == "qkv" else "plain"))
            if kind in ("silu", "qkv"):
                assert lin.fold_norm((torch.rand(K, device=dev) + 0.5).bfloat16())
            lins.append(lin)
        x = torch.randn(M, K, device=dev).bfloat16()
        nw = torch.ones(K, device=dev).bfloat16()
        ncols = N // 2 if kind == "silu" else (hq * D if kind == "qkv" else N)
        out = torch.zeros(M, ncols, dtype=torch.bfloat16, device=dev)
        kv = dict(positions=torch.arange(M, dtype=torch.int32, device=dev),
                  slots=torch.arange(M, dtype=torch.int32, device=dev),
                  cos_sin=torch.zeros(4096, 128, device=dev),
                  k_cache=torch.zeros(64, hkv, BS, D, dtype=torch.bfloat16, device=dev),
                  v_cache=torch.zeros(64, hkv, BS, D, dtype=torch.bfloat16, device=dev), hq=hq, hkv=hkv)
        res = {}
        ref = None
        for var in VARIANTS:
            for lin in lins:
                lin.dec_sk = var if var is not None else False

            def run():
                for lin in lins:
                    if kind == "silu":
                        ops.linear(x, lin, out=out, norm=(nw, 1e-6))
                    elif kind == "qkv":
                        ops.linear(x, lin, out=out, norm=(nw, 1e-6), qkv=kv)
                    else:
                        ops.linear(x, lin, out=out, residual=out)
            try:
                out.zero_()
                run()
                torch.cuda.synchronize()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    run()
                torch.cuda.current_stream().wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    run()
                for _ in range(3):
                    g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.iters):
                    g.replay()
                e1.record()
                e1.synchronize()
                us = 1e3 * e0.elapsed_time(e1) / (a.iters * COPIES)
            except RuntimeError as ex:
                res[str(var)] = f"error {str(ex)[:80]}"
                continue
            if kind != "res":  # (residual outputs accumulate over replays)
                out.zero_()
                run()
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                elif not torch.allclose(out.float(), ref.float(), atol=2e-2, rtol=2e-2):
                    res[str(var)] = "MISMATCH"
                    continue
            res[str(var)] = round(us, 2)
        mb = N * K * 2 / 1e6
        print(json.dumps({"model": a.model, "proj": name, "M": M, "N": N, "K": K, "weight_MB": round(mb, 1),
                          "us_per_launch": res, "fault": int(ops.fault_word(dev)[0].item())}), flush=True)


if __name__ == "__main__":
    main()
