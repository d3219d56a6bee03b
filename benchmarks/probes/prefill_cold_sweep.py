"""Prefill GEMM decompositions at serving M, COLD weights vs back-to-back (MI355X, Qwen2.5-1.5B).

The engine's start-up tuner (ops.tune_prefill) ranks the prefill candidates for M >= 128 by
back-to-back launches (weights warm in the Infinity Cache / L2). Inside a prefill step every GEMM
reads its weights cold. This times every candidate both ways, plus hipBLASLt (torch.mm, oracle)
cold, and prints the best of each per (shape, M).

    python benchmarks/probes/prefill_cold_sweep.py [--ms 320,448,640] [--model llama8b] [--only 1024,1025]
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

SHAPES = {"qwen": [("qkv", 2048, 1536), ("o", 1536, 1536), ("gate_up", 17920, 1536), ("down", 1536, 8960)],
          "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="320,448,640")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--model", default="qwen", choices=sorted(SHAPES))
    ap.add_argument("--only", default="", help="comma list of tile codes to time (default: every candidate)")
    ap.add_argument("--norm", action="store_true", help="with the folded RMSNorm row scale (qkv / gate_up in a step)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.native()
    ws = ops.workspace(dev)
    flush = torch.empty(512 * 2**20, dtype=torch.uint8, device=dev)

    def cold(run):
        tot = 0.0
        for _ in range(a.iters):
            C.prefetch(flush, 1024)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            run()
            s1.record()
            s1.synchronize()
            tot += s0.elapsed_time(s1)
        return 1e3 * tot / a.iters

    def warm(run):
        run()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.iters):
            run()
        s1.record()
        s1.synchronize()
        return 1e3 * s0.elapsed_time(s1) / a.iters

    cands = ops.PREFILL_CANDIDATES + ops.PREFILL_RING_CANDIDATES
    cands += [(t, s) for t in (1025, 769) for s in range(9) if (t, s) not in cands]  # persistent: tail slices
    only = {int(c) for c in a.only.split(",") if c}
    for name, N, K in SHAPES[a.model]:
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        wp = ops.pack_weight(w)
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            rows = {}
            for bn, sk in cands + [("tile", 0), ("tile3", 0)]:
                if only and (not isinstance(bn, int) or bn not in only):
                    continue
                kw = dict(waves=-1) if bn == "tile" else dict(waves=-2) if bn == "tile3" else ops._plan_kw((bn, sk), M)

                if a.norm:
                    kw = dict(kw, rownorm=True, eps=1e-6)

                def run(kw=kw):
                    C.gemm(x, wp, N, K, out, 0, ws=ws, **kw)
                try:
                    run()
                except RuntimeError:
                    continue
                rows[f"{bn}/{sk}"] = (round(cold(run), 2), round(warm(run), 2))
            torch.mm(x, w.t())  # hipBLASLt's first call per shape selects its algorithm: not timed
            torch.cuda.synchronize()
            blas = (round(cold(lambda: torch.mm(x, w.t())), 2), round(warm(lambda: torch.mm(x, w.t())), 2))
            bc = min(rows, key=lambda k: rows[k][0])
            bw = min(rows, key=lambda k: rows[k][1])
            print(json.dumps({"shape": name, "M": M, "best_cold": [bc, rows[bc]], "best_warm": [bw, rows[bw]],
                              "default_0/0": rows.get("0/0"), "tile": rows.get("tile/0"), "tile3": rows.get("tile3/0"), "hipblaslt": blas,
                              "all": rows}), flush=True)


if __name__ == "__main__":
    main()
