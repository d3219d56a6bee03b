"""Decode GEMM decomposition sweep with the column-tile width per block (MI355X, M = 8).

A block of the weight-streaming kernel owns NTB 16-column tiles; its waves split the block's
K-slice. Activation bytes per block are K_slice x 8 rows x 2 B against weight bytes
K_slice x 16 NTB x 2 B, so NTB sets the activation share of the vector-memory stream
(1/2 at NTB = 1, 1/8 at NTB = 4) while split-K restores the block count. Spans from the
launch timeline, weights cycled through > 600 MB of copies.

    python benchmarks/gemm_ntb_sweep.py [--shape down]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from benchmarks.tlgraph import timeline_graph  # noqa: E402
from vgate import ops  # noqa: E402

SHAPES = {"down": (1536, 8960), "o_proj": (1536, 1536), "lm_head": (151936, 1536)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="down,o_proj")
    a = ap.parse_args()
    C = ops.native()
    M = 8
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    for name in a.shape.split(","):
        N, K = SHAPES[name]
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        ncopy = max(2, math.ceil(600e6 / (N * K * 2)))
        lins = [ops.Linear(w) for _ in range(ncopy)]
        res = torch.randn(M, N, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        rows = []
        combos = [(0, 0, 0)] + [(ntb, wv, sk) for ntb in (1, 2, 4) for wv in (4, 8) for sk in (1, 2, 3, 4, 6, 8)]
        for ntb, wv, sk in combos:
            if name == "lm_head" and sk > 1:
                continue

            def fns():
                for i in range(12):
                    C.gemm(x, lins[i % ncopy].wp, N, K, out, 0, res=res, ws=ws, waves=wv, splitk=sk, ntb=ntb)
            spans, wall = timeline_graph(C, fns)
            vals = [v for vs in spans.values() for v in vs]
            rows.append({"ntb": ntb, "waves": wv, "splitk": sk, "span_us": round(sum(vals[1:]) / (len(vals) - 1), 2),
                         "wall_us": round(wall / 12, 2)})
        best = min(rows, key=lambda r: r["wall_us"])
        print(json.dumps({"shape": name, "N": N, "K": K, "auto": rows[0], "best": best,
                          "all": sorted(rows, key=lambda r: r["wall_us"])[:12]}), flush=True)


if __name__ == "__main__":
    main()
