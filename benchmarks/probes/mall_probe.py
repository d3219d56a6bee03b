"""Does a default-policy read sweep (ops prefetch) make the next decode GEMM stream its
weights from the 256 MB Infinity Cache (MALL) instead of HBM? (MI355X)

For each Qwen2.5-1.5B projection at M = 8, hipGraphs of 20 launches cycle through > 600 MB
of weight copies (every launch cold in L2 and MALL) in three forms:
  gemm              : the GEMM alone;
  prefetch + gemm   : a 256-block read sweep of the same weights right before the GEMM;
  prefetch          : the sweep alone.
Block spans come from the launch timeline (TLScope): the GEMM span with and without the
sweep in front is the MALL-hit speed-up; the sweep span is its cost when it cannot be hidden.

    python benchmarks/probes/mall_probe.py
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402
from tlgraph import timeline_graph  # noqa: E402

SHAPES = [("qkv", 2048, 1536, "plain", 0), ("o_proj", 1536, 1536, "plain", 0), ("gate_up", 17920, 1536, "silu", 2),
          ("down", 1536, 8960, "plain", 0)]


def main():
    C = ops.native()
    M = 8
    ws = ops.workspace(torch.device("cuda"))
    for name, N, K, layout, epi in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        ncopy = max(2, math.ceil(600e6 / (N * K * 2)))
        lins = [ops.Linear(w, layout=layout) for _ in range(ncopy)]
        out = torch.empty(M, N // 2 if epi == 2 else N, device="cuda", dtype=torch.bfloat16)
        reps = 20

        def gemm(i):
            C.gemm(x, lins[i % ncopy].wp, N, K, out, epi, ws=ws)

        res = {"shape": name, "MB": round(N * K * 2 / 1e6, 1)}
        for form in ("gemm", "prefetch+gemm", "prefetch"):
            def fns():
                for i in range(reps):
                    if form != "gemm":
                        C.prefetch(lins[i % ncopy].wp, 256)
                    if form != "prefetch":
                        gemm(i)
            spans, wall = timeline_graph(C, fns)
            res[form] = {k: round(sum(v[1:]) / max(1, len(v) - 1), 2) for k, v in spans.items()}
            res[form]["wall_per_iter_us"] = round(wall / reps, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
