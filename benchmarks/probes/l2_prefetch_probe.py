"""Would L2-resident weights shorten the latency-bound decode GEMMs? (MI355X, M = 8, Qwen2.5-1.5B)

Block spans (launch timeline, one hipGraph) of the qkv and o_proj decode GEMMs in three cache states:
  cold      — a down_proj-sized GEMM (27.5 MB, its own cold copy) streams, then the target reads its
              weights for the first time (the serving step's state);
  warm      — the target GEMM runs twice back to back (its second run reads what the first left in
              the XCDs' L2s / the Infinity Cache: the upper bound of any prefetch);
  prefetch  — the target GEMM runs, then the down-sized stream, then the target again (does a
              prefetch made one kernel earlier survive the next kernel's weight stream?).
Weights cycle through > 600 MB of copies, so "cold" is cold.

    python benchmarks/probes/l2_prefetch_probe.py
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from benchmarks.tlgraph import timeline_graph  # noqa: E402
from vgate import ops  # noqa: E402


def main():
    C = ops.native()
    M, H, inter = 8, 1536, 8960
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    x = torch.randn(M, inter, device=dev).bfloat16()
    shapes = {"qkv": (2048, H), "o": (H, H), "down": (H, inter)}
    lins = {}
    for name, (N, K) in shapes.items():
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        ncopy = max(3, math.ceil(700e6 / (N * K * 2)))
        lins[name] = [ops.Linear(w, layout="plain") for _ in range(ncopy)]
    outs = {n: torch.empty(M, N, device=dev, dtype=torch.bfloat16) for n, (N, _) in shapes.items()}
    ctr = {"down": 0}

    xs = {K: x[:, :K].contiguous() for K in (H, inter)}

    def gemm(name, i):
        N, K = shapes[name]
        lin = lins[name][i % len(lins[name])]
        C.gemm(xs[K], lin.wp, N, K, outs[name], 0, ws=ws)

    def down():
        ctr["down"] += 1
        gemm("down", ctr["down"])

    reps = 12
    res = {}
    for tgt in ("qkv", "o"):
        variants = {
            "cold": lambda: [(down(), gemm(tgt, i)) for i in range(reps)],
            "warm": lambda: [(down(), gemm(tgt, i), gemm(tgt, i)) for i in range(reps)],
            "prefetch": lambda: [(gemm(tgt, i), down(), gemm(tgt, i)) for i in range(reps)],
        }
        for vn, fn in variants.items():
            spans, wall = timeline_graph(C, fn)
            seq = spans["gemm"]
            per = len(seq) // reps
            # the target's measured launch is the last of each rep's group
            tv = [seq[r * per + per - 1] for r in range(1, reps)]
            dv = [seq[r * per + (0 if vn != "prefetch" else 1)] for r in range(1, reps)]
            res[f"{tgt}_{vn}"] = {"target_span_us": round(sum(tv) / len(tv), 2),
                                  "down_span_us": round(sum(dv) / len(dv), 2)}
            print(json.dumps({tgt: vn, **res[f"{tgt}_{vn}"]}), flush=True)
    print(json.dumps({"l2_prefetch_probe": res}), flush=True)


if __name__ == "__main__":
    main()
