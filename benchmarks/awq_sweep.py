"""AWQ W4A16 decode GEMM sweep on the MI355X (Qwen2.5-1.5B shapes, M = 8, group 128):
split-K of the LDS-shared-activation kernel (awq_dec_kernel) and the K-split kernel
(waves forced), block spans from the launch timeline, weights cycled through > 600 MB.

    python benchmarks/awq_sweep.py
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from benchmarks.mall_probe import timeline_graph  # noqa: E402
from vgate import ops  # noqa: E402

SHAPES = [("qkv", 2048, 1536, "plain"), ("o_proj", 1536, 1536, "plain"), ("gate_up", 17920, 1536, "silu"),
          ("down", 1536, 8960, "plain")]


def main():
    C = ops.native()
    M, g = 8, 128
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    for name, N, K, layout in SHAPES:
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev)
        scales = (torch.rand(K // g, N, device=dev) * 0.02 + 0.005).bfloat16()
        zeros = torch.randint(0, 16, (K // g, N), device=dev).float().bfloat16()
        ncopy = max(2, math.ceil(400e6 / (N * K // 2)))
        lins = [ops.Linear(None, awq={"qint": q, "scales": scales, "zeros": zeros, "group": g,
                                      "silu": layout == "silu"}) for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev).bfloat16()
        res = torch.randn(M, N, device=dev).bfloat16()
        epi = 2 if layout == "silu" else 0
        out = torch.empty(M, N // 2 if epi == 2 else N, device=dev, dtype=torch.bfloat16)
        rows = []
        for waves, sk in [(0, 0), (0, 1), (0, 2), (0, 3), (0, 4), (0, 6), (0, 8), (4, 0), (8, 0), (8, 2)]:
            def fns():
                for i in range(12):
                    L = lins[i % ncopy]
                    C.gemm(x, L.wp, N, K, out, epi, res=None if epi else res, ws=ws, waves=waves, splitk=sk,
                           awq_scales=L.scales, awq_zeros=L.zeros, group=g)
            spans, wall = timeline_graph(C, fns)
            vals = [v for vs in spans.values() for v in vs]
            rows.append({"waves": waves, "splitk": sk, "span_us": round(sum(vals[1:]) / (len(vals) - 1), 2),
                         "wall_us": round(wall / 12, 2)})
        print(json.dumps({"shape": name, "N": N, "K": K, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
