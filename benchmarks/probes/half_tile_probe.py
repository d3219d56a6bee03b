"""Half-tile decode blocks (path 5, gemm_block: 8 of a 16-column tile per block over the whole K)
against the production decode plans at M = 8 (MI355X, Qwen2.5-1.5B o_proj / down_proj, residual
epilogue): block spans in a hipGraph, weights cycling through > 600 MB of copies (cold), each
launch behind a gate_up-sized stream as in a step.

    python benchmarks/probes/half_tile_probe.py

(Measured negative and removed: profiles/r6_half_tile_negative.log. path=5 now runs the default plan.)
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
from vgate.ops import reference as ref  # noqa: E402


def main():
    C = ops.native()
    M, H, inter = 8, 1536, 8960
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    skw, fault = ops.sk_workspace(dev), ops.fault_word(dev)
    shapes = {"o": (H, H), "down": (H, inter)}
    res = {}
    for name, (N, K) in shapes.items():
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        ncopy = max(3, math.ceil(700e6 / (N * K * 2)))
        lins = [ops.Linear(w) for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16()
        want = ref.linear_ref(x.cpu(), w.cpu(), None, r.cpu()).float()
        variants = {"plan_w16_sk2": dict(waves=16, splitk=2), "plan_w8": dict(waves=8, splitk=1),
                    "half_w4": dict(waves=4, path=5), "half_w8": dict(waves=8, path=5),
                    "half_w12": dict(waves=12, path=5), "half_w16": dict(waves=16, path=5)}
        for vn, kw in variants.items():
            out = r.clone()
            C.gemm(x, lins[0].wp, N, K, out, 0, res=out, ws=ws, sk_ws=skw, fault=fault, **kw)
            err = float((out.float().cpu() - want).norm() / want.norm())
            outs = [r.clone() for _ in range(ncopy)]

            def fn(kw=kw):
                for i in range(12):
                    C.gemm(x, lins[i % ncopy].wp, N, K, outs[i % ncopy], 0, res=outs[i % ncopy], ws=ws,
                           sk_ws=skw, fault=fault, **kw)
            spans, wall = timeline_graph(C, fn)
            seq = [v for k, v in spans.items()][0]
            res[f"{name}_{vn}"] = {"span_us": round(sum(seq[1:]) / (len(seq) - 1), 2),
                                   "wall_per_launch_us": round(wall / 12, 2), "rel_err": round(err, 5)}
            print(json.dumps({name: vn, **res[f"{name}_{vn}"]}), flush=True)
    print(json.dumps({"half_tile_probe": res, "fault": int(fault[0].item())}), flush=True)


if __name__ == "__main__":
    main()
