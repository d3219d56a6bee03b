"""bf16 decode GEMM sweep on the MI355X (Qwen2.5-1.5B shapes, M = 8): the tile-per-block kernels
(gemm_decode.h gemm_kernel, the launcher's plan) against the register-stationary kernel
(csrc/kernels/gemm_kx.h, path 4) over (waves, K slices, tiles per GROUP block); the qkv / gate_up
rows also as the RMSNorm hand-off consumer (NORM 3, as in-engine). Block spans from the launch
timeline, weights cycled through > 400 MB (cold).

    python benchmarks/dense_kx_sweep.py        (DKX_SHAPES=gate_up,down ...)
"""
from __future__ import annotations

import json
import math
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from benchmarks.awq_sweep import block_stats  # noqa: E402
from benchmarks.tlgraph import timeline_graph  # noqa: E402
from vgate import ops  # noqa: E402

SHAPES = [("qkv", 2048, 1536, "plain"), ("o_proj", 1536, 1536, "plain"), ("gate_up", 17920, 1536, "silu"),
          ("down", 1536, 8960, "plain")]
# (path, waves, splitk, ntb): path 0 = tile kernels (launcher's plan / forced waves, slices), 3 = stream-K
# (waves 4 / 8, blocks per CU 1 / 2 in splitk, k-steps per group 4 / 8 in ntb), 4 = register-stationary
CFGS = {
    "qkv": [(0, 0, 0, 0), (4, 0, 0, 0), (4, 8, 1, -12), (4, 6, 2, -12), (4, 16, 1, -12)],
    "o_proj": [(0, 0, 0, 0), (4, 0, 0, 0), (4, 8, 1, -12), (4, 6, 2, -12), (4, 12, 1, -13)],
    "gate_up": [(0, 0, 0, 0), (4, 0, 0, 0), (4, 8, 0, -12), (4, 6, 0, -12), (4, 12, 2, -13), (4, 12, 1, -13)],
    "down": [(0, 0, 0, 0), (4, 0, 0, 0), (4, 8, 4, -13), (3, 0, 0, 0), (3, 4, 0, 0), (3, 0, 2, 0), (3, 4, 2, 0),
             (3, 0, 0, 4), (0, 16, 2, 0), (0, 8, 4, 0), (0, 8, 3, 0), (0, 4, 4, 0), (0, 8, 8, 0)],
}


def main():
    C = ops.native()
    M = 8
    only = os.environ.get("DKX_SHAPES")
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    skw = dict(sk_ws=ops.sk_workspace(dev), fault=ops.fault_word(dev))
    for name, N, K, layout in SHAPES:
        if only and name not in only.split(","):
            continue
        epi = 2 if layout == "silu" else 0
        ncopy = max(2, math.ceil(400e6 / (N * K * 2)))
        w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
        lins = [ops.Linear(w.clone(), kind="silu" if layout == "silu" else "plain") for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev).bfloat16()
        res = torch.randn(M, N, device=dev).bfloat16()
        out = torch.empty(M, N // 2 if epi == 2 else N, device=dev, dtype=torch.bfloat16)
        ssp = x.float().pow(2).reshape(M, K // 16, 16).sum(-1).contiguous()
        cfgs = list(CFGS[name])
        if name in ("qkv", "gate_up"):
            cfgs += [c + ("norm3",) for c in cfgs[:2]]
        rows, ref = [], None
        for cfg in cfgs:
            path, waves, sk, ntb = cfg[:4]
            nkw = dict(ssp_in=ssp, eps=1e-6) if len(cfg) > 4 else {}

            def call(L):
                C.gemm(x, L.wp, N, K, out, epi, res=None if epi else res, ws=ws, waves=waves, splitk=sk, ntb=ntb,
                       path=path, **skw, **nkw)

            call(lins[0])
            torch.cuda.synchronize()
            got = out.float().clone()
            if not nkw and path == 0:
                ref = got
            err = float((got - ref).norm() / ref.norm()) if (ref is not None and not nkw) else None

            def fns():
                for i in range(12):
                    call(lins[i % ncopy])
            spans, wall = timeline_graph(C, fns)
            vals = [v for vs in spans.values() for v in vs]
            bs = block_stats(C, lambda: call(lins[0]))
            rows.append({"path": path, "waves": waves, "splitk": sk, "ntb": ntb, "norm": 3 if nkw else 0,
                         "kernel": sorted(spans)[0] if spans else None,
                         "span_us": round(sum(vals[1:]) / (len(vals) - 1), 2), "wall_us": round(wall / 12, 2),
                         "rel_err_vs_tile": None if err is None else round(err, 5), "blocks": bs})
        print(json.dumps({"shape": name, "N": N, "K": K, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
