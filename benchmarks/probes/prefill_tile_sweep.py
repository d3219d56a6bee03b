"""Prefill GEMM tile / K-split sweep at mid M (the engine's multi-prompt prefill steps: 8 prompts of
~50 tokens land in one 384- or 512-token step), MI355X: every forced (tile, K slices) of the
packed-weight prefill kernels vs the launcher's choice, hipBLASLt as the oracle.

tile codes (GemmArgs.ntb on the prefill path): 0 launcher, 64 / 128 = v1 128 x 64 / 128 x 128,
256 = v2 256 x 128 (3-deep ring), 512 = v2 256 x 256, 768 = v4 256 x 128, 1024 = v4 256 x 256,
1280 / 1281 = v2 128 x 128 on a 4-deep ring (4 / 8 waves), 640 / 641 = v2 128 x 64 (4 / 8 waves),
2560 / 2561 = v2 64 x 512 / 128 x 320 (8 waves). --cold flushes the Infinity Cache before every launch.

    python benchmarks/prefill_tile_sweep.py [--ms 384,512] [--model qwen]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from benchmarks.prefill_gemm_bench import SHAPES, timeit  # noqa: E402
from vgate import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="384,512")
    ap.add_argument("--model", default="qwen")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tiles", default="0,64,128,256,512,768,1024")
    ap.add_argument("--sks", default="0,1,2,3,4,6")
    ap.add_argument("--cold", action="store_true", help="Infinity Cache flushed before every launch (in-step weights)")
    ap.add_argument("--projs", default="", help="comma list of projections to sweep (default all)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.native()
    ws = ops.workspace(dev)
    cold = ops._cold_timer(dev) if a.cold else None

    def tm(fn):
        return 1000.0 * cold(fn, a.iters) if cold is not None else timeit(fn, a.iters)
    for proj, N, K in SHAPES[a.model]:
        if a.projs and proj not in a.projs.split(","):
            continue
        torch.manual_seed(N + K)
        w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        wp = ops.pack_weight(w)
        for M in [int(m) for m in a.ms.split(",")]:
            x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            ref = x.float() @ w.float().t()
            lib = tm(lambda: torch.mm(x, w.t()))
            res = {}
            for bn in [int(v) for v in a.tiles.split(",")]:
                for sk in [int(v) for v in a.sks.split(",")]:
                    if bn == 0 and sk != 0:
                        continue
                    try:
                        us = tm(lambda: C.gemm(x, wp, N, K, out, 0, ws=ws, path=1, ntb=bn, splitk=sk))
                    except RuntimeError:
                        continue
                    err = ((out.float() - ref).norm() / ref.norm()).item()
                    if err > 1e-2:
                        res[f"{bn}/{sk}"] = "BAD"
                        continue
                    res[f"{bn}/{sk}"] = round(us, 2)
            best = min((v, k) for k, v in res.items() if v != "BAD")
            print(json.dumps({"proj": proj, "M": M, "cold": a.cold, "N": N, "K": K, "hipblaslt_us": round(lib, 2), "auto_us": res.get("0/0"),
                              "best": best[1], "best_us": best[0], "all": res}), flush=True)


if __name__ == "__main__":
    main()
