"""Hand-written LDS-tiled prefill GEMM (gemm_prefill.hip) vs hipBLASLt (torch.mm, used here
ONLY as the oracle / bar) on the SURVEY.md §2.4 projection shapes (MI355X).

For every (model shape, M) both run the same bf16 x[M,K] . W[N,K]^T with random operands,
timed over --iters back-to-back launches (CUDA events); prints TFLOP/s of each and the ratio.
The packed-weight kernel gets its tile width from the launcher heuristic (ntb=0) unless
--bn forces one.

    python benchmarks/prefill_gemm_bench.py [--ms 128,512,2048,4096] [--models qwen,llama8b,llama70b_tp8]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402

SHAPES = {  # name: [(proj, N, K)]
    "qwen": [("qkv", 2048, 1536), ("o", 1536, 1536), ("gate_up", 17920, 1536), ("down", 1536, 8960)],
    "llama8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)],
    "llama70b_tp8": [("qkv", 1280, 8192), ("o", 8192, 1024), ("gate_up", 7168, 8192), ("down", 8192, 3584)],
}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return 1e3 * s.elapsed_time(e) / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="128,256,512,1024,2048,4096")
    ap.add_argument("--models", default="qwen,llama8b,llama70b_tp8")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bn", type=int, default=0)
    ap.add_argument("--tuned", action="store_true",
                    help="report the decomposition the engine's start-up tuner (ops.tune_prefill) would pick: "
                         "the fastest of ops.PREFILL_CANDIDATES (+ the ring candidates at 64 < M <= 1024) unless "
                         "within 5%% of the heuristic")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    C = ops.native()
    ws = ops.workspace(dev)
    rows = []
    for model in a.models.split(","):
        for proj, N, K in SHAPES[model]:
            torch.manual_seed(N + K)
            w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
            wp = ops.pack_weight(w)
            for M in [int(m) for m in a.ms.split(",")]:
                x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
                out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                ours = timeit(lambda: C.gemm(x, wp, N, K, out, 0, ws=ws, path=1, ntb=a.bn), a.iters)
                pick = (a.bn, 0)
                if a.tuned:
                    t = {}
                    extra = ops.PREFILL_RING_CANDIDATES if 64 < M <= 1024 else []  # as ops.tune_prefill
                    for bn, sk in ops.PREFILL_CANDIDATES + extra:
                        try:
                            t[(bn, sk)] = timeit(lambda: C.gemm(x, wp, N, K, out, 0, ws=ws, path=1, ntb=bn, splitk=sk),
                                                 a.iters)
                        except RuntimeError:
                            continue
                    best = min(t, key=t.get)
                    if t[best] < 0.95 * t[(0, 0)]:
                        pick, ours = best, t[best]
                    C.gemm(x, wp, N, K, out, 0, ws=ws, path=1, ntb=pick[0], splitk=pick[1])
                lib = timeit(lambda: torch.mm(x, w.t()), a.iters)
                err = ((out.float() - (x.float() @ w.float().t())).norm() / (x.float() @ w.float().t()).norm()).item()
                fl = 2.0 * M * N * K
                r = {"model": model, "proj": proj, "M": M, "N": N, "K": K, "ours_us": round(ours, 2),
                     "hipblaslt_us": round(lib, 2), "ours_tflops": round(fl / ours / 1e6, 1),
                     "hipblaslt_tflops": round(fl / lib / 1e6, 1), "ratio_vs_lib": round(lib / ours, 3),
                     "rel_err": round(err, 5), "plan": list(pick)}
                rows.append(r)
                print(json.dumps(r), flush=True)
    geo = 1.0
    for r in rows:
        geo *= r["ratio_vs_lib"]
    print(json.dumps({"summary": {"n": len(rows), "geomean_ratio_vs_hipblaslt": round(geo ** (1 / len(rows)), 3),
                                  "min_ratio": min(r["ratio_vs_lib"] for r in rows)}}), flush=True)


if __name__ == "__main__":
    main()
