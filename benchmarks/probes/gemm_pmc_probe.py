"""One prefill GEMM shape, one tile code, repeated: the target of a rocprofv3 --pmc pass.

    rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES ... -- python3 benchmarks/probes/gemm_pmc_probe.py \
        --M 2048 --N 28672 --K 4096 --code 1024 --reps 20
"""
from __future__ import annotations

import argparse
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=2048)
    ap.add_argument("--N", type=int, default=28672)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--code", type=int, default=1024)
    ap.add_argument("--slices", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--norm", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    w = (torch.rand(a.N, a.K, device=dev) * 2 - 1).div(math.sqrt(a.K)).bfloat16()
    wp = ops.pack_weight(w)
    x = (torch.rand(a.M, a.K, device=dev) * 2 - 1).bfloat16()
    out = torch.empty(a.M, a.N, dtype=torch.bfloat16, device=dev)
    kw = ops._plan_kw((a.code, a.slices), a.M)
    if a.norm:
        kw.update(rownorm=True, eps=1e-6)
    C = ops.native()
    ws = ops.workspace(dev)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    C.gemm(x, wp, a.N, a.K, out, 0, ws=ws, **kw)
    torch.cuda.synchronize()
    s0.record()
    for _ in range(a.reps):
        C.gemm(x, wp, a.N, a.K, out, 0, ws=ws, **kw)
    s1.record()
    s1.synchronize()
    us = 1e3 * s0.elapsed_time(s1) / a.reps
    print({"M": a.M, "N": a.N, "K": a.K, "code": a.code, "us": round(us, 2),
           "tflops": round(2 * a.M * a.N * a.K / us / 1e6, 1)}, flush=True)


if __name__ == "__main__":
    main()
