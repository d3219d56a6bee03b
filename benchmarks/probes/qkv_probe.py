"""Where does the fused QKV GEMM's time go? (MI355X, M = 8, Qwen2.5-1.5B shapes)

Block spans (launch timeline) of the decode QKV projection with its fusions switched on one
at a time: plain GEMM, + deferred RMSNorm row scale, + bias, + RoPE / paged KV-cache write
epilogue, all of them (the engine's form). Weights cycle through > 600 MB of copies.

    python benchmarks/probes/qkv_probe.py
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
    M, H, hq, hkv = 8, 1536, 12, 2
    N = (hq + 2 * hkv) * 128
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    x = torch.randn(M, H, device=dev).bfloat16()
    w = (torch.randn(N, H, device=dev) / math.sqrt(H)).bfloat16()
    bias = (torch.randn(N, device=dev) * 0.02).bfloat16()
    ncopy = max(2, math.ceil(600e6 / (N * H * 2)))
    lins_plain = [ops.Linear(w, layout="plain") for _ in range(ncopy)]
    lins_qkv = [ops.Linear(w, bias=bias, layout="qkv") for _ in range(ncopy)]
    nblk = 4096
    kc = torch.zeros(nblk, hkv, 16, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    pos = torch.arange(M, dtype=torch.int32, device=dev) * 7 + 40
    slots = torch.arange(M, dtype=torch.int32, device=dev) * 16 * 37 + 3
    cos_sin = torch.randn(4096, 128, device=dev)
    q_out = torch.empty(M, hq * 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    reps = 20
    forms = {
        "plain": lambda i: C.gemm(x, lins_plain[i % ncopy].wp, N, H, out, 0, ws=ws),
        "rownorm": lambda i: C.gemm(x, lins_plain[i % ncopy].wp, N, H, out, 0, ws=ws, rownorm=True),
        "bias": lambda i: C.gemm(x, lins_plain[i % ncopy].wp, N, H, out, 0, ws=ws, bias=bias),
        "qkv_epi": lambda i: C.gemm(x, lins_qkv[i % ncopy].wp, N, H, q_out, 3, ws=ws, positions=pos, slots=slots,
                                    cos_sin=cos_sin, k_cache=kc, v_cache=vc, hq=hq, hkv=hkv),
        "qkv_epi+bias+rownorm": lambda i: C.gemm(x, lins_qkv[i % ncopy].wp, N, H, q_out, 3, ws=ws, bias=bias,
                                                 positions=pos, slots=slots, cos_sin=cos_sin, k_cache=kc,
                                                 v_cache=vc, hq=hq, hkv=hkv, rownorm=True),
    }
    res = {}
    for name, fn in forms.items():
        spans, wall = timeline_graph(C, lambda: [fn(i) for i in range(reps)])
        vals = [v for k, v in spans.items()][0]
        res[name] = {"span_us": round(sum(vals[1:]) / (len(vals) - 1), 2), "wall_per_launch_us": round(wall / reps, 2)}
    print(json.dumps({"qkv_probe": res}), flush=True)


if __name__ == "__main__":
    main()
