"""Fused decode MLP (csrc/kernels/mlp_fused.hip) vs the two-GEMM path, standalone on the MI355X.

Runs L distinct layers back to back (as a decode step does: each layer's weights are cold, 2.3 GB
for Qwen2.5-1.5B's 28 MLPs), times the sequence with events, and prints the per-workgroup phase
stamps of one fused launch (s_memrealtime, 100 MHz): x staged, gate_up done, h stored, h polled,
down done, ticket, end — medians / p90 / max over the grid relative to the launch's first start.

    python benchmarks/mlp_probe.py [--M 8] [--layers 28] [--H 1536] [--I 8960]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402

PHASES = ["start", "setup_done", "x_issued", "x_landed", "x_staged", "gate_up_done_all_waves", "h_stored", "h_polled",
          "down_done", "ticket", "end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8)
    ap.add_argument("--layers", type=int, default=28)
    ap.add_argument("--H", type=int, default=1536)
    ap.add_argument("--I", type=int, default=8960)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--slices", type=int, default=0)
    ap.add_argument("--b-early", type=int, default=0)
    a = ap.parse_args()
    ops.FUSED_MLP = True
    dev = torch.device("cuda:0")
    H, I, M = a.H, a.I, a.M
    g = torch.Generator(device=dev).manual_seed(0)
    layers = []
    for _ in range(a.layers):
        wgu = (torch.randn(2 * I, H, device=dev, generator=g) / math.sqrt(H)).bfloat16()
        gu = ops.Linear(wgu, kind="silu")
        gamma = (torch.rand(H, device=dev, generator=g) + 0.5).bfloat16()
        gu.fold_norm(gamma)
        dn = ops.Linear((torch.randn(H, I, device=dev, generator=g) / math.sqrt(I)).bfloat16())
        layers.append((gu, dn, gamma))
    x = torch.randn(M, H, device=dev, generator=g).bfloat16()
    epoch = torch.zeros(4, dtype=torch.int32, device=dev)
    mid = torch.empty(M, I, dtype=torch.bfloat16, device=dev)

    def fused():
        epoch.add_(1)
        for li, (gu, dn, _) in enumerate(layers):
            assert ops.mlp_decode(x, gu, dn, x, x, 1e-6, li, epoch, slices=a.slices, b_early=a.b_early)

    def unfused():
        for gu, dn, gamma in layers:
            ops.linear(x, gu, out=mid, norm=(gamma, 1e-6))
            ops.linear(mid, dn, out=x, residual=x)

    res = {}
    for name, fn in (("fused", fused), ("two_gemm", unfused)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.iters):
            fn()
        s1.record()
        s1.synchronize()
        res[name + "_us_per_layer"] = round(1e3 * s0.elapsed_time(s1) / (a.iters * a.layers), 2)
    res["weights_mb_per_layer"] = round((2 * I * H + H * I) * 2 / 1e6, 1)
    res["fused_tb_s"] = round(res["weights_mb_per_layer"] / res["fused_us_per_layer"], 2)
    res["two_gemm_tb_s"] = round(res["weights_mb_per_layer"] / res["two_gemm_us_per_layer"], 2)
    print(json.dumps(res), flush=True)

    # phase stamps of one fused launch (the middle layer, cold weights: the previous layers evict it)
    G = 256
    dbg = torch.zeros(G * 16, dtype=torch.int64, device=dev)
    epoch.add_(1)
    for li, (gu, dn, _) in enumerate(layers):
        kw = {"dbg": dbg} if li == a.layers // 2 else {}
        ops.native().mlp_decode(x, gu.wp, dn.wp, H, I, x, x, 1e-6, ops.mlp_workspace(dev, H, I), epoch, li,
                                a.slices, 0, b_early=a.b_early, **kw)
    torch.cuda.synchronize()
    st = dbg.view(G, 16).cpu().double()
    t0 = st[:, 0].min()
    out = {}
    for i, ph in enumerate(PHASES):
        col = st[:, i]
        col = col[col > 0]
        if col.numel() == 0:
            continue
        rel = (col - t0) / 100.0  # us
        q = torch.quantile(rel, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        out[ph] = {"p10": round(q[0].item(), 2), "p50": round(q[1].item(), 2), "p90": round(q[2].item(), 2),
                   "max": round(rel.max().item(), 2), "n": int(col.numel())}
    print(json.dumps({"phases_us_from_first_start": out}), flush=True)
    print(json.dumps({"mlp_error": ops.mlp_error(dev)}), flush=True)


if __name__ == "__main__":
    main()
