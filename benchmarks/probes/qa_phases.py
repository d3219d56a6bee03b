"""Phases of the fused QKV projection + decode attention launch (csrc/kernels/qkv_attn.hip) on the
MI355X, Qwen2.5-1.5B decode shape (batch 8, ctx 100): per-block [start, end] stamps of every block
of the launch (launch timeline) and the attention phase stamps of block (sequence 0, KV head 0,
partition 0) wave 0 (AttnArgs::dbg_ts, 100 MHz s_memrealtime): entry (0) -> metadata (1) -> query
granules seen (6) -> chunk done (2) -> partials in LDS (5) -> output stored (3). Times are relative
to the launch's first block start; medians over 40 launches with cold weights (a ring of copies).

    python benchmarks/qa_phases.py [--ctx 100] [--batch 8]
"""
from __future__ import annotations

import argparse
import json
import math
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402
from vgate.ops import reference as ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=100)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hq", type=int, default=12)
    ap.add_argument("--hkv", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=1536)
    a = ap.parse_args()
    C = ops.native()
    dev = torch.device("cuda")
    S, H, D, BS, part, maxlen = a.batch, a.hidden, 128, 16, 512, 2048
    hq, hkv = a.hq, a.hkv
    N = (hq + 2 * hkv) * D
    nbs = maxlen // BS
    nblocks = S * nbs + 8
    bt = torch.randperm(nblocks)[: S * nbs].view(S, nbs).int().to(dev)
    kc = (torch.randn(nblocks, hkv, BS, D, device=dev) * 0.5).bfloat16()
    vc = torch.randn_like(kc)
    cl = torch.full((S,), a.ctx, dtype=torch.int32, device=dev)
    pos = cl - 1
    slots = (bt[torch.arange(S, device=dev), (pos // BS).long()] * BS + pos % BS).int()
    qs = torch.arange(S + 1, dtype=torch.int32, device=dev)
    x = torch.randn(S, H, device=dev).bfloat16()
    gamma = (torch.rand(H, device=dev) + 0.5).bfloat16()
    copies = 24  # cold weights: 24 copies of the projection (> the 256 MB MALL)
    lins = []
    for _ in range(copies):
        lin = ops.Linear((torch.randn(N, H, device=dev) / math.sqrt(H)).bfloat16(),
                         bias=(torch.randn(N, device=dev) * 0.1).bfloat16(), layout="qkv")
        lin.fold_norm(gamma)
        lins.append(lin)
    cs = ref.rope_cos_sin(4096, D, 1e6, device=dev)
    P = maxlen // part
    po = torch.empty(S, hq, P, D, device=dev)
    pml = torch.empty(S, hq, P, 2, device=dev)
    q = torch.empty(S, hq * D, dtype=torch.bfloat16, device=dev)
    o = torch.empty(S, hq * D, dtype=torch.bfloat16, device=dev)
    dbg = torch.zeros(16, dtype=torch.int64, device=dev)
    buf = torch.zeros(1 << 16, dtype=torch.int64, device=dev)
    rows = []
    for it in range(48):
        dbg.zero_()
        buf.zero_()
        C.timeline_start(buf)
        ops.linear(x, lins[it % copies], out=q, norm=(gamma, 1e-6),
                   qkv=dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kc, v_cache=vc, hq=hq, hkv=hkv),
                   attn=dict(block_tables=bt, context_lens=cl, query_start=qs, out=o, part_o=po, part_ml=pml,
                             part_size=part, scale=D ** -0.5, dbg_ts=dbg))
        torch.cuda.synchronize()
        C.timeline_stop()
        ents = C.timeline_entries()
        if it < 8 or not ents:
            continue
        name, off, nb = ents[0]
        st = buf[off: off + 2 * nb].view(nb, 2).cpu()
        t0 = int(st[:, 0].min())
        ncons = S * P * hkv
        nprod = nb - ncons
        prod_end = (st[:nprod, 1] - t0).float() / 100.0
        cons = st[nprod:]
        work = [i for i in range(ncons) if (i % S) < S and (i // S) % P == 0]  # partition 0 blocks do the work
        cons_end = (cons[work, 1] - t0).float() / 100.0
        d = dbg.cpu().tolist()
        rows.append({"kernel": name, "gemm_end_med": float(prod_end.median()), "gemm_end_max": float(prod_end.max()),
                     "attn_end_med": float(cons_end.median()), "attn_end_max": float(cons_end.max()),
                     "b0_start": (d[0] - t0) / 100.0, "b0_meta": (d[1] - t0) / 100.0, "b0_q_seen": (d[6] - t0) / 100.0,
                     "b0_chunk_done": (d[2] - t0) / 100.0, "b0_lds": (d[5] - t0) / 100.0, "b0_stored": (d[3] - t0) / 100.0})
    out = {"ctx": a.ctx, "batch": S, "hq": hq, "hkv": hkv, "kernel": rows[0]["kernel"] if rows else None}
    for k in rows[0]:
        if k != "kernel":
            out[k] = round(statistics.median(r[k] for r in rows), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
