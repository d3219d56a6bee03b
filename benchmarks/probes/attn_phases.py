"""Decode-attention phase timing on the MI355X: 100 MHz s_memrealtime stamps written by wave 0
of block (sequence 0, KV head 0, partition 0) of the unified attention kernel (AttnArgs::dbg_ts):
entry (0) -> metadata loaded (1) -> first chunk's K/V landed (4) -> chunk loop done (2) ->
waves' partials in LDS (5) -> merged output stored (3). Medians over 50 launches, in us.

    python benchmarks/attn_phases.py
"""
from __future__ import annotations

import json
import math
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def main():
    C = ops.native()
    S, Hq, Hkv, D, bs, nblk = 8, 12, 2, 128, 16, 4096
    kc = torch.randn(nblk, Hkv, bs, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, bs, D, device="cuda").bfloat16()
    for ctx in (32, 64, 128, 256, 512):
        maxb = 2048 // bs
        bt = torch.randperm(nblk, device="cuda")[: S * maxb].view(S, maxb).int().contiguous()
        cl = torch.full((S,), ctx, dtype=torch.int32, device="cuda")
        qs = torch.arange(S + 1, dtype=torch.int32, device="cuda")
        q = torch.randn(S, Hq * D, device="cuda").bfloat16()
        out = torch.empty(S, Hq * D, device="cuda").bfloat16()
        ts = torch.full((S,), -1, dtype=torch.int32, device="cuda")
        tq = torch.zeros(S, dtype=torch.int32, device="cuda")
        part = 512
        P = 2048 // part
        po = torch.empty(S, Hq, P, D, device="cuda")
        pml = torch.empty(S, Hq, P, 2, device="cuda")
        dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
        ph = []
        for _ in range(50):
            dbg.zero_()
            C.attention(q, Hq * D, kc, vc, bt, cl, qs, ts, tq, out, po, pml, Hq, Hkv, part, 1 / math.sqrt(D), 0,
                        ops.attn_tickets(q.device), dbg)
            torch.cuda.synchronize()
            ph.append(dbg.cpu().tolist())

        def us(i, j):
            return round(statistics.median((x[j] - x[i]) / 100.0 for x in ph), 3)
        print(json.dumps({"ctx": ctx, "meta_us": us(0, 1), "first_kv_us": us(1, 4), "loop_rest_us": us(4, 2),
                          "partials_to_lds_us": us(2, 5), "merge_store_us": us(5, 3), "total_block_us": us(0, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
