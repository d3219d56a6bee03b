"""Decode-attention phase timing on the MI355X: s_memtime stamps written by block (0,0,0)
of the unified attention kernel (AttnArgs::dbg_ts) — entry, metadata loaded, chunk loop
done, merge/store done — to see where a short-context decode launch spends its time.

    python benchmarks/attn_phases.py
"""
from __future__ import annotations

import json
import math
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def main():
    C = ops.native()
    S, Hq, Hkv, D, bs, nblk = 8, 12, 2, 128, 16, 4096
    kc = torch.randn(nblk, Hkv, bs, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, bs, D, device="cuda").bfloat16()
    for ctx in (32, 64, 128, 256):
        maxb = 2048 // bs
        bt = torch.randperm(nblk, device="cuda")[: S * maxb].view(S, maxb).int().contiguous()
        cl = torch.full((S,), ctx, dtype=torch.int32, device="cuda")
        qs = torch.arange(S + 1, dtype=torch.int32, device="cuda")
        q = torch.randn(S, Hq * D, device="cuda").bfloat16()
        out = torch.empty(S, Hq * D, device="cuda").bfloat16()
        ts = torch.full((S,), -1, dtype=torch.int32, device="cuda")
        tq = torch.zeros(S, dtype=torch.int32, device="cuda")
        part = 256
        P = 2048 // part
        po = torch.empty(S, Hq, P, D, device="cuda")
        pml = torch.empty(S, Hq, P, 2, device="cuda")
        dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
        ph = []
        for _ in range(30):
            dbg.zero_()
            C.attention(q, Hq * D, kc, vc, bt, cl, qs, ts, tq, out, po, pml, Hq, Hkv, part, 1 / math.sqrt(D), 0,
                        ops.attn_tickets(q.device), dbg)
            torch.cuda.synchronize()
            d = dbg.cpu().tolist()
            ph.append(d)
        # clock rate from the 100 MHz realtime stamps
        rates = [(x[3] - x[0]) / max(1, (x[7] - x[6])) * 100.0 for x in ph if x[7] > x[6]]  # ticks per us
        rate = statistics.median(rates) if rates else 2400.0
        def us(i, j):
            return round(statistics.median((x[j] - x[i]) / rate for x in ph), 3)
        rec = {"ctx": ctx, "ticks_per_us": round(rate, 1), "meta_us": us(0, 1), "loop_us": us(1, 2),
               "merge_store_us": us(2, 3), "total_block_us": us(0, 3)}
        if ctx > 32:  # chunk-1 sub-phases: loads landed -> QK -> softmax -> V to LDS -> PV
            rec.update(qk_us=us(8, 9), softmax_us=us(9, 10), v_lds_us=us(10, 11), pv_us=us(11, 12))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
