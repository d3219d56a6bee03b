"""Phase stamps of the AWQ decode kernel (awq_dec_kernel, first and last block): x staged
(1), LDS barrier passed (2), weight stream + MFMAs done (3), epilogue done (4),
split-K combine (5) — microseconds from the block's start, Qwen2.5-1.5B shapes at M = 8,
weights cycled through > 400 MB so every launch streams from HBM.

    python benchmarks/awq_phases.py
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402

SHAPES = [("gate_up", 17920, 1536, "silu"), ("down", 1536, 8960, "plain")]


def main():
    C = ops.native()
    M, g = 8, 128
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    for name, N, K, layout in SHAPES:
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev)
        scales = (torch.rand(K // g, N, device=dev) * 0.02 + 0.005).bfloat16()
        zeros = torch.randint(0, 16, (K // g, N), device=dev).float().bfloat16()
        ncopy = max(2, math.ceil(400e6 / (N * K // 2)))
        lins = [ops.Linear(None, awq={"qint": q, "scales": scales, "zeros": zeros, "group": g,
                                      "silu": layout == "silu"}) for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev).bfloat16()
        epi = 2 if layout == "silu" else 0
        out = torch.empty(M, N // 2 if epi == 2 else N, device=dev, dtype=torch.bfloat16)
        for sk in (0, 2):
            buf = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
            reps = 12
            rows = []
            for i in range(reps):
                L = lins[i % ncopy]
                buf.zero_()
                C.timeline_start(buf)
                C.gemm(x, L.wp, N, K, out, epi, ws=ws, splitk=sk, awq_scales=L.scales, awq_zeros=L.zeros, group=g,
                       awq_szp=L.szp)
                C.timeline_stop()
                torch.cuda.synchronize()
                ents = C.timeline_entries()
                if not ents:
                    continue
                _, off, nb = ents[-1]
                t = buf[off: off + 2 * nb].cpu().tolist()
                nblk = nb - 8
                starts = [t[2 * b] for b in range(nblk) if t[2 * b] > 0]
                ends = [t[2 * b + 1] for b in range(nblk) if t[2 * b + 1] > 0]
                ph = t[2 * nblk: 2 * nblk + 16]
                first = [round((v - ph[0]) / 100.0, 2) if v else None for v in ph[:6]]
                last = [round((v - ph[8]) / 100.0, 2) if v else None for v in ph[8:14]]
                rows.append({"span_us": round((max(ends) - min(starts)) / 100.0, 2),
                             "start_skew_us": round((max(starts) - min(starts)) / 100.0, 2),
                             "first_block": first, "last_block": last, "blocks": nblk})
            rows = rows[2:]  # drop the cold ones
            avg = {k: round(sum(r[k] for r in rows) / len(rows), 2) for k in ("span_us", "start_skew_us")}
            print(json.dumps({"shape": name, "splitk": sk, "blocks": rows[0]["blocks"], **avg,
                              "phases_first_block": rows[-1]["first_block"], "phases_last_block": rows[-1]["last_block"]}),
                  flush=True)


if __name__ == "__main__":
    main()
