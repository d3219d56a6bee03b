"""Per-block timeline of the decode GEMMs on the MI355X (s_memrealtime, 10 ns ticks):
every block stamps its start and end (GemmArgs::dbg_ts), so one launch shows the span,
the per-block duration distribution, the dispatch skew and the tail — the data needed to
tell a latency-bound kernel from an imbalanced one.

    python benchmarks/gemm_blocks.py
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402

SHAPES = [("qkv", 2048, 1536, "plain"), ("o_proj", 1536, 1536, "plain"), ("gate_up", 17920, 1536, "silu"),
          ("down", 1536, 8960, "plain"), ("lm_head", 151936, 1536, "plain")]


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(int(len(xs) * p / 100), len(xs) - 1)] if xs else 0


def main():
    C = ops.native()
    M = 8
    for name, N, K, layout in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        ncopy = max(1, math.ceil(600e6 / (N * K * 2)))
        lins = [ops.Linear(w, layout=layout) for _ in range(ncopy)]
        out = torch.empty(M, lins[0].out_features, device="cuda",
                          dtype=torch.float32 if name == "lm_head" else torch.bfloat16)
        res = torch.randn(M, N, device="cuda").bfloat16() if name in ("o_proj", "down") else None
        ts = torch.zeros(2 * 65536, dtype=torch.int64, device="cuda")
        runs = []
        for it in range(ncopy + 3):
            lin = lins[it % ncopy]
            ts.zero_()
            kw = dict(ws=ops.workspace(x.device), dbg_ts=ts)
            if res is not None:
                kw["res"] = res
            epi = 2 if layout == "silu" else (1 if name == "lm_head" else 0)
            C.gemm(x, lin.wp, lin.N, lin.K, out, epi, **kw)
            torch.cuda.synchronize()
            t = ts.view(-1, 2).cpu()
            started = t[:, 0] > 0
            st = t[started, 0].tolist()
            en = [e for e in t[started, 1].tolist() if e > 0]
            if it >= 2:
                t0 = min(st)
                runs.append({"blocks": len(st), "span_us": (max(en) - t0) / 100.0,
                             "dur_med_us": pct([e - s for s, e in t[started].tolist() if e > 0], 50) / 100.0,
                             "dur_p90_us": pct([e - s for s, e in t[started].tolist() if e > 0], 90) / 100.0,
                             "dur_max_us": max(e - s for s, e in t[started].tolist() if e > 0) / 100.0,
                             "start_p90_us": (pct(st, 90) - t0) / 100.0, "start_max_us": (max(st) - t0) / 100.0,
                             "end_p10_us": (pct(en, 10) - t0) / 100.0, "end_p50_us": (pct(en, 50) - t0) / 100.0})
        best = min(runs, key=lambda r: r["span_us"])
        print(json.dumps({"shape": name, **{k: round(v, 2) if isinstance(v, float) else v for k, v in best.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
