"""Idle-GPU gaps of the serving loop from a rocprofv3 ``--kernel-trace`` database (rocpd SQLite).

Splits the trace into engine steps at every embedding launch (the first kernel of a step) and
reports, over the decode steps, the median gap in front of the step (previous step's last
kernel end -> embedding start) and after each of the step's first kernels, plus the median
sum of all gaps inside a step. rocprof's per-kernel durations cannot show where the device
waits for the host (graph submission, metadata upload, the sampled-token copy).

    python benchmarks/trace_gaps.py gpurun_out/prof/run_results.db [--first 6]
"""
from __future__ import annotations

import argparse
import json
import re
import sqlite3
import statistics


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name).replace("void ", "").replace("vgate::", "")
    return re.sub(r"<.*$", "", name)[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first", type=int, default=6, help="gaps after the first N kernels of a step")
    ap.add_argument("--min-kernels", type=int, default=100, help="steps with fewer launches are skipped (prefill, eager)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("PRAGMA table_info(kernels)")]
    s_col = next(x for x in cols if x in ("start", "start_ns", "begin"))
    e_col = next(x for x in cols if x in ("end", "end_ns", "stop"))
    rows = sorted(c.execute(f"select name, {s_col}, {e_col} from kernels"), key=lambda r: r[1])
    steps, cur = [], []
    for r in rows:
        if "embedding" in r[0] and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    if cur:
        steps.append(cur)
    before, inner, span = [], [], []
    after = [[] for _ in range(a.first)]
    names = None
    prev_end = None
    for st in steps:
        if prev_end is not None and len(st) >= a.min_kernels:
            before.append((st[0][1] - prev_end) / 1e3)
            gaps = [(st[i + 1][1] - st[i][2]) / 1e3 for i in range(len(st) - 1)]
            for i in range(min(a.first, len(gaps))):
                after[i].append(gaps[i])
            inner.append(sum(g for g in gaps if g > 0))
            span.append((st[-1][2] - st[0][1]) / 1e3)
            names = names or [short(x[0]) for x in st[: a.first]]
        prev_end = max(x[2] for x in st)
    med = lambda v: round(statistics.median(v), 2) if v else None  # noqa: E731
    print(json.dumps({"decode_steps": len(span), "step_span_us_med": med(span), "gap_before_step_us_med": med(before),
                      "gaps_inside_step_us_med": med(inner),
                      "gap_after_first_kernels_us_med": {f"{i}:{names[i] if names else i}": med(v)
                                                        for i, v in enumerate(after)}}))


if __name__ == "__main__":
    main()
