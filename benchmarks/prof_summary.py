"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd SQLite, ``*_results.db``) per
kernel *shape*: the demangled name shortened to its template head plus the launch grid, so
the decode GEMMs (same kernel, different N) show up as separate rows.

    python benchmarks/prof_summary.py gpurun_out/prof/run_results.db [--top 30] [--vgate-only]
"""
from __future__ import annotations

import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)  # drop the argument list
    name = name.replace("void ", "").replace("vgate::", "")
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--vgate-only", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count from kernels")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    total = 0.0
    for name, dur, gx, gy, gz, wx, lds, vgpr in rows:
        if a.vgate_only and "vgate" not in name:
            continue
        key = (short(name), f"{gx // max(wx, 1)}x{gy}x{gz} wg{wx} lds{lds} v{vgpr}")
        e = agg[key]
        e[0] += 1
        e[1] += dur / 1e3
        e[2] = max(e[2], dur / 1e3)
        total += dur / 1e3
    print(f"{'kernel':70s} {'launch':34s} {'calls':>7s} {'avg_us':>8s} {'max_us':>8s} {'total_ms':>9s} {'%':>5s}")
    for (k, shape), (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{k:70s} {shape:34s} {n:7d} {tot / n:8.2f} {mx:8.2f} {tot / 1e3:9.2f} {100 * tot / total:5.1f}")
    print(f"total kernel time {total / 1e3:.1f} ms over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main()
