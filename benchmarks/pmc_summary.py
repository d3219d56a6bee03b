"""Summarise a rocprofv3 ``--pmc <COUNTER> --output-format csv`` run per kernel shape
(template head + grid): calls, mean counter value, mean duration and — for FETCH_SIZE /
WRITE_SIZE (KiB) — the bytes per launch and the effective bandwidth. Under counter
collection every dispatch is serialised, so durations are per-kernel in isolation.

    python benchmarks/pmc_summary.py gpurun_out/pmc_fetch/run_counter_collection.csv [--top 25]
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name).replace("void ", "").replace("vgate::", "")
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--all", action="store_true", help="include non-vgate (torch) kernels")
    a = ap.parse_args()
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    with open(a.csv, newline="") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not a.all and "vgate::" not in name:
                continue
            key = (r["Counter_Name"], short(name), int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])))
            g = agg[key]
            g[0] += 1
            g[1] += float(r["Counter_Value"])
            g[2] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for counter in sorted({k[0] for k in agg}):
        rows = sorted(((k[1:], v) for k, v in agg.items() if k[0] == counter), key=lambda kv: -kv[1][1])[: a.top]
        bytes_counter = counter in ("FETCH_SIZE", "WRITE_SIZE")
        print(f"== {counter}")
        hdr = f"{'kernel':60s} {'blocks':>7s} {'calls':>6s} {'avg':>14s} {'avg_us':>8s}"
        print(hdr + ("   MB/launch   GB/s" if bytes_counter else ""))
        for (k, blocks), (n, v, us) in rows:
            line = f"{k:60s} {blocks:7d} {n:6d} {v / n:14.1f} {us / n:8.2f}"
            if bytes_counter:
                mb = v / n * 1024 / 1e6
                line += f"   {mb:9.2f} {mb * 1e3 / max(us / n, 1e-9):7.0f}"
            print(line)

if __name__ == "__main__":
    main()
