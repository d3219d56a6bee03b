#!/usr/bin/env python3
"""Merge per-scenario JSON files (``run_scenario_cli.py``) into one report .json + .md
(reference benchmarks/_aggregate_results.py), scenarios ordered by start time.

    python benchmarks/aggregate_results.py benchmarks/results/scenarios --out benchmarks/results/report
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

from bench_load import format_markdown  # noqa: E402


def aggregate(src: Path) -> dict:
    runs = []
    for f in sorted(src.glob("*.json")):
        try:
            r = json.loads(f.read_text())
        except json.JSONDecodeError:
            continue
        if isinstance(r, dict) and "scenario" in r and "throughput" in r:
            runs.append(r)
    runs.sort(key=lambda r: r["scenario"].get("started", 0))
    return {r["scenario"]["name"]: r for r in runs}


def to_markdown(results: dict, title: str) -> str:
    md = [f"# {title}", "", "| scenario | req/s | p50 s | p99 s | tok/s |", "|---|---|---|---|---|"]
    for name, r in results.items():
        md.append(f"| {name} | {r['throughput']['requests_per_second']:.2f} | {r['latency']['p50_s']:.4f} | "
                  f"{r['latency']['p99_s']:.4f} | {r['throughput'].get('tokens_per_second', 0):.1f} |")
    md.append("")
    for name, r in results.items():
        md.append(format_markdown(r, title=name))
        md.append("")
    return "\n".join(md)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("src")
    ap.add_argument("--out", default=None)
    ap.add_argument("--title", default="V-Gate benchmark report")
    a = ap.parse_args()
    res = aggregate(Path(a.src))
    if not res:
        sys.exit(f"no scenario results in {a.src}")
    out = Path(a.out) if a.out else Path(a.src) / "report"
    out.with_suffix(".json").write_text(json.dumps(res, indent=2))
    out.with_suffix(".md").write_text(to_markdown(res, a.title))
    print(f"wrote {out.with_suffix('.md')} ({len(res)} scenarios)")


if __name__ == "__main__":
    main()
