"""What the device does between two engine steps, from a rocprofv3 database recorded with
``--kernel-trace --memory-copy-trace`` (rocpd SQLite).

For every decode step (split at the embedding launch, the first kernel of a step) it lists the
dispatches and copies from the end of the previous step's sampler to the step's embedding
kernel, and reports the median idle time of that boundary. Kernel-only traces cannot show it:
the metadata upload and the sampled-id download are not kernels when they go through hipMemcpy.

    python benchmarks/step_boundary.py run_results.db [--show 2]
"""
from __future__ import annotations

import argparse
import json
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--show", type=int, default=2, help="boundaries to print event by event")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    ks = con.execute("select start, end, name from kernels order by start").fetchall()
    try:
        cs = con.execute("select c.start, c.end, c.size, s.string from rocpd_memory_copy c "
                         "left join rocpd_string s on c.name_id = s.id").fetchall()
    except sqlite3.OperationalError:
        cs = []
    ev = sorted([(s, e, "K", n) for s, e, n in ks] + [(s, e, "C", f"{name} {sz} B") for s, e, sz, name in cs])
    emb = [i for i, x in enumerate(ev) if x[2] == "K" and "embedding_kernel" in x[3]]
    rows, shown = [], 0
    for i0 in emb:
        j = i0 - 1
        while j > 0 and i0 - j < 8 and not (ev[j][2] == "K" and "sample" in ev[j][3]):
            j -= 1
        if j <= 0 or i0 - j >= 8 or "sample" not in ev[j][3]:
            continue  # not a decode step boundary (first step, prefill-only, eager paths)
        t_end = ev[j][1]
        between = ev[j + 1: i0]
        busy = sum(e - s for s, e, _, _ in between)
        rows.append(((ev[i0][0] - t_end) / 1e3, busy / 1e3, len(between)))
        if shown < a.show and len(rows) > len(emb) // 2:
            shown += 1
            print(f"# boundary {len(rows)} (us from the sampler's end)")
            for s, e, kind, name in ev[j: i0 + 1]:
                print(f"  {(s - t_end) / 1e3:8.2f} {(e - t_end) / 1e3:8.2f} {kind} {name[:70]}")
    if not rows:
        print(json.dumps({"boundaries": 0}))
        return
    gaps = [r[0] for r in rows]
    print(json.dumps({"boundaries": len(rows), "sampler_end_to_next_step_us_med": round(statistics.median(gaps), 2),
                      "p90": round(sorted(gaps)[int(0.9 * (len(gaps) - 1))], 2),
                      "ops_between_med": statistics.median(r[2] for r in rows),
                      "busy_between_us_med": round(statistics.median(r[1] for r in rows), 2)}))


if __name__ == "__main__":
    main()
