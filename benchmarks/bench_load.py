#!/usr/bin/env python3
"""Closed-loop load generator against a RUNNING V-Gate server (full HTTP path:
security -> batcher -> cache -> backend).

Same CLI and result schema as the reference tool (reference
benchmarks/bench_load.py:160-279, :356-383) so existing scripts keep working:

  * ``--concurrency`` in-flight requests (asyncio semaphore), ``--requests`` total;
  * throughput = requests / wall time, failures included;
  * percentiles use the index ``min(int(n * p / 100), n - 1)`` over sorted latencies;
  * batching / cache sections are the DIFF of ``/stats`` before and after the run;
  * ``--stream`` consumes SSE, reports client TTFT percentiles, and counts tokens
    from the server's ``vgate_stream_tokens_total`` counter (a delta may carry
    several tokens).

Additions: ``--unique`` makes every prompt unique (defeats the result cache, the
setting of the published baseline), ``--output json|markdown``.

    python benchmarks/bench_load.py --url http://127.0.0.1:8000 -c 8 -n 40 --unique
"""
from __future__ import annotations

import argparse
import asyncio
import json
import re
import statistics
import time
from pathlib import Path

DEFAULT_PROMPTS = [
    "Explain the concept of machine learning in one paragraph.",
    "Write a Python function that computes the Fibonacci sequence.",
    "What are the benefits of using a load balancer?",
    "Summarize the CAP theorem in two sentences.",
]


def percentile(xs: list[float], p: float) -> float:
    if not xs:
        return 0.0
    s = sorted(xs)
    return s[min(int(len(s) * p / 100), len(s) - 1)]


def counter_value(metrics_text: str, name: str) -> float:
    """Sum of all samples of a Prometheus counter in text exposition format."""
    total = 0.0
    pat = re.compile(rf"^{re.escape(name)}(?:\{{[^}}]*\}})?\s+([0-9.eE+-]+)")
    for line in metrics_text.splitlines():
        m = pat.match(line)
        if m:
            total += float(m.group(1))
    return total


def load_prompts(path: str | None) -> list[str]:
    if not path:
        return list(DEFAULT_PROMPTS)
    lines = [ln.strip() for ln in Path(path).read_text(encoding="utf-8").splitlines() if ln.strip()]
    return lines or list(DEFAULT_PROMPTS)


async def _one(session, url, prompt, max_tokens, headers):
    body = {"model": "default", "messages": [{"role": "user", "content": prompt}], "max_tokens": max_tokens}
    t0 = time.perf_counter()
    try:
        async with session.post(url, json=body, headers=headers) as r:
            data = await r.json(content_type=None)
            ok = r.status == 200
    except Exception:  # noqa: BLE001 - a failed request counts, it never aborts the run
        return {"ok": False, "latency_s": time.perf_counter() - t0, "tokens": 0}
    toks = (data.get("usage") or {}).get("completion_tokens", 0) if ok and isinstance(data, dict) else 0
    return {"ok": ok, "latency_s": time.perf_counter() - t0, "tokens": toks}


async def _one_stream(session, url, prompt, max_tokens, headers):
    body = {"model": "default", "messages": [{"role": "user", "content": prompt}], "max_tokens": max_tokens,
            "stream": True}
    t0 = time.perf_counter()
    ttft, chunks, ok = None, 0, False
    try:
        async with session.post(url, json=body, headers=headers) as r:
            if r.status != 200:
                return {"ok": False, "latency_s": time.perf_counter() - t0, "content_chunks": 0, "ttft_s": None}
            async for raw in r.content:
                line = raw.decode("utf-8", "replace").strip()
                if not line.startswith("data:"):
                    continue
                payload = line[5:].strip()
                if payload == "[DONE]":
                    ok = True
                    break
                try:
                    ev = json.loads(payload)
                except json.JSONDecodeError:
                    continue
                if "error" in ev:
                    break
                delta = (ev.get("choices") or [{}])[0].get("delta", {})
                if delta.get("content"):
                    chunks += 1
                    if ttft is None:
                        ttft = time.perf_counter() - t0
    except Exception:  # noqa: BLE001
        ok = False
    return {"ok": ok, "latency_s": time.perf_counter() - t0, "content_chunks": chunks, "ttft_s": ttft}


async def run_load_test(base_url: str, concurrency: int, total_requests: int, prompts: list[str],
                        max_tokens: int = 64, api_key: str | None = None, stream: bool = False,
                        unique: bool = False) -> dict:
    import aiohttp
    headers = {"Authorization": f"Bearer {api_key}"} if api_key else None
    chat = f"{base_url.rstrip('/')}/v1/chat/completions"
    send = _one_stream if stream else _one
    conn = aiohttp.TCPConnector(limit=max(concurrency * 2, 16))
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=600)) as s:
        async def get(path, text=False):
            async with s.get(f"{base_url.rstrip('/')}{path}", headers=headers) as r:
                return await (r.text() if text else r.json(content_type=None))

        before = await get("/stats")
        tok0 = counter_value(await get("/metrics", True), "vgate_stream_tokens_total") if stream else 0.0
        sem = asyncio.Semaphore(concurrency)

        async def bounded(i):
            p = prompts[i % len(prompts)]
            if unique:
                p = f"[{i}] {p}"
            async with sem:
                return await send(s, chat, p, max_tokens, headers)

        t0 = time.perf_counter()
        res = await asyncio.gather(*(bounded(i) for i in range(total_requests)))
        wall = time.perf_counter() - t0
        after = await get("/stats")
        tok1 = counter_value(await get("/metrics", True), "vgate_stream_tokens_total") if stream else 0.0

    lat = [r["latency_s"] for r in res if r["ok"]]
    fails = sum(not r["ok"] for r in res)
    total_tokens = int(round(tok1 - tok0)) if stream else sum(r["tokens"] for r in res)
    b0, b1 = before.get("batcher", {}), after.get("batcher", {})
    c0, c1 = before.get("cache", {}), after.get("cache", {})

    def d(a, b, k):
        return b.get(k, 0) - a.get(k, 0)

    nreq, nbat = d(b0, b1, "total_requests"), d(b0, b1, "total_batches")
    hits, miss = d(c0, c1, "hits"), d(c0, c1, "misses")
    latency = {"mean_s": round(statistics.mean(lat), 4) if lat else 0, "p50_s": round(percentile(lat, 50), 4),
               "p95_s": round(percentile(lat, 95), 4), "p99_s": round(percentile(lat, 99), 4),
               "max_s": round(max(lat), 4) if lat else 0}
    throughput = {"total_tokens": total_tokens,
                  "tokens_per_second": round(total_tokens / wall, 2) if wall > 0 else 0,
                  "requests_per_second": round(total_requests / wall, 2) if wall > 0 else 0}
    if stream:
        tt = [r["ttft_s"] for r in res if r["ok"] and r.get("ttft_s") is not None]
        latency.update(ttft_mean_s=round(statistics.mean(tt), 4) if tt else 0,
                       ttft_p50_s=round(percentile(tt, 50), 4), ttft_p95_s=round(percentile(tt, 95), 4))
        throughput["content_chunks"] = sum(r["content_chunks"] for r in res)
    return {
        "config": {"concurrency": concurrency, "total_requests": total_requests,
                   "unique_prompts": total_requests if unique else len(prompts), "max_tokens": max_tokens,
                   "stream": stream},
        "wall_time_s": round(wall, 4),
        "failures": fails,
        "latency": latency,
        "throughput": throughput,
        "batching": {"requests": nreq, "batches": nbat,
                     "average_batch_size": round(nreq / nbat, 2) if nbat > 0 else 0,
                     "deduplicated": d(b0, b1, "total_deduplicated"),
                     "avg_queue_time_s": b1.get("avg_queue_time_s", 0), "avg_ttft_s": b1.get("avg_ttft_s", 0),
                     "avg_tpot_s": b1.get("avg_tpot_s", 0)},
        "cache": {"hits": hits, "misses": miss,
                  "hit_rate": round(hits / (hits + miss), 4) if hits + miss > 0 else 0},
    }


def format_markdown(r: dict, title: str = "V-Gate Load Benchmark") -> str:
    c, lat, thr, b, ch = r["config"], r["latency"], r["throughput"], r["batching"], r["cache"]
    out = [f"## {title}", "",
           f"- Concurrency: {c['concurrency']}", f"- Total requests: {c['total_requests']}",
           f"- Unique prompts: {c['unique_prompts']}", f"- max_tokens: {c['max_tokens']}",
           f"- Streaming: {c['stream']}", f"- Wall time: {r['wall_time_s']} s", f"- Failures: {r['failures']}", "",
           "| Metric | Value |", "|---|---|",
           f"| Throughput | {thr['requests_per_second']} req/s |",
           f"| Tokens/s | {thr['tokens_per_second']} |",
           f"| Latency mean | {lat['mean_s']} s |", f"| Latency p50 | {lat['p50_s']} s |",
           f"| Latency p95 | {lat['p95_s']} s |", f"| Latency p99 | {lat['p99_s']} s |",
           f"| Latency max | {lat['max_s']} s |"]
    if c["stream"]:
        out += [f"| TTFT mean | {lat['ttft_mean_s']} s |", f"| TTFT p50 | {lat['ttft_p50_s']} s |",
                f"| TTFT p95 | {lat['ttft_p95_s']} s |"]
    out += [f"| Batches | {b['batches']} (avg size {b['average_batch_size']}) |",
            f"| Deduplicated | {b['deduplicated']} |",
            f"| Cache hits / misses | {ch['hits']} / {ch['misses']} (hit rate {ch['hit_rate']}) |"]
    return "\n".join(out)


def main() -> None:
    ap = argparse.ArgumentParser(description="V-Gate concurrent load benchmark (hits a running server)")
    ap.add_argument("--url", default="http://localhost:8000")
    ap.add_argument("--concurrency", "-c", type=int, default=8)
    ap.add_argument("--requests", "-n", type=int, default=80)
    ap.add_argument("--prompt-file", default=None)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--api-key", default=None)
    ap.add_argument("--stream", action="store_true")
    ap.add_argument("--unique", action="store_true", help="make every prompt unique (no cache hits)")
    ap.add_argument("--output", choices=["json", "markdown"], default="markdown")
    a = ap.parse_args()
    r = asyncio.run(run_load_test(a.url, a.concurrency, a.requests, load_prompts(a.prompt_file), a.max_tokens,
                                  a.api_key, a.stream, a.unique))
    print(json.dumps(r, indent=2) if a.output == "json" else format_markdown(r, f"Load Benchmark: {a.url}"))


if __name__ == "__main__":
    main()
