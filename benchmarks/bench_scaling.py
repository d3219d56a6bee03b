#!/usr/bin/env python3
"""Gateway + N worker scaling harness (split deployment, real processes, real HTTP).

Starts one gateway and N dry-run workers as separate OS processes (each its own
process group, reaped on exit), points the gateway at the workers through
``VGATE_WORKER__ENDPOINTS``, and drives the gateway with the closed-loop load
generator. Every worker has a declared synthetic capacity (latency per generation x
concurrent slots), so the ideal throughput of N workers is N x slots / latency and
the measured efficiency isolates the gateway/transport overhead — the quantity the
reference's scaling study reports (reference benchmarks/bench_scaling.py:1028-1045,
results 2.00x@2 and 3.89x@4 workers).

Optional: ``--client-procs K`` splits the load over K separate client processes that
start on a shared wall-clock barrier (benchmarks/_load_client.py), so the client is
never the bottleneck. ``--engine native`` runs real native-engine workers instead of
dry-run ones (one GPU each via HIP_VISIBLE_DEVICES).

Experiments beyond the worker sweep (``--experiments``), after the reference's
gateway-ceiling study (reference benchmarks/bench_scaling.py:342-572):

* ``admission`` — 4 workers, gateway ``batch.max_batch_size`` swept over
  {capacity, shipped default, --admission}: below N x capacity the gateway's own
  permit count is the ceiling, invisible from outside.
* ``saturation`` — 8 workers (2x the pool capacity of anything else measured), load
  from 1/2/4 separate client PROCESSES whose offered concurrency grows with their
  count; throughput over ONE common wall-clock window; gateway CPU (from
  /proc/<pid>/stat) and host CPU busy recorded, so a flat total is attributable.
* ``source`` — generation cost 100/50/25 ms at far-above-demand pool capacity: a
  concurrency-bound gateway ceiling moves with latency, a CPU-bound one does not.

    python benchmarks/bench_scaling.py --workers 1 2 4 --repeats 3
    python benchmarks/bench_scaling.py --experiments workers admission saturation source
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(ROOT))

from bench_load import DEFAULT_PROMPTS, run_load_test  # noqa: E402


def port_free(port: int) -> bool:
    with socket.socket() as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)  # as uvicorn binds (TIME_WAIT is fine)
        try:
            s.bind(("127.0.0.1", port))
            return True
        except OSError:
            return False


def wait_ports_free(ports, timeout=30.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if all(port_free(p) for p in ports):
            return
        time.sleep(0.2)
    raise RuntimeError(f"ports still busy: {ports}")


def wait_http(url: str, timeout: float = 120.0) -> None:
    import urllib.request
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            with urllib.request.urlopen(url, timeout=2) as r:
                if r.status == 200:
                    return
        except Exception:  # noqa: BLE001
            time.sleep(0.2)
    raise RuntimeError(f"{url} not ready after {timeout}s")


class Proc:
    """A child server process in its own process group (killed as a group)."""

    def __init__(self, env: dict, log: Path):
        self.log = open(log, "w")
        self.p = subprocess.Popen([sys.executable, str(ROOT / "main.py")], cwd=str(ROOT), env=env,
                                  stdout=self.log, stderr=subprocess.STDOUT, start_new_session=True)

    def stop(self):
        if self.p.poll() is None:
            try:
                os.killpg(self.p.pid, signal.SIGTERM)
                self.p.wait(timeout=15)
            except Exception:  # noqa: BLE001
                os.killpg(self.p.pid, signal.SIGKILL)
                self.p.wait(timeout=15)
        self.log.close()


def base_env(**kw) -> dict:
    env = dict(os.environ)
    env.update({"VGATE_LOGGING__LEVEL": "WARNING", "PYTHONPATH": str(ROOT)})
    env.update({k: str(v) for k, v in kw.items()})
    return env


def start_topology(n_workers: int, args, logdir: Path):
    gw_port, w0 = args.gateway_port, args.worker_port
    ports = [gw_port] + [w0 + i for i in range(n_workers)]
    wait_ports_free(ports)
    procs = []
    for i in range(n_workers):
        env = dict(VGATE_ROLE="worker", VGATE_SERVER__HOST="127.0.0.1", VGATE_SERVER__PORT=w0 + i)
        if args.engine == "dry-run":
            env.update(VGATE_DRY_RUN="true", VGATE_DRYRUN_SIMULATED_LATENCY_MS=args.latency_ms,
                       VGATE_DRYRUN_MAX_CONCURRENCY=args.capacity)
        else:
            env.update(VGATE_DRY_RUN="false", VGATE_MODEL__ENGINE_TYPE="native", HIP_VISIBLE_DEVICES=str(i))
        procs.append(Proc(base_env(**env), logdir / f"worker{i}.log"))
    for i in range(n_workers):
        wait_http(f"http://127.0.0.1:{w0 + i}/health", args.boot_timeout)
    eps = json.dumps([f"http://127.0.0.1:{w0 + i}" for i in range(n_workers)])
    gw = Proc(base_env(VGATE_ROLE="gateway", VGATE_SERVER__HOST="127.0.0.1", VGATE_SERVER__PORT=gw_port,
                       VGATE_WORKER__ENDPOINTS=eps, VGATE_BATCH__MAX_BATCH_SIZE=args.admission,
                       VGATE_CACHE__ENABLED="false", VGATE_WORKER__ROUTING=args.routing),
              logdir / "gateway.log")
    procs.append(gw)
    wait_http(f"http://127.0.0.1:{gw_port}/ready", args.boot_timeout)
    return procs


def proc_cpu_seconds(pid: int):
    """utime+stime of one process from /proc (None if unreadable)."""
    try:
        f = Path(f"/proc/{pid}/stat").read_text().rsplit(")", 1)[1].split()
        return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return None


def host_busy_seconds():
    """Busy CPU-seconds of the whole host (all cores) from /proc/stat."""
    try:
        v = [int(x) for x in Path("/proc/stat").read_text().splitlines()[0].split()[1:]]
        idle = v[3] + (v[4] if len(v) > 4 else 0)
        return (sum(v[:8]) - idle) / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError):
        return None


def run_client_procs(url: str, procs: int, conc_each: int, requests_each: int, max_tokens: int, tag: str) -> dict:
    """`procs` separate load-generator processes over one shared window.

    Throughput = every completed request / (first start .. last end) — not a sum of
    per-process rates, which over non-coinciding windows biases upward with the
    process count (the axis being varied). A shared start barrier removes most of the
    skew; the residual is reported."""
    start_at = time.time() + 1.0 + 0.3 * procs
    stamp = int(time.time() * 1000)
    ps = [subprocess.Popen([sys.executable, str(Path(__file__).parent / "_load_client.py"), "--url", url,
                            "--requests", str(requests_each), "--concurrency", str(conc_each), "--max-tokens",
                            str(max_tokens), "--start-at", f"{start_at:.3f}", "--tag", f"{tag}-{stamp}-{k}"],
                           stdout=subprocess.PIPE, text=True) for k in range(procs)]
    outs = []
    for p in ps:
        out, _ = p.communicate(timeout=900)
        if p.returncode != 0:
            raise RuntimeError(f"load client exited {p.returncode}")
        outs.append(json.loads(out.strip().splitlines()[-1]))
    t0 = min(o["t_start"] for o in outs)
    t1 = max(o["t_end"] for o in outs)
    if t1 <= t0:
        raise RuntimeError(f"measurement window {t1 - t0:.3f}s is unusable (clock jump?)")
    lat = sorted(x for o in outs for x in o["latencies"])
    n = sum(o["requests"] for o in outs)

    def pct(q):
        return round(lat[min(int(len(lat) * q), len(lat) - 1)], 4) if lat else 0.0
    return {"wall_time_s": round(t1 - t0, 3), "requests": n, "failures": sum(o["failures"] for o in outs),
            "start_skew_s": round(max(o["t_start"] for o in outs) - t0, 3),
            "throughput": {"requests_per_second": round(n / (t1 - t0), 2)},
            "latency": {"p50_s": pct(0.50), "p95_s": pct(0.95), "p99_s": pct(0.99)}}


def run_clients(url: str, args) -> dict:
    if args.client_procs <= 1:
        return asyncio.run(run_load_test(url, args.concurrency, args.requests, DEFAULT_PROMPTS, args.max_tokens,
                                         stream=False, unique=True))
    return run_client_procs(url, args.client_procs, max(1, args.concurrency // args.client_procs),
                            args.requests // args.client_procs, args.max_tokens, "sweep")


class topology:
    """Context manager: a gateway + n dry-run workers with the given knobs."""

    def __init__(self, args, n_workers, logdir, **over):
        self.a = argparse.Namespace(**{**vars(args), **over})
        self.n, self.logdir = n_workers, logdir

    def __enter__(self):
        self.procs = start_topology(self.n, self.a, self.logdir)
        self.gateway_pid = self.procs[-1].p.pid
        return self

    def __exit__(self, *exc):
        for p in self.procs:
            p.stop()


def gen_seconds(latency_ms: float, max_tokens: int) -> float:
    return (latency_ms + 2.0 * max_tokens) / 1e3  # DryRunBackend cost model (backends/base.py)


def warm(a) -> None:
    """Untimed warm-up: the gateway's keep-alive pool and the workers' first-request paths."""
    run_client_procs(f"http://127.0.0.1:{a.gateway_port}", 1, a.concurrency, 2 * a.concurrency, a.max_tokens, "warm")


def exp_workers(a, logdir) -> list:
    gen_s = gen_seconds(a.latency_ms, a.max_tokens)
    rows = []
    for n in a.workers:
        with topology(a, n, logdir):
            warm(a)
            runs = [run_clients(f"http://127.0.0.1:{a.gateway_port}", a) for _ in range(a.repeats)]
        rps = statistics.median(r["throughput"]["requests_per_second"] for r in runs)
        ideal = n * a.capacity / gen_s if a.engine == "dry-run" else None
        rows.append({"workers": n, "rps_median": rps, "runs": [r["throughput"]["requests_per_second"] for r in runs],
                     "p50_s": statistics.median(r["latency"]["p50_s"] for r in runs),
                     "p99_s": statistics.median(r["latency"]["p99_s"] for r in runs),
                     "failures": sum(r["failures"] for r in runs), "ideal_rps": round(ideal, 2) if ideal else None,
                     "efficiency_vs_ideal": round(rps / ideal, 3) if ideal else None})
        print(json.dumps(rows[-1]), flush=True)
    base = rows[0]["rps_median"] / rows[0]["workers"]
    for r in rows:
        r["speedup_vs_1"] = round(r["rps_median"] / base, 3) if base else None
        r["scaling_efficiency"] = round(r["rps_median"] / (base * r["workers"]), 3) if base else None
    return rows


def exp_admission(a, logdir) -> list:
    """Gateway admission window (batch.max_batch_size) as a ceiling (ref bench_scaling.py:342-383)."""
    from vgate.config import BatchConfig
    default = BatchConfig().max_batch_size
    gen_s = gen_seconds(a.latency_ms, a.max_tokens)
    rows = []
    for adm in sorted({a.capacity, default, a.admission}):
        with topology(a, a.ceiling_workers, logdir, admission=adm):
            warm(a)
            r = run_client_procs(f"http://127.0.0.1:{a.gateway_port}", 1, a.concurrency, a.requests,
                                 a.max_tokens, f"adm{adm}")
        pool = a.ceiling_workers * a.capacity
        rows.append({"admission": adm, "workers": a.ceiling_workers, "is_shipped_default": adm == default,
                     "binding": adm < pool, "predicted_rps": round(min(adm, pool) / gen_s, 1),
                     "measured_rps": r["throughput"]["requests_per_second"], "p95_s": r["latency"]["p95_s"],
                     "failures": r["failures"]})
        print(json.dumps(rows[-1]), flush=True)
    return rows


def exp_saturation(a, logdir) -> dict:
    """8 workers, 1/2/4 client processes, offered concurrency grows with the process count
    (ref bench_scaling.py:386-470)."""
    gen_s = gen_seconds(a.latency_ms, a.max_tokens)
    rows = []
    with topology(a, a.saturation_workers, logdir, admission=a.admission * 8) as topo:
        warm(a)
        for procs in (1, 2, 4):
            g0, h0 = proc_cpu_seconds(topo.gateway_pid), host_busy_seconds()
            r = run_client_procs(f"http://127.0.0.1:{a.gateway_port}", procs, a.concurrency, a.requests,
                                 a.max_tokens, f"sat{procs}")
            g1, h1 = proc_cpu_seconds(topo.gateway_pid), host_busy_seconds()
            w = r["wall_time_s"]
            rows.append({"client_processes": procs, "offered_concurrency": procs * a.concurrency,
                         "total_rps": r["throughput"]["requests_per_second"], "window_s": w,
                         "start_skew_s": r["start_skew_s"],
                         "gateway_cores": round((g1 - g0) / w, 2) if None not in (g0, g1) else None,
                         "host_cores_busy": round((h1 - h0) / w, 2) if None not in (h0, h1) else None,
                         "host_cores_total": os.cpu_count(), "p95_s": r["latency"]["p95_s"],
                         "failures": r["failures"]})
            print(json.dumps(rows[-1]), flush=True)
    return {"workers": a.saturation_workers, "pool_capacity_rps": round(a.saturation_workers * a.capacity / gen_s, 1),
            "rows": rows}


def exp_source(a, logdir) -> list:
    """Vary generation cost at far-above-demand pool capacity (ref bench_scaling.py:520-560): a
    concurrency-bound ceiling scales with 1/latency, a CPU-bound one stays flat."""
    rows = []
    for lat in a.source_latencies:
        n = a.saturation_workers
        with topology(a, n, logdir, latency_ms=lat, capacity=a.capacity * 4, admission=a.admission * 8) as topo:
            warm(a)
            g0, h0 = proc_cpu_seconds(topo.gateway_pid), host_busy_seconds()
            r = run_client_procs(f"http://127.0.0.1:{a.gateway_port}", 2, a.concurrency * 3, a.requests,
                                 a.max_tokens, f"src{lat}")
            g1, h1 = proc_cpu_seconds(topo.gateway_pid), host_busy_seconds()
        w = r["wall_time_s"]
        gen_s = gen_seconds(lat, a.max_tokens)
        rows.append({"latency_ms": lat, "pool_capacity_rps": round(n * a.capacity * 4 / gen_s, 1),
                     "concurrency_bound_rps": round(2 * a.concurrency * 3 / gen_s, 1),
                     "measured_rps": r["throughput"]["requests_per_second"],
                     "gateway_cores": round((g1 - g0) / w, 2) if None not in (g0, g1) else None,
                     "host_cores_busy": round((h1 - h0) / w, 2) if None not in (h0, h1) else None,
                     "p95_s": r["latency"]["p95_s"], "failures": r["failures"]})
        print(json.dumps(rows[-1]), flush=True)
    return rows


def report(res: dict, a) -> str:
    md = [f"# Gateway + worker scaling (dry-run workers, {os.cpu_count()}-CPU host)", "",
          "Generated by `benchmarks/bench_scaling.py`; dry-run workers declare their capacity "
          f"({a.capacity} concurrent generations x {a.latency_ms:.0f} ms + 2 ms/token, max_tokens={a.max_tokens}), "
          "so ideal throughput is arithmetic. Unique prompts: no cache hit or dedup stands in for work.", ""]
    if "workers" in res:
        md += ["## Worker sweep", "", "| workers | req/s (median) | runs | ideal | efficiency vs ideal | speedup | "
               "p50 s | p99 s | failures |", "|---|---|---|---|---|---|---|---|---|"]
        for r in res["workers"]:
            md.append(f"| {r['workers']} | {r['rps_median']} | {r['runs']} | {r['ideal_rps']} | "
                      f"{r['efficiency_vs_ideal']} | {r['speedup_vs_1']}x | {r['p50_s']} | {r['p99_s']} | "
                      f"{r['failures']} |")
        md.append("")
    if "admission" in res:
        md += ["## Admission window as a ceiling", "", "| max_batch_size | workers | binding | predicted req/s | "
               "measured req/s | p95 s | failures | |", "|---|---|---|---|---|---|---|---|"]
        for r in res["admission"]:
            md.append(f"| {r['admission']} | {r['workers']} | {r['binding']} | {r['predicted_rps']} | "
                      f"{r['measured_rps']} | {r['p95_s']} | {r['failures']} | "
                      f"{'**shipped default**' if r['is_shipped_default'] else ''} |")
        md.append("")
    if "saturation" in res:
        s = res["saturation"]
        md += [f"## Saturation: {s['workers']} workers ({s['pool_capacity_rps']} req/s of pool capacity)", "",
               "| client procs | offered conc | total req/s | window s | start skew s | gateway cores | "
               "host cores busy | p95 s | failures |", "|---|---|---|---|---|---|---|---|---|"]
        for r in s["rows"]:
            md.append(f"| {r['client_processes']} | {r['offered_concurrency']} | {r['total_rps']} | {r['window_s']} | "
                      f"{r['start_skew_s']} | {r['gateway_cores']} | {r['host_cores_busy']} / "
                      f"{r['host_cores_total']} | {r['p95_s']} | {r['failures']} |")
        md.append("")
    if "source" in res:
        md += ["## Ceiling source: vary generation cost", "", "| latency ms | pool capacity req/s | "
               "offered-concurrency bound req/s | measured req/s | gateway cores | host cores busy | p95 s | "
               "failures |", "|---|---|---|---|---|---|---|---|"]
        for r in res["source"]:
            md.append(f"| {r['latency_ms']} | {r['pool_capacity_rps']} | {r['concurrency_bound_rps']} | "
                      f"{r['measured_rps']} | {r['gateway_cores']} | {r['host_cores_busy']} | {r['p95_s']} | "
                      f"{r['failures']} |")
        rs = res["source"]
        top = max(r["measured_rps"] for r in rs)
        spread = (max(r["measured_rps"] for r in rs) - min(r["measured_rps"] for r in rs)) / top
        md += ["", f"Reading: the measured ceiling stays within {100 * spread:.0f}% across a 4x change in generation "
               f"cost (peak {top:.0f} req/s) while the pool and the offered concurrency allow far more, so it is "
               "not concurrency-bound (no thread pool in the path: `RemoteBackend` awaits an aiohttp pool on the "
               "event loop). The gateway process sits near one core "
               f"({max(r['gateway_cores'] or 0 for r in rs)} cores at most): the remaining ceiling is the "
               "single event loop's CPU per request. The reference's ceiling on its 16-CPU host was ~183 req/s, "
               "bound by a 20-thread executor (reference benchmarks/results/scaling.md:123-181); scaling past one "
               "event loop is a gateway-replica question (k8s/, several gateway pods behind a Service)."]
        md.append("")
    return "\n".join(md) + "\n"


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--experiments", nargs="+", default=["workers"],
                    choices=["workers", "admission", "saturation", "source"])
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--requests", type=int, default=480)
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--max-tokens", type=int, default=1)
    ap.add_argument("--latency-ms", type=float, default=100.0)
    ap.add_argument("--capacity", type=int, default=4, help="concurrent generations per dry-run worker")
    ap.add_argument("--admission", type=int, default=64, help="gateway max_batch_size (admission window)")
    ap.add_argument("--ceiling-workers", type=int, default=4)
    ap.add_argument("--saturation-workers", type=int, default=8)
    ap.add_argument("--source-latencies", type=float, nargs="+", default=[100.0, 50.0, 25.0])
    ap.add_argument("--routing", default="least_inflight", choices=["round_robin", "least_inflight"])
    ap.add_argument("--engine", default="dry-run", choices=["dry-run", "native"])
    ap.add_argument("--client-procs", type=int, default=1)
    ap.add_argument("--gateway-port", type=int, default=8110)
    ap.add_argument("--worker-port", type=int, default=8111)
    ap.add_argument("--boot-timeout", type=float, default=300.0)
    ap.add_argument("--out", default=str(ROOT / "benchmarks" / "results" / "scaling"))
    a = ap.parse_args()
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    logdir = out.parent / "logs"
    logdir.mkdir(exist_ok=True)
    res = {"config": vars(a)}
    runners = {"workers": exp_workers, "admission": exp_admission, "saturation": exp_saturation,
               "source": exp_source}
    for e in a.experiments:
        res[e] = runners[e](a, logdir)
    out.with_suffix(".json").write_text(json.dumps(res, indent=2))
    md = report(res, a)
    out.with_suffix(".md").write_text(md)
    print(md)


if __name__ == "__main__":
    main()
