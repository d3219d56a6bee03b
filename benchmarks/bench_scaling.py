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

    python benchmarks/bench_scaling.py --workers 1 2 4 --repeats 3
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


def run_clients(url: str, args) -> dict:
    if args.client_procs <= 1:
        return asyncio.run(run_load_test(url, args.concurrency, args.requests, DEFAULT_PROMPTS, args.max_tokens,
                                         stream=False, unique=True))
    start_at = time.time() + 2.0
    per = args.requests // args.client_procs
    conc = max(1, args.concurrency // args.client_procs)
    ps = [subprocess.Popen([sys.executable, str(Path(__file__).parent / "_load_client.py"), "--url", url,
                            "--requests", str(per), "--concurrency", str(conc), "--max-tokens",
                            str(args.max_tokens), "--start-at", str(start_at), "--tag", str(k)],
                           stdout=subprocess.PIPE, text=True) for k in range(args.client_procs)]
    outs = [json.loads(p.communicate(timeout=600)[0].strip().splitlines()[-1]) for p in ps]
    t0 = min(o["t_start"] for o in outs)
    t1 = max(o["t_end"] for o in outs)
    lat = sorted(x for o in outs for x in o["latencies"])
    n = sum(o["requests"] for o in outs)
    fails = sum(o["failures"] for o in outs)
    return {"wall_time_s": t1 - t0, "failures": fails,
            "throughput": {"requests_per_second": round(n / (t1 - t0), 2)},
            "latency": {"p50_s": lat[min(len(lat) // 2, len(lat) - 1)] if lat else 0,
                        "p99_s": lat[min(int(len(lat) * 0.99), len(lat) - 1)] if lat else 0}}


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--requests", type=int, default=480)
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--max-tokens", type=int, default=1)
    ap.add_argument("--latency-ms", type=float, default=100.0)
    ap.add_argument("--capacity", type=int, default=4, help="concurrent generations per dry-run worker")
    ap.add_argument("--admission", type=int, default=64, help="gateway max_batch_size (admission window)")
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
    gen_s = (a.latency_ms + 2.0 * a.max_tokens) / 1e3  # DryRunBackend cost model
    rows = []
    for n in a.workers:
        procs = start_topology(n, a, logdir)
        try:
            runs = [run_clients(f"http://127.0.0.1:{a.gateway_port}", a) for _ in range(a.repeats)]
        finally:
            for p in procs:
                p.stop()
        rps = statistics.median(r["throughput"]["requests_per_second"] for r in runs)
        ideal = n * a.capacity / gen_s if a.engine == "dry-run" else None
        rows.append({"workers": n, "rps_median": rps, "runs": [r["throughput"]["requests_per_second"] for r in runs],
                     "p50_s": statistics.median(r["latency"]["p50_s"] for r in runs),
                     "p99_s": statistics.median(r["latency"]["p99_s"] for r in runs),
                     "failures": sum(r["failures"] for r in runs), "ideal_rps": ideal,
                     "efficiency_vs_ideal": round(rps / ideal, 3) if ideal else None})
        print(json.dumps(rows[-1]), flush=True)
    base = rows[0]["rps_median"] / rows[0]["workers"]
    for r in rows:
        r["speedup_vs_1"] = round(r["rps_median"] / (base * 1), 3) if base else None
        r["scaling_efficiency"] = round(r["rps_median"] / (base * r["workers"]), 3) if base else None
    res = {"config": vars(a), "rows": rows}
    out.with_suffix(".json").write_text(json.dumps(res, indent=2))
    md = ["| workers | req/s (median) | speedup | efficiency | ideal req/s | p50 s | p99 s | failures |",
          "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        md.append(f"| {r['workers']} | {r['rps_median']} | {r['speedup_vs_1']}x | {r['scaling_efficiency']} | "
                  f"{r['ideal_rps']} | {r['p50_s']} | {r['p99_s']} | {r['failures']} |")
    out.with_suffix(".md").write_text("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
