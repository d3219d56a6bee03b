"""Headline benchmark: req/s + p50/p99 end-to-end latency of ``POST /v1/chat/completions``
(Qwen2.5-1.5B-Instruct architecture, bf16, random-init weights, synthetic unique
prompts) at fixed client concurrency — the reference's published metric
(6.47 req/s, p50 1.19 s, p99 1.53 s at concurrency 8, max_tokens 64).

Every rank is one GPU running a full V-Gate stack (gateway + native engine) as a
DP serving replica behind a real HTTP/1.1 server on 127.0.0.1 (vgate.api.server by
default, ``--server uvicorn`` for uvicorn/h11); a closed-loop
client in the same process keeps ``--concurrency`` requests in flight against it
through the full path (HTTP -> security -> cache/dedup/admission -> engine ->
JSON). One "step" = ``--requests-per-step`` requests (40 = the reference run).
``value`` is the whole-job aggregate (sum over ranks of requests / max wall time).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
    ... bench.py --gpus N --tp T   # N/T replicas, each a T-way tensor-parallel engine (RCCL / xGMI):
                                   # rank 0 of each TP group serves HTTP, the others follow its steps
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import time

os.environ.setdefault("VGATE_LOGGING__LEVEL", "WARNING")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_REQ_S = 6.47
LAST_T_RUN = 0.0  # perf_counter origin of the last run_load's ``starts``
BENCH_KEY = "vgate-bench-key"
METRIC = "req/s + p50/p99 end-to-end latency, {model} /v1/chat/completions at fixed concurrency"

WORDS = ("the quick brown fox jumps over a lazy dog while engineers measure latency throughput memory "
         "bandwidth kernels scheduling batching caching tokens requests gateway worker cluster").split()


def make_prompt(rank: int, i: int) -> str:
    # unique, ~24-word prompts (the reference load test used unique prompts: no cache hits)
    h = (rank * 1_000_003 + i * 7919) & 0xFFFFFFFF
    words = [WORDS[(h >> (k % 24)) % len(WORDS) ^ 0] if k % 3 else WORDS[(h + k * 31) % len(WORDS)] for k in range(22)]
    return f"Request {rank}-{i}: " + " ".join(words) + "?"


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(int(len(xs) * p / 100), len(xs) - 1)] if xs else 0.0


async def run_load(port: int, n: int, concurrency: int, max_tokens: int, rank: int, start_idx: int,
                   model: str = "Qwen/Qwen2.5-1.5B-Instruct", api_key: str | None = None, client: str = "lean"):
    """Closed loop: ``concurrency`` requests in flight, ``n`` in all (reference bench_load.py:160-212).
    ``client`` "lean" = vgate.utils.http1 keep-alive pool (the default: the load generator shares
    this process's event loop with the server, so its own per-request cost would be charged to
    the server), "aiohttp" = the reference's client library."""
    lat, starts, fails, tokens = [], [], 0, 0
    sem = asyncio.Semaphore(concurrency)
    path = "/v1/chat/completions"
    headers = {"Authorization": f"Bearer {api_key}"} if api_key else None

    def body_of(i):
        return {"model": model, "messages": [{"role": "user", "content": make_prompt(rank, start_idx + i)}],
                "max_tokens": max_tokens}

    if client == "aiohttp":
        import aiohttp
        conn = aiohttp.TCPConnector(limit=concurrency * 2)
        session = aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=300), headers=headers)

        async def post(body):
            async with session.post(f"http://127.0.0.1:{port}{path}", json=body) as r:
                return r.status, await r.json()
    else:
        from vgate.utils.http1 import Http1Pool
        session = Http1Pool("127.0.0.1", port, headers=headers)

        async def post(body):
            status, _, data = await session.request("POST", path, json.dumps(body).encode())
            return status, json.loads(data)

    async def one(i):
        nonlocal fails, tokens
        async with sem:
            body = body_of(i)
            t0 = time.perf_counter()
            try:
                status, data = await post(body)
                if status != 200:
                    fails += 1
                else:
                    tokens += data["usage"]["completion_tokens"]
            except Exception:  # noqa: BLE001
                fails += 1
            lat.append(time.perf_counter() - t0)
            starts.append(t0 - t_run)

    global LAST_T_RUN
    try:
        t_run = t0 = LAST_T_RUN = time.perf_counter()
        await asyncio.gather(*(one(i) for i in range(n)))
        wall = time.perf_counter() - t0
    finally:
        await session.close()
    return lat, fails, tokens, wall, starts


def engine_model_cfg(args, rank: int, local: int) -> dict:
    import torch
    return {"model_id": args.model, "quantization": args.quantization, "engine_type": "native",
            "random_init": True, "max_model_len": 2048, "max_num_seqs": 256,
            "max_num_batched_tokens": 2048, "num_kv_blocks": args.kv_blocks, "enforce_eager": args.eager,
            # device_count() does not initialise HIP: with --engine-process the parent must
            # not touch the GPU before it spawns the engine core
            "device": f"cuda:{local}" if torch.cuda.device_count() > 0 else "cpu",
            # every rank of a TP group uses the same seed (one replica); replicas differ
            "seed": 1234 + rank // args.tp, "tensor_parallel_size": args.tp,
            "engine_process": bool(args.engine_process) and args.tp == 1,
            **({"idle_batch_window_ms": args.idle_window_ms} if args.idle_window_ms is not None else {})}


async def serve_and_bench(args, rank: int, world: int, dist_ok: bool, client=None, group=None):
    import torch
    from vgate.api.app import create_app
    from vgate.api.server import make_server
    from vgate.config import VGateConfig

    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = VGateConfig(
        role="gateway",
        model=engine_model_cfg(args, rank, local),
        batch={"max_batch_size": args.concurrency},
        cache={"enabled": True, "maxsize": 1000},
        logging={"level": "WARNING", "json_format": True},
        # --security: bearer auth + the sliding-window rate limiter on the hot path (BASELINE
        # config 5: high-QPS rate limiter on); the key's limit is far above the offered load
        security={"enabled": bool(args.security),
                  "api_keys": [{"key": BENCH_KEY, "name": "bench", "rate_limit": 10_000_000}],
                  "rate_limiting": {"enabled": True, "window_seconds": 60}},
    )
    app = create_app(cfg)
    port = args.port + local
    # the in-process server is stopped by this script, never by a signal: leave the process's
    # handlers alone (a profiler's native SIGINT/SIGTERM handler is not restorable from Python)
    server = make_server(app, "127.0.0.1", port, args.server)
    srv_task = asyncio.create_task(server.serve())
    t_boot = time.perf_counter()
    while not server.started:
        if srv_task.done():
            srv_task.result()
            raise RuntimeError("server exited during startup")
        await asyncio.sleep(0.1)
    boot_s = time.perf_counter() - t_boot

    def barrier():
        if dist_ok:
            import torch.distributed as dist
            dist.barrier(group=group)
        # this rank's GPU explicitly: the bare call syncs the calling thread's current device,
        # which is cuda:0 unless this thread happened to construct the engine
        if not args.engine_process and torch.cuda.is_available():
            torch.cuda.synchronize(local)

    per_step = args.requests_per_step
    key = BENCH_KEY if args.security else None

    async def load(n, start_idx):
        if client is None:  # default: the load loop shares this process's event loop / GIL
            return await run_load(port, n, args.concurrency, args.max_tokens, rank, start_idx, args.model, key,
                                  args.client)
        # the load generator is its own process (as the reference's bench_load.py against a
        # running server): one command line in, one result line out; the server keeps serving
        # on this event loop while the reply is awaited off-loop
        cmd = {"port": port, "n": n, "concurrency": args.concurrency, "max_tokens": args.max_tokens,
               "rank": rank, "start_idx": start_idx, "model": args.model, "api_key": key, "client": args.client}
        client.stdin.write(json.dumps(cmd) + "\n")
        client.stdin.flush()
        line = await asyncio.get_running_loop().run_in_executor(None, client.stdout.readline)
        if not line:
            raise RuntimeError("load client exited")
        r = json.loads(line)
        return r["lat"], r["fails"], r["tokens"], r["wall"], r.get("starts", [])

    # warmup (also captures the hipGraph buckets this load uses)
    if args.warmup > 0:
        await load(per_step * args.warmup, 10_000_000)
    # buckets first seen during warmup ran eagerly; the engine captures them once idle
    backend = app.state.vgate.engine.backend
    stats = getattr(backend, "stats", None)
    t_cap = time.perf_counter()
    await asyncio.sleep(0.3)  # the engine core's stats snapshot is pushed every 0.25 s
    while callable(stats) and stats().get("pending_captures", 0) and time.perf_counter() - t_cap < 120:
        await asyncio.sleep(0.05)
    eng = app.state.vgate.engine
    inner = getattr(eng.backend, "engine", None)
    if hasattr(inner, "reset_peaks"):
        inner.reset_peaks()
    barrier()
    # server event-loop lag during the timed region (a stalled loop delays every response)
    lag = {"max_ms": 0.0, "at_s": 0.0}

    async def lag_monitor(t_ref):
        while True:
            t = time.perf_counter()
            await asyncio.sleep(0.005)
            d = 1e3 * (time.perf_counter() - t - 0.005)
            if d > lag["max_ms"]:
                lag["max_ms"], lag["at_s"] = d, t - t_ref
    import gc
    gcs = {"max_ms": 0.0, "n2": 0, "t": 0.0}

    def gc_cb(phase, info):
        if phase == "start":
            gcs["t"] = time.perf_counter()
        elif info.get("generation") == 2 or time.perf_counter() - gcs["t"] > 0.005:
            gcs["n2"] += info.get("generation") == 2
            gcs["max_ms"] = max(gcs["max_ms"], 1e3 * (time.perf_counter() - gcs["t"]))
    gc.callbacks.append(gc_cb)
    prof = None
    if args.profile_loop:  # the serving event loop's own work in the timed region (this thread only)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    snap0 = eng.backend.stats() if hasattr(eng.backend, "stats") else {}
    rcache = getattr(getattr(app.state.vgate, "batcher", None), "cache", None)
    rc0 = rcache.hits if rcache is not None else None
    t0 = time.perf_counter()
    mon = asyncio.create_task(lag_monitor(t0))
    lat, fails, tokens, _, starts = await load(per_step * args.steps, 0)
    mon.cancel()
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(40)
    gc.callbacks.remove(gc_cb)
    barrier()
    wall = time.perf_counter() - t0
    snap = eng.backend.stats() if hasattr(eng.backend, "stats") else {}
    # timed-region forensics (p99): eager (graph-miss) steps and captures INSIDE the timed region
    snap = dict(snap)
    if rc0 is not None:  # gateway result-cache hits in the timed region (unique prompts: 0)
        snap["timed_result_cache_hits"] = rcache.hits - rc0
    for k in ("graph_misses_eager", "graph_captures", "steps", "graph_hits", "idle_ms", "prefill_steps", "waves",
              "wave_requests", "coalesce_ms", "busy_ms", "collect_wait_ms", "sum_step_ms", "sum_cycle_ms",
              "sum_gpu_ms", "gpu_steps", "prefix_cache_hits"):
        if k in snap and k in snap0:
            snap[f"timed_{k}"] = snap[k] - snap0[k]
    # per-step averages over the timed region only (the snapshot's avg_* are since boot, warm-up
    # and captures included): the engine's busy time per step, the device time of the timed steps
    ts = snap.get("timed_steps") or 0
    if ts and "timed_busy_ms" in snap:
        snap["timed_avg_step_ms"] = round(snap["timed_busy_ms"] / ts, 3)
        snap["timed_avg_cycle_ms"] = round(snap["timed_sum_cycle_ms"] / ts, 3)
        snap["timed_avg_gpu_ms"] = round(snap["timed_sum_gpu_ms"] / max(1, snap["timed_gpu_steps"]), 3)
    if "wave_sum_ms" in snap and "wave_sum_ms" in snap0:
        nw = max(1, snap.get("timed_waves", 0))
        snap["wave_breakdown_ms"] = [round((a - b) / nw, 3) for a, b in zip(snap["wave_sum_ms"], snap0["wave_sum_ms"])]
    # wave-boundary trace (in-process engine, lean client: one clock): per timed wave, last finish
    # in the engine -> idle start, -> first response received by the client, -> the client's first
    # new request sent, -> that request reaching the engine, -> the last of the wave arriving
    trace = None
    wl = list(getattr(inner, "wave_log", []))
    if wl and starts and client is None:
        t_run_abs = LAST_T_RUN
        sends = sorted(t_run_abs + s for s in starts)
        recvs = sorted(t_run_abs + s + la for s, la in zip(starts, lat))
        import bisect as _bs
        parts = {k: [] for k in ("finish_to_idle", "finish_to_first_recv", "first_recv_to_first_send",
                                 "first_send_to_first_arrival", "first_to_last_arrival")}
        for fin, idle0, a0, a1, _ in wl:
            if fin < t0:
                continue
            i = _bs.bisect_left(recvs, fin)
            j = _bs.bisect_left(sends, fin)
            if i >= len(recvs) or j >= len(sends):
                continue
            parts["finish_to_idle"].append(idle0 - fin)
            parts["finish_to_first_recv"].append(recvs[i] - fin)
            parts["first_recv_to_first_send"].append(sends[j] - recvs[i])
            parts["first_send_to_first_arrival"].append(a0 - sends[j])
            parts["first_to_last_arrival"].append(a1 - a0)
        trace = {k: round(1e3 * sorted(v)[len(v) // 2], 3) for k, v in parts.items() if v}
        # per-wave medians of the engine's own boundary phases (the cumulative means of the snapshot
        # carry the first timed wave's idle, which started before the timed region: ~3 ms per wave
        # of bias over 100 waves)
        tw = [w for w in wl if w[2] >= t0]
        if tw:
            med = lambda xs: round(1e3 * sorted(xs)[len(xs) // 2], 3)  # noqa: E731
            trace["wave_breakdown_median_ms"] = [med([a0 - i0 for _, i0, a0, _, _ in tw]),
                                                 med([a1 - a0 for _, _, a0, a1, _ in tw]),
                                                 med([st - a1 for _, _, _, a1, st in tw])]
    server.should_exit = True
    await srv_task
    slow = sorted(zip(lat, starts), reverse=True)[:8]
    return {"lat": lat, "fails": fails, "tokens": tokens, "wall": wall, "boot_s": boot_s,
            "slowest": [[round(st, 3), round(la, 4)] for la, st in slow],
            "loop_lag_max_ms": round(lag["max_ms"], 2), "loop_lag_at_s": round(lag["at_s"], 3),
            "gc_gen2_collections": gcs["n2"], "gc_max_pause_ms": round(gcs["max_ms"], 2),
            "n": per_step * args.steps, "engine": snap, "wave_trace_ms": trace}


def run_follower(args, rank: int) -> None:
    """A TP follower rank: the same engine config as its group's serving rank, then the step loop."""
    from vgate.backends.native import engine_config_from
    from vgate.config import ModelConfig
    from vgate.runtime.engine import LLMEngine

    local = int(os.environ.get("LOCAL_RANK", "0"))
    eng = LLMEngine(engine_config_from(ModelConfig(**engine_model_cfg(args, rank, local))))
    eng.follower_loop()


def client_loop():
    """--client-proc: one JSON load command per stdin line -> one JSON result per stdout line."""
    for line in sys.stdin:
        c = json.loads(line)
        lat, fails, tokens, wall, starts = asyncio.run(run_load(c["port"], c["n"], c["concurrency"], c["max_tokens"],
                                                        c["rank"], c["start_idx"], c["model"], c["api_key"],
                                                        c.get("client", "lean")))
        sys.stdout.write(json.dumps({"lat": lat, "fails": fails, "tokens": tokens, "wall": wall, "starts": starts}) + "\n")
        sys.stdout.flush()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree of each replica (divides the world)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--requests-per-step", type=int, default=40)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--kv-blocks", type=int, default=4096)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--idle-window-ms", type=float, default=None,
                    help="model.idle_batch_window_ms (0 = no idle admission window; default: config.yaml's)")
    ap.add_argument("--port", type=int, default=18100)
    ap.add_argument("--security", action="store_true", help="bearer auth + rate limiter on the request path")
    ap.add_argument("--engine-process", action="store_true",
                    help="run the engine core in its own process (model.engine_process)")
    ap.add_argument("--client-process", action="store_true",
                    help="run the load loop in a separate client process (default: in the server process; "
                         "measured slower on the 1-GPU box: 68 vs 81 req/s, profiles/r1_bench_client_modes.log)")
    ap.add_argument("--client-proc", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--profile-loop", action="store_true",
                    help="cProfile the serving event loop over the timed region (stats to stderr; slows it)")
    ap.add_argument("--server", default="vgate", choices=["vgate", "uvicorn"],
                    help="HTTP server: vgate.api.server (default) or uvicorn (h11)")
    ap.add_argument("--client", default="lean", choices=["lean", "aiohttp"],
                    help="load-generator HTTP client: vgate.utils.http1 (default) or aiohttp")
    ap.add_argument("--switch-interval-us", type=float,
                    default=float(os.environ.get("VGATE_SWITCH_INTERVAL_US", "0")),
                    help="sys.setswitchinterval for the server process (0 = Python default 5 ms)")
    args = ap.parse_args()
    if args.switch_interval_us > 0:
        sys.setswitchinterval(args.switch_interval_us * 1e-6)
    if args.client_proc:
        client_loop()
        return

    # start the load-client process before anything here touches the GPU
    client = None
    is_follower = args.tp > 1 and int(os.environ.get("RANK", "0")) % args.tp != 0
    if args.client_process and not is_follower:
        client = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--client-proc"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world % args.tp:
        raise SystemExit(f"--tp {args.tp} does not divide the world size {world}")
    dp = world // args.tp
    dist_ok = False
    leaders = None  # process group of the serving ranks (rank 0 of every TP group)
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # single node: gloo over loopback, independent of whether the hostname resolves
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        # DP replicas share no tensors (gloo coordinates them); TP groups run RCCL over xGMI
        backend = "nccl" if args.tp > 1 and torch.cuda.device_count() > 0 else "gloo"
        dist.init_process_group(backend)
        if args.tp > 1:
            leaders = dist.new_group(list(range(0, world, args.tp)), backend="gloo")
        dist_ok = True
    if args.tp > 1 and rank % args.tp:
        # TP follower: join its group's engine and execute rank 0's steps until it shuts down
        run_follower(args, rank)
        res = None
    else:
        try:
            res = asyncio.run(serve_and_bench(args, rank, world, dist_ok, client, group=leaders))
        finally:
            if client is not None:
                client.stdin.close()
                client.wait(timeout=30)
    if dist_ok:
        import torch.distributed as dist
        allr = [None] * world
        dist.barrier()
        dist.all_gather_object(allr, res)
        allr = [r for r in allr if r is not None]
    else:
        allr = [res]
    if rank == 0:
        model_name = args.model.split("/")[-1]
        lat = [x for r in allr for x in r["lat"]]
        total = sum(r["n"] for r in allr)
        wall = max(r["wall"] for r in allr)
        value = total / wall
        toks = sum(r["tokens"] for r in allr)
        out = {
            "metric": METRIC.format(model="Qwen2.5-1.5B" if model_name == "Qwen2.5-1.5B-Instruct" else model_name), "value": round(value, 3), "unit": "req/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * wall / args.steps, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / BASELINE_REQ_S, 3),
            # weight precision of the run: int4 weights with bf16 activations for AWQ
            "dtype": "w4a16" if (args.quantization or "").lower() == "awq" else "bf16",
            "data": f"synthetic unique prompts, random-init weights ({model_name} architecture)",
            "config": {"model": model_name, "quantization": args.quantization or "none",
                       "security_rate_limiter": bool(args.security),
                       "load_client": ("separate process" if args.client_process else "in-process") + f" ({args.client})",
                       "http_server": args.server,
                       "engine_core": "separate process" if args.engine_process else "in-process", "global_batch": args.concurrency * dp,
                       "seq_len": args.max_tokens,
                       "parallelism": f"dp{dp}" if args.tp == 1 else f"dp{dp}xtp{args.tp}",
                       "concurrency_per_gpu": args.concurrency, "max_tokens": args.max_tokens,
                       "requests_per_step_per_gpu": args.requests_per_step},
            "p50_s": round(pct(lat, 50), 4), "p99_s": round(pct(lat, 99), 4),
            "mean_s": round(sum(lat) / max(1, len(lat)), 4),
            "generated_tokens_per_s": round(toks / wall, 1),
            "failures": sum(r["fails"] for r in allr),
            # timed region only: engine busy time per step (schedule + launch + wait + process; with
            # asynchronous scheduling the cycles of consecutive steps overlap, so avg_cycle can exceed
            # it), the mean schedule -> processed cycle, the device time of the timed steps
            "engine_avg_step_ms": allr[0]["engine"].get("timed_avg_step_ms"),
            "engine_avg_cycle_ms": allr[0]["engine"].get("timed_avg_cycle_ms"),
            "engine_avg_gpu_ms": allr[0]["engine"].get("timed_avg_gpu_ms"),
            "boot_s": round(max(r["boot_s"] for r in allr), 1),
            "max_s": round(max(lat), 4) if lat else 0.0,
            "timed_engine_steps": allr[0]["engine"].get("timed_steps"),
            # the engine thread idle (nothing queued, no step in flight) and the steps that carried
            # prompt tokens, over the timed region: at concurrency c the requests run in waves of c
            # that start together, so every wave boundary waits for the next c requests' HTTP path
            "timed_engine_idle_ms": allr[0]["engine"].get("timed_idle_ms"),
            # the engine thread's timed wall time, split: idle (nothing to do) + coalesce (the idle
            # admission window waiting for the rest of a wave) + busy (steps); accounted / wall
            "timed_engine_coalesce_ms": allr[0]["engine"].get("timed_coalesce_ms"),
            "timed_engine_busy_ms": allr[0]["engine"].get("timed_busy_ms"),
            "timed_engine_collect_wait_ms": allr[0]["engine"].get("timed_collect_wait_ms"),
            "timed_wall_ms": round(1e3 * allr[0]["wall"], 3),
            "timed_wall_ms_accounted": (round(sum(allr[0]["engine"].get(k, 0.0) for k in
                                                  ("timed_idle_ms", "timed_coalesce_ms", "timed_busy_ms")), 3)
                                        if "timed_busy_ms" in allr[0]["engine"] else None),
            "timed_prefill_steps": allr[0]["engine"].get("timed_prefill_steps"),
            # reuse in the timed region: KV blocks served by the prefix cache (the chat template's
            # shared head; every prompt is unique) and gateway result-cache hits (must be 0)
            "timed_prefix_cache_hit_blocks": allr[0]["engine"].get("timed_prefix_cache_hits"),
            "timed_result_cache_hits": allr[0]["engine"].get("timed_result_cache_hits"),
            # per idle -> busy transition: [idle start -> first arrival, first -> last arrival of the
            # wave, last arrival -> step start] in ms, and the requests per transition
            "wave_breakdown_ms": ((allr[0].get("wave_trace_ms") or {}).get("wave_breakdown_median_ms")
                                  or allr[0]["engine"].get("wave_breakdown_ms")),
            # medians over the timed waves (rank 0, in-process client): where a wave boundary's idle goes
            "wave_trace_ms": allr[0].get("wave_trace_ms"),
            "timed_waves": allr[0]["engine"].get("timed_waves"),
            "timed_wave_requests": allr[0]["engine"].get("timed_wave_requests"),
            "timed_eager_steps": allr[0]["engine"].get("timed_graph_misses_eager"),
            "timed_graph_captures": allr[0]["engine"].get("timed_graph_captures"),
            "max_gpu_step_ms": allr[0]["engine"].get("max_gpu_step_ms"),
            "max_gpu_step_bucket": allr[0]["engine"].get("max_gpu_step_bucket"),
            "max_cycle_ms": allr[0]["engine"].get("max_cycle_ms"),
            "max_cycle_tokens_seqs": allr[0]["engine"].get("max_cycle_tokens_seqs"),
            # p99 forensics: the slowest requests as [start offset s, latency s] (rank 0) and
            # the serving event loop's worst lag inside the timed region
            "slowest_requests": allr[0].get("slowest"),
            "loop_lag_max_ms": allr[0].get("loop_lag_max_ms"), "loop_lag_at_s": allr[0].get("loop_lag_at_s"),
            "gc_gen2_collections": allr[0].get("gc_gen2_collections"), "gc_max_pause_ms": allr[0].get("gc_max_pause_ms"),
        }
        print(json.dumps(out), flush=True)
    if dist_ok:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
