"""``POST /v1/benchmark`` against an in-process V-Gate server on the MI355X (BASELINE config 4:
Llama-3 70B, ``/v1/benchmark`` rounds=5; also usable for any model / TP=1).

The server runs the native engine with random-init weights of the named architecture; the
endpoint pushes every configured prompt through the full batcher path per round and reports
latency / TTFT / TPOT / throughput (the reference's response shape, main.py:593-688).

    python benchmarks/bench_endpoint.py --model meta-llama/Meta-Llama-3-70B --rounds 5
    # BASELINE config 4: Llama-3-70B TP=8 over xGMI (RCCL + the custom all-reduce), one command:
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        benchmarks/bench_endpoint.py --model meta-llama/Meta-Llama-3-70B --rounds 5 --tp 8
"""
from __future__ import annotations

import argparse
import asyncio
import contextlib
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("VGATE_LOGGING__LEVEL", "WARNING")


def model_cfg(a, local: int) -> dict:
    import torch
    return {"model_id": a.model, "quantization": a.quantization, "engine_type": "native", "random_init": True,
            "max_model_len": 2048, "max_num_seqs": 64, "max_num_batched_tokens": 2048,
            "num_kv_blocks": a.kv_blocks, "device": f"cuda:{local}" if torch.cuda.device_count() > 0 else "cpu",
            "seed": 7, "tensor_parallel_size": a.tp}


async def main_async(a):
    import httpx
    import torch
    import uvicorn

    from vgate.api.app import create_app
    from vgate.config import VGateConfig

    cfg = VGateConfig(
        role="gateway",
        model=model_cfg(a, int(os.environ.get("LOCAL_RANK", "0"))),
        batch={"max_batch_size": a.concurrency},
        cache={"enabled": False},
        logging={"level": "WARNING", "json_format": True},
    )
    t0 = time.perf_counter()
    app = create_app(cfg)
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=a.port, log_level="warning",
                                           access_log=False, lifespan="on"))
    server.capture_signals = contextlib.nullcontext
    task = asyncio.create_task(server.serve())
    while not server.started:
        if task.done():
            task.result()
            raise RuntimeError("server exited during startup")
        await asyncio.sleep(0.2)
    boot = time.perf_counter() - t0
    prompts = [f"Benchmark prompt {i}: describe the memory hierarchy of an accelerator in detail." for i in
               range(a.prompts)]
    async with httpx.AsyncClient(timeout=3600) as c:
        # warm-up round (captures the decode graphs this load uses)
        await c.post(f"http://127.0.0.1:{a.port}/v1/benchmark",
                     json={"prompts": prompts, "max_tokens": a.max_tokens, "rounds": 1})
        r = await c.post(f"http://127.0.0.1:{a.port}/v1/benchmark",
                         json={"prompts": prompts, "max_tokens": a.max_tokens, "rounds": a.rounds})
        body = r.json()
    stats = app.state.vgate.engine.backend.stats() if hasattr(app.state.vgate.engine.backend, "stats") else {}
    server.should_exit = True
    await task
    out = {"model": a.model.split("/")[-1], "quantization": a.quantization or "none", "tp": a.tp,
           "status": r.status_code, "boot_s": round(boot, 1), "benchmark": body,
           "engine": {k: stats.get(k) for k in ("avg_step_ms", "avg_gpu_ms", "kv_usage", "steps")}}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Meta-Llama-3-70B")
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--prompts", type=int, default=8)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--kv-blocks", type=int, default=4096)
    ap.add_argument("--port", type=int, default=18300)
    ap.add_argument("--tp", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="tensor-parallel degree (= the torchrun world: rank 0 serves, the others follow)")
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    if a.tp > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if torch.cuda.device_count() > 0 else "gloo")
        if rank % a.tp:
            from vgate.backends.native import engine_config_from
            from vgate.config import ModelConfig
            from vgate.runtime.engine import LLMEngine
            LLMEngine(engine_config_from(ModelConfig(**model_cfg(a, int(os.environ.get("LOCAL_RANK", "0")))))) \
                .follower_loop()
            dist.destroy_process_group()
            return
    asyncio.run(main_async(a))
    if a.tp > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
