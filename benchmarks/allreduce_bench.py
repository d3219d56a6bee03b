"""Latency of the custom all-reduce kernels (csrc/kernels/allreduce.hip) per message size, world
size and blocks per call, with every rank a process on ONE MI355X (IPC-mapped buffers of the same
device: the same mapping and protocol a node's 8 GPUs use over xGMI, but the "peer" reads are
local HBM, so this measures the kernels' synchronisation + copy cost, not xGMI bandwidth).

For each world size (2, 4, 8) and VGATE_AR_BLOCKS value, W processes form a gloo group, create
the CustomAllReduce, and time ``--iters`` back-to-back calls per (size, one-shot / two-shot) with
CUDA events after a barrier; the slowest rank's mean per call is reported (one JSON line each).

    python benchmarks/allreduce_bench.py [--worlds 2,4,8] [--blocks 16,32,64,128]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import traceback
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SIZES = [64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, blocks, iters, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VGATE_AR_BLOCKS=str(blocks))
        import torch
        import torch.distributed as dist

        from vgate.parallel.custom_allreduce import CustomAllReduce

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        ar = CustomAllReduce(dist.group.WORLD, rank, world, dev, max_bytes=8 << 20)
        rows = []
        for nbytes in SIZES:
            t = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=dev)
            for mode, two in (("one_shot", -1), ("two_shot", 1)):
                for _ in range(5):
                    ar.all_reduce(t, two_shot=two)
                torch.cuda.synchronize()
                dist.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    ar.all_reduce(t, two_shot=two)
                e1.record()
                e1.synchronize()
                us = 1e3 * e0.elapsed_time(e1) / iters
                rows.append((nbytes, mode, us))
        ar.check()
        out = [None] * world
        dist.all_gather_object(out, rows)
        if rank == 0:
            q.put(("ok", out))
        ar.close()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put(("err", traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--blocks", default="16,32,64,128")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    for world in [int(w) for w in a.worlds.split(",")]:
        for blocks in [int(b) for b in a.blocks.split(",")]:
            q = ctx.Queue()
            port = _port()
            procs = [ctx.Process(target=_rank, args=(r, world, port, blocks, a.iters, q)) for r in range(world)]
            for p in procs:
                p.start()
            try:
                kind, res = q.get(timeout=300)
            finally:
                for p in procs:
                    p.join(timeout=60)
                    if p.is_alive():
                        p.kill()
            if kind != "ok":
                print(json.dumps({"world": world, "blocks": blocks, "error": res[-2000:]}), flush=True)
                sys.exit(1)
            for i, (nbytes, mode, _) in enumerate(res[0]):
                worst = max(r[i][2] for r in res)
                print(json.dumps({"world": world, "blocks": blocks, "bytes": nbytes, "mode": mode,
                                  "us": round(worst, 2), "GB_per_s": round(nbytes / worst / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
