"""Medium-M GEMM paths (the mixed prefill + decode steps of a serving load, 16 < M < 128) on MI355X.

For every projection shape of a model and every M bucket, times the engine's default path at that
M (csrc/kernels/gemm_decode.h launch_m: the K-split decode kernels / the LDS tile kernel) against
every prefill-kernel decomposition (gemm_prefill.hip, ops.PREFILL_CANDIDATES), all on the layer's
real epilogue-free product, back-to-back launches timed with events. Prints one JSON line per
(shape, M) with the default time, the best candidate and its time.

    python benchmarks/medium_m_bench.py [--model Qwen/Qwen2.5-1.5B-Instruct] [--ms 24,32,48,64,96]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402
from vgate.models.config import resolve_arch  # noqa: E402


def shapes(arch):
    H, I, D = arch.hidden_size, arch.intermediate_size, arch.head_dim
    q = arch.num_heads * D
    kv = arch.num_kv_heads * D
    return {"qkv": (q + 2 * kv, H), "o": (H, q), "gate_up": (2 * I, H), "down": (H, I)}


def timed_hot(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return 1e3 * s.elapsed_time(e) / iters


_COLD = None


def timed(fn, iters):
    """Per-launch time with the Infinity Cache flushed before each launch (cold weights, as inside a
    decode step); --hot: back-to-back launches instead."""
    if HOT:
        return timed_hot(fn, iters)
    fn()
    return 1e3 * _COLD(fn, iters)


HOT = False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--ms", default="24,32,48,64,96")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--hot", action="store_true", help="back-to-back launches (weights resident in the MALL)")
    a = ap.parse_args()
    global HOT, _COLD
    HOT = a.hot
    arch = resolve_arch(a.model)
    dev = torch.device("cuda:0")
    C = ops.native()
    _COLD = ops._cold_timer(dev)
    ws = ops.workspace(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for name, (N, K) in shapes(arch).items():
        wp = ops.pack_weight((torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16())
        for M in (int(m) for m in a.ms.split(",")):
            x = torch.rand(M, K, device=dev, generator=g).bfloat16()
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            base = timed(lambda: C.gemm(x, wp, N, K, out, 0, ws=ws), a.iters)
            times = {}
            for bn, sk in ops.PREFILL_CANDIDATES + ops.MID_CANDIDATES:
                try:
                    times[(bn, sk)] = timed(lambda: C.gemm(x, wp, N, K, out, 0, ws=ws, **ops._plan_kw((bn, sk), M)),
                                            a.iters)
                except RuntimeError:
                    continue
            best = min(times, key=times.get)
            print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "default_us": round(base, 2),
                              "best": best, "best_us": round(times[best], 2),
                              "speedup": round(base / times[best], 2),
                              "all": {f"{k[0]}/{k[1]}": round(v, 1) for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
