"""GPU micro-benchmarks (run on the MI355X box):

  1. per-kernel floor: N trivial launches captured in one hipGraph, replayed;
  2. decode GEMM sweep: every Qwen2.5-1.5B projection at M=8 over (waves, split-K),
     each timed as 20 launches inside a hipGraph (no host overhead), reporting
     us/launch and effective weight bandwidth. The launches cycle through enough
     weight copies (> 512 MB) that every launch streams its weights from HBM, as in
     the real forward (the 256 MB MALL would otherwise serve a repeated matrix);
  3. decode attention (unified kernel) and the sampler at the bench shape.

    python benchmarks/micro_gpu.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def graph_time(fn, reps=20, iters=30):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / (iters * reps))
    return best  # us per launch


def floor():
    x = torch.randn(1, 128, device="cuda").bfloat16()
    w = torch.ones(128, device="cuda").bfloat16()
    y = torch.empty_like(x)
    C = ops.native()
    return {"trivial_kernel_us": round(graph_time(lambda: C.rmsnorm(x, None, w, y, 1e-6), reps=100), 3)}


SHAPES = [  # name, N, K, layout, out_f32
    ("qkv", 2048, 1536, "plain", False),
    ("o_proj", 1536, 1536, "plain", False),
    ("gate_up", 17920, 1536, "silu", False),
    ("down", 1536, 8960, "plain", False),
    ("lm_head", 151936, 1536, "plain", True),
]


def sweep(M=8, quick=False):
    out = []
    for name, N, K, layout, f32 in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        ncopy = max(1, math.ceil(512e6 / (N * K * 2)))
        lins = [ops.Linear(w, layout=layout) for _ in range(ncopy)]
        lin = lins[0]
        cyc = {"i": 0}

        def nxt():
            cyc["i"] = (cyc["i"] + 1) % ncopy
            return lins[cyc["i"]]
        res = torch.randn(M, N, device="cuda").bfloat16() if name in ("o_proj", "down") else None
        y = torch.empty(M, lin.out_features, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
        nbytes = N * K * 2
        rows = []
        waves = [1, 2, 4, 8, 16] if not quick else [4, 8]
        splits = [1, 2, 4, 8] if name not in ("gate_up", "lm_head") else [1, 2]
        for wv in waves:
            for sk in splits:
                try:
                    t = graph_time(lambda: ops.linear(x, nxt(), out=y, residual=res, out_f32=f32, waves=wv, splitk=sk))
                except Exception as e:  # noqa: BLE001
                    rows.append({"waves": wv, "splitk": sk, "error": str(e)[:80]})
                    continue
                rows.append({"waves": wv, "splitk": sk, "us": round(t, 2), "TBps": round(nbytes / t / 1e6, 2)})
        auto = graph_time(lambda: ops.linear(x, nxt(), out=y, residual=res, out_f32=f32))
        best = min((r for r in rows if "us" in r), key=lambda r: r["us"])
        out.append({"shape": name, "N": N, "K": K, "M": M, "auto_us": round(auto, 2),
                    "auto_TBps": round(nbytes / auto / 1e6, 2), "best": best, "all": rows})
        print(json.dumps(out[-1]), flush=True)
    return out


def attention_bench(S=8, ctx=64, Hq=12, Hkv=2, D=128, part=2048, max_len=4096):
    """Decode attention (S sequences, 1 query token each) through the unified kernel."""
    bs, nblk = 16, 4096
    kc = torch.randn(nblk, Hkv, bs, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, bs, D, device="cuda").bfloat16()
    mb = (ctx + bs - 1) // bs
    bt = torch.randperm(nblk, device="cuda")[: S * mb].view(S, mb).int().contiguous()
    cl = torch.full((S,), ctx, dtype=torch.int32, device="cuda")
    qs = torch.arange(S + 1, dtype=torch.int32, device="cuda")
    q = torch.randn(S, Hq * D, device="cuda").bfloat16()
    out = torch.empty(S, Hq * D, device="cuda").bfloat16()
    ts = torch.full((S,), -1, dtype=torch.int32, device="cuda")
    tq = torch.zeros(S, dtype=torch.int32, device="cuda")
    P = (max_len + part - 1) // part
    po = torch.empty(S, Hq, P, D, device="cuda")
    pml = torch.empty(S, Hq, P, 2, device="cuda")
    bt = torch.cat([bt, torch.zeros(S, max_len // bs - mb, dtype=torch.int32, device="cuda")], 1).contiguous()
    t = graph_time(lambda: ops.attention(q, Hq * D, kc, vc, bt, cl, qs, ts, tq, out, po, pml, Hq, Hkv, part,
                                         1 / math.sqrt(D)))
    return {"attention_decode": {"S": S, "ctx": ctx, "part": part, "Hq": Hq, "Hkv": Hkv, "us": round(t, 2)}}


def sampler_sweep(V=151936):
    out = {}
    for B in (1, 8, 32, 256):
        logits = torch.randn(B, V, device="cuda") * 2
        z = torch.zeros(B, device="cuda")
        t = torch.full((B,), 0.7, device="cuda")
        p = torch.full((B,), 0.9, device="cuda")
        k = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        sd = torch.arange(B, dtype=torch.int64, device="cuda")
        of = torch.zeros(B, dtype=torch.int64, device="cuda")
        o = torch.empty(B, dtype=torch.int32, device="cuda")
        out[f"B{B}_greedy"] = round(graph_time(lambda: ops.sample(logits, z, p, k, sd, of, out=o)), 2)
        out[f"B{B}_top_p"] = round(graph_time(lambda: ops.sample(logits, t, p, k, sd, of, out=o)), 2)
    return {"sampler_sweep_us": out}


def sampler_bench(B=8, V=151936):
    logits = torch.randn(B, V, device="cuda") * 2
    temp = torch.full((B,), 0.7, device="cuda")
    topp = torch.full((B,), 0.9, device="cuda")
    topk = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    seeds = torch.arange(B, dtype=torch.int64, device="cuda")
    offs = torch.zeros(B, dtype=torch.int64, device="cuda")
    out = torch.empty(B, dtype=torch.int32, device="cuda")
    res = {}
    for name, tp in (("top_p0.9", topp), ("plain", torch.ones_like(topp))):
        t = graph_time(lambda: ops.sample(logits, temp, tp, topk, seeds, offs, out=out))
        res[name] = round(t, 2)
    t = graph_time(lambda: ops.sample(logits, torch.zeros_like(temp), topp, topk, seeds, offs, out=out))
    res["greedy"] = round(t, 2)
    return {"sampler_us": res, "B": B, "V": V}


def prefill_sweep():
    """M > 16: N-split tile kernel (forced, waves=-1) vs the K-split decode kernel family
    (forced with waves=4), weights cycled through > 512 MB as in sweep()."""
    for name, N, K, layout, f32 in SHAPES[:4]:
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        ncopy = max(1, math.ceil(512e6 / (N * K * 2)))
        lins = [ops.Linear(w, layout=layout) for _ in range(ncopy)]
        cyc = {"i": 0}

        def nxt():
            cyc["i"] = (cyc["i"] + 1) % ncopy
            return lins[cyc["i"]]
        row = {"shape": name}
        for M in (24, 64, 192, 384, 1024):
            x = torch.randn(M, K, device="cuda").bfloat16()
            y = torch.empty(M, lins[0].out_features, device="cuda", dtype=torch.bfloat16)
            t_tile = graph_time(lambda: ops.linear(x, nxt(), out=y, waves=-1), reps=10, iters=10)
            t_old = graph_time(lambda: ops.linear(x, nxt(), out=y, waves=4), reps=10, iters=10)
            row[f"M{M}"] = {"tile_us": round(t_tile, 1), "ksplit_us": round(t_old, 1)}
        print(json.dumps(row), flush=True)


def engine_sweep(M=8, quick=False):
    """The decode GEMMs exactly as the engine issues them for Qwen2.5-1.5B (folded norm +
    QKV epilogue on qkv, residual on o/down, folded norm + SiLU on gate_up, folded norm +
    f32 on the LM head), swept over (waves, splitk); weights cycled through > 512 MB."""
    from vgate.ops import reference as ref
    H, I, hq, hkv, D, V = 1536, 8960, 12, 2, 128, 151936
    eps = 1e-6
    g = (torch.rand(H, device="cuda") + 0.5).bfloat16()
    pos = torch.arange(M, dtype=torch.int32, device="cuda") + 40
    slots = torch.arange(M, dtype=torch.int32, device="cuda") * 16 + 5
    cs = ref.rope_cos_sin(4096, D, 1e6, device="cuda")
    kc = torch.zeros(256, hkv, 16, D, device="cuda").bfloat16()
    vc = torch.zeros_like(kc)
    shapes = [("qkv", (hq + 2 * hkv) * D, H, "qkv"), ("o_proj", H, hq * D, "plain"),
              ("gate_up", 2 * I, H, "silu"), ("down", H, I, "plain"), ("lm_head", V, H, "plain")]
    for name, N, K, layout in shapes:
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
        b = (torch.randn(N, device="cuda") * 0.1).bfloat16() if name == "qkv" else None
        ncopy = max(1, math.ceil(512e6 / (N * K * 2)))
        lins = []
        for _ in range(ncopy):
            lin = ops.Linear(w, bias=b, layout=layout)
            if name in ("qkv", "gate_up", "lm_head"):
                lin.fold_norm(g)
            lins.append(lin)
        cyc = {"i": 0}

        def nxt():
            cyc["i"] = (cyc["i"] + 1) % ncopy
            return lins[cyc["i"]]
        x = torch.randn(M, K, device="cuda").bfloat16()
        f32 = name == "lm_head"
        y = torch.empty(M, lins[0].out_features if name != "qkv" else hq * D, device="cuda",
                        dtype=torch.float32 if f32 else torch.bfloat16)
        res = torch.randn(M, N, device="cuda").bfloat16() if name in ("o_proj", "down") else None
        kw = dict(out=y, residual=res, out_f32=f32)
        if name in ("qkv", "gate_up", "lm_head"):
            kw["norm"] = (g, eps)
        if name == "qkv":
            kw["qkv"] = dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kc, v_cache=vc, hq=hq, hkv=hkv)
        rows = []
        waves = [2, 4, 8] if quick else [1, 2, 4, 8, 16]
        splits = [1, 2] if name in ("gate_up", "lm_head") else [1, 2, 3, 4, 6, 8]
        for wv in waves:
            for sk in splits:
                t = graph_time(lambda: ops.linear(x, nxt(), waves=wv, splitk=sk, **kw))
                rows.append({"waves": wv, "splitk": sk, "us": round(t, 2), "TBps": round(N * K * 2 / t / 1e6, 2)})
        auto = graph_time(lambda: ops.linear(x, nxt(), **kw))
        best = min(rows, key=lambda r: r["us"])
        print(json.dumps({"shape": name, "M": M, "auto_us": round(auto, 2), "auto_TBps": round(N * K * 2 / auto / 1e6, 2),
                          "best": best, "all": rows}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--M", type=int, default=8)
    ap.add_argument("--only", default=None, choices=[None, "attn", "sampler", "gemm", "prefill", "engine"])
    a = ap.parse_args()
    print(json.dumps(floor()), flush=True)
    if a.only == "prefill":
        prefill_sweep()
        return
    if a.only == "engine":
        engine_sweep(a.M, a.quick)
        return
    if a.only == "gemm":
        sweep(a.M, a.quick)
        return
    for ctx in (64, 256, 512, 1024, 2048, 4096):
        for part in (64, 128, 256, 512):
            r = attention_bench(ctx=ctx, part=part)
            kv = 8 * 2 * ctx * 128 * 2 * 2  # S x Hkv x ctx x D x (K, V) x bf16
            r["attention_decode"]["TBps"] = round(kv / r["attention_decode"]["us"] / 1e6, 2)
            print(json.dumps(r), flush=True)
    if a.only == "attn":
        return
    print(json.dumps(sampler_bench()), flush=True)
    print(json.dumps(sampler_sweep()), flush=True)
    sweep(a.M, a.quick)


if __name__ == "__main__":
    main()
