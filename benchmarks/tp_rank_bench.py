"""One TP rank's decode step on ONE MI355X: the model sharded exactly as rank ``--rank`` of a
``--tp``-way group (default Llama-3-70B TP=8: qkv 8192 -> 1280, o 1024 -> 8192, gate_up 8192 ->
7168, down 3584 -> 8192, LM head 8192 -> 16032), random-init weights, collectives stubbed
(``TPGroup(simulated=True)``: the all-reduces are no-ops, the logits all-gather replicates the
local shard). Reports

* the per-rank decode step (whole hipGraph replayed, CUDA events) — the compute part of a TP=8
  step; the 2 x 80 + 1 all-reduces and the all-gather add their latencies on a real node
  (``benchmarks/allreduce_bench.py`` gives the kernels' same-GPU latency per size);
* per projection: the in-graph kernel span (launch timeline, benchmarks/timeline.py), its
  weight bytes and the effective TB/s;
* with ``--sweep``: the in-context decode decomposition table (waves, split-K, tiles per block)
  per projection, as benchmarks/decode_sweep.py does for the TP=1 models.

    python benchmarks/tp_rank_bench.py [--model llama-3-70b] [--tp 8] [--batch 8] [--ctx 128] [--sweep]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from vgate.parallel.comm import TPGroup  # noqa: E402
from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402

KINDS = ("qkv", "o", "gate_up", "down")
# (waves, split-K, tiles per block) candidates for the large-K per-rank shapes (0 = heuristic)
# ("kx", waves, slices, tiles code): the register-stationary kernel; ("sk", waves, blocks/CU, group): stream-K
RANK_CANDIDATES = {
    "qkv": [(0, 0, 0), (8, 3, 0), (8, 4, 0), (4, 4, 0), ("kx", 0, 0, 0), ("kx", 0, 2, 0), ("kx", 0, 4, 0),
            ("kx", 8, 3, 0), ("kx", 0, 2, -13), ("sk", 8, 1, 4), ("sk", 4, 1, 8), ("sk", 8, 1, 8)],
    "o": [(0, 0, 0), (2, 1, 1), (4, 1, 1), (8, 1, 1), ("kx", 0, 0, 0), ("kx", 0, 1, 0), ("kx", 0, 1, -13),
          ("sk", 4, 1, 4)],
    "gate_up": [(0, 0, 0), (4, 1, 0), (8, 1, 0), ("kx", 0, 2, 0), ("kx", 8, 2, 0), ("kx", 0, 3, 0),
                ("sk", 4, 1, 8), ("sk", 8, 1, 8)],
    "down": [(0, 0, 0), ("sk", 4, 1, 8), (8, 1, 1), (4, 1, 1), (8, 2, 1), ("kx", 0, 0, 0), ("kx", 0, 2, 0),
             ("kx", 0, 2, -13), ("sk", 8, 1, 8)],
    "lm_head": [(0, 0, 0), (8, 1, 1), (8, 1, 2), (4, 1, 2)],
}


def layer_kinds(live):
    """Assign each launch of a decode step to a projection kind by position: per layer
    qkv GEMM -> attention -> o GEMM -> gate_up GEMM -> down GEMM; the f32 GEMM is the LM head."""
    out = []
    nxt = None
    for x in live:
        n = x["kernel"]
        if n.startswith("gemm_sk_"):  # stream-K launches carry their role in the name
            k = {"gemm_sk_qkv": "qkv", "gemm_sk_gate_up": "gate_up", "gemm_sk_f32": "lm_head"}.get(n)
            if k is None:
                k, nxt = (nxt or "?"), None
            elif k == "qkv":
                nxt = "o"
            elif k == "gate_up":
                nxt = "down"
        elif n.startswith("gemm_qkv"):
            k, nxt = "qkv", "o"
        elif n.startswith("attention") or n.startswith("attn"):
            k = "attention"
        elif n.startswith("gemm_gate_up"):
            k, nxt = "gate_up", "down"
        elif n.startswith("gemm_f32"):
            k = "lm_head"
        elif n.startswith("gemm"):
            k = nxt or "?"
            nxt = None
        else:
            k = n
        out.append(k)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--sweep", action="store_true", help="in-context decode decomposition table per projection")
    ap.add_argument("--kinds", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--fused-ar", action="store_true",
                    help="o_proj / down_proj all-reduce in their epilogue against a one-rank loopback region "
                         "(prices the fused exchange's in-kernel cost; no peers)")
    a = ap.parse_args()
    if a.sweep:  # the sweep's (0, 0, 0) row is the launcher heuristic, not the measured table
        from vgate.models import transformer
        transformer.APPLY_DECODE_PLANS = False
    from decode_sweep import set_plan, time_step
    from timeline import measure

    tp = TPGroup(rank=a.rank, size=a.tp, simulated=True)
    if a.fused_ar:
        from vgate.parallel.custom_allreduce import LoopbackFused

        tp.custom_ar = LoopbackFused(torch.device("cuda:0"))
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda:0", max_model_len=2048, max_num_seqs=64,
                                 max_num_batched_tokens=2048, num_kv_blocks=1024, warmup=False,
                                 tensor_parallel_size=a.tp, prefill_autotune=False), tp=tp)
    eng.runner.defer_capture = False
    eng.async_sched = False
    m = eng.model
    sh = m.shard
    shapes = {"qkv": m.layers[0].qkv, "o": m.layers[0].o, "gate_up": m.layers[0].gate_up, "down": m.layers[0].down,
              "lm_head": m.lm_head}
    print(json.dumps({"model": a.model, "tp": a.tp, "rank": a.rank, "hq": sh.hq, "hkv": sh.hkv,
                      "shapes": {k: [lin.N, lin.K] for k, lin in shapes.items()},
                      "weight_GB_per_rank": round(m.weight_bytes() / 1e9, 2)}), flush=True)
    for i in range(a.batch):
        ids = [100 + (i * 131 + j * 17) % 5000 for j in range(a.ctx)]
        eng.add_request(f"r{i}", prompt_ids=ids,
                        params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=100000, ignore_eos=True))
    eng._drain_inbox()
    for _ in range(3):
        eng.step()
    base = time_step(eng, a.iters)
    print(json.dumps({"per_rank_step_us": round(base, 1), "batch": a.batch, "ctx": a.ctx,
                      "note": ("o / down all-reduce fused in the epilogue against a loopback region (no peers); "
                               "embedding all-reduce and logits all-gather stubbed") if a.fused_ar
                      else "compute only; collectives stubbed"}), flush=True)
    summary, live, _, _ = measure(eng)
    kinds = layer_kinds(live)
    agg = {}
    for x, k in zip(live, kinds):
        g = agg.setdefault(k, [0, 0.0, 0.0])
        g[0] += 1
        g[1] += x["span_us"]
        g[2] += x["gap_after_us"]
    rows = {}
    for k, (n, span, gap) in agg.items():
        r = {"n": n, "avg_span_us": round(span / n, 2), "avg_gap_after_us": round(gap / n, 2)}
        if k in shapes:
            nb = shapes[k].nbytes()
            r["weight_MB"] = round(nb / 1e6, 2)
            r["TB_per_s"] = round(nb / (span / n) / 1e6, 2)
        rows[k] = r
    # on a real TP node each step adds its collectives as launches: the embedding all-reduce and the
    # logits all-gather, plus one all-reduce per row-parallel GEMM unless it runs in the GEMM's epilogue
    # (decode rows, model.tp_fused_allreduce: gemm_epilogue.h epilogue_ar)
    nl = len(m.layers)
    print(json.dumps({"timeline_step_us": summary["step_us"], "launches": summary["launches"],
                      "collective_launches_per_real_step": {"fused_all_reduce": 2, "separate_all_reduce": 2 + 2 * nl},
                      "sum_gap_us": summary["sum_gap_us"], "per_kind": rows}), flush=True)
    if not a.sweep:
        return
    best = {}
    for kind in a.kinds.split(","):
        res = []
        for cfg in RANK_CANDIDATES[kind]:
            set_plan(eng.model, kind, cfg)
            try:
                us = time_step(eng, a.iters)
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"kind": kind, "cfg": cfg, "error": str(ex)[:200]}), flush=True)
                continue
            res.append((us, cfg))
            print(json.dumps({"kind": kind, "cfg": cfg, "step_us": round(us, 1)}), flush=True)
        us, cfg = min(res)
        heur = next((u for u, c in res if c == (0, 0, 0)), float("nan"))
        best[kind] = {"cfg": cfg, "step_us": round(us, 1), "heuristic_step_us": round(heur, 1)}
        set_plan(eng.model, kind, cfg)
    print(json.dumps({"best": best, "final_step_us": round(time_step(eng, a.iters), 1)}), flush=True)


if __name__ == "__main__":
    main()
