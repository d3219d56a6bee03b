"""Measured decode-GEMM decompositions (M <= 16) per weight shape, applied to every matching
Linear at model construction (``Linear.dec_waves / dec_splitk / dec_ntb``; 0 = the launcher's
heuristic, csrc/kernels/gemm_decode.h ``plan``).

Entries come from in-context sweeps: every candidate (waves per block, K slices, column tiles
per block) re-captures the decode hipGraph and times the WHOLE step, all other projections at
their current plan (benchmarks/decode_sweep.py for TP = 1 models, benchmarks/tp_rank_bench.py
--sweep for one TP rank's shapes). A shape missing here measured best on the heuristic.

Key: (N, K, layout, weight kind) of the packed weight; layout "qkv" / "silu" / "plain".
Value: (waves, K slices, column tiles per block) of the tile-per-block kernels, ("kx", waves, K
slices, tiles code) for the register-stationary kernel (path 4; 0 = its own grid rule), or
("sk", waves, blocks per CU, k-steps per register group) for the stream-K kernel
(csrc/kernels/gemm_streamk.hip: one equal share of the weight stream per CU), which wins on the
large matrices where the tile count leaves CUs uneven (benchmarks/probes/sk_probe.py,
profiles/r4_streamk_probe.log).
"""
from __future__ import annotations

PLANS: dict[tuple[int, int, str, str], tuple] = {
    # Llama-3-70B TP = 8, one rank, batch 8, ctx 128: round-5 in-context sweep with the register-stationary
    # and stream-K candidates (profiles/r5_tp8_rank_sweep.log; round 3: profiles/r3_tp8_rank_sweep.log)
    (1280, 8192, "qkv", "dense"): ("kx", 8, 3, 0),  # 80 tiles x 3 K slices, 8 waves (tile kernel 8 x 3: +56 us)
    (8192, 1024, "plain", "dense"): ("kx", 0, 1, 0),  # o_proj: 512 one-tile blocks (tile kernel 2 x 1: +13 us)
    (7168, 8192, "silu", "dense"): (4, 1, 0),    # gate_up: 448 one-tile blocks at 4 waves (heuristic 8: +67 us)
    # down_proj (8192, 3584): the heuristic tile plan (stream-K 4 x 1 x 8, the round-4 entry: +94 us since the
    # round-5 wait fixes). A rank with the fused row-parallel all-reduce (the TP default) runs o / down on
    # the tile kernels with the all-reduce epilogue whatever the entry says (vgate/ops linear: path 0 with ar)
    (16032, 8192, "plain", "dense"): (8, 1, 1),  # LM head shard
    # Llama-3-8B, batch 8 (r4 probe, profiles/r4_streamk_probe.log): qkv on stream-K (13.6 vs 15.1 us per
    # launch); gate_up and down_proj on 4-wave tile blocks (39.0 vs 41.3, 21.1 vs 21.9 us)
    (6144, 4096, "qkv", "dense"): ("sk", 8, 1, 4),
    (28672, 4096, "silu", "dense"): (4, 1, 0),
    (4096, 14336, "plain", "dense"): (4, 1, 1),
    # Qwen2.5-1.5B bf16 gate_up on the register-stationary kernel (one block per CU owning 4-5 whole
    # tiles, every weight fragment requested at once; csrc/kernels/gemm_kx.h): 10.5 vs 11.9 us per
    # launch as the hand-off consumer, cold weights (benchmarks/probes/dense_kx_sweep.py,
    # profiles/r5_dense_kx_sweep.log). qkv / o_proj / down_proj stay on the tile kernels there.
    (17920, 1536, "silu", "dense"): ("kx", 0, 0, 0),
    # Qwen2.5-1.5B AWQ int4: no entries — every int4 decode GEMM runs the register-stationary kernel
    # (csrc/kernels/gemm_awq_kx.hip) on its own grid rule (round 3's awq_stream / wide plans:
    # profiles/r3_awq_decode_sweep.log)
}


def apply(model) -> int:
    """Set the measured plan on every Linear of ``model`` whose shape has one; returns how many."""
    n = 0
    lins = [lin for L in model.layers for lin in (L.qkv, L.o, L.gate_up, L.down)] + [model.lm_head]
    for lin in lins:
        p = PLANS.get((lin.N, lin.K, lin.layout, lin.kind))
        if p is not None:
            if p[0] == "sk":
                lin.dec_sk = tuple(p[1:])
            elif p[0] == "kx":
                lin.dec_path = 4
                lin.dec_waves, lin.dec_splitk, lin.dec_ntb = p[1:]
            else:
                lin.dec_waves, lin.dec_splitk, lin.dec_ntb = p
            n += 1
    return n
