"""In-engine sweep of the decode-GEMM decomposition per projection kind (MI355X).

Builds the engine (random init), runs the prefill and a few decode steps of ``--batch``
sequences, then for every candidate (waves, splitk, ntb) of one projection kind (qkv, o,
gate_up, down, lm_head) re-captures the decode hipGraph and times ``--iters`` back-to-back
replays of the WHOLE step (CUDA events). Every other kind keeps its current setting, so the
deltas are in-context: cold weights from HBM, activations from the previous kernel, real
inter-kernel boundaries. Prints one JSON line per (kind, config) and a final JSON line with
the best config per kind (the table the model applies: vgate/models/decode_plans.py).

    python benchmarks/decode_sweep.py [--batch 8] [--ctx 64] [--kinds qkv,o,gate_up,down]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402

CANDIDATES = {
    "qkv": [(0, 0, 0), (8, 1, 0), (4, 1, 0), (8, 2, 0), (4, 2, 0), (4, 4, 0), (2, 4, 0), (8, 4, 0), (2, 2, 0),
            (1, 4, 0)],
    "o": [(0, 0, 0), (8, 1, 1), (4, 1, 1), (8, 2, 1), (4, 2, 1), (4, 3, 1), (4, 4, 1), (2, 4, 1), (8, 4, 1),
          (2, 8, 1), (1, 8, 1)],
    "gate_up": [(0, 0, 0), (0, 0, -8), (4, 1, 0), (2, 1, 0), (1, 1, 0), (8, 1, 0), (2, 2, 0), (1, 2, 0), (2, 1, 2),
                (4, 1, 2), (8, 1, 2), (4, 1, 4), (8, 1, 4)],
    "down": [(0, 0, 0), (8, 2, 1), (8, 3, 1), (8, 4, 1), (4, 4, 1), (4, 6, 1), (4, 8, 1), (8, 8, 1),
             (2, 8, 1), (1, 8, 1), (4, 5, 1), (8, 6, 1), (2, 6, 1)],
    "lm_head": [(0, 0, 0), (8, 1, 2), (4, 1, 2), (2, 1, 2), (1, 1, 2), (4, 1, 4), (2, 1, 1), (4, 1, 1)],
}
# int4 (AWQ) layers: the register-stationary kernel (csrc/kernels/gemm_awq_kx.hip); ntb -12 / -13 / -14
# force 1 / 2 / 4 tiles per GROUP block with the given (waves, K slices), -2 the K-split awq_gemm_kernel
CANDIDATES_AWQ = {
    "qkv": [(0, 0, 0), (8, 1, -12), (16, 1, -12), (6, 2, -12), (4, 0, -2)],
    "o": [(0, 0, 0), (8, 1, -12), (16, 1, -12), (6, 2, -12), (12, 1, -13), (4, 0, -2)],
    "gate_up": [(0, 0, 0), (8, 0, -12), (16, 0, -12), (6, 0, -12)],
    "down": [(0, 0, 0), (8, 4, -13), (8, 3, -13), (16, 2, -12), (12, 3, -12), (8, 8, -14), (4, 0, -2)],
    "lm_head": [(0, 0, 0)],
}


def lins(model, kind):
    if kind == "lm_head":
        return [model.lm_head]
    attr = {"qkv": "qkv", "o": "o", "gate_up": "gate_up", "down": "down"}[kind]
    return [getattr(L, attr) for L in model.layers]


def set_plan(model, kind, cfg):
    """cfg: (waves, K slices, tiles code) of the tile kernels, ("kx", waves, slices, tiles code) of the
    register-stationary kernel (path 4) or ("sk", waves, blocks per CU, group) of stream-K."""
    for lin in lins(model, kind):
        lin.dec_path, lin.dec_sk = 0, False
        if cfg[0] == "kx":
            lin.dec_path = 4
            lin.dec_waves, lin.dec_splitk, lin.dec_ntb = cfg[1:]
        elif cfg[0] == "sk":
            lin.dec_sk = tuple(cfg[1:])
            lin.dec_waves, lin.dec_splitk, lin.dec_ntb = 0, 0, 0
        else:
            lin.dec_waves, lin.dec_splitk, lin.dec_ntb = cfg


def time_step(eng, iters):
    r = eng.runner
    for k in list(r.graphs):
        del r.graphs[k]
    eng.step()  # captures the bucket (non-deferred) and runs it
    eng._drain_inflight()
    torch.cuda.synchronize()
    (key,) = [k for k in r.graphs]
    g = r.graphs[key]
    for _ in range(5):
        g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    e.synchronize()
    return 1e3 * s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=64)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--kinds", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--baseline-only", action="store_true", help="time the default plans only")
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda:0", max_model_len=2048, max_num_seqs=64,
                                 max_num_batched_tokens=2048, num_kv_blocks=2048, warmup=False,
                                 quantization=a.quantization))
    eng.runner.defer_capture = False
    eng.async_sched = False
    for i in range(a.batch):
        ids = [100 + (i * 131 + j * 17) % 5000 for j in range(a.ctx)]
        eng.add_request(f"r{i}", prompt_ids=ids,
                        params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=100000, ignore_eos=True))
    eng._drain_inbox()
    for _ in range(3):
        eng.step()
    base = time_step(eng, a.iters)
    print(json.dumps({"baseline_us": round(base, 1)}), flush=True)
    if a.baseline_only:
        for _ in range(2):
            print(json.dumps({"repeat_us": round(time_step(eng, a.iters), 1)}), flush=True)
        return
    best = {}
    for kind in a.kinds.split(","):
        res = []
        for cfg in (CANDIDATES_AWQ if a.quantization == "awq" else CANDIDATES)[kind]:
            set_plan(eng.model, kind, cfg)
            try:
                us = time_step(eng, a.iters)
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"kind": kind, "cfg": cfg, "error": str(ex)[:200]}), flush=True)
                continue
            res.append((us, cfg))
            print(json.dumps({"kind": kind, "cfg": cfg, "step_us": round(us, 1)}), flush=True)
        us, cfg = min(res)
        best[kind] = {"cfg": cfg, "step_us": round(us, 1)}
        set_plan(eng.model, kind, cfg)  # keep the winner while sweeping the next kind
    print(json.dumps({"best": best, "final_step_us": round(time_step(eng, a.iters), 1)}), flush=True)


if __name__ == "__main__":
    main()
