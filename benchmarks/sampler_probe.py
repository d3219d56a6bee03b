"""Sampler cost on the logits the benchmarked model really produces (MI355X).

Runs a few decode steps of the random-init Qwen2.5-1.5B engine, keeps the logits the
sampler saw, then times ``ops.sample`` on them (hipGraph replay, like the engine) for the
request defaults (T=0.7, top_p=0.9), plain temperature sampling and greedy, and reports
the logits spread and nucleus size (what decides the number of rejection passes).

    python benchmarks/sampler_probe.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from benchmarks.micro_gpu import graph_time  # noqa: E402
from vgate import ops  # noqa: E402
from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402


def main():
    eng = LLMEngine(EngineConfig(model="Qwen/Qwen2.5-1.5B-Instruct", device="cuda:0", max_model_len=512,
                                 max_num_seqs=8, max_num_batched_tokens=512, num_kv_blocks=512,
                                 enforce_eager=True, warmup=False))
    seen = []
    orig = ops.sample

    def spy(logits, *a, **k):
        if logits.shape[0] == 8 and len(seen) < 4:
            seen.append(logits.detach().clone())
        return orig(logits, *a, **k)

    import vgate.runtime.model_runner as mr
    mr.ops.sample = spy
    for i in range(8):
        eng.add_request(f"p{i}", prompt=f"Request {i}: the quick brown fox jumps over the lazy dog {i}?",
                        params=SamplingParams(temperature=0.7, top_p=0.9, max_tokens=6, ignore_eos=True))
    eng.run_until_idle()
    mr.ops.sample = orig
    assert seen, "no batch-8 step observed"
    logits = seen[-1]
    B, V = logits.shape
    lg = logits.float()
    p = torch.softmax(lg / 0.7, -1)
    ps, _ = p.sort(-1, descending=True)
    nucleus = (ps.cumsum(-1) < 0.9).sum(-1) + 1
    stats = {"B": B, "V": V, "logit_std": round(lg.std(-1).mean().item(), 3),
             "logit_max_minus_mean": round((lg.max(-1).values - lg.mean(-1)).mean().item(), 3),
             "nucleus_sizes": nucleus.tolist(), "top1_prob": [round(v, 4) for v in ps[:, 0].tolist()]}
    dev = logits.device
    temp = torch.full((B,), 0.7, device=dev)
    topp = torch.full((B,), 0.9, device=dev)
    topk = torch.full((B,), -1, dtype=torch.int32, device=dev)
    seeds = torch.arange(B, dtype=torch.int64, device=dev)
    offs = torch.zeros(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.int32, device=dev)
    res = {}
    for name, t, tp in (("T0.7_top_p0.9", temp, topp), ("T0.7", temp, torch.ones_like(topp)),
                        ("greedy", torch.zeros_like(temp), topp)):
        res[name] = round(graph_time(lambda: orig(logits, t, tp, topk, seeds, offs, out=out)), 2)
    rnd = torch.randn(B, V, device=dev) * 2
    res["randn2_T0.7_top_p0.9"] = round(graph_time(lambda: orig(rnd, temp, topp, topk, seeds, offs, out=out)), 2)
    print(json.dumps({"sampler_probe": stats, "sampler_us": res}), flush=True)
    # segments per row (B * nseg blocks): more segments = less sweep work per block, more arrivals
    # per meeting
    C = ops.native()
    for cap in (16, 32, 64, 128):
        C.set_sample_nseg(cap)
        r = {"nseg": C.sample_segments(B, V)}
        for name, t, tp in (("T0.7_top_p0.9", temp, topp), ("greedy", torch.zeros_like(temp), topp)):
            r[name] = round(graph_time(lambda: orig(logits, t, tp, topk, seeds, offs, out=out)), 2)
        print(json.dumps({"nseg_cap": cap, **r}), flush=True)
    C.set_sample_nseg(64)
    # pass kernels (pass 0 + R rejection rounds as launches, last-arriver merges) vs the in-launch
    # meetings only (-1)
    for rl in (-1, 0, 1, 2):
        C.set_sample_round_launches(rl)
        r = {"round_launches": rl}
        for name, t, tp in (("T0.7_top_p0.9", temp, topp), ("T0.7", temp, torch.ones_like(topp)),
                            ("greedy", torch.zeros_like(temp), topp)):
            r[name] = round(graph_time(lambda: orig(logits, t, tp, topk, seeds, offs, out=out)), 2)
        print(json.dumps(r), flush=True)
    C.set_sample_round_launches(2)


if __name__ == "__main__":
    main()
