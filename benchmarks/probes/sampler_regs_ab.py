"""Sampler A/B: register-resident rejection rounds (sampling.hip sample_gran_kernel, next round's
noise computed while the row's segments meet) vs the memory-sweep rounds, on near-uniform logits
(random-init LM heads: an ~86k-token nucleus at T 0.7 / top-p 0.9, most batches of 8 need round 2+).
One hipGraph of 64 sampler calls with distinct offsets (distinct draws), device time per call.

    python benchmarks/probes/sampler_regs_ab.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from vgate import ops  # noqa: E402


def main():
    C = ops.native()
    dev = torch.device("cuda")
    torch.manual_seed(5)
    B, V, n = 8, 151936, 64
    L = (torch.randn(B, V, device=dev) * 0.8).contiguous()
    t = torch.full((B,), 0.7, device=dev)
    tp = torch.full((B,), 0.9, device=dev)
    tk = torch.full((B,), -1, dtype=torch.int32, device=dev)
    seeds = torch.arange(B, device=dev, dtype=torch.int64) * 7 + 3
    offs = [torch.full((B,), i, dtype=torch.int64, device=dev) for i in range(n)]
    outs = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(n)]
    res = {}
    got = {}
    for regs in (True, False, True, False):
        C.set_sample_regs(regs)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(n):
                ops.sample(L, t, top_p=tp, top_k=tk, seeds=seeds, offsets=offs[i], out=outs[i])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(n):
                ops.sample(L, t, top_p=tp, top_k=tk, seeds=seeds, offsets=offs[i], out=outs[i])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            best = min(best, 1e3 * e0.elapsed_time(e1) / n)
        key = "regs" if regs else "memory"
        res[key] = min(res.get(key, 1e9), round(best, 2))
        got[key] = torch.stack(outs).cpu()
    C.set_sample_regs(True)
    print(json.dumps({"sampler_us_per_call": res, "identical_tokens": bool(torch.equal(got["regs"], got["memory"])),
                      "fault": int(ops.fault_word(dev)[0].item())}), flush=True)


if __name__ == "__main__":
    main()
