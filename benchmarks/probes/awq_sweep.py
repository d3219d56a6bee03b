"""AWQ W4A16 decode GEMM sweep on the MI355X (Qwen2.5-1.5B shapes, M = 8, group 128): the
register-stationary kernel (csrc/kernels/gemm_awq_kx.hip, ntb = -12) over (waves, K slices) per
shape against its own grid rule (0, 0, 0) and the older int4 kernels; block spans from the launch
timeline, weights cycled through > 400 MB (cold), the decode split-K granule workspace as in-engine.

    python benchmarks/awq_sweep.py            (AWQ_SWEEP_CFGS="w:sk:ntb,..." / AWQ_SWEEP_SHAPES=down,...)
"""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from benchmarks.tlgraph import timeline_graph  # noqa: E402


def block_stats(C, fn):
    """One launch in a graph with timeline slots: per-block duration / start percentiles (us)."""
    buf = torch.zeros(1 << 16, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    C.timeline_start(buf)
    with torch.cuda.graph(g, stream=s):
        fn()
    used = C.timeline_stop()
    ents = C.timeline_entries()
    out = {}
    for _ in range(3):
        buf.zero_()
        g.replay()
        torch.cuda.synchronize()
    t = buf[:used].view(-1, 2).cpu().double()
    for name, off, nb in ents:
        blk = t[off // 2: off // 2 + nb]
        blk = blk[blk[:, 0] > 0]
        if len(blk) == 0:
            continue
        st = (blk[:, 0] - blk[:, 0].min()) / 100.0
        du = (blk[:, 1] - blk[:, 0]) / 100.0
        q = lambda v, p: round(float(v.quantile(p)), 2)  # noqa: E731
        out = {"blocks": len(blk), "dur_p10": q(du, 0.1), "dur_med": q(du, 0.5), "dur_p90": q(du, 0.9),
               "dur_max": round(float(du.max()), 2), "start_p90": q(st, 0.9), "start_max": round(float(st.max()), 2),
               "span": round(float((blk[:, 1].max() - blk[:, 0].min()) / 100.0), 2)}
    return out
from vgate import ops  # noqa: E402

SHAPES = [("qkv", 2048, 1536, "plain"), ("o_proj", 1536, 1536, "plain"), ("gate_up", 17920, 1536, "silu"),
          ("down", 1536, 8960, "plain")]


def main():
    import os
    C = ops.native()
    M, g = int(os.environ.get("AWQ_SWEEP_M", "8")), 128
    only = os.environ.get("AWQ_SWEEP_SHAPES")
    dev = torch.device("cuda")
    ws = ops.workspace(dev)
    skw = dict(sk_ws=ops.sk_workspace(dev), fault=ops.fault_word(dev))
    for name, N, K, layout in SHAPES:
        if only and name not in only.split(","):
            continue
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev)
        scales = (torch.rand(K // g, N, device=dev) * 0.02 + 0.005).bfloat16()
        zeros = torch.randint(0, 16, (K // g, N), device=dev).float().bfloat16()
        ncopy = max(2, math.ceil(400e6 / (N * K // 2)))
        lins = [ops.Linear(None, awq={"qint": q, "scales": scales, "zeros": zeros, "group": g,
                                      "silu": layout == "silu"}) for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev).bfloat16()
        res = torch.randn(M, N, device=dev).bfloat16()
        epi = 2 if layout == "silu" else 0
        out = torch.empty(M, N // 2 if epi == 2 else N, device=dev, dtype=torch.bfloat16)
        rows = []
        # ntb: 0 = launcher's choice (register-stationary kernel), -12 / -13 / -14 = that kernel with 1 / 2 / 4
        # tiles per GROUP block and the forced (waves, slices), -2 = K-split awq_gemm_kernel
        cfgs = {"qkv": [(0, 0, 0), (8, 1, -12)],
                "o_proj": [(0, 0, 0), (8, 1, -12)],
                "gate_up": [(0, 0, 0), (4, 0, -2)],
                "down": [(0, 0, 0), (16, 1, -12), (12, 1, -12), (8, 4, -13), (8, 3, -13), (16, 2, -13), (16, 1, -13),
                         (14, 1, -12)]}[name]
        if os.environ.get("AWQ_SWEEP_CFGS"):
            cfgs = [tuple(int(v) for v in c.split(":")) for c in os.environ["AWQ_SWEEP_CFGS"].split(",")]
        ssp = (x.float().pow(2).reshape(M, K // 16, 16).sum(-1)).contiguous()
        if name in ("qkv", "gate_up"):
            cfgs = cfgs + [(w_, s_, n_, "norm3") for (w_, s_, n_) in cfgs[:1]]
        for cfg in cfgs:
            waves, sk, ntb = cfg[:3]
            nkw = dict(ssp_in=ssp, eps=1e-6) if len(cfg) > 3 else {}
            def fns():
                for i in range(12):
                    L = lins[i % ncopy]
                    C.gemm(x, L.wp, N, K, out, epi, res=None if epi else res, ws=ws, waves=waves, splitk=sk,
                           awq_scales=L.scales, awq_zeros=L.zeros, group=g, awq_szp=L.szp, ntb=ntb, **skw, **nkw)
            spans, wall = timeline_graph(C, fns)
            vals = [v for vs in spans.values() for v in vs]
            w_us = wall / 12
            L0 = lins[0]
            bs = block_stats(C, lambda: C.gemm(x, L0.wp, N, K, out, epi, res=None if epi else res, ws=ws, waves=waves,
                                               splitk=sk, awq_scales=L0.scales, awq_zeros=L0.zeros, group=g,
                                               awq_szp=L0.szp, ntb=ntb, **skw, **nkw))
            rows.append({"waves": waves, "splitk": sk, "ntb": ntb, "norm": 3 if nkw else 0, "span_us": round(sum(vals[1:]) / (len(vals) - 1), 2),
                         "wall_us": round(w_us, 2), "eff_TBps": round(lins[0].nbytes() / w_us / 1e6, 2), "blocks": bs})
        print(json.dumps({"shape": name, "N": N, "K": K, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
