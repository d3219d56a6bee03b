"""Launch-timeline helper of the kernel sweeps: capture a callable in a hipGraph with the in-kernel
timeline slots on (TLScope, csrc/kernels/common.h), replay it and return each launch's block spans."""
from __future__ import annotations

from collections import defaultdict

import torch

TICKS_PER_US = 100.0


def timeline_graph(C, fns, reps=3):
    """Capture fns() in a graph with timeline slots, replay, return {name: [spans_us]}."""
    buf = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fns()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    C.timeline_start(buf)
    with torch.cuda.graph(g, stream=s):
        fns()
    used = C.timeline_stop()
    ents = C.timeline_entries()
    spans = defaultdict(list)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall = []
    for _ in range(reps):
        buf.zero_()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        wall.append(e0.elapsed_time(e1) * 1e3)
    t = buf[:used].view(-1, 2).cpu()
    for name, off, nb in ents:
        blk = t[off // 2: off // 2 + nb]
        ok = blk[:, 0] > 0
        if ok.any():
            spans[name].append((int(blk[ok, 1].max()) - int(blk[ok, 0].min())) / 100.0)
    return spans, min(wall)

