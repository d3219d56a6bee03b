"""Does hipGraphLaunch block the host when the SAME graph exec is still running on the
device? Times the host-side cost of back-to-back replays of one ~1 ms graph vs
alternating two identical graphs (MI355X, torch.cuda.CUDAGraph = hipGraphExec).

    python benchmarks/probes/graph_relaunch_probe.py
"""
import json
import time

import torch


def main():
    dev = torch.device("cuda")
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    outs = [torch.empty_like(a) for _ in range(2)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.mm(a, b, out=outs[0])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graphs = []
    for i in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(8):
                torch.mm(a, b, out=outs[i])
        graphs.append(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    graphs[0].replay()
    torch.cuda.synchronize()
    one = time.perf_counter() - t0
    res = {"graph_device_ms": round(1e3 * one, 3)}
    for name, seq in (("same_exec", [0] * 8), ("alternating", [0, 1] * 4)):
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for i in seq:
            t = time.perf_counter()
            graphs[i].replay()
            host.append(1e3 * (time.perf_counter() - t))
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        res[name] = {"host_ms_per_replay_call": [round(x, 3) for x in host], "enqueue_all_ms": round(1e3 * t_enq, 3),
                     "total_ms": round(1e3 * (time.perf_counter() - t0), 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
