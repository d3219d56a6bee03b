"""Custom one-shot all-reduce (csrc/kernels/allreduce.hip) on a real MI355X: 2 processes
share the box's one GPU (each maps the other's uncached IPC buffer, exactly as two GPUs
of a node map each other's over xGMI) and compare against the bf16 sum computed locally
from the same seeded inputs (fp32 accumulation in rank order -> bf16: bit-exact).
Covers in-place / out-of-place, sizes from one 16-byte vector to 4 MiB, many consecutive
calls (epoch parity), and replay from a captured hipGraph."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2


def _inputs(n, it, world):
    out = []
    for r in range(world):
        g = torch.Generator().manual_seed(1000 * it + 17 * r + n)
        out.append(torch.randn(n, generator=g).bfloat16())
    return out


def _expect(xs):
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x in xs:
        acc += x.float()
    return acc.bfloat16()


def _worker(rank, port, q, WORLD=2, modes=(0,)):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from vgate.parallel.custom_allreduce import CustomAllReduce
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ar = CustomAllReduce(dist.group.WORLD, rank, WORLD, dev, max_bytes=4 << 20)
        it = 0
        for two_shot in modes:  # (one process group for every form: a spawn per form cost ~3 s of tier time)
            it = _one_mode(ar, dist, dev, rank, WORLD, two_shot, it)
        dist.barrier()
        ar.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))


def _one_mode(ar, dist, dev, rank, WORLD, two_shot, it):
    for n in [8, 64, 4096, 8 * 1536, 64 * 8192, 2 << 20]:
        for rep in range(3):
            it += 1
            xs = _inputs(n, it, WORLD)
            t = xs[rank].to(dev)
            if rep == 1:
                out = torch.empty_like(t)
                ar.all_reduce(t, out, two_shot=two_shot)
            else:
                out = ar.all_reduce(t, two_shot=two_shot)
            torch.cuda.synchronize()
            ar.check()
            assert torch.equal(out.cpu(), _expect(xs)), (rank, n, rep)
    # captured into a hipGraph: replays read the static input, epochs advance on device
    n = 8 * 4096
    static = torch.zeros(n, dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.all_reduce(static.clone(), two_shot=two_shot)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        res = ar.all_reduce(static, two_shot=two_shot)
    for rep in range(4):
        it += 1
        xs = _inputs(n, it, WORLD)
        static.copy_(xs[rank].to(dev))
        g.replay()
        torch.cuda.synchronize()
        ar.check()
        assert torch.equal(res.cpu(), _expect(xs)), (rank, "graph", two_shot, rep)
    dist.barrier()
    return it


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,modes", [(2, (0, 1)), (3, (-1, 1))])
def test_custom_allreduce_processes_one_gpu(world, modes):
    """One-shot (-1 / auto at 2 ranks) and two-shot (reduce-scatter + all-gather, 1) forms, 2 and
    3 ranks sharing the GPU: bit-exact vs the fp32 rank-order sum, eager and graph-replayed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, world, modes)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, msg = q.get(timeout=200)
        res[r] = msg
    for p in procs:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res
