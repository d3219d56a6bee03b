"""TP row-parallel decode GEMM with the all-reduce in its epilogue (gemm_epilogue.h epilogue_ar)
against the fp32 references: out = bf16(sum over ranks of x_r @ W_r^T) + residual.

* one rank against a loopback region (world 1): every decode path that ends in the epilogue
  (one-tile and two-tile blocks, granule and slab split-K, the K-split int4 kernel), repeated
  calls (per-tile epochs alternate the parity buffers) and hipGraph replay;
* two ranks in ONE process on two streams, each with its own region, the kernels running
  concurrently and meeting through each other's arrival words: both ranks store the same bits,
  equal to the reference sum, and no wait timed out.
Engine level (two processes sharing the GPU, graph == eager == TP 1): tests/test_tp_gpu.py.
"""
import math
from types import SimpleNamespace

import pytest
import torch

from vgate import ops
from vgate.ops import reference as ref
from vgate.parallel.custom_allreduce import SIGNAL_BYTES, LoopbackFused

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.fixture(scope="module")
def loop():
    lb = LoopbackFused(torch.device(DEV))
    yield lb
    assert ops.native().ar_error(lb.own) == 0, "a fused all-reduce wait gave up"
    lb.close()


def _dense(N, K, seed):
    torch.manual_seed(seed)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    return w, ops.Linear(w)


@pytest.mark.parametrize("M", [1, 16])
@pytest.mark.parametrize("N,K,waves,splitk,ntb", [
    (1024, 2048, 0, 0, 0),     # launcher heuristic
    (8192, 1024, 2, 1, 1),     # Llama-3-70B TP = 8 o_proj plan
    (1536, 8960, 4, 2, 1),     # two K slices: granule combine
    (1536, 8960, 4, 3, 1),     # three slices: slab + ticket combine
    (2048, 1536, 4, 1, 2),     # two-tile blocks (prefetched epilogue operands)
])
def test_fused_ar_loopback(loop, M, N, K, waves, splitk, ntb):
    w, lin = _dense(N, K, M + N + K + splitk)
    lin.dec_waves, lin.dec_splitk, lin.dec_ntb = waves, splitk, ntb
    x = torch.randn(M, K, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    want = ref.linear_ref(x, w, None, res)
    outs = []
    for _ in range(3):  # epochs 1..3: both parity buffers
        out = res.clone()
        ops.linear(x, lin, out=out, residual=out, ar=loop)
        outs.append(out)
    torch.cuda.synchronize()
    assert _rel(outs[0], want) < 1e-2
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_fused_ar_loopback_graph(loop):
    w, lin = _dense(2048, 1536, 5)
    x = torch.randn(8, 1536, device=DEV).bfloat16()
    res = torch.randn(8, 2048, device=DEV).bfloat16()
    out = torch.empty_like(res)
    ops.linear(x, lin, out=out, residual=res, ar=loop)
    eager = out.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            ops.linear(x, lin, out=out, residual=res, ar=loop)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)


def test_fused_ar_loopback_awq(loop):
    torch.manual_seed(3)
    M, N, K, g = 8, 512, 1024, 128
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    lin = ops.Linear(None, kind="awq", awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g})
    x = torch.randn(M, K, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    out = res.clone()
    ops.linear(x, lin, out=out, residual=out, ar=loop)
    assert _rel(out, ref.linear_ref(x, wd, None, res)) < 2e-2


@pytest.mark.parametrize("M,N,K,splitk", [(8, 1024, 2048, 0), (4, 2048, 4096, 2)])
def test_fused_ar_two_ranks_two_streams(M, N, K, splitk):
    """Two ranks' GEMMs in flight together on two streams, exchanging through their regions."""
    C = ops.native()
    nbytes = SIGNAL_BYTES + int(C.ar_fused_bytes())
    bases = [C.ar_alloc(nbytes), C.ar_alloc(nbytes)]
    try:
        torch.manual_seed(M + N + K)
        ws = [(torch.randn(N, K, device=DEV) / math.sqrt(2 * K)).bfloat16() for _ in range(2)]
        lins = [ops.Linear(w) for w in ws]
        for lin in lins:
            lin.dec_splitk = splitk
            lin.dec_waves = 4 if splitk else 0
        xs = [torch.randn(M, K, device=DEV).bfloat16() for _ in range(2)]
        res = torch.randn(M, N, device=DEV).bfloat16()
        want = (xs[0].float() @ ws[0].float().t() + xs[1].float() @ ws[1].float().t()).bfloat16().float() + res.float()
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for it in range(3):
            outs = [torch.empty_like(res) for _ in range(2)]
            torch.cuda.synchronize()
            for r in (0, 1):
                rank = SimpleNamespace(bases=bases, rank=r, fused_off=SIGNAL_BYTES)
                with torch.cuda.stream(streams[r]):
                    ops.linear(xs[r], lins[r], out=outs[r], residual=res, ar=rank)
            torch.cuda.synchronize()
            assert C.ar_error(bases[0]) == 0 and C.ar_error(bases[1]) == 0, "a fused wait gave up"
            assert torch.equal(outs[0], outs[1]), it  # replicated: the same bits on every rank
            assert _rel(outs[0], want) < 1e-2
    finally:
        torch.cuda.synchronize()
        for b in bases:
            C.ar_free(b)
