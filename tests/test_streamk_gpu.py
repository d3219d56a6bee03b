"""Stream-K decode GEMM (csrc/kernels/gemm_streamk.hip) against the fp32 references and the
tile-per-block decode kernel: every epilogue (plain + residual, f32, SiLU*mul with the folded
RMSNorm, QKV + bias + RoPE + paged KV write), the real projection shapes whose tiles split over
2-4 blocks, rows 1..16 (activation packing XP 4 / 2 / 1), bit-identical repeats (the owner adds
the published partials in block order) and hipGraph replay (the owner clears its slots)."""
import math

import pytest
import torch

from vgate import ops
from vgate.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.fixture(autouse=True)
def _sk():
    old = ops.STREAMK_DECODE
    ops.STREAMK_DECODE = True
    yield
    ops.STREAMK_DECODE = old
    assert int(ops.fault_word(DEV)[0].item()) & 4 == 0, "a stream-K partial poll gave up"


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K", [(1536, 8960), (1536, 1536), (2048, 1536), (1280, 8192), (8192, 1024), (4096, 14336)])
def test_streamk_plain_residual(M, N, K):
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    lin = ops.Linear(w)
    res = torch.randn(M, N, device=DEV).bfloat16()
    out = res.clone()
    ops.linear(x, lin, out=out, residual=out)
    assert _rel(out, ref.linear_ref(x, w, None, res)) < 1e-2
    out2 = res.clone()
    ops.linear(x, lin, out=out2, residual=out2)
    assert torch.equal(out, out2)  # bit-reproducible
    y = ops.linear(x, lin, out_f32=True)
    assert _rel(y, ref.linear_ref(x, w, None, None, True)) < 1e-3


@pytest.mark.parametrize("M", [1, 8, 16])
@pytest.mark.parametrize("H,I", [(1536, 8960), (4096, 3584)])
def test_streamk_silu_folded_norm(M, H, I):
    torch.manual_seed(M + H + I)
    x = (torch.randn(M, H, device=DEV) * 2).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    wg = (torch.randn(I, H, device=DEV) / math.sqrt(H)).bfloat16()
    wu = (torch.randn(I, H, device=DEV) / math.sqrt(H)).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), layout="silu")
    assert gu.fold_norm(nw)
    h = ops.linear(x, gu, norm=(nw, 1e-6))
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel(h, ref.silu_mul_linear_ref(xn, wg, wu)) < 2e-2


@pytest.mark.parametrize("M", [1, 8])
def test_streamk_qkv_rope_kv(M):
    torch.manual_seed(40 + M)
    H, D, BS, hq, hkv = 1536, 128, 16, 12, 2
    x = torch.randn(M, H, device=DEV).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    N = (hq + 2 * hkv) * D
    wq = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    lin = ops.Linear(wq, bias=b, layout="qkv")
    assert lin.fold_norm(nw)
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(64 * BS, device=DEV)[:M].int()
    cos_sin = ref.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc = torch.zeros(64, hkv, BS, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    q = torch.empty(M, hq * D, dtype=torch.bfloat16, device=DEV)
    ops.linear(x, lin, out=q, norm=(nw, 1e-6), qkv=dict(positions=pos, slots=slots, cos_sin=cos_sin, k_cache=kc,
                                                          v_cache=vc, hq=hq, hkv=hkv))
    kr, vr = torch.zeros_like(kc), torch.zeros_like(vc)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    y = ref.linear_ref(xn, wq, b)
    ref.rope_kv_ref(y, pos, slots, cos_sin, kr, vr, hq, hkv, D)
    assert _rel(q, y[:, : hq * D]) < 2e-2
    assert _rel(kc, kr) < 2e-2 and _rel(vc, vr) < 2e-2


def test_streamk_graph_replay():
    torch.manual_seed(3)
    M, N, K = 8, 1536, 8960
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    lin = ops.Linear(w)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.linear(x, lin, out=out)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.linear(x, lin, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.linear(x, lin, out=out)
    want = ref.linear_ref(x, w)
    for i in range(4):
        x.copy_(torch.randn(M, K, device=DEV).bfloat16())
        want = ref.linear_ref(x, w)
        g.replay()
        torch.cuda.synchronize()
        assert _rel(out, want) < 1e-2, i
