"""Fused decode MLP (csrc/kernels/mlp_fused.hip) against the fp32 reference and the two-GEMM path.

out = residual + down(silu(gate(xn)) * up(xn)), xn = RMSNorm(x) * gamma (gamma folded into gate_up).
"""
import math

import pytest
import torch

from vgate import ops
from vgate.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.fixture(autouse=True, scope="module")
def _native():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    ops.native()
    keep = ops.FUSED_MLP
    ops.FUSED_MLP = True  # the kernel under test, whatever the engine default
    yield
    ops.FUSED_MLP = keep


def _layers(H, I, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    wg = (torch.randn(I, H, device=DEV, generator=g) / math.sqrt(H)).bfloat16()
    wu = (torch.randn(I, H, device=DEV, generator=g) / math.sqrt(H)).bfloat16()
    wd = (torch.randn(H, I, device=DEV, generator=g) / math.sqrt(I)).bfloat16()
    gamma = (torch.rand(H, device=DEV, generator=g) + 0.5).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), kind="silu")
    assert gu.fold_norm(gamma)
    dn = ops.Linear(wd)
    return gu, dn, (wg, wu, wd, gamma)


def _reference(x, dense, eps=1e-6, residual=True):
    wg, wu, wd, gamma = dense
    xn, _ = ref.rmsnorm_ref(x.cpu(), gamma.cpu(), eps)
    h = ref.silu_mul_linear_ref(xn, wg.cpu(), wu.cpu())
    return ref.linear_ref(h, wd.cpu(), None, x.cpu() if residual else None)


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("H,I,slices", [(1536, 8960, 0), (1024, 4096, 8), (1024, 4096, 4)])
def test_mlp_fused_matches_reference_and_two_gemms(M, H, I, slices):
    """Qwen2.5-1.5B (8 slices: SiLU tiles 4 / 5 per workgroup, down shares evening the bytes out) and a
    smaller shape at 8 and 4 slices (other tile / piece splits)."""
    gu, dn, dense = _layers(H, I, 100 + M)
    x = (torch.randn(M, H, device=DEV) * 2).bfloat16()
    epoch = torch.zeros(4, dtype=torch.int32, device=DEV)
    yref = _reference(x, dense)
    # two-GEMM path (the kernels the fused launch replaces)
    mid = ops.linear(x, gu, norm=(dense[3], 1e-6))
    y2 = ops.linear(mid, dn, residual=x)
    # fused, in place (out = x = residual, as the model runs it)
    y = x.clone()
    epoch += 1
    assert ops.mlp_decode(y, gu, dn, y, y, 1e-6, 5, epoch, slices=slices)
    torch.cuda.synchronize()
    assert ops.mlp_error(DEV) == 0
    assert _rel_err(y.cpu(), yref) < 1e-2
    assert _rel_err(y, y2) < 1e-2
    # deterministic: the same input again (next epoch) is bit-identical
    y3 = x.clone()
    epoch += 1
    assert ops.mlp_decode(y3, gu, dn, y3, y3, 1e-6, 5, epoch, slices=slices)
    assert torch.equal(y3, y)


def test_mlp_fused_no_residual_and_out_of_place():
    H, I = 1536, 8960
    gu, dn, dense = _layers(H, I, 7)
    M = 8
    x = torch.randn(M, H, device=DEV).bfloat16()
    out = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    epoch = torch.ones(4, dtype=torch.int32, device=DEV)
    assert ops.mlp_decode(x, gu, dn, out, None, 1e-6, 0, epoch)
    assert _rel_err(out.cpu(), _reference(x, dense, residual=False)) < 1e-2
    # the layer index separates the tags of two launches that share an epoch
    out2 = torch.empty_like(out)
    x2 = torch.randn(M, H, device=DEV).bfloat16()
    assert ops.mlp_decode(x2, gu, dn, out2, None, 1e-6, 1, epoch)
    assert _rel_err(out2.cpu(), _reference(x2, dense, residual=False)) < 1e-2
    assert ops.mlp_error(DEV) == 0


def test_mlp_fused_graph_replay():
    """Captured with the epoch bump in the graph (as the engine's embedding kernel does it): every
    replay reads its own h, results equal the eager launch for new inputs."""
    H, I = 1536, 8960
    gu, dn, dense = _layers(H, I, 11)
    M = 8
    xin = torch.randn(M, H, device=DEV).bfloat16()
    buf = xin.clone()
    epoch = torch.zeros(4, dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            buf.copy_(xin)
            epoch.add_(1)
            assert ops.mlp_decode(buf, gu, dn, buf, buf, 1e-6, 3, epoch)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        buf.copy_(xin)
        epoch.add_(1)
        ops.mlp_decode(buf, gu, dn, buf, buf, 1e-6, 3, epoch)
    for seed in range(3):
        xin.copy_(torch.randn(M, H, device=DEV, generator=torch.Generator(device=DEV).manual_seed(seed)).bfloat16())
        g.replay()
        torch.cuda.synchronize()
        assert _rel_err(buf.cpu(), _reference(xin, dense)) < 1e-2
    assert ops.mlp_error(DEV) == 0


def test_mlp_fused_declines_unfit_shapes():
    # Llama-3-8B (H = 4096: the x fragments of a block exceed the staged form) and > 16 rows: not fused
    gu, dn, _ = _layers(4096, 14336, 3)
    epoch = torch.ones(4, dtype=torch.int32, device=DEV)
    x = torch.randn(8, 4096, device=DEV).bfloat16()
    assert not ops.mlp_decode(x, gu, dn, x, x, 1e-6, 0, epoch)
    gu2, dn2, _ = _layers(1536, 8960, 4)
    x2 = torch.randn(17, 1536, device=DEV).bfloat16()
    assert not ops.mlp_decode(x2, gu2, dn2, x2, x2, 1e-6, 0, epoch)
