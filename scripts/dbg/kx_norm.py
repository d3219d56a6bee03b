"""Debug: int4 kx kernel NORM modes x XP x slices vs the dequantised reference."""
import torch
from vgate import ops
from vgate.ops import reference as ref

DEV = "cuda"
C = ops.native()
ws = ops.workspace(torch.device(DEV))
torch.manual_seed(0)
K, g = 1536, 128
for N in (1536, 8960 * 2):
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    sc = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zz = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    wd = ref.awq_dequant_ref(q, sc, zz, g).to(DEV)
    lin = ops.Linear(None, awq={"qint": q, "scales": sc.to(DEV), "zeros": zz.to(DEV), "group": g})
    for M in (8, 16):
        h = torch.randn(M, K, device=DEV).bfloat16()
        gamma = (torch.rand(K, device=DEV) + 0.5).bfloat16()
        xn, _ = ref.rmsnorm_ref(h, gamma, 1e-6)
        want = ref.linear_ref(xn, wd)
        hg = (h.float() * gamma.float()).bfloat16()
        ssp = h.float().pow(2).reshape(M, K // 16, 16).sum(-1).contiguous()
        for sk in (1, 2, 3):
            for w in (0, 4):
                kw = dict(ws=ws, awq_scales=lin.scales, awq_zeros=lin.zeros, group=g, awq_szp=lin.szp, ntb=-12,
                          waves=w, splitk=sk)
                o1 = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
                C.gemm(h, lin.wp, N, K, o1, 0, norm_w=gamma, eps=1e-6, **kw)
                o3 = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
                C.gemm(hg, lin.wp, N, K, o3, 0, eps=1e-6, ssp_in=ssp, **kw)
                o0 = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
                C.gemm(xn.bfloat16(), lin.wp, N, K, o0, 0, **kw)
                torch.cuda.synchronize()
                e = lambda o: ((o.float() - want).norm() / want.norm()).item()
                bad_rows = lambda o: [m for m in range(M) if ((o[m].float() - want[m]).norm() / want[m].norm()).item() > 0.02]
                print(f"N={N} M={M} sk={sk} w={w}: norm0 {e(o0):.4f} norm1 {e(o1):.4f} {bad_rows(o1)} "
                      f"norm3 {e(o3):.4f} {bad_rows(o3)}", flush=True)
