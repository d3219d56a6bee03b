"""Which rows of a flash mixed step (decode rows + K-split prefill tiles) differ between identical launches."""
import math
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from vgate import ops  # noqa: E402

DEV = "cuda"


def diag(Hq, Hkv):
    C = ops.native()
    torch.manual_seed(200 + Hq + Hkv)
    D = 128
    qlens = [1, 33, 64, 65, 200, 1]
    ctxs = [40, 33, 300, 65, 456, 77]
    S = len(qlens)
    maxb = max(ctxs) // 16 + 2
    nblk = S * maxb + 4
    g = torch.Generator(device="cpu").manual_seed(5)
    kc = torch.randn(nblk, Hkv, 16, D, generator=g).bfloat16().to(DEV)
    vc = torch.randn(nblk, Hkv, 16, D, generator=g).bfloat16().to(DEV)
    bt = (torch.randperm(nblk)[: S * maxb]).reshape(S, maxb).int().to(DEV)
    qs = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(qs[-1])
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    stride = (Hq + 2 * Hkv) * D
    qkv = torch.randn(T, stride, device=DEV).bfloat16()
    ts, tq = ops.prefill_tiles(qlens, ops.flash_lead(Hq, Hkv))
    ts, tq = ts + [-1] * 5, tq + [0] * 5
    ts = torch.tensor(ts, dtype=torch.int32, device=DEV)
    tq = torch.tensor(tq, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    C.set_flash_prefill(1)
    P = 4
    po = torch.empty(S, Hq, P, D, device=DEV)
    pml = torch.empty(S, Hq, P, 2, device=DEV)
    out = torch.zeros(T, Hq * D, device=DEV).bfloat16()
    ops.attention(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out, po, pml, Hq, Hkv, 512, scale)
    H = 1536
    xg = torch.randn(448, 8960, device=DEV).bfloat16()
    wg = ops.Linear((torch.randn(H, 8960, device=DEV) / 95.0).bfloat16())
    yg = torch.empty(448, H, dtype=torch.bfloat16, device=DEV)
    for it in range(8):
        if it % 2:  # a split-K prefill GEMM (its fp32 slabs in the same workspace) + its reduce in between
            C.gemm(xg, wg.wp, H, 8960, yg, 0, ws=ops.workspace(DEV), path=1, ntb=1281, splitk=3)
        out3 = torch.zeros_like(out)
        ops.attention(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out3, po, pml, Hq, Hkv, 512, scale)
        d3 = (out.float() - out3.float()).abs().sum(1)
        rows = torch.nonzero(d3).flatten().tolist()
        print(Hq, Hkv, "gemm before" if it % 2 else "", "rows differing", rows[:40], len(rows), flush=True)
    C.set_flash_prefill(-1)


if __name__ == "__main__":
    for hq, hkv in ((12, 2), (8, 1), (32, 8)):
        diag(hq, hkv)
