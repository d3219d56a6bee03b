import math, sys
sys.path.insert(0, ".")
import torch
from vgate import ops
from vgate.ops import reference as ref
DEV = "cuda"
def _rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))
def diag(hq, hkv, S, mode):
    """Decode-only step: the QKV projection with the decode attention in its launch (qkv_attn.hip on
    the decode tile kernel, gemm_kx.h kx_qa_kernel on the register-stationary bf16 / int4 kernels)
    == the two-launch path (q and the K / V cache bit-exact, attention within bf16 rounding of the
    fp32 reference), contexts of 1 .. 1000 tokens (two partitions, several chunks per wave, the new
    token first / last in its cache block), K slices combined in-launch (sk 2: granules, 3: slabs),
    and a second launch on the cleared granules."""
    torch.manual_seed(40 + S + hq + len(mode))
    H, D, BS, part, maxlen = 1536, 128, 16, 512, 1024
    nbs = maxlen // BS
    N = (hq + 2 * hkv) * D
    ctxs = [100, 1, 33, 257, 700, 512, 513, 31, 64, 65, 1000, 2, 128, 300, 17, 90][:S]
    nblocks = S * nbs + 3
    bt = torch.randperm(nblocks)[: S * nbs].view(S, nbs).int().to(DEV)
    kc = (torch.randn(nblocks, hkv, BS, D, device=DEV) * 0.5).bfloat16()
    vc = torch.randn(nblocks, hkv, BS, D, device=DEV).bfloat16()
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    pos = cl - 1
    slots = (bt[torch.arange(S, device=DEV), (pos // BS).long()] * BS + pos % BS).int()
    qs = torch.arange(S + 1, dtype=torch.int32, device=DEV)
    x = torch.randn(S, H, device=DEV).bfloat16()
    gamma = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    if mode.startswith("awq"):
        g = 128
        qi = torch.randint(0, 16, (N, H), dtype=torch.int32)
        sc = (torch.rand(H // g, N) * 0.02 + 0.005).bfloat16()
        zr = torch.randint(0, 16, (H // g, N)).float().bfloat16()
        lin = ops.Linear(None, awq={"qint": qi, "scales": sc.to(DEV), "zeros": zr.to(DEV), "group": g,
                                    "layout": "qkv"})
        if mode == "awq_sk2":
            lin.dec_waves, lin.dec_splitk, lin.dec_ntb = 6, 2, -12
    else:
        lin = ops.Linear(w, bias=b, layout="qkv")
        assert lin.fold_norm(gamma)
        if mode.startswith("tile_sk"):
            lin.dec_waves, lin.dec_splitk = 8, int(mode[-1])
        elif mode.startswith("kx"):
            lin.dec_path = 4
            lin.dec_waves, lin.dec_splitk, lin.dec_ntb = (8, 3, 0) if mode == "kx_sk3" else (0, 0, 0)
    cs = ref.rope_cos_sin(2048, D, 1e6, device=DEV)
    P = maxlen // part
    part_o = torch.empty(S, hq, P, D, dtype=torch.float32, device=DEV)
    part_ml = torch.empty(S, hq, P, 2, dtype=torch.float32, device=DEV)
    C = ops.native()
    # the layer's o_proj as the third role (bf16 modes): resid += attn @ Wo^T + the hand-off sums
    lo = ops.Linear((torch.randn(H, hq * D, device=DEV) / math.sqrt(hq * D)).bfloat16())
    resid0 = torch.randn(S, H, device=DEV).bfloat16()
    with_o = not mode.startswith("awq")

    def run(fuse, kcx, vcx):
        ops.FUSE_QKV_ATTN = fuse
        ops.step_tag(DEV).add_(1)  # (the model's embedding launch bumps it every step)
        q = torch.empty(S, hq * D, dtype=torch.bfloat16, device=DEV)
        o = torch.zeros(S, hq * D, dtype=torch.bfloat16, device=DEV)
        r = resid0.clone()
        ssp = torch.zeros(S, H // 16, dtype=torch.float32, device=DEV)
        fa = dict(block_tables=bt, context_lens=cl, query_start=qs, out=o, part_o=part_o, part_ml=part_ml,
                  part_size=part, scale=D ** -0.5)
        if with_o:
            fa.update(oproj=dict(lin=lo, out=r, residual=r, ssp_out=ssp), layer=3)
        ops.linear(x, lin, out=q, norm=(gamma, 1e-6),
                   qkv=dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kcx, v_cache=vcx, hq=hq, hkv=hkv),
                   attn=fa)
        flags = fa.get("fused", 0)
        if with_o and not flags & 2:
            ops.linear(o, lo, out=r, residual=r, norm_out=(None, ssp, gamma))
        return q, o, r, ssp, flags

    fault0 = int(ops.fault_word(DEV)[0])
    try:
        kc1, vc1 = kc.clone(), vc.clone()
        buf = torch.zeros(1 << 16, dtype=torch.int64, device=DEV)
        C.timeline_start(buf)
        q1, o1, r1, ss1, flags = run(True, kc1, vc1)
        torch.cuda.synchronize()
        C.timeline_stop()
        names = [e[0] for e in C.timeline_entries()]
        q1b, o1b, r1b, _, _ = run(True, kc1, vc1)
        kc2, vc2 = kc.clone(), vc.clone()
        q2, o2, r2, ss2, flags2 = run(False, kc2, vc2)
        torch.cuda.synchronize()
    finally:
        ops.FUSE_QKV_ATTN = True
    assert (int(ops.fault_word(DEV)[0]) & ~fault0 & 32) == 0, "a fused attention wait gave up"
    if mode.startswith("tile"):  # the same GEMM blocks: bit-exact
        assert torch.equal(q1, q2) and torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    else:  # the fused register-stationary launch holds <= 8 waves: another K split, bf16 rounding apart
        assert _rel_err(q1, q2) < 1e-2 and _rel_err(kc1, kc2) < 1e-2 and _rel_err(vc1, vc2) < 1e-2
    assert torch.equal(q1b, q1) and torch.equal(o1b, o1)
    for qq, kk, vv, oo in ((q1, kc1, vc1, o1), (q2, kc2, vc2, o2)):
        ro = ref.attention_ref(qq.view(S, hq, D), kk, vv, bt, cl, qs, hq, hkv, D ** -0.5).view(S, hq * D)
        assert _rel_err(oo, ro) < 1e-2
    print(mode, S, hq, hkv, "flags", flags, "flags_b?", "names", names)
    d = (r1b.float() - r1.float()).abs()
    print("max |r1b - r1|", float(d.max()), "rows differing", sorted(set(torch.nonzero(d > 0)[:, 0].tolist())))
    ro = ref.linear_ref(o1, lo.dense_weight(), None, resid0)
    print("rel r1 vs ref", _rel_err(r1, ro), "rel r1b vs ref", _rel_err(r1b, ro), "rel r2 vs ref", _rel_err(r2, ro))
    cols = sorted(set((torch.nonzero(d > 0)[:, 1] // 16).tolist()))
    print("tiles differing", cols[:40], len(cols))

if __name__ == "__main__":
    for S in (8, 5, 16):
        for i in range(2):
            diag(12, 2, S, "tile")
