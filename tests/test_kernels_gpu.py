"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference.

Run on an MI355X: ``python -m pytest tests -m gpu``. Shapes include the real
Qwen2.5-1.5B / Llama-3 projection sizes.
"""
import math
import os

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
    ops.native()  # must load: no silent fallback
    yield


@pytest.mark.parametrize("M,N,K", [(1, 2048, 1536), (8, 1536, 1536), (8, 1536, 8960), (17, 256, 512),
                                   (33, 4096, 4096), (64, 6144, 4096), (100, 512, 1024), (300, 1024, 2048)])
def test_gemm_plain(M, N, K):
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    lin = ops.Linear(w)
    y = ops.linear(x, lin)
    yr = ref.linear_ref(x, w)
    assert _rel_err(y, yr) < 1e-2


def test_gemm_bias_residual_f32():
    torch.manual_seed(1)
    M, N, K = 8, 2048, 1536
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=DEV).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    lin = ops.Linear(w, bias=b)
    assert _rel_err(ops.linear(x, lin), ref.linear_ref(x, w, b)) < 1e-2
    lin2 = ops.Linear(w)
    assert _rel_err(ops.linear(x, lin2, residual=r), ref.linear_ref(x, w, None, r)) < 1e-2
    y32 = ops.linear(x, lin2, out_f32=True)
    assert y32.dtype == torch.float32
    assert _rel_err(y32, ref.linear_ref(x, w, out_f32=True)) < 5e-3
    # in-place residual (out aliases residual), as the model's o_proj/down_proj do
    r2 = r.clone()
    ops.linear(x, lin2, out=r2, residual=r2)
    assert _rel_err(r2, ref.linear_ref(x, w, None, r)) < 1e-2


@pytest.mark.parametrize("M", [1, 8, 40])
def test_gemm_silu(M):
    torch.manual_seed(2)
    I, K = 8960 // 4, 1536
    x = torch.randn(M, K, device=DEV).bfloat16()
    wg = (torch.randn(I, K, device=DEV) / math.sqrt(K)).bfloat16()
    wu = (torch.randn(I, K, device=DEV) / math.sqrt(K)).bfloat16()
    lin = ops.Linear(torch.cat([wg, wu]), kind="silu")
    y = ops.linear(x, lin)
    assert y.shape == (M, I)
    assert _rel_err(y, ref.silu_mul_linear_ref(x, wg, wu)) < 1e-2
    if M <= 16:  # decode blocks of 2 / 4 SiLU tiles (forced), with the RMSNorm prologue
        nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
        xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
        for ntb, waves in [(2, 2), (2, 4), (4, 4)]:
            lin.dec_waves, lin.dec_splitk, lin.dec_ntb = waves, 1, ntb
            yt = ops.linear(x, lin, norm=(nw, 1e-6))
            assert _rel_err(yt, ref.silu_mul_linear_ref(xn, wg, wu)) < 1e-2, (ntb, waves)


def test_gemm_asymmetric_identity():
    # A = I with an asymmetric B catches transposed C writes (cdna_hip_programming.md §3)
    K = 64
    x = torch.eye(16, K, device=DEV).bfloat16()
    w = torch.arange(32 * K, device=DEV, dtype=torch.float32).reshape(32, K).remainder(7).bfloat16()
    y = ops.linear(x, ops.Linear(w))
    assert torch.equal(y.float(), (x.float() @ w.float().t()))


def test_awq_gemm():
    torch.manual_seed(3)
    M, N, K, g = 8, 512, 1024, 128
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    lin = ops.Linear(None, kind="awq", awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g})
    x = torch.randn(M, K, device=DEV).bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    assert _rel_err(ops.linear(x, lin), ref.linear_ref(x, wd)) < 2e-2


@pytest.mark.parametrize("H", [1536, 4096, 8192])
def test_rmsnorm(H):
    torch.manual_seed(4)
    x = torch.randn(13, H, device=DEV).bfloat16()
    r = torch.randn(13, H, device=DEV).bfloat16()
    w = torch.randn(H, device=DEV).bfloat16()
    y = ops.rmsnorm(x, w, 1e-6)
    yr, _ = ref.rmsnorm_ref(x, w, 1e-6)
    assert _rel_err(y, yr) < 1e-2
    r2 = r.clone()
    y2 = ops.rmsnorm(x, w, 1e-6, residual=r2)
    yr2, sr = ref.rmsnorm_ref(x, w, 1e-6, r)
    assert torch.equal(r2, sr)
    assert _rel_err(y2, yr2) < 1e-2


def test_embedding_vocab_shard():
    table = torch.randn(100, 64, device=DEV).bfloat16()
    ids = torch.tensor([0, 5, 99, 100, 150, 42], device=DEV, dtype=torch.int32)
    out = ops.embedding(ids, table, vstart=50)
    assert torch.equal(out, ref.embedding_ref(ids, table, 50))


def test_rope_kv():
    torch.manual_seed(5)
    Hq, Hkv, D, BS, T = 12, 2, 128, 16, 37
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).bfloat16()
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(64 * BS, device=DEV)[:T].int()
    slots[3] = -1
    cs = ref.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc = torch.zeros(64, Hkv, BS, D, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    a, kc2, vc2 = qkv.clone(), kc.clone(), vc.clone()
    ops.rope_kv(a, pos, slots, cs, kc, vc, Hq, Hkv, D)
    ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, Hq, Hkv, D)
    assert _rel_err(a, qkv) < 1e-2
    assert _rel_err(kc, kc2) < 1e-2
    assert torch.equal(vc, vc2)


def _make_cache(num_blocks, Hkv, D=128, BS=16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    kc = torch.randn(num_blocks, Hkv, BS, D, generator=g).bfloat16().to(DEV)
    vc = torch.randn(num_blocks, Hkv, BS, D, generator=g).bfloat16().to(DEV)
    return kc, vc


@pytest.mark.parametrize("Hq,Hkv", [(12, 2), (32, 8), (8, 1), (64, 8), (32, 2)])
@pytest.mark.parametrize("ctxs", [[1, 7, 33, 100], [513, 2048, 1500, 64], [5]])
def test_attention_decode(Hq, Hkv, ctxs):
    torch.manual_seed(6)
    D, BS = 128, 16
    S = len(ctxs)
    maxb = 2048 // BS
    nblk = S * maxb + 8
    kc, vc = _make_cache(nblk, Hkv)
    perm = torch.randperm(nblk - 1)[: S * maxb] + 1
    bt = perm.reshape(S, maxb).int().to(DEV)
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    q = torch.randn(S, Hq * D, device=DEV).bfloat16()
    part = 512
    P = (maxb * BS + part - 1) // part
    po = torch.empty(S, Hq, P, D, device=DEV)
    pml = torch.empty(S, Hq, P, 2, device=DEV)
    out = torch.zeros(S, Hq * D, device=DEV).bfloat16()
    scale = 1 / math.sqrt(D)
    ops.attention_decode(q, Hq * D, kc, vc, bt, cl, out, po, pml, Hq, Hkv, part, scale)
    r = ref.attention_ref(q.view(S, Hq, D), kc, vc, bt, cl, torch.arange(S + 1, dtype=torch.int32), Hq, Hkv, scale)
    assert _rel_err(out.view(S, Hq, D), r) < 2e-2


@pytest.mark.parametrize("Hq,Hkv", [(12, 2), (32, 8), (16, 16)])
def test_attention_prefill_chunked(Hq, Hkv):
    torch.manual_seed(7)
    D, BS = 128, 16
    qlens = [1, 17, 64, 5, 130]
    ctxs = [1, 17, 100, 300, 130]  # ctx > qlen => chunked prefill against earlier cache
    S = len(qlens)
    maxb = 32
    nblk = S * maxb + 4
    kc, vc = _make_cache(nblk, Hkv, seed=1)
    bt = (torch.randperm(nblk)[: S * maxb]).reshape(S, maxb).int().to(DEV)
    qs = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(qs[-1])
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    stride = (Hq + 2 * Hkv) * D  # q lives inside a fused qkv row
    qkv = torch.randn(T, stride, device=DEV).bfloat16()
    ts, tq = ops.prefill_tiles(qlens)
    ts = torch.tensor(ts, dtype=torch.int32, device=DEV)
    tq = torch.tensor(tq, dtype=torch.int32, device=DEV)
    out = torch.zeros(T, Hq * D, device=DEV).bfloat16()
    scale = 1 / math.sqrt(D)
    ops.attention_prefill(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out, Hq, Hkv, scale)
    q = qkv[:, : Hq * D].reshape(T, Hq, D)
    r = ref.attention_ref(q, kc, vc, bt, cl, qs.cpu(), Hq, Hkv, scale)
    assert _rel_err(out.view(T, Hq, D), r) < 2e-2


@pytest.mark.parametrize("Hq,Hkv", [(12, 2), (32, 8)])
@pytest.mark.parametrize("qlens,ctxs", [([2048], [2048]), ([4096], [4096]), ([1024, 2048], [3072, 2048])])
def test_attention_prefill_long(Hq, Hkv, qlens, ctxs):
    """Prefill attention at prompt lengths 2048 / 4096 (whole prompt in one step) and a chunked
    prefill (1024 new queries against 2048 cached tokens) next to a fresh 2048 prompt, against
    the fp32 reference."""
    torch.manual_seed(71 + sum(qlens))
    D = 128
    S = len(qlens)
    maxb = max(ctxs) // 16
    nblk = S * maxb + 4
    kc, vc = _make_cache(nblk, Hkv, seed=2)
    bt = (torch.randperm(nblk)[: S * maxb]).reshape(S, maxb).int().to(DEV)
    qs = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(qs[-1])
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    stride = (Hq + 2 * Hkv) * D
    qkv = torch.randn(T, stride, device=DEV).bfloat16()
    ts, tq = ops.prefill_tiles(qlens)
    ts = torch.tensor(ts, dtype=torch.int32, device=DEV)
    tq = torch.tensor(tq, dtype=torch.int32, device=DEV)
    out = torch.zeros(T, Hq * D, device=DEV).bfloat16()
    scale = 1 / math.sqrt(D)
    ops.attention_prefill(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out, Hq, Hkv, scale)
    q = qkv[:, : Hq * D].reshape(T, Hq, D)
    r = ref.attention_ref(q, kc, vc, bt, cl, qs.cpu(), Hq, Hkv, scale)
    assert _rel_err(out.view(T, Hq, D), r) < 2e-2


def test_sample_greedy_and_topk1():
    torch.manual_seed(8)
    B, V = 6, 151936
    logits = torch.randn(B, V, device=DEV) * 3
    out = ops.sample(logits, temperature=torch.zeros(B, device=DEV))
    assert torch.equal(out.long().cpu(), logits.argmax(-1).cpu())
    t = torch.ones(B, device=DEV)
    out2 = ops.sample(logits, temperature=t, top_k=torch.ones(B, dtype=torch.int32, device=DEV),
                      seeds=torch.arange(B, device=DEV), offsets=torch.zeros(B, dtype=torch.int64, device=DEV))
    assert torch.equal(out2.long().cpu(), logits.argmax(-1).cpu())


def test_sample_distribution_topk_topp():
    V = 1000
    logits = torch.full((1, V), -10.0, device=DEV)
    logits[0, :4] = torch.tensor([2.0, 1.5, 1.0, 0.2], device=DEV)
    n = 3000
    L = logits.expand(n, V).contiguous()
    t = torch.ones(n, device=DEV)
    seeds = torch.arange(n, device=DEV, dtype=torch.int64) * 7919 + 1
    offs = torch.zeros(n, dtype=torch.int64, device=DEV)
    # top_k = 2 -> only tokens 0/1 with ratio e^2 : e^1.5
    out = ops.sample(L, t, top_k=torch.full((n,), 2, dtype=torch.int32, device=DEV), seeds=seeds, offsets=offs)
    o = out.cpu()
    assert set(o.tolist()) <= {0, 1}
    p0 = (o == 0).float().mean().item()
    exp0 = math.exp(2.0) / (math.exp(2.0) + math.exp(1.5))
    assert abs(p0 - exp0) < 0.04
    # top_p = 0.7 -> nucleus {0, 1} (p0=.47 < .7, p0+p1=.76 >= .7)
    out = ops.sample(L, t, top_p=torch.full((n,), 0.7, device=DEV), seeds=seeds, offsets=offs)
    assert set(out.cpu().tolist()) <= {0, 1}
    # determinism
    out_b = ops.sample(L, t, top_p=torch.full((n,), 0.7, device=DEV), seeds=seeds, offsets=offs)
    assert torch.equal(out, out_b)
    # plain multinomial hits the tail sometimes, never invalid ids
    out = ops.sample(L, t, seeds=seeds, offsets=offs)
    assert int(out.max()) < V and int(out.min()) >= 0


def test_sample_segmented_matches_single_block_and_distribution():
    """Small batches split each row over many blocks (per-row meeting counters); the
    Gumbel noise is indexed by token, so the draw is identical to one block per row."""
    torch.manual_seed(21)
    V = 151936
    base = torch.full((V,), -30.0, device=DEV)
    hot = torch.tensor([5, 77_000, 151_935, 40_000, 123_456], device=DEV)
    base[hot] = torch.tensor([2.0, 1.6, 1.2, 0.8, 0.0], device=DEV)
    B = 4
    L = base.expand(B, V).contiguous()
    seeds = torch.tensor([3, 5, 7, 11], device=DEV, dtype=torch.int64)
    t = torch.full((B,), 1.0, device=DEV)
    for kw in ({}, {"top_p": torch.full((B,), 0.8, device=DEV)}, {"top_k": torch.full((B,), 3, dtype=torch.int32, device=DEV)}):
        counts = torch.zeros(V, dtype=torch.long)
        for off in range(150):
            offs = torch.full((B,), off, dtype=torch.int64, device=DEV)
            seg = ops.sample(L, t, seeds=seeds, offsets=offs, **kw)
            # the same rows inside a 300-row batch run one block per row
            big = 300
            Lb = base.expand(big, V).contiguous()
            kwb = {k: v.repeat(big // B) for k, v in kw.items()}
            one = ops.sample(Lb, t.repeat(big // B), seeds=seeds.repeat(big // B),
                             offsets=offs.repeat(big // B), **kwb)[:B]
            assert torch.equal(seg, one), (kw, off)
            counts += torch.bincount(seg.long().cpu(), minlength=V)
        n = counts.sum().item()
        p = torch.softmax(base.cpu(), -1)
        if "top_p" in kw:
            allowed = hot[:3].cpu()   # .40 + .27 < .8 <= .40 + .27 + .18
        elif "top_k" in kw:
            allowed = hot[:3].cpu()
        else:
            allowed = hot.cpu()
        assert counts[allowed].sum().item() == n
        q = p[allowed] / p[allowed].sum()
        emp = counts[allowed].double() / n
        assert (emp - q.double()).abs().max().item() < 0.07, (kw, emp, q)


def _nucleus_probs(row: torch.Tensor, temp: float, top_p: float) -> torch.Tensor:
    """Exact target of top-p sampling: token j is inside iff the tempered mass strictly
    above x_j is < top_p (the token crossing top_p is included); renormalised."""
    p = torch.softmax(row.double() / temp, -1)
    above = torch.stack([p[row > v].sum() for v in row])
    keep = above < top_p
    q = torch.where(keep, p, torch.zeros_like(p))
    return q / q.sum()


@pytest.mark.parametrize("B", [8, 512])
def test_sample_top_p_frequent_rejection(B):
    """A flat head with a small nucleus: the first Gumbel candidate is rejected ~70% of the
    time, so later rejection rounds decide the draw. Their acceptance statistics must be
    measured against the ROW max of pass 0 (regression: a later round read the previous
    round's partial and degenerated into the argmax)."""
    V = 4096
    hot = torch.tensor([1.0, 0.9, 0.8, 0.7, 0.6, 0.5, 0.4, 0.3, 0.2, 0.1])
    row = torch.full((V,), -40.0)
    idx = torch.arange(0, 10) * 397 + 11
    row[idx] = hot
    q = _nucleus_probs(row, 1.0, 0.3)
    allowed = (q > 0).nonzero().flatten()
    assert 2 <= len(allowed) <= 4
    L = row.to(DEV).expand(B, V).contiguous()
    t = torch.ones(B, device=DEV)
    tp = torch.full((B,), 0.3, device=DEV)
    counts = torch.zeros(V, dtype=torch.long)
    reps = max(1, 6000 // B)
    for off in range(reps):
        seeds = torch.arange(B, device=DEV, dtype=torch.int64) * 104729 + 17
        offs = torch.full((B,), off, dtype=torch.int64, device=DEV)
        out = ops.sample(L, t, top_p=tp, seeds=seeds, offsets=offs)
        counts += torch.bincount(out.long().cpu(), minlength=V)
    n = counts.sum().item()
    assert counts[allowed].sum().item() == n, "sampled outside the nucleus"
    emp = counts.double() / n
    assert (emp[allowed] - q[allowed]).abs().max().item() < 0.03, (emp[allowed], q[allowed])


def test_sample_segmented_matches_row_kernel_across_batch_sizes():
    """The segmented sampler (every block gathers its row's tagged partials itself) draws what the
    one-block-per-row kernel draws — same Gumbel noise, same acceptance tests — while the batch size
    ALTERNATES between launches (8 -> 4 -> 16 -> 8 ...: the rows' granule layout must not move with
    nseg, round-4 ADVICE: rows of a smaller batch wrote into a larger batch's row regions and a row
    whose epoch had not moved matched them), for greedy / temperature / top-p / top-k rows, then under
    hipGraph replay (> 64 replays: the per-row epoch keeps the tags apart)."""
    torch.manual_seed(40)
    V = 151936
    C = ops.native()
    L = (torch.randn(16, V, device=DEV) * 0.8).contiguous()
    t = torch.full((16,), 0.7, device=DEV)
    t[0] = 0.0  # a greedy row
    tp = torch.full((16,), 0.9, device=DEV)
    tk = torch.full((16,), -1, dtype=torch.int32, device=DEV)
    tk[2] = 50
    tk[5] = 20
    tp[5] = 0.5
    tp[1] = 1.0  # plain temperature row
    seeds = torch.arange(16, device=DEV, dtype=torch.int64) * 7 + 3
    try:
        for off in range(90):
            B = (8, 4, 16, 8, 2, 16)[off % 6]
            offs = torch.full((B,), off, dtype=torch.int64, device=DEV)
            args = (L[:B], t[:B])
            kw = dict(top_p=tp[:B], top_k=tk[:B], seeds=seeds[:B], offsets=offs)
            assert C.sample_segments(B, V) > 1
            a = ops.sample(*args, **kw).clone()
            C.set_sample_nseg(1)
            b = ops.sample(*args, **kw)
            C.set_sample_nseg(64)
            assert torch.equal(a, b), (off, B, a, b)
        B = 8
        offs = torch.full((B,), 7, dtype=torch.int64, device=DEV)
        out = torch.empty(B, dtype=torch.int32, device=DEV)
        kw = dict(top_p=tp[:B], top_k=tk[:B], seeds=seeds[:B], offsets=offs)
        want = ops.sample(L[:B], t[:B], **kw).clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                ops.sample(L[:B], t[:B], out=out, **kw)
        torch.cuda.current_stream().wait_stream(s)
        for i in range(70):
            out.fill_(-1)
            g.replay()
            if i % 10 == 5:  # other batch sizes between replays
                ops.sample(L[:4], t[:4], top_p=tp[:4], top_k=tk[:4], seeds=seeds[:4], offsets=offs[:4])
            torch.cuda.synchronize()
            assert torch.equal(out, want)
        assert int(ops.fault_word(DEV)[0].item()) & 16 == 0, "a sampler row wait gave up"
    finally:
        C.set_sample_nseg(64)


def test_sample_logprob():
    torch.manual_seed(9)
    logits = torch.randn(4, 5000, device=DEV)
    lp = torch.empty(4, device=DEV)
    out = ops.sample(logits, temperature=torch.zeros(4, device=DEV), out_logprob=lp)
    exp = torch.log_softmax(logits, -1).gather(1, out.long()[:, None]).squeeze(1)
    assert torch.allclose(lp, exp, atol=1e-3)


# ---------------------------------------------------------------- fused GEMM v2
@pytest.mark.parametrize("M,N,K", [(8, 1536, 1536), (8, 1536, 8960), (40, 2048, 1536), (200, 512, 1024)])
@pytest.mark.parametrize("splitk", [1, 3, 8])
def test_gemm_splitk_residual_inplace(M, N, K, splitk):
    """In-launch split-K through fp32 slabs + a ticket (the two-slice granule combine: the decode
    plans / test_gemm_norm_splitk); repeated launches re-use the self-resetting tickets."""
    torch.manual_seed(10)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    exp = ref.linear_ref(x, w, None, r)
    lin = ops.Linear(w)
    for _ in range(3):  # repeated launches: split-K tickets must self-reset
        r2 = r.clone()
        ops.linear(x, lin, out=r2, residual=r2, splitk=splitk)
        assert _rel_err(r2, exp) < 1e-2


def test_gemm_norm_prologue_and_row_gather():
    torch.manual_seed(11)
    T, H, N = 37, 1536, 4096
    x = torch.randn(T, H, device=DEV).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    idx = torch.tensor([36, 0, 17, 5], dtype=torch.int32, device=DEV)
    y = ops.linear(x, ops.Linear(w), out_f32=True, norm=(nw, 1e-6), row_idx=idx)
    xn, _ = ref.rmsnorm_ref(x[idx.long()], nw, 1e-6)
    assert _rel_err(y, ref.linear_ref(xn, w, out_f32=True)) < 1e-2
    # silu + norm
    wg = (torch.randn(512, H, device=DEV) / math.sqrt(H)).bfloat16()
    wu = (torch.randn(512, H, device=DEV) / math.sqrt(H)).bfloat16()
    y2 = ops.linear(x, ops.Linear(torch.cat([wg, wu]), kind="silu"), norm=(nw, 1e-6))
    xn2, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel_err(y2, ref.silu_mul_linear_ref(xn2, wg, wu)) < 1e-2


@pytest.mark.parametrize("hq,hkv", [(12, 2), (8, 1)])
def test_gemm_qkv_rope_kv_epilogue(hq, hkv):
    torch.manual_seed(12)
    T, H, D, BS = 21, 1536, 128, 16
    N = (hq + 2 * hkv) * D
    x = torch.randn(T, H, device=DEV).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    pos = torch.randint(0, 1000, (T,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(32 * BS, device=DEV)[:T].int()
    slots[4] = -1
    cs = ref.rope_cos_sin(1024, D, 1e6, device=DEV)
    kc = torch.zeros(32, hkv, BS, D, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    lin = ops.Linear(w, bias=b, layout="qkv")
    q = ops.linear(x, lin, norm=(nw, 1e-6), qkv=dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kc,
                                                      v_cache=vc, hq=hq, hkv=hkv))
    # reference: norm -> linear(+bias) -> rope + kv write
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    qkv = ref.linear_ref(xn, w, b)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, hq, hkv, D)
    assert _rel_err(q, qkv[:, : hq * D]) < 1e-2
    assert _rel_err(kc, kc2) < 1e-2 and _rel_err(vc, vc2) < 1e-2
    assert torch.equal(lin.dense_weight(), w)


@pytest.mark.parametrize("hq,hkv", [(12, 2), (8, 1), (32, 8)])
@pytest.mark.parametrize("S", [1, 5, 8, 16])
@pytest.mark.parametrize("mode", ["tile", "tile_sk2", "tile_sk3", "kx", "kx_sk3", "awq", "awq_sk2"])
def test_qkv_attention_fused(hq, hkv, S, mode):
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

    def run(fuse, kcx, vcx):
        ops.FUSE_QKV_ATTN = fuse
        q = torch.empty(S, hq * D, dtype=torch.bfloat16, device=DEV)
        o = torch.zeros(S, hq * D, dtype=torch.bfloat16, device=DEV)
        ops.linear(x, lin, out=q, norm=(gamma, 1e-6),
                   qkv=dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kcx, v_cache=vcx, hq=hq, hkv=hkv),
                   attn=dict(block_tables=bt, context_lens=cl, query_start=qs, out=o, part_o=part_o,
                             part_ml=part_ml, part_size=part, scale=D ** -0.5))
        return q, o

    fault0 = int(ops.fault_word(DEV)[0])
    try:
        kc1, vc1 = kc.clone(), vc.clone()
        buf = torch.zeros(1 << 16, dtype=torch.int64, device=DEV)
        C.timeline_start(buf)
        q1, o1 = run(True, kc1, vc1)
        torch.cuda.synchronize()
        C.timeline_stop()
        names = [e[0] for e in C.timeline_entries()]
        q1b, o1b = run(True, kc1, vc1)
        kc2, vc2 = kc.clone(), vc.clone()
        q2, o2 = run(False, kc2, vc2)
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
    fused = {"qkv_attn", "kx_qa", "awq_kx_qa"}
    assert fused & set(names), names  # the decode kernel took the fused launch


def test_awq_norm_splitk():
    torch.manual_seed(13)
    M, N, K, g = 8, 1536, 1536, 128
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    lin = ops.Linear(None, awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g})
    x = torch.randn(M, K, device=DEV).bfloat16()
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    for sk in (1, 4):
        y = ops.linear(x, lin, norm=(nw, 1e-6), splitk=sk)
        assert _rel_err(y, ref.linear_ref(xn, wd)) < 2e-2


@pytest.mark.parametrize("M", [1, 5, 16, 24])
@pytest.mark.parametrize("g", [64, 128])
@pytest.mark.parametrize("sk", [0, 3])
def test_awq_decode_kernel_shapes(M, g, sk):
    """AWQ decode kernel (waves split N over an LDS copy of x, M <= 16) == dequantised
    reference for plain + residual, silu pairs and group 64 / 128; M = 24 takes the
    K-split kernel. Also == the K-split kernel (waves forced) on the same inputs."""
    torch.manual_seed(40 + M + g + sk)
    N, K = 1024, 2048
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    x = torch.randn(M, K, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    lin = ops.Linear(None, awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g})
    y = ops.linear(x, lin, residual=res, splitk=sk)
    assert _rel_err(y, ref.linear_ref(x, wd, None, res)) < 2e-2
    y_ks = ops.linear(x, lin, residual=res, waves=4)
    assert _rel_err(y, y_ks) < 1e-2
    silu = ops.Linear(None, awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g,
                                 "silu": True})
    ys = ops.linear(x, silu, splitk=sk)
    assert _rel_err(ys, ref.silu_mul_linear_ref(x, wd[: N // 2], wd[N // 2:])) < 2e-2


@pytest.mark.parametrize("M", [1, 5, 8, 16])
@pytest.mark.parametrize("producer", ["dense", "awq"])
def test_awq_norm_handoff(M, producer):
    """RMSNorm hand-off of the int4 decode path: a residual GEMM writes out, hg = bf16(out * gamma)
    and per-16-column sums of out^2; the int4 consumers (qkv K-split kernel, SiLU stream kernel,
    split-K) read hg with the row scale from those sums == the gamma-in-registers mode."""
    torch.manual_seed(90 + M)
    H, Kin, g = 1536, 2048, 128
    x = torch.randn(M, Kin, device=DEV).bfloat16()
    res = torch.randn(M, H, device=DEV).bfloat16()
    gamma = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    if producer == "dense":
        wo = (torch.randn(H, Kin, device=DEV) / math.sqrt(Kin)).bfloat16()
        lo = ops.Linear(wo)
        h_ref = ref.linear_ref(x, wo, None, res)
    else:
        qo = torch.randint(0, 16, (H, Kin), dtype=torch.int32)
        so = (torch.rand(Kin // g, H) * 0.004 + 0.001).bfloat16()
        zo = torch.randint(0, 16, (Kin // g, H)).float().bfloat16()
        lo = ops.Linear(None, kind="awq", awq={"qint": qo, "scales": so.to(DEV), "zeros": zo.to(DEV), "group": g})
        h_ref = ref.linear_ref(x, ref.awq_dequant_ref(qo, so, zo, g).to(DEV), None, res)
    h = res.clone()
    hg = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    ssp = torch.empty(M, H // 16, dtype=torch.float32, device=DEV)
    ops.linear(x, lo, out=h, residual=h, norm_out=(hg, ssp, gamma))
    assert _rel_err(h, h_ref) < 2e-2
    assert torch.equal(hg, (h.float() * gamma.float()).bfloat16())
    torch.testing.assert_close(ssp, h.float().pow(2).reshape(M, H // 16, 16).sum(-1), rtol=1e-5, atol=1e-4)
    for N, layout, sk in [(2048, "qkv", 0), (2 * 4480, "silu", 0), (1536, "plain", 3)]:
        q = torch.randint(0, 16, (N, H), dtype=torch.int32)
        sc = (torch.rand(H // g, N) * 0.004 + 0.001).bfloat16()
        zz = torch.randint(0, 16, (H // g, N)).float().bfloat16()
        lin = ops.Linear(None, kind="awq", awq={"qint": q, "scales": sc.to(DEV), "zeros": zz.to(DEV), "group": g,
                                                "layout": layout})
        if layout == "qkv":
            continue  # covered through the engine (needs the cache operands); plain + silu here
        out_n = torch.empty(M, lin.out_features, dtype=torch.bfloat16, device=DEV)
        out_h = torch.empty_like(out_n)
        ops.linear(h, lin, out=out_n, norm=(gamma, 1e-6), splitk=sk)
        ops.linear(hg, lin, out=out_h, prenorm=(ssp, 1e-6), splitk=sk)
        assert _rel_err(out_h, out_n) < 1e-2, (layout, _rel_err(out_h, out_n))


@pytest.mark.parametrize("kernel", [0, -2, -12])
@pytest.mark.parametrize("N,K", [(17920, 1536), (1536, 8960), (2048, 1536)])
def test_awq_decode_kernels_each(kernel, N, K):
    """Every AWQ decode kernel on the Qwen2.5-1.5B shapes (M = 8, group 128, RMSNorm gamma in
    registers): 0 = launcher's choice (the register-stationary kernel, gemm_awq_kx.hip), -2 = the
    K-split awq_gemm_kernel (TP / group-64 fallback), -12 = the register-stationary kernel forced;
    == the dequantised fp32 reference."""
    torch.manual_seed(N + K + kernel)
    M, g = 8, 128
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    silu = N == 17920
    lin = ops.Linear(None, awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g,
                                "silu": silu})
    x = torch.randn(M, K, device=DEV).bfloat16()
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    out = torch.empty(M, N // 2 if silu else N, device=DEV, dtype=torch.bfloat16)
    ops.native().gemm(x, lin.wp, N, K, out, 2 if silu else 0, norm_w=nw, eps=1e-6, ws=ops.workspace(x.device),
                      awq_scales=lin.scales, awq_zeros=lin.zeros, group=g, awq_szp=lin.szp,
                      waves=4 if kernel == -2 else 0, ntb=kernel)
    want = ref.silu_mul_linear_ref(xn, wd[: N // 2], wd[N // 2:]) if silu else ref.linear_ref(xn, wd)
    assert _rel_err(out, want) < 2e-2


@pytest.mark.parametrize("M", [1, 8, 16])
@pytest.mark.parametrize("N,K,w,sk,tb", [(2 * 8960, 1536, 0, 0, 1), (4096 * 2, 1536, 6, 0, 1), (1536, 8960, 0, 0, 1),
                                         (1536, 8960, 8, 4, 2), (1536, 1536, 0, 0, 1), (1024, 2048, 8, 8, 4)])
def test_dense_kx_decode(M, N, K, w, sk, tb):
    """The register-stationary decode kernel on bf16 weights (path 4; ntb = -12 / -13 / -14 with the
    given waves / K slices, or its own grid rule) == the fp32 reference and the tile kernels: plain +
    residual, the hand-off producer (hg-free bf16 form: out + per-tile sums of squares), SiLU pairs with
    the folded-gamma row scale (NORM 2) and as the hand-off consumer (NORM 3)."""
    torch.manual_seed(900 + M + N // 64 + K // 128 + w + sk + tb)
    C = ops.native()
    dev = torch.device(DEV)
    kw = dict(ws=ops.workspace(dev), sk_ws=ops.sk_workspace(dev), fault=ops.fault_word(dev), path=4, waves=w,
              splitk=sk, ntb={1: -12 if (w or sk) else 0, 2: -13, 4: -14}[tb])
    wt = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    lin = ops.Linear(wt)
    x = torch.randn(M, K, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C.gemm(x, lin.wp, N, K, out, 0, res=res, **kw)
    assert _rel_err(out, ref.linear_ref(x, wt, None, res)) < 1e-2
    tile = torch.empty_like(out)
    C.gemm(x, lin.wp, N, K, tile, 0, res=res, ws=kw["ws"])
    assert _rel_err(out, tile) < 5e-3
    h = res.clone()
    ssp_n = torch.empty(M, N // 16, dtype=torch.float32, device=DEV)
    C.gemm(x, lin.wp, N, K, h, 0, res=h, ssp_out=ssp_n, **kw)
    assert torch.equal(h, out)
    torch.testing.assert_close(ssp_n, h.float().pow(2).reshape(M, N // 16, 16).sum(-1), rtol=1e-5, atol=1e-4)
    # SiLU pairs, RMSNorm gamma folded into W: row scale from x (NORM 2) / from the producer's sums (NORM 3)
    silu = ops.Linear(wt.clone(), kind="silu")
    gamma = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    assert silu.fold_norm(gamma)
    xn, _ = ref.rmsnorm_ref(x, gamma, 1e-6)
    want = ref.silu_mul_linear_ref(xn, wt[: N // 2], wt[N // 2:])
    ys = torch.empty(M, N // 2, device=DEV, dtype=torch.bfloat16)
    C.gemm(x, silu.wp, N, K, ys, 2, rownorm=True, eps=1e-6, **kw)
    assert _rel_err(ys, want) < 2e-2
    if K // 16 <= 128:
        ssp = x.float().pow(2).reshape(M, K // 16, 16).sum(-1).contiguous()
        yh = torch.empty_like(ys)
        C.gemm(x, silu.wp, N, K, yh, 2, eps=1e-6, ssp_in=ssp, **kw)
        assert _rel_err(yh, want) < 2e-2
        assert _rel_err(yh, ys) < 1e-2


@pytest.mark.parametrize("M", [1, 5, 8, 13, 16])
@pytest.mark.parametrize("N,K,w,sk,tb", [(2 * 8960, 1536, 0, 0, 1), (4096 * 2, 1536, 0, 0, 1), (2 * 8960, 1536, 8, 0, 1),
                                         (1536, 8960, 0, 0, 1), (1536, 1536, 0, 0, 1), (1536, 1536, 6, 2, 1),
                                         (1024, 2048, 4, 3, 1), (2048, 1536, 16, 1, 1), (1536, 8960, 12, 4, 2),
                                         (1536, 8960, 8, 8, 4), (1536, 1536, 6, 1, 2)])
def test_awq_kx_decode(M, N, K, w, sk, tb):
    """The register-stationary int4 decode kernel (gemm_awq_kx.hip; ntb = -12 / -13 / -14 forces it with
    1 / 2 / 4 tiles per GROUP block and the given waves / K slices, 0 = its own choice) == the
    dequantised fp32 reference: WIDE blocks (one per CU, 4-5 or 2 tiles each) and GROUP blocks (1-4
    tiles, 1-8 K slices: granules / slabs), XP = 2 (M <= 8) and XP = 1; plain + residual, RMSNorm
    gamma in registers + SiLU pairs, the hand-off consumer (x = h * gamma, row scale from the
    producer's per-tile sums) and the hand-off producer (hg, sums). (Multi-tile GROUP blocks take the
    plain / residual / producer GEMMs; the norm consumers fall back on one-tile blocks.)"""
    torch.manual_seed(700 + M + N // 64 + K // 128 + w + sk + tb)
    C = ops.native()
    ws = ops.workspace(torch.device(DEV))
    g = 128
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    awq = {"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g}
    lin = ops.Linear(None, awq=dict(awq))
    kw = dict(ws=ws, awq_scales=lin.scales, awq_zeros=lin.zeros, group=g, awq_szp=lin.szp, ntb={1: -12, 2: -13, 4: -14}[tb],
              waves=w, splitk=sk, sk_ws=ops.sk_workspace(torch.device(DEV)), fault=ops.fault_word(torch.device(DEV)))
    x = torch.randn(M, K, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C.gemm(x, lin.wp, N, K, out, 0, res=res, **kw)
    want = ref.linear_ref(x, wd, None, res)
    assert _rel_err(out, want) < 2e-2
    # hand-off producer: h = x W^T + res, hg = bf16(h * gamma), per-16-column sums of h^2
    gamma_n = (torch.rand(N, device=DEV) + 0.5).bfloat16()
    h = res.clone()
    hg = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ssp_n = torch.empty(M, N // 16, dtype=torch.float32, device=DEV)
    C.gemm(x, lin.wp, N, K, h, 0, res=h, hg_out=hg, hg_gamma=gamma_n, ssp_out=ssp_n, **kw)
    assert torch.equal(h, out)
    assert torch.equal(hg, (h.float() * gamma_n.float()).bfloat16())
    torch.testing.assert_close(ssp_n, h.float().pow(2).reshape(M, N // 16, 16).sum(-1), rtol=1e-5, atol=1e-4)
    # RMSNorm gamma in registers + SiLU pairs, and the hand-off consumer of the same rows
    silu = ops.Linear(None, awq=dict(awq, silu=True))
    skw = dict(kw, awq_scales=silu.scales, awq_zeros=silu.zeros, awq_szp=silu.szp)
    hx = torch.randn(M, K, device=DEV).bfloat16()
    gamma = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    xn, _ = ref.rmsnorm_ref(hx, gamma, 1e-6)
    want_s = ref.silu_mul_linear_ref(xn, wd[: N // 2], wd[N // 2:])
    ys = torch.empty(M, N // 2, device=DEV, dtype=torch.bfloat16)
    C.gemm(hx, silu.wp, N, K, ys, 2, norm_w=gamma, eps=1e-6, **skw)
    assert _rel_err(ys, want_s) < 2e-2
    if K // 16 <= 128:  # the producer's sums in the prefetched form (and the plain one past it)
        hgx = (hx.float() * gamma.float()).bfloat16()
        ssp = hx.float().pow(2).reshape(M, K // 16, 16).sum(-1).contiguous()
        yh = torch.empty_like(ys)
        C.gemm(hgx, silu.wp, N, K, yh, 2, eps=1e-6, ssp_in=ssp, **skw)
        assert _rel_err(yh, want_s) < 2e-2
        assert _rel_err(yh, ys) < 1e-2


@pytest.mark.parametrize("M", [17, 40, 64])
@pytest.mark.parametrize("w,sk", [(0, 0), (8, 0), (4, 3), (2, 6), (1, 12)])
def test_awq_mid_gemm(M, w, sk):
    """The int4 medium-M kernel (awq_mid_kernel, path 2: int4 fragments straight to registers, x by
    m-tile pairs in LDS with the gamma / x^2 / activation-sum pass, wide or K-split + reduce) ==
    the dequantised fp32 reference: plain + residual, gamma-in-registers RMSNorm + SiLU pairs (the
    1120-tile gate_up shape), and QKV + bias + RoPE + paged KV write."""
    torch.manual_seed(500 + M + 3 * w + sk)
    C = ops.native()
    ws = ops.workspace(torch.device(DEV))
    K, g, D, BS, hq, hkv = 1536, 128, 128, 16, 12, 2

    def awq_lin(N, silu=False, layout="plain", bias=None):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32)
        scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
        zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
        lin = ops.Linear(None, bias=bias, awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV),
                                               "group": g, "silu": silu, "layout": layout})
        return lin, ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)

    def kw(lin):
        return dict(ws=ws, awq_scales=lin.scales, awq_zeros=lin.zeros, group=g, awq_szp=lin.szp, path=2, waves=w,
                    splitk=sk)
    x = torch.randn(M, K, device=DEV).bfloat16()
    lin, wd = awq_lin(1536)
    res = torch.randn(M, 1536, device=DEV).bfloat16()
    out = res.clone()
    C.gemm(x, lin.wp, 1536, K, out, 0, res=out, **kw(lin))
    assert _rel_err(out, ref.linear_ref(x, wd, None, res)) < 2e-2
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    gu, wgu = awq_lin(2 * 8960, silu=True)
    ys = torch.empty(M, 8960, device=DEV, dtype=torch.bfloat16)
    C.gemm(x, gu.wp, 2 * 8960, K, ys, 2, norm_w=nw, eps=1e-6, **kw(gu))
    assert _rel_err(ys, ref.silu_mul_linear_ref(xn, wgu[:8960], wgu[8960:])) < 2e-2
    N = (hq + 2 * hkv) * D
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    lq, wq = awq_lin(N, layout="qkv", bias=b)
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=DEV)
    nblk = (M + BS - 1) // BS + 8
    slots = torch.randperm(nblk * BS, device=DEV)[:M].int()
    cs = ref.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc = torch.zeros(nblk, hkv, BS, D, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    qo = torch.empty(M, hq * D, dtype=torch.bfloat16, device=DEV)
    C.gemm(x, lq.wp, N, K, qo, 3, bias=b, norm_w=nw, eps=1e-6, positions=pos, slots=slots, cos_sin=cs, k_cache=kc,
           v_cache=vc, hq=hq, hkv=hkv, **kw(lq))
    qkv = ref.linear_ref(xn, wq, b)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, hq, hkv, D)
    assert _rel_err(qo, qkv[:, : hq * D]) < 2e-2
    assert _rel_err(kc, kc2) < 2e-2 and _rel_err(vc, vc2) < 2e-2


@pytest.mark.parametrize("M", [40, 256])
def test_awq_prefill_dequant_path(M):
    """Long AWQ steps: int4 -> bf16 fragment-packed scratch (gamma folded) + the bf16 prefill /
    tile kernels, for plain + residual, SiLU and norm; no library copy exists."""
    torch.manual_seed(77 + M)
    g, K = 128, 1536
    for N, silu in ((1536, False), (2048, True)):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32)
        scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
        zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
        wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
        lin = ops.Linear(None, awq={"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g,
                                    "silu": silu})
        assert not hasattr(lin, "wl")  # no resident bf16 copy
        x = torch.randn(M, K, device=DEV).bfloat16()
        nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
        xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
        if silu:
            y = ops.linear(x, lin, norm=(nw, 1e-6))
            assert _rel_err(y, ref.silu_mul_linear_ref(xn, wd[: N // 2], wd[N // 2:])) < 2e-2
        else:
            res = torch.randn(M, N, device=DEV).bfloat16()
            y = ops.linear(x, lin, residual=res.clone(), norm=(nw, 1e-6))
            assert _rel_err(y, ref.linear_ref(xn, wd, None, res)) < 2e-2


@pytest.mark.parametrize("Hq,Hkv", [(12, 2), (32, 8), (64, 8)])
def test_unified_attention_mixed_batch(Hq, Hkv):
    """decode rows (qlen 1, incl. split-K partitions) + prefill chunks in one launch."""
    torch.manual_seed(14)
    D, BS = 128, 16
    qlens = [1, 1, 37, 1, 16, 3]
    ctxs = [700, 5, 100, 1500, 16, 40]
    S = len(qlens)
    maxb = 128
    nblk = S * maxb + 4
    kc, vc = _make_cache(nblk, Hkv, seed=3)
    bt = (torch.randperm(nblk)[: S * maxb]).reshape(S, maxb).int().to(DEV)
    qs = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(qs[-1])
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    q = torch.randn(T, Hq * D, device=DEV).bfloat16()
    ts, tq = ops.prefill_tiles([ql if ql > 1 else 0 for ql in qlens])
    ts = torch.tensor(ts + [-1, -1], dtype=torch.int32, device=DEV)  # + padding tiles
    tq = torch.tensor(tq + [0, 0], dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    r = ref.attention_ref(q.view(T, Hq, D), kc, vc, bt, cl, qs.cpu(), Hq, Hkv, scale)
    for part in (64, 256, 1024, 256):  # repeated: in-launch partition tickets must self-reset
        P = (maxb * BS + part - 1) // part
        po = torch.empty(S, Hq, P, D, device=DEV)
        pml = torch.empty(S, Hq, P, 2, device=DEV)
        out = torch.zeros(T, Hq * D, device=DEV).bfloat16()
        ops.attention(q, Hq * D, kc, vc, bt, cl, qs, ts, tq, out, po, pml, Hq, Hkv, part, scale)
        assert _rel_err(out.view(T, Hq, D), r) < 2e-2


@pytest.mark.parametrize("T", [5, 40])
@pytest.mark.parametrize("waves", [1, 4, 16])
def test_deferred_norm_all_wave_counts(T, waves):
    """Fused RMSNorm (deferred row scale, per-wave ssq partials) == rmsnorm_ref -> linear_ref,
    for every wave decomposition, and bit-reproducible run to run."""
    torch.manual_seed(15 + T + waves)
    H, N = 1536, 2048
    x = (torch.randn(T, H, device=DEV) * 3).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    lin = ops.Linear(w)
    y = ops.linear(x, lin, norm=(nw, 1e-6), waves=waves)
    y2 = ops.linear(x, lin, norm=(nw, 1e-6), waves=waves)
    xn, _ = ref.rmsnorm_ref(x.cpu(), nw.cpu(), 1e-6)
    r = ref.linear_ref(xn, w.cpu())
    assert _rel_err(y.float().cpu(), r.float()) < 1e-2
    assert torch.equal(y, y2)


@pytest.mark.parametrize("T", [3, 8, 40])
def test_gemm_folded_norm(T):
    """RMSNorm gamma folded into the packed weight (row scale only in the kernel) == gamma path."""
    torch.manual_seed(30 + T)
    H, N = 1536, 4096
    x = (torch.randn(T, H, device=DEV) * 2).bfloat16()
    g = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    xn, _ = ref.rmsnorm_ref(x.cpu(), g.cpu(), 1e-6)
    r = ref.linear_ref(xn, w.cpu())
    plain = ops.Linear(w)
    folded = ops.Linear(w)
    assert folded.fold_norm(g)
    y1 = ops.linear(x, plain, norm=(g, 1e-6))
    y2 = ops.linear(x, folded, norm=(g, 1e-6))
    assert _rel_err(y1.float().cpu(), r.float()) < 1e-2
    assert _rel_err(y2.float().cpu(), r.float()) < 1e-2
    # silu layout too (the fold is along K, the row permutation along N)
    wg = torch.cat([w[:1024], w[1024:2048]])
    f2 = ops.Linear(wg, kind="silu")
    f2.fold_norm(g)
    y3 = ops.linear(x, f2, norm=(g, 1e-6))
    assert _rel_err(y3.float().cpu(), ref.silu_mul_linear_ref(xn, w[:1024].cpu(), w[1024:2048].cpu()).float()) < 1e-2


@pytest.mark.parametrize("T,splitk,waves", [(8, 2, 4), (8, 4, 2), (3, 3, 8), (16, 4, 4)])
def test_gemm_norm_splitk(T, splitk, waves):
    """Deferred RMSNorm under in-launch split-K: each slice publishes its partial sum of
    squares next to its slab, the last arriver scales the summed tile (gamma in registers,
    folded gamma, SiLU and the QKV epilogue)."""
    torch.manual_seed(60 + T + splitk)
    H, N = 1536, 1024
    x = (torch.randn(T, H, device=DEV) * 2).bfloat16()
    g = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    xn, _ = ref.rmsnorm_ref(x.cpu(), g.cpu(), 1e-6)
    r = ref.linear_ref(xn, w.cpu())
    kw = dict(waves=waves, splitk=splitk)
    y1 = ops.linear(x, ops.Linear(w), norm=(g, 1e-6), **kw)
    folded = ops.Linear(w)
    folded.fold_norm(g)
    y2 = ops.linear(x, folded, norm=(g, 1e-6), **kw)
    assert _rel_err(y1.float().cpu(), r.float()) < 1e-2
    assert _rel_err(y2.float().cpu(), r.float()) < 1e-2
    f3 = ops.Linear(w, kind="silu")
    f3.fold_norm(g)
    y3 = ops.linear(x, f3, norm=(g, 1e-6), **kw)
    assert _rel_err(y3.float().cpu(), ref.silu_mul_linear_ref(xn, w[:512].cpu(), w[512:].cpu()).float()) < 1e-2
    # QKV epilogue (Qwen2.5-1.5B heads) with the folded norm, as the engine runs it
    hq, hkv, D, BS = 12, 2, 128, 16
    wq = (torch.randn((hq + 2 * hkv) * D, H, device=DEV) / math.sqrt(H)).bfloat16()
    b = (torch.randn(wq.shape[0], device=DEV) * 0.1).bfloat16()
    pos = torch.randint(0, 1000, (T,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(32 * BS, device=DEV)[:T].int()
    cs = ref.rope_cos_sin(1024, D, 1e6, device=DEV)
    kc = torch.zeros(32, hkv, BS, D, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    lq = ops.Linear(wq, bias=b, layout="qkv")
    lq.fold_norm(g)
    q = ops.linear(x, lq, norm=(g, 1e-6), qkv=dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kc, v_cache=vc,
                                                     hq=hq, hkv=hkv), **kw)
    qkv = ref.linear_ref(xn.to(DEV), wq, b)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, hq, hkv, D)
    assert _rel_err(q, qkv[:, : hq * D]) < 1e-2
    assert _rel_err(kc, kc2) < 1e-2 and _rel_err(vc, vc2) < 1e-2


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 7, 8, 9, 16])
def test_gemm_small_batch_activation_packing(M):
    """Decode batches <= 4 / <= 8 pack 4 / 2 k-steps of activations per load (DPP unpack)."""
    torch.manual_seed(40 + M)
    K = 1536
    x = torch.randn(M, K, device=DEV).bfloat16()
    g = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    for N, kind in ((1536, "plain"), (1024, "silu")):
        w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
        lin = ops.Linear(w, kind=kind) if kind == "silu" else ops.Linear(w)
        wc = w.cpu()
        r_res = torch.randn(M, N // (2 if kind == "silu" else 1), device=DEV).bfloat16()
        for waves in (1, 4, 8):
            for sk in ((1, 2) if kind == "plain" else (1,)):
                if kind == "silu":
                    y = ops.linear(x, lin, norm=(g, 1e-6), waves=waves)
                    xn, _ = ref.rmsnorm_ref(x.cpu(), g.cpu(), 1e-6)
                    r = ref.silu_mul_linear_ref(xn, wc[: N // 2], wc[N // 2:])
                else:
                    out = r_res.clone()
                    y = ops.linear(x, lin, out=out, residual=out, waves=waves, splitk=sk)
                    r = ref.linear_ref(x.cpu(), wc, None, r_res.cpu())
                assert _rel_err(y.float().cpu(), r.float()) < 1e-2, (N, kind, waves, sk)


@pytest.mark.parametrize("M", [17, 40, 64, 100, 384])
def test_gemm_tile_kernel_prefill_shapes(M):
    """M > 16 with waves=-1 forces the N-split tile kernel (shared LDS copy of x): residual, folded-norm
    SiLU, f32 + row gather and the QKV epilogue against the fp32 references."""
    torch.manual_seed(50 + M)
    K1, N1 = 2240, 1536
    x = torch.randn(M, K1, device=DEV).bfloat16()
    w = (torch.randn(N1, K1, device=DEV) / math.sqrt(K1)).bfloat16()
    r = torch.randn(M, N1, device=DEV).bfloat16()
    out = r.clone()
    ops.linear(x, ops.Linear(w), out=out, residual=out, waves=-1)
    assert _rel_err(out.float().cpu(), ref.linear_ref(x.cpu(), w.cpu(), None, r.cpu()).float()) < 1e-2
    # folded-norm SiLU (gate_up shape class)
    H, I = 1536, 1024
    xh = (torch.randn(M, H, device=DEV) * 2).bfloat16()
    g = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    wg = (torch.randn(2 * I, H, device=DEV) / math.sqrt(H)).bfloat16()
    lin = ops.Linear(wg, kind="silu")
    lin.fold_norm(g)
    y = ops.linear(xh, lin, norm=(g, 1e-6), waves=-1)
    xn, _ = ref.rmsnorm_ref(xh.cpu(), g.cpu(), 1e-6)
    assert _rel_err(y.float().cpu(), ref.silu_mul_linear_ref(xn, wg[:I].cpu(), wg[I:].cpu()).float()) < 1e-2
    # f32 logits over a gathered row subset (LM head with > 16 sequences)
    idx = torch.randperm(M, device=DEV)[: max(17, M // 2)].int()
    wl = (torch.randn(4096, H, device=DEV) / math.sqrt(H)).bfloat16()
    lf = ops.linear(xh, ops.Linear(wl), out_f32=True, row_idx=idx, waves=-1)
    assert _rel_err(lf.cpu(), ref.linear_ref(xh[idx.long()].cpu(), wl.cpu(), out_f32=True)) < 1e-2


@pytest.mark.parametrize("M,K", [(17, 1536), (100, 2048), (448, 1536), (448, 8960), (640, 2304)])
def test_gemm_tile3_two_deep_pipeline(M, K):
    """waves=-2 forces the two-deep-pipeline tile kernel (gemm_tile3_kernel; K % 256 == 0, any number
    of stages incl. the loop's early exits): residual, folded-norm SiLU and f32 + row gather against
    the fp32 references, and bit-identical to the one-deep tile kernel (same k order per block)."""
    torch.manual_seed(70 + M + K)
    N = 1536
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    lin = ops.Linear(w)
    out3, out1 = r.clone(), r.clone()
    ops.linear(x, lin, out=out3, residual=out3, waves=-2)
    ops.linear(x, lin, out=out1, residual=out1, waves=-1)
    assert _rel_err(out3.float().cpu(), ref.linear_ref(x.cpu(), w.cpu(), None, r.cpu()).float()) < 1e-2
    assert torch.equal(out3, out1)
    I = 1024
    g = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    wg = (torch.randn(2 * I, K, device=DEV) / math.sqrt(K)).bfloat16()
    ls = ops.Linear(wg, kind="silu")
    ls.fold_norm(g)
    y = ops.linear(x, ls, norm=(g, 1e-6), waves=-2)
    xn, _ = ref.rmsnorm_ref(x.cpu(), g.cpu(), 1e-6)
    assert _rel_err(y.float().cpu(), ref.silu_mul_linear_ref(xn, wg[:I].cpu(), wg[I:].cpu()).float()) < 1e-2
    idx = torch.randperm(M, device=DEV)[: max(17, M // 2)].int()
    lf = ops.linear(x, lin, out_f32=True, row_idx=idx, waves=-2)
    assert _rel_err(lf.cpu(), ref.linear_ref(x[idx.long()].cpu(), w.cpu(), out_f32=True)) < 1e-2
    # QKV epilogue (bias + folded-norm row scale + RoPE + paged KV write), the prefill step's qkv form
    hq, hkv, D, BS = 12, 2, 128, 16
    Nq = (hq + 2 * hkv) * D
    wq = (torch.randn(Nq, K, device=DEV) / math.sqrt(K)).bfloat16()
    bq = (torch.randn(Nq, device=DEV) * 0.1).bfloat16()
    lq = ops.Linear(wq, bias=bq, layout="qkv")
    lq.fold_norm(g)
    pos = torch.randint(0, 1000, (M,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(64 * BS, device=DEV)[:M].int()
    cs = ref.rope_cos_sin(1024, D, 1e6, device=DEV)
    outs = []
    for wv in (-2, -1):
        kc = torch.zeros(64, hkv, BS, D, device=DEV).bfloat16()
        vc = torch.zeros_like(kc)
        q = ops.linear(x, lq, norm=(g, 1e-6), waves=wv, qkv=dict(positions=pos, slots=slots, cos_sin=cs,
                                                                 k_cache=kc, v_cache=vc, hq=hq, hkv=hkv))
        outs.append((q, kc, vc))
    xq = ref.linear_ref(xn, wq.cpu(), bq.cpu())
    kc2, vc2 = torch.zeros(64, hkv, BS, D).bfloat16(), torch.zeros(64, hkv, BS, D).bfloat16()
    ref.rope_kv_ref(xq, pos.cpu(), slots.cpu(), cs.cpu(), kc2, vc2, hq, hkv, D)
    (q3, k3, v3), (q1, k1, v1) = outs
    assert _rel_err(q3.float().cpu(), xq[:, : hq * D].float()) < 1e-2
    assert _rel_err(k3.float().cpu(), kc2.float()) < 1e-2 and _rel_err(v3.float().cpu(), vc2.float()) < 1e-2
    assert torch.equal(q3, q1) and torch.equal(k3, k1) and torch.equal(v3, v1)


def test_tile_kernel_no_residual_small_k_large_m():
    """The tile kernels prefetch every m-tile's epilogue words; without a residual (a TP follower's
    row-parallel GEMM) those reads must stay inside the packed weights at any M (round 6: M x N past
    a 256 x 256 matrix faulted the TP = 2 tests)."""
    torch.manual_seed(77)
    M, N, K = 640, 256, 256
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    y = ops.linear(x, ops.Linear(w), waves=-1)
    torch.cuda.synchronize()
    assert _rel_err(y.float().cpu(), ref.linear_ref(x.cpu(), w.cpu()).float()) < 1e-2


@pytest.mark.parametrize("layout", ["plain", "silu", "qkv"])
def test_awq_long_step_dequant_path(layout):
    """AWQ linear at M > 64 (a prefill step): int4 -> bf16 scratch (awq_dequant, RMSNorm gamma folded
    in) + the bf16 prefill kernel == the dequantised fp32 reference, for every epilogue."""
    torch.manual_seed(60)
    M, N, K, g = 256, 2048, 1536, 128
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    scales = (torch.rand(K // g, N) * 0.02 + 0.005).bfloat16()
    zeros = torch.randint(0, 16, (K // g, N)).float().bfloat16()
    wd = ref.awq_dequant_ref(q, scales, zeros, g).to(DEV)
    awq = {"qint": q, "scales": scales.to(DEV), "zeros": zeros.to(DEV), "group": g, "silu": layout == "silu"}
    if layout == "qkv":
        awq["layout"] = "qkv"
    lin = ops.Linear(None, awq=awq)
    assert lin.layout == layout and M >= ops.AWQ_DEQUANT_MIN_M
    assert _rel_err(lin.dense_weight().float(), wd.float()) < 1e-2  # original row order restored
    x = torch.randn(M, K, device=DEV).bfloat16()
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    if layout == "qkv":  # hq = 12, hkv = 2 heads of 128 -> N = 2048
        D, BS, hq, hkv = 128, 16, 12, 2
        pos = torch.randint(0, 1000, (M,), dtype=torch.int32, device=DEV)
        slots = torch.randperm(64 * BS, device=DEV)[:M].int()
        cs = ref.rope_cos_sin(1024, D, 1e6, device=DEV)
        kc = torch.zeros(64, hkv, BS, D, device=DEV).bfloat16()
        vc = torch.zeros_like(kc)
        qo = ops.linear(x, lin, norm=(nw, 1e-6), qkv=dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kc,
                                                          v_cache=vc, hq=hq, hkv=hkv))
        qkv = ref.linear_ref(xn, wd)
        kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
        ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, hq, hkv, D)
        assert _rel_err(qo, qkv[:, : hq * D]) < 2e-2
        assert _rel_err(kc, kc2) < 2e-2 and _rel_err(vc, vc2) < 2e-2
        return
    y = ops.linear(x, lin, norm=(nw, 1e-6))
    if layout == "silu":
        assert _rel_err(y, ref.silu_mul_linear_ref(xn, wd[: N // 2], wd[N // 2:])) < 2e-2
    else:
        assert _rel_err(y, ref.linear_ref(xn, wd)) < 2e-2


@pytest.mark.parametrize("M", [128, 200, 1024, 4096])
@pytest.mark.parametrize("bn,sk", [(0, 0), (64, 0), (128, 0), (64, 3), (256, 0), (256, 2), (512, 0), (512, 2),
                                   (1024, 0), (1024, 3), (768, 0), (768, 2), (1280, 0), (1281, 2), (640, 3),
                                   (641, 0), (1025, 0), (769, 0)])
def test_prefill_lds_gemm_all_epilogues(M, bn, sk):
    """The LDS-tiled MFMA prefill kernel (gemm_prefill.hip, path=1) on the decode kernels'
    fragment-packed weights, against the fp32 references: plain + in-place residual,
    folded-norm SiLU*mul, folded-norm QKV + bias + RoPE + paged KV write (rows past M masked,
    M not a multiple of the 128-row tile), for both tile widths and the heuristic, and with
    K split over blocks (partials + the deterministic reduce kernel; the heuristic splits the
    small grids of M = 128 / 200 by itself)."""
    torch.manual_seed(70 + M + bn)
    H, D, BS, hq, hkv, I = 1536, 128, 16, 12, 2, 1024
    x = (torch.randn(M, H, device=DEV) * 1.5).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    # plain + residual (o_proj / down class), K = 2 x H to cover a longer K loop
    K2 = 2 * H
    x2 = torch.randn(M, K2, device=DEV).bfloat16()
    w = (torch.randn(H, K2, device=DEV) / math.sqrt(K2)).bfloat16()
    res = torch.randn(M, H, device=DEV).bfloat16()
    out = res.clone()
    ops.native().gemm(x2, ops.Linear(w).wp, H, K2, out, 0, res=out, ws=ops.workspace(DEV), path=1, ntb=bn,
                      splitk=sk)
    assert _rel_err(out, ref.linear_ref(x2, w, None, res)) < 1e-2
    # SiLU*mul with the folded RMSNorm (gate_up class)
    wg = (torch.randn(I, H, device=DEV) / math.sqrt(H)).bfloat16()
    wu = (torch.randn(I, H, device=DEV) / math.sqrt(H)).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), layout="silu")
    assert gu.fold_norm(nw)
    h = torch.empty(M, I, dtype=torch.bfloat16, device=DEV)
    ops.native().gemm(x, gu.wp, 2 * I, H, h, 2, ws=ops.workspace(DEV), rownorm=True, eps=1e-6, path=1, ntb=bn,
                      splitk=sk)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel_err(h, ref.silu_mul_linear_ref(xn, wg, wu)) < 2e-2
    # QKV + bias + RoPE + paged KV write with the folded norm
    N = (hq + 2 * hkv) * D
    wq = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=DEV)
    nblk = (M + BS - 1) // BS + 8
    slots = torch.randperm(nblk * BS, device=DEV)[:M].int()
    slots[min(4, M - 1)] = -1
    cs = ref.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc = torch.zeros(nblk, hkv, BS, D, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    lq = ops.Linear(wq, bias=b, layout="qkv")
    assert lq.fold_norm(nw)
    q = torch.empty(M, hq * D, dtype=torch.bfloat16, device=DEV)
    ops.native().gemm(x, lq.wp, N, H, q, 3, bias=b, ws=ops.workspace(DEV), rownorm=True, eps=1e-6, positions=pos,
                      slots=slots, cos_sin=cs, k_cache=kc, v_cache=vc, hq=hq, hkv=hkv, path=1, ntb=bn, splitk=sk)
    qkv = ref.linear_ref(xn, wq, b)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, hq, hkv, D)
    assert _rel_err(q, qkv[:, : hq * D]) < 2e-2
    assert _rel_err(kc, kc2) < 2e-2 and _rel_err(vc, vc2) < 2e-2


@pytest.mark.parametrize("M", [200, 448, 640])
@pytest.mark.parametrize("bn,sk", [(2560, 0), (2561, 0), (2560, 2), (2561, 3)])
def test_prefill_wide_tiles(M, bn, sk):
    """The wide-N mid-M prefill tiles (gemm_prefill.hip: 64 x 512 and 128 x 320) against
    the fp32 references: plain + in-place residual and folded-norm SiLU*mul, N = 2560 (both tiles
    divide it), rows past M masked, K split + reduce."""
    torch.manual_seed(90 + M + bn + sk)
    H, N = 1536, 2560
    x = (torch.randn(M, H, device=DEV) * 1.5).bfloat16()
    w = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    out = res.clone()
    ops.native().gemm(x, ops.Linear(w).wp, N, H, out, 0, res=out, ws=ops.workspace(DEV), path=1, ntb=bn, splitk=sk)
    assert _rel_err(out, ref.linear_ref(x, w, None, res)) < 1e-2
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    wg = (torch.randn(N // 2, H, device=DEV) / math.sqrt(H)).bfloat16()
    wu = (torch.randn(N // 2, H, device=DEV) / math.sqrt(H)).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), layout="silu")
    assert gu.fold_norm(nw)
    h = torch.empty(M, N // 2, dtype=torch.bfloat16, device=DEV)
    ops.native().gemm(x, gu.wp, N, H, h, 2, ws=ops.workspace(DEV), rownorm=True, eps=1e-6, path=1, ntb=bn, splitk=sk)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel_err(h, ref.silu_mul_linear_ref(xn, wg, wu)) < 2e-2


@pytest.mark.parametrize("M,N,K,slices", [(448, 2560, 1536, 0), (1024, 7168, 1024, 0), (2048, 3584, 2048, 0),
                                          (640, 5120, 4096, 0), (2048, 9216, 1024, 0), (2048, 6144, 4096, 0),
                                          (640, 5120, 4096, 7), (448, 2560, 1536, 3)])
@pytest.mark.parametrize("bn", [1025, 769])
def test_prefill_persistent_k_split_tail(M, N, K, slices, bn):
    """The persistent 4-phase prefill kernel (gemm_prefill4sk_kernel): whole rounds of tiles, then the
    last round's tiles as 2-6 K slices met in-launch (the owner adds the published partials in
    slice order), or unsplit where the tail already fills the chip; tails of several rounds (Llama-3-8B
    qkv_proj at 2048 rows: 192 tiles x 4 slices; forced 7 slices of 60 tiles). Against the fp32 references
    (plain + residual, folded-norm SiLU*mul with the partial sums of squares), bit-identical on a
    repeat (fixed add order, tickets reset by the owner), and the fault word clear (no ticket poll
    gave up)."""
    torch.manual_seed(M + N + K + bn)
    fw = ops.fault_word(DEV)
    fw.zero_()
    x = (torch.randn(M, K, device=DEV) * 1.5).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    lin = ops.Linear(w)
    res = torch.randn(M, N, device=DEV).bfloat16()
    outs = []
    for _ in range(2):
        out = res.clone()
        ops.native().gemm(x, lin.wp, N, K, out, 0, res=out, ws=ops.workspace(DEV), path=1, ntb=bn, splitk=slices,
                          fault=fw)
        outs.append(out)
    assert _rel_err(outs[0], ref.linear_ref(x, w, None, res)) < 1e-2
    assert torch.equal(outs[0], outs[1])
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    wg = (torch.randn(N // 2, K, device=DEV) / math.sqrt(K)).bfloat16()
    wu = (torch.randn(N // 2, K, device=DEV) / math.sqrt(K)).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), layout="silu")
    assert gu.fold_norm(nw)
    hs = []
    for _ in range(2):
        h = torch.empty(M, N // 2, dtype=torch.bfloat16, device=DEV)
        ops.native().gemm(x, gu.wp, N, K, h, 2, ws=ops.workspace(DEV), rownorm=True, eps=1e-6, path=1, ntb=bn,
                          splitk=slices, fault=fw)
        hs.append(h)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel_err(hs[0], ref.silu_mul_linear_ref(xn, wg, wu)) < 2e-2
    assert torch.equal(hs[0], hs[1])
    torch.cuda.synchronize()
    assert int(fw[0].item()) == 0


@pytest.mark.parametrize("M", [17, 24, 40, 48, 64])
@pytest.mark.parametrize("w,s_long,s_short", [(0, 0, 0), (4, 6, 2), (4, 8, 3), (2, 12, 4), (1, 16, 6), (4, 7, 16),
                                              (8, 0, 0)])
def test_mid_gemm_all_epilogues(M, w, s_long, s_short):
    """The medium-M kernel (gemm_mid.hip, path=2: x slice DMA'd into LDS, every weight fragment of a
    wave's tile slice in flight, K slices combined by the reduce kernel) against the fp32
    references: plain + in-place residual over a long K (192 k-steps), folded-norm SiLU*mul,
    folded-norm QKV + bias + RoPE + paged KV write; rows past M (partial m-tiles) masked; the
    heuristic and forced (tiles per block, K slices) decompositions."""
    torch.manual_seed(170 + M + 7 * w + s_short)
    H, D, BS, hq, hkv, I = 1536, 128, 16, 12, 2, 1024
    C, ws = ops.native(), ops.workspace(DEV)
    x = (torch.randn(M, H, device=DEV) * 1.5).bfloat16()
    nw = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    K2 = 4 * H
    x2 = torch.randn(M, K2, device=DEV).bfloat16()
    wd = (torch.randn(H, K2, device=DEV) / math.sqrt(K2)).bfloat16()
    res = torch.randn(M, H, device=DEV).bfloat16()
    out = res.clone()
    C.gemm(x2, ops.Linear(wd).wp, H, K2, out, 0, res=out, ws=ws, path=2, waves=w, splitk=s_long)
    assert _rel_err(out, ref.linear_ref(x2, wd, None, res)) < 1e-2
    wg = (torch.randn(I, H, device=DEV) / math.sqrt(H)).bfloat16()
    wu = (torch.randn(I, H, device=DEV) / math.sqrt(H)).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), layout="silu")
    assert gu.fold_norm(nw)
    h = torch.empty(M, I, dtype=torch.bfloat16, device=DEV)
    C.gemm(x, gu.wp, 2 * I, H, h, 2, ws=ws, rownorm=True, eps=1e-6, path=2, waves=w, splitk=s_short)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel_err(h, ref.silu_mul_linear_ref(xn, wg, wu)) < 2e-2
    N = (hq + 2 * hkv) * D
    wq = (torch.randn(N, H, device=DEV) / math.sqrt(H)).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=DEV)
    nblk = (M + BS - 1) // BS + 8
    slots = torch.randperm(nblk * BS, device=DEV)[:M].int()
    slots[min(4, M - 1)] = -1
    cs = ref.rope_cos_sin(4096, D, 1e6, device=DEV)
    kc = torch.zeros(nblk, hkv, BS, D, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    lq = ops.Linear(wq, bias=b, layout="qkv")
    assert lq.fold_norm(nw)
    q = torch.empty(M, hq * D, dtype=torch.bfloat16, device=DEV)
    C.gemm(x, lq.wp, N, H, q, 3, bias=b, ws=ws, rownorm=True, eps=1e-6, positions=pos, slots=slots, cos_sin=cs,
           k_cache=kc, v_cache=vc, hq=hq, hkv=hkv, path=2, waves=w, splitk=s_short)
    qkv = ref.linear_ref(xn, wq, b)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref.rope_kv_ref(qkv, pos, slots, cs, kc2, vc2, hq, hkv, D)
    assert _rel_err(q, qkv[:, : hq * D]) < 2e-2
    assert _rel_err(kc, kc2) < 2e-2 and _rel_err(vc, vc2) < 2e-2


@pytest.mark.parametrize("M", [1, 8, 16, 20, 32, 48, 64])
@pytest.mark.parametrize("I,K", [(8960, 1536), (1000 * 8, 2048), (128, 512)])
def test_mid_wide_gemm_silu(M, I, K):
    """The wide medium-M kernel (one block per CU owning whole tiles, K in 16-k-step parts met in
    LDS, x by m-tile pairs): Qwen2.5-1.5B gate_up (1120 tiles: 4-5 per block, idle part-waves in the
    4-tile blocks), a 1000-tile / 64-k-step shape and a one-block-per-tile one, folded-norm SiLU*mul
    against the fp32 reference."""
    torch.manual_seed(300 + M + I)
    x = (torch.randn(M, K, device=DEV) * 1.5).bfloat16()
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    wg = (torch.randn(I, K, device=DEV) / math.sqrt(K)).bfloat16()
    wu = (torch.randn(I, K, device=DEV) / math.sqrt(K)).bfloat16()
    gu = ops.Linear(torch.cat([wg, wu]), layout="silu")
    assert gu.fold_norm(nw)
    h = torch.empty(M, I, dtype=torch.bfloat16, device=DEV)
    ops.native().gemm(x, gu.wp, 2 * I, K, h, 2, ws=ops.workspace(DEV), rownorm=True, eps=1e-6, path=2, waves=8)
    xn, _ = ref.rmsnorm_ref(x, nw, 1e-6)
    assert _rel_err(h, ref.silu_mul_linear_ref(xn, wg, wu)) < 2e-2


def test_mid_gemm_plans_in_linear():
    """ops.linear consults a medium bucket's plan: a tuned entry routes 16 < M <= 64 rows to the
    medium kernel, MEDIUM_DEFAULT keeps the default path, and both agree with the reference."""
    torch.manual_seed(77)
    K = 1536
    lin = ops.Linear((torch.randn(2048, K, device=DEV) / math.sqrt(K)).bfloat16())
    x = torch.randn(48, K, device=DEV).bfloat16()
    want = ref.linear_ref(x, lin.dense_weight())
    for cfg in [ops.MEDIUM_DEFAULT, (ops.MID_BASE - 4, 0), (ops.MID_BASE - 2, 4), (ops.MID_BASE - 8, 0), (64, 0)]:
        lin.prefill_plan = {48: cfg, 128: (0, 0)}
        assert _rel_err(ops.linear(x, lin), want) < 1e-2, cfg
    assert ops._plan_kw((ops.MID_BASE - 4, 3), 48) == dict(path=2, waves=4, splitk=3)
    assert ops._plan_kw(ops.MEDIUM_DEFAULT, 48) == {}


def test_kernel_copy_host_device_round_trip():
    """ops.host_device_copy: pinned host -> device and device -> pinned host by the copy kernel
    (16-B pieces, sizes rounded up to 16 inside both tensors), ordered on the current stream."""
    C = ops.native()
    src = torch.randint(0, 2**31 - 1, (4096,), dtype=torch.int32).pin_memory()
    dev = torch.zeros(4096, dtype=torch.int32, device=DEV)
    back = torch.zeros(4096, dtype=torch.int32).pin_memory()
    for nbytes in (16, 4000, 16384):
        dev.zero_()
        back.zero_()
        C.kernel_copy(dev, src, nbytes)
        C.kernel_copy(back, dev, nbytes)
        torch.cuda.synchronize()
        n = (nbytes + 15) // 16 * 4
        assert torch.equal(back[:n], src[:n]), nbytes
        assert int(back[n:].abs().sum()) == 0 and int(dev[n:].abs().sum()) == 0
    with pytest.raises(RuntimeError):
        C.kernel_copy(dev, src, 4096 * 4 + 16)  # past the tensors


def test_tune_prefill_plans_match_heuristic_results():
    """ops.tune_prefill: plans for every planned M bucket, and a planned (tile, K-slices) linear
    gives the launcher's result within bf16 split-K rounding for plain / SiLU / residual layers."""
    torch.manual_seed(71)
    K = 1536
    lins = [ops.Linear((torch.randn(2048, K, device=DEV) / math.sqrt(K)).bfloat16()),
            ops.Linear((torch.randn(2 * 2240, K, device=DEV) / math.sqrt(K)).bfloat16(), kind="silu")]
    plans = ops.tune_prefill(lins, [128, 384])
    assert set(plans) == {(2048, K), (2 * 2240, K)}
    for lin in lins:
        assert set(lin.prefill_plan) == {128, 384}
        for M in (100, 384):  # 100 rows: below the prefill path, the plan is not consulted
            x = torch.randn(M, K, device=DEV).bfloat16()
            res = torch.randn(M, lin.out_features, device=DEV).bfloat16() if lin.layout == "plain" else None
            y = ops.linear(x, lin, residual=res)
            plan, lin.prefill_plan = lin.prefill_plan, {}
            y0 = ops.linear(x, lin, residual=res)
            lin.prefill_plan = plan
            assert _rel_err(y, y0) < 1e-2, (lin.layout, M)


@pytest.mark.parametrize("M", [3, 8, 12])
def test_decode_gemm_register_groups_bit_identical(M):
    """The decode GEMM's register group size (k-steps per in-flight group: auto, the round-2
    rule, forced 6 / 8 / 10 / 12) changes only how the loads are batched, never the per-wave
    accumulation order: every size gives the same bits, and matches the fp32 reference
    (down_proj shape with residual + split-K, gate_up SiLU with folded RMSNorm)."""
    C = ops.native()
    torch.manual_seed(70 + M)
    try:
        for N, K, kind, waves, splitk in ((1536, 8960, "plain", 8, 2), (1024, 1536, "silu", 2, 1),
                                          (2048, 1536, "plain", 8, 1)):
            x = torch.randn(M, K, device=DEV).bfloat16()
            w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
            g = (torch.rand(K, device=DEV) + 0.5).bfloat16()
            lin = ops.Linear(w, kind=kind) if kind == "silu" else ops.Linear(w)
            if kind == "silu":
                lin.fold_norm(g)
            res = torch.randn(M, N // (2 if kind == "silu" else 1), device=DEV).bfloat16()
            outs = []
            for u in (0, -1, 6, 8, 10, 12):
                C.set_dec_u(u)
                if kind == "silu":
                    y = ops.linear(x, lin, norm=(g, 1e-6), waves=waves, splitk=splitk)
                else:
                    y = res.clone()
                    ops.linear(x, lin, out=y, residual=y, waves=waves, splitk=splitk)
                outs.append(y)
            for u, y in zip((0, -1, 6, 8, 10, 12), outs):
                assert torch.equal(y, outs[0]), (N, K, kind, u)
            if kind == "silu":
                xn, _ = ref.rmsnorm_ref(x.cpu(), g.cpu(), 1e-6)
                r = ref.silu_mul_linear_ref(xn, w.cpu()[: N // 2], w.cpu()[N // 2:])
            else:
                r = ref.linear_ref(x.cpu(), w.cpu(), None, res.cpu())
            assert _rel_err(outs[0].float().cpu(), r.float()) < 1e-2, (N, K, kind)
    finally:
        C.set_dec_u(-100)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (12, 2), (8, 1), (16, 16)])
def test_flash_prefill_matches_tile_kernel_and_reference(Hq, Hkv):
    """Flash prefill (64- / 32-query blocks x the G heads of a KV head, K / V double-buffered in LDS
    by DMA) == the 16-query tile kernel and the fp32 reference: ragged prompts, chunked prefill
    against cached tokens, padding tiles of a graph bucket (tile_seq = -1), and a mixed step with
    decode rows through the unified launch (decode rows keep the decode kernel)."""
    C = ops.native()
    torch.manual_seed(200 + Hq + Hkv)
    D = 128
    qlens = [1, 33, 64, 65, 200, 1]
    ctxs = [40, 33, 300, 65, 456, 77]
    S = len(qlens)
    maxb = max(ctxs) // 16 + 2
    nblk = S * maxb + 4
    kc, vc = _make_cache(nblk, Hkv, seed=5)
    bt = (torch.randperm(nblk)[: S * maxb]).reshape(S, maxb).int().to(DEV)
    qs = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(qs[-1])
    cl = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    stride = (Hq + 2 * Hkv) * D
    qkv = torch.randn(T, stride, device=DEV).bfloat16()
    ts, tq = ops.prefill_tiles(qlens, ops.flash_lead(Hq, Hkv))  # the engine's tile order
    ts, tq = ts + [-1] * 5, tq + [0] * 5  # a bucket's padding tiles
    ts = torch.tensor(ts, dtype=torch.int32, device=DEV)
    tq = torch.tensor(tq, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    outs = []
    try:
        for on in (1, 0):
            C.set_flash_prefill(on)
            out = torch.zeros(T, Hq * D, device=DEV).bfloat16()
            ops.attention_prefill(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out, Hq, Hkv, scale)
            outs.append(out)
        q = qkv[:, : Hq * D].reshape(T, Hq, D)
        r = ref.attention_ref(q, kc, vc, bt, cl, qs.cpu(), Hq, Hkv, scale)
        assert _rel_err(outs[0].view(T, Hq, D), r) < 2e-2
        assert _rel_err(outs[0], outs[1]) < 1e-2
        # mixed step: the unified launch with decode rows (query length 1 sequences) and prefill tiles
        C.set_flash_prefill(1)
        P = 4
        po = torch.empty(S, Hq, P, D, device=DEV)
        pml = torch.empty(S, Hq, P, 2, device=DEV)
        out = torch.zeros(T, Hq * D, device=DEV).bfloat16()
        ops.attention(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out, po, pml, Hq, Hkv, 512, scale)
        assert _rel_err(out.view(T, Hq, D), r) < 2e-2
        # the K split (ranges of >= 4 chunks as two halves met through the workspace, ctx 300 / 456
        # here) is deterministic and matches the unsplit kernel
        assert ops.FLASH_SPLIT
        out2 = torch.zeros_like(out)
        ops.attention(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out2, po, pml, Hq, Hkv, 512, scale)
        assert torch.equal(out, out2)
        ops.FLASH_SPLIT = False
        out3 = torch.zeros_like(out)
        ops.attention(qkv, stride, kc, vc, bt, cl, qs, ts, tq, out3, po, pml, Hq, Hkv, 512, scale)
        assert _rel_err(out, out3) < 1e-2
    finally:
        ops.FLASH_SPLIT = True
        C.set_flash_prefill(-1)
