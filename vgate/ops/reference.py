"""Pure-PyTorch fp32 reference implementations of every vgate kernel.

Two roles:
  * numerics oracle for the HIP kernels (tests compare GPU kernels against these),
  * the CPU execution path, so the whole engine (scheduler, KV manager, sampler
    bookkeeping, HTTP stack) runs and is tested on a machine without a GPU.

They are deliberately written for clarity, not speed.
"""
from __future__ import annotations

import math

import torch


def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None):
    """Returns (y, new_residual). Mirrors HF RMSNorm rounding (normalise in f32, cast, scale)."""
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
    else:
        s = x
    xf = s.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    y = ((xf * inv).to(x.dtype).float() * w.float()).to(x.dtype)
    return y, (s if residual is not None else None)


def embedding_ref(ids: torch.Tensor, table: torch.Tensor, vstart: int = 0) -> torch.Tensor:
    local = ids.long() - vstart
    ok = (local >= 0) & (local < table.shape[0])
    out = table[local.clamp(0, table.shape[0] - 1)]
    return out * ok.unsqueeze(-1).to(out.dtype)


def linear_ref(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, out_f32=False):
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if out_f32:
        return y
    y = y.to(torch.bfloat16)
    if residual is not None:
        y = (y.float() + residual.float()).to(torch.bfloat16)
    return y


def silu_mul_linear_ref(x: torch.Tensor, w_gate: torch.Tensor, w_up: torch.Tensor) -> torch.Tensor:
    g = x.float() @ w_gate.float().t()
    u = x.float() @ w_up.float().t()
    return (torch.nn.functional.silu(g) * u).to(torch.bfloat16)


def rope_cos_sin(max_pos: int, dim: int, theta: float, scaling: dict | None = None,
                 device="cpu") -> torch.Tensor:
    """[max_pos, dim] f32 table: first half cos, second half sin (NeoX layout)."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    elif scaling and scaling.get("rope_type", scaling.get("type")) == "linear":
        inv = inv / scaling.get("factor", 1.0)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def rope_kv_ref(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D):
    """In-place NeoX rotary on q,k of `qkv` [T, (Hq+2Hkv)*D]; writes k,v to the paged cache."""
    T = qkv.shape[0]
    if T == 0:
        return
    v3 = qkv.view(T, Hq + 2 * Hkv, D)
    half = D // 2
    cs = cos_sin[positions.long()]  # [T, D]
    c, s = cs[:, None, :half], cs[:, None, half:]
    qk = v3[:, : Hq + Hkv].float()
    x1, x2 = qk[..., :half], qk[..., half:]
    rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(qkv.dtype)
    v3[:, : Hq + Hkv] = rot
    if slots is None:
        return
    BS = k_cache.shape[2]
    sl = slots.long()
    ok = sl >= 0
    if ok.any():
        idx = torch.nonzero(ok).squeeze(-1)
        blk, off = sl[idx] // BS, sl[idx] % BS
        k_cache[blk, :, off] = v3[idx, Hq:Hq + Hkv]
        v_cache[blk, :, off] = v3[idx, Hq + Hkv:]


def _gather_kv(cache, table_row, n):
    BS = cache.shape[2]
    nb = (n + BS - 1) // BS
    blocks = table_row[:nb].long()
    kv = cache[blocks]  # [nb, H, BS, D]
    return kv.permute(1, 0, 2, 3).reshape(cache.shape[1], nb * BS, cache.shape[3])[:, :n]


def attention_ref(q, k_cache, v_cache, block_tables, context_lens, query_start, Hq, Hkv, scale):
    """Varlen causal attention over the paged cache. q: [T, Hq, D] (any row stride).

    query_start: [S+1] cumulative query counts (decode: arange(S+1)).
    Returns [T, Hq, D] in q.dtype.
    """
    T = q.shape[0]
    D = q.shape[-1]
    out = torch.zeros(T, Hq, D, dtype=q.dtype, device=q.device)
    G = Hq // Hkv
    qs = query_start.tolist()
    cl = context_lens.tolist()
    for s in range(len(cl)):
        a, b = qs[s], qs[s + 1]
        ql, ctx = b - a, cl[s]
        if ql <= 0 or ctx <= 0:
            continue
        K = _gather_kv(k_cache, block_tables[s], ctx).float()  # [Hkv, ctx, D]
        V = _gather_kv(v_cache, block_tables[s], ctx).float()
        K = K.repeat_interleave(G, dim=0)
        V = V.repeat_interleave(G, dim=0)
        qq = q[a:b].float().transpose(0, 1)  # [Hq, ql, D]
        sc = (qq @ K.transpose(1, 2)) * scale  # [Hq, ql, ctx]
        qpos = torch.arange(ctx - ql, ctx, device=q.device)[:, None]
        kpos = torch.arange(ctx, device=q.device)[None, :]
        sc = sc.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(sc, dim=-1)
        out[a:b] = (p @ V).transpose(0, 1).to(q.dtype)
    return out


def sample_ref(logits, temperature, top_p, top_k, generators=None):
    """Reference sampler (sort based). Returns int32 [B]."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32)
    for i in range(B):
        row = logits[i].float()
        t = float(temperature[i]) if temperature is not None else 0.0
        if t <= 1e-5:
            out[i] = int(torch.argmax(row))
            continue
        probs = torch.softmax(row / t, dim=-1)
        sp, si = torch.sort(probs, descending=True)
        keep = torch.ones_like(sp, dtype=torch.bool)
        k = int(top_k[i]) if top_k is not None else -1
        if 0 < k < V:
            keep[k:] = False
        p = float(top_p[i]) if top_p is not None else 1.0
        if p < 1.0:
            csum = torch.cumsum(sp, 0)
            excl = csum - sp
            keep &= excl < p
        sp = sp * keep
        g = generators[i] if generators is not None else None
        j = torch.multinomial(sp.cpu(), 1, generator=g)
        out[i] = int(si[j])
    return out


def awq_dequant_ref(qint: torch.Tensor, scales: torch.Tensor, zeros: torch.Tensor, group: int):
    """qint: [N, K] int (0..15); scales/zeros: [K/group, N] -> bf16 [N, K] weight (w = (q - z) * s)."""
    N, K = qint.shape
    s = scales.float().t().repeat_interleave(group, dim=1)  # [N, K]
    z = zeros.float().t().repeat_interleave(group, dim=1)
    return ((qint.float() - z) * s).to(torch.bfloat16)
