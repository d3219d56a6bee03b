"""Decoder-only transformer (Qwen2 / Llama families) on the vgate kernel set.

One forward pass = one engine step over a flat token batch (any mix of decode
tokens and prefill chunks), reading all step metadata from device buffers
(:class:`vgate.runtime.step_meta.StepView`) so the identical code path is
captured into a hipGraph per token-count bucket.

Per layer (TP degree t, Megatron layout):
    x    = rmsnorm(resid)                              K2
    qkv  = x @ Wqkv^T + b           column-parallel    K3 (MFMA, fused bias)
    rope(q, k); k, v -> paged cache                    K4
    a    = paged attention(q)       heads sharded      K5 / K6
    resid = resid + a @ Wo^T        row-parallel       K7 (+residual epilogue) -> C1 all-reduce
    x    = rmsnorm(resid)                              K2
    h    = silu(x Wg^T) * (x Wu^T)  column-parallel    K8 (fused SiLU*mul epilogue)
    resid = resid + h @ Wd^T        row-parallel       K9 (+residual epilogue) -> C1
The residual add of a row-parallel GEMM is applied by TP rank 0 only, so the
all-reduce of the partial outputs yields resid + sum(partials) on every rank
with no extra kernel.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from vgate import ops
from vgate.models.config import ModelArch
from vgate.parallel.comm import TPGroup

# the measured per-shape decode decompositions (vgate/models/decode_plans.py) at model construction;
# the decode sweeps turn this off to time the launcher's heuristic
APPLY_DECODE_PLANS = True
# TP comm / compute overlap of long steps: row-parallel GEMMs of >= TP_OVERLAP_MIN_TOKENS rows run in
# TP_OVERLAP_CHUNKS row chunks, chunk i's all-reduce on a side stream under chunk i+1's GEMM
TP_OVERLAP_CHUNKS = 4
TP_OVERLAP_MIN_TOKENS = 256


@dataclass
class LayerWeights:
    in_norm: torch.Tensor
    qkv: ops.Linear
    o: ops.Linear
    post_norm: torch.Tensor
    gate_up: ops.Linear
    down: ops.Linear


class ShardSpec:
    """Per-rank sizes for a TP degree."""

    def __init__(self, arch: ModelArch, tp: TPGroup):
        self.tp = tp
        t, r = tp.size, tp.rank
        if arch.num_heads % t:
            raise ValueError(f"num_heads {arch.num_heads} not divisible by tp {t}")
        self.hq = arch.num_heads // t
        if arch.num_kv_heads >= t:
            if arch.num_kv_heads % t:
                raise ValueError("num_kv_heads not divisible by tp")
            self.hkv = arch.num_kv_heads // t
            self.kv_head0 = r * self.hkv
        else:  # replicate KV heads across ranks (e.g. Qwen 2 KV heads at tp 4/8)
            if t % arch.num_kv_heads:
                raise ValueError("tp not a multiple of num_kv_heads")
            self.hkv = 1
            self.kv_head0 = r // (t // arch.num_kv_heads)
        self.q_head0 = r * self.hq
        if arch.intermediate_size % (16 * t):
            raise ValueError("intermediate_size must split into 16-row tiles per rank")
        self.inter = arch.intermediate_size // t
        self.inter0 = r * self.inter
        vpad = ((arch.vocab_size + 16 * t - 1) // (16 * t)) * 16 * t
        self.vocab_padded = vpad
        self.vocab = vpad // t
        self.vocab0 = r * self.vocab


class DecoderModel:
    def __init__(self, arch: ModelArch, device: torch.device | str, tp: TPGroup | None = None,
                 quantization: str | None = None, seed: int = 0, weights_path: str | None = None,
                 max_model_len: int = 4096):
        self.arch = arch
        self.device = torch.device(device)
        self.tp = tp or TPGroup()
        self.shard = ShardSpec(arch, self.tp)
        self.quant = (quantization or "").lower() or None
        if self.device.type == "cuda" and arch.head_dim != 128:
            raise ValueError("the gfx950 attention kernels require head_dim == 128")
        self.max_model_len = max_model_len
        self.scale = 1.0 / math.sqrt(arch.head_dim)
        if weights_path:
            from vgate.models.weights import load_checkpoint
            load_checkpoint(self, weights_path)
        else:
            from vgate.models.weights import random_init
            random_init(self, seed)
        if self.device.type == "cuda" and self.quant == "awq":
            # long AWQ steps: int4 -> bf16 dequant of one matrix at a time into a shared scratch
            # (ops.linear), sized once here so graph capture never allocates
            lins = [lin for L in self.layers for lin in (L.qkv, L.o, L.gate_up, L.down)]
            ops.reserve_awq_scratch(self.device, max(lin.N * lin.K for lin in lins if lin.kind == "awq"))
        if self.device.type == "cuda":
            self.fold_norms()
        if APPLY_DECODE_PLANS:  # measured decode decompositions per shape
            from vgate.models import decode_plans
            decode_plans.apply(self)
        table_len = max(max_model_len, 16) + 1
        self.cos_sin = ops.ref.rope_cos_sin(table_len, arch.head_dim, arch.rope_theta, arch.rope_scaling,
                                            device=self.device)
        # TP comm/compute overlap for long steps (prefill): row-parallel GEMMs run in row
        # chunks and chunk i's all-reduce runs on a side stream while chunk i+1's GEMM runs
        self.tp_overlap_chunks = TP_OVERLAP_CHUNKS
        self.tp_overlap_min_tokens = TP_OVERLAP_MIN_TOKENS
        self.comm_stream = (torch.cuda.Stream(self.device)
                            if self.device.type == "cuda" and self.tp.size > 1 else None)

    def fold_norms(self) -> int:
        """Fold every RMSNorm weight into the packed matrix of the GEMM that consumes it
        (qkv <- input_layernorm, gate_up <- post_attention_layernorm, LM head <- final norm);
        the fused GEMMs then apply only the deferred per-row scale. Dense bf16 only."""
        n = 0
        for L in self.layers:
            n += L.qkv.fold_norm(L.in_norm) + L.gate_up.fold_norm(L.post_norm)
        return n + self.lm_head.fold_norm(self.final_norm)

    # ------------------------------------------------------------------ sizes
    @property
    def num_kv_heads_local(self) -> int:
        return self.shard.hkv

    @property
    def num_heads_local(self) -> int:
        return self.shard.hq

    def weight_bytes(self) -> int:
        n = self.embed.numel() * 2 + self.final_norm.numel() * 2 + self.lm_head.nbytes()
        for L in self.layers:
            n += L.qkv.nbytes() + L.o.nbytes() + L.gate_up.nbytes() + L.down.nbytes() + 4 * L.in_norm.numel()
        return n

    # ---------------------------------------------------------------- forward
    def _row_parallel(self, x: torch.Tensor, lin, resid: torch.Tensor, first: bool, norm_out: tuple | None = None) -> None:
        """resid = all_reduce(x @ W^T [+ resid on TP rank 0]) for a row-parallel linear
        (o_proj / down_proj). With TP and >= tp_overlap_min_tokens rows the GEMM runs in
        row chunks (multiples of 16) and each chunk's all-reduce is issued on the comm
        stream as soon as that chunk is written, so RCCL (or the custom xGMI kernel) moves
        chunk i while the MFMA GEMM computes chunk i+1; the main stream joins the comm
        stream before the next layer reads ``resid``. Fork/join through events, so the
        pattern is captured into the prefill hipGraphs as well."""
        tp = self.tp
        T = x.shape[0]
        nch = self.tp_overlap_chunks if tp.size > 1 and T >= self.tp_overlap_min_tokens else 1
        car = tp.custom_ar if tp.size > 1 else None
        if nch <= 1 and car is not None and norm_out is None and resid.is_cuda and car.fuses(lin, x, resid):
            # decode rows: the all-reduce runs in the GEMM's epilogue (every rank sums the ranks'
            # fp32 partials in rank order, then adds the residual): one launch, no copy-in
            ops.linear(x, lin, out=resid, residual=resid, ar=car)
            car.calls += 1
            return
        if nch <= 1:
            ops.linear(x, lin, out=resid, residual=resid if first else None, norm_out=norm_out)
            if tp.size > 1:
                tp.all_reduce(resid)
            return
        bounds = sorted({min(T, 16 * ((T * i // nch + 15) // 16)) for i in range(nch)} | {T})
        if bounds[0] != 0:
            bounds.insert(0, 0)
        side = self.comm_stream if resid.is_cuda else None
        main = torch.cuda.current_stream(resid.device) if side is not None else None
        for a, b in zip(bounds[:-1], bounds[1:]):
            r = resid[a:b]
            ops.linear(x[a:b], lin, out=r, residual=r if first else None)
            if side is None:
                tp.all_reduce(r)
                continue
            ev = torch.cuda.Event()
            ev.record(main)
            with torch.cuda.stream(side):
                side.wait_event(ev)
                tp.all_reduce(r)
        if side is not None:
            main.wait_stream(side)

    def forward(self, sv, kv_caches, part_size: int, return_hidden: bool = False) -> torch.Tensor:
        """One step. ``sv`` is a StepView (token/seq metadata views, bucket sizes T and S).

        Returns f32 logits [S, vocab] for the sample rows (one per sequence), or with
        ``return_hidden`` the residual stream [T, H] after the last layer (embeddings).
        GPU: 4 fused GEMM launches + 1 attention launch per layer (RMSNorm, RoPE, KV
        write, bias, SiLU*mul and residual adds all live inside them).
        """
        if self.device.type != "cuda":
            return self._forward_reference(sv, kv_caches, part_size, return_hidden)
        a = self.arch
        sh = self.shard
        tp = self.tp
        T, S = sv.T, sv.S
        D = a.head_dim
        dev = self.device
        # RMSNorms are folded into the consuming GEMMs (deferred row scale), so a layer is
        # qkv GEMM -> attention -> o GEMM (+residual) -> gate_up GEMM -> down GEMM (+residual).
        resid = ops.embedding(sv.ids, self.embed, vstart=sh.vocab0, prev=sv.prev_tokens)
        if tp.size > 1:
            tp.all_reduce(resid)
        q = torch.empty(T, sh.hq * D, dtype=torch.bfloat16, device=dev)
        attn = torch.empty(T, sh.hq * D, dtype=torch.bfloat16, device=dev)
        mlp = torch.empty(T, sh.inter, dtype=torch.bfloat16, device=dev)
        P = max(1, (self.max_model_len + part_size - 1) // part_size)
        part_o = torch.empty(S, sh.hq, P, D, dtype=torch.float32, device=dev)
        part_ml = torch.empty(S, sh.hq, P, 2, dtype=torch.float32, device=dev)
        first = tp.is_first
        eps = a.rms_eps
        # int4 decode steps: the residual GEMMs (o_proj, down_proj) hand the NEXT RMSNorm over —
        # h * gamma plus per-tile sums of h^2 — so the int4 qkv / gate_up kernels read normed rows
        # (no gamma loads, no x^2 pass; ops.linear norm_out / prenorm)
        # decode steps (TP = 1): the residual GEMMs (o_proj, down_proj) hand the NEXT RMSNorm over — the
        # per-(row, 16-column tile) sums of h^2 of the rows they store — so the consumer (qkv, gate_up)
        # applies the row scale from them: no x^2 pass beside its weight stream (ops.linear norm_out /
        # prenorm). int4 consumers also get hg = h * gamma (their weights carry no gamma); bf16 consumers
        # read h itself (gamma folded into the packed weights), except on a stream-K plan (no hand-off there)
        hand = tp.size == 1 and T <= 16 and dev.type == "cuda"
        awq = self.quant == "awq"
        if hand:
            hg = torch.empty(T, a.hidden_size, dtype=torch.bfloat16, device=dev) if awq else None
            ssp = torch.empty(T, a.hidden_size // 16, dtype=torch.float32, device=dev)
        nl = len(self.layers)

        def takes(lin) -> bool:  # a consumer of the hand-off
            return hand and (awq or (lin.norm_gamma is not None and not lin.dec_sk))

        # decode-only steps (T <= S: no prefill tiles, StepMeta.tile_cap): the decode attention rides in
        # the QKV projection's launch (ops.linear attn=, csrc/kernels/qkv_attn.hip)
        fuse_attn = T <= S and T <= 16
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            qkv_args = dict(positions=sv.positions, slots=sv.slots, cos_sin=self.cos_sin, k_cache=kc, v_cache=vc,
                            hq=sh.hq, hkv=sh.hkv)
            fa = dict(block_tables=sv.block_tables, context_lens=sv.context_lens, query_start=sv.query_start,
                      out=attn, part_o=part_o, part_ml=part_ml, part_size=part_size,
                      scale=self.scale) if fuse_attn else None
            if li > 0 and takes(L.qkv):
                ops.linear(hg if awq else resid, L.qkv, out=q, prenorm=(ssp, eps), qkv=qkv_args, attn=fa)
            else:
                ops.linear(resid, L.qkv, out=q, norm=(L.in_norm, eps), qkv=qkv_args, attn=fa)
            if fa is None:
                ops.attention(q, sh.hq * D, kc, vc, sv.block_tables, sv.context_lens, sv.query_start, sv.tile_seq,
                              sv.tile_q0, attn, part_o, part_ml, sh.hq, sh.hkv, part_size, self.scale)
            gu = takes(L.gate_up)
            self._row_parallel(attn, L.o, resid, first, norm_out=(hg, ssp, L.post_norm) if gu else None)
            if gu:
                ops.linear(hg if awq else resid, L.gate_up, out=mlp, prenorm=(ssp, eps))
            else:
                ops.linear(resid, L.gate_up, out=mlp, norm=(L.post_norm, eps))
            nq = li + 1 < nl and takes(self.layers[li + 1].qkv)
            self._row_parallel(mlp, L.down, resid, first, norm_out=(hg, ssp, self.layers[li + 1].in_norm) if nq else None)
        self.last_resid = resid  # the post-all-reduce residual (replicated over TP): consistency guard
        if return_hidden:
            return resid
        logits = ops.linear(resid, self.lm_head, out_f32=True, norm=(self.final_norm, eps), row_idx=sv.sample_idx)
        if tp.size > 1:
            logits = tp.all_gather_lastdim(logits)
        return logits[:, : a.vocab_size]

    def _forward_reference(self, sv, kv_caches, part_size: int, return_hidden: bool = False) -> torch.Tensor:
        """Same math with the fp32 reference ops, one op at a time (CPU path)."""
        a = self.arch
        sh = self.shard
        tp = self.tp
        T = sv.T
        D = a.head_dim
        dev = self.device
        resid = ops.embedding(sv.ids, self.embed, vstart=sh.vocab0)
        if tp.size > 1:
            tp.all_reduce(resid)
        x = torch.empty_like(resid)
        attn = torch.empty(T, sh.hq * D, dtype=torch.bfloat16, device=dev)
        qkv = torch.empty(T, (sh.hq + 2 * sh.hkv) * D, dtype=torch.bfloat16, device=dev)
        mlp = torch.empty(T, sh.inter, dtype=torch.bfloat16, device=dev)
        first = tp.is_first
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            ops.rmsnorm(resid, L.in_norm, a.rms_eps, out=x)
            ops.linear(x, L.qkv, out=qkv)
            ops.rope_kv(qkv, sv.positions, sv.slots, self.cos_sin, kc, vc, sh.hq, sh.hkv, D)
            self._attention_cpu(qkv, attn, kc, vc, sv)
            self._row_parallel(attn, L.o, resid, first)
            ops.rmsnorm(resid, L.post_norm, a.rms_eps, out=x)
            ops.linear(x, L.gate_up, out=mlp)
            self._row_parallel(mlp, L.down, resid, first)
        self.last_resid = resid
        if return_hidden:
            return resid
        xs = resid.index_select(0, sv.sample_idx.long())
        xn = ops.rmsnorm(xs, self.final_norm, a.rms_eps)
        logits = ops.linear(xn, self.lm_head, out_f32=True)
        if tp.size > 1:
            logits = tp.all_gather_lastdim(logits)
        return logits[:, : a.vocab_size]

    def _attention_cpu(self, qkv, attn, kc, vc, sv):
        sh = self.shard
        D = self.arch.head_dim
        n = int(sv.num_tokens)
        nseq = int(sv.num_seqs)
        if n == 0 or nseq == 0:
            return
        T = qkv.shape[0]
        q = qkv[:, : sh.hq * D].reshape(T, sh.hq, D)
        qs = sv.query_start[: nseq + 1]
        o = ops.ref.attention_ref(q[:n], kc, vc, sv.block_tables[:nseq], sv.context_lens[:nseq], qs,
                                  sh.hq, sh.hkv, self.scale)
        attn[:n] = o.reshape(n, sh.hq * D)

    # ------------------------------------------------------------- reference
    @torch.no_grad()
    def reference_logits(self, token_ids: list[int], return_hidden: bool = False) -> torch.Tensor:
        """Dense fp32 forward of one sequence (no KV cache, no custom kernels) -> [len, vocab]
        (or, with ``return_hidden``, the final-RMSNorm hidden states [len, H]).

        Used by tests as the oracle for the engine's kernel path (TP=1 only).
        """
        assert self.tp.size == 1
        a = self.arch
        D = a.head_dim
        ids = torch.tensor(token_ids, device=self.device)
        n = len(token_ids)
        r = self.embed[ids].float()
        cs = self.cos_sin[:n]
        c, s = cs[:, None, : D // 2], cs[:, None, D // 2:]

        def rope(t):
            x1, x2 = t[..., : D // 2], t[..., D // 2:]
            return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)

        def norm(t, w):
            return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + a.rms_eps) * w.float()

        mask = torch.full((n, n), float("-inf"), device=self.device).triu(1)
        G = a.num_heads // a.num_kv_heads
        for L in self.layers:
            x = norm(r, L.in_norm)
            wqkv = L.qkv.dense_weight().float()
            qkv = x @ wqkv.t()
            if L.qkv.bias is not None:
                qkv = qkv + L.qkv.bias.float()
            q = qkv[:, : a.q_size].view(n, a.num_heads, D)
            k = qkv[:, a.q_size: a.q_size + a.kv_size].view(n, a.num_kv_heads, D)
            v = qkv[:, a.q_size + a.kv_size:].view(n, a.num_kv_heads, D)
            q, k = rope(q), rope(k)
            k = k.repeat_interleave(G, 1)
            v = v.repeat_interleave(G, 1)
            sc = torch.einsum("qhd,khd->hqk", q, k) * self.scale + mask
            o = torch.einsum("hqk,khd->qhd", torch.softmax(sc, -1), v).reshape(n, -1)
            r = r + o @ L.o.dense_weight().float().t()
            x = norm(r, L.post_norm)
            gu = L.gate_up.dense_weight().float()
            I = gu.shape[0] // 2
            h = torch.nn.functional.silu(x @ gu[:I].t()) * (x @ gu[I:].t())
            r = r + h @ L.down.dense_weight().float().t()
        x = norm(r, self.final_norm)
        if return_hidden:
            return x
        w = self.embed if a.tie_embeddings else self.lm_head.dense_weight()
        return (x @ w.float().t())[:, : a.vocab_size]
