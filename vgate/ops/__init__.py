"""vgate compute ops: gfx950 HIP kernels (``vgate._C``) with fp32 torch references.

Dispatch rule: GPU tensors ALWAYS go to the native HIP kernels — if the
extension is missing on a GPU machine the op raises (no silent eager fallback);
CPU tensors use the reference implementations in :mod:`vgate.ops.reference`.
"""
from __future__ import annotations

import math
import os

import torch

from . import reference as ref

_C = None
_C_ERR: Exception | None = None


def _dev_key(device) -> str:
    """Key of the per-device buffers below: "cuda" and "cuda:<current>" name the same device."""
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def native():
    """Return the compiled extension module, building it in-tree if needed."""
    global _C, _C_ERR
    if _C is not None:
        return _C
    try:
        from vgate import _C as mod  # type: ignore
        _C = mod
        _configure(mod)
    except ImportError as e:  # pragma: no cover - depends on build state
        if os.environ.get("VGATE_AUTOBUILD", "1") == "1":
            try:
                import importlib
                import sys
                from pathlib import Path
                sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "csrc"))
                import build as _build  # type: ignore
                _build.build(verbose=False)
                _C = importlib.import_module("vgate._C")
                _configure(_C)
                return _C
            except Exception as e2:  # noqa: BLE001
                _C_ERR = e2
        else:
            _C_ERR = e
        raise RuntimeError(f"vgate native extension unavailable: {_C_ERR}") from _C_ERR
    return _C


def _configure(mod) -> None:
    """Runtime knobs of the extension that default from the environment on the Python side (none
    left: the sampler's pass-kernel and round-launch variants were deleted in round 5)."""


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------------------- packing
def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> fragment-major [N/16, K/32, 4, 16, 8] (see csrc/kernels/gemm.hip)."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0, (N, K)
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def unpack_weight(wp: torch.Tensor, N: int, K: int) -> torch.Tensor:
    return wp.reshape(N // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(N, K)


def interleave_gate_up(w_gate: torch.Tensor, w_up: torch.Tensor) -> torch.Tensor:
    """Rows ordered [G0 U0 G1 U1 ...] in 16-row tiles for the fused SiLU*mul epilogue."""
    I, K = w_gate.shape
    assert I % 16 == 0
    return torch.stack([w_gate.reshape(I // 16, 16, K), w_up.reshape(I // 16, 16, K)], 1).reshape(2 * I, K)


def unpack_awq(packed: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """Inverse of :func:`pack_awq`: int32 [N/16, K/128, 64, 4] -> int4 values [N, K] (int32)."""
    w = packed.to(torch.int64) & 0xFFFFFFFF
    w = w.reshape(N // 16, K // 128, 4, 16, 4)  # nt, kq, g, r, u
    j = torch.arange(8, dtype=torch.int64, device=packed.device)
    shifts = (j & 1) * 16 + (j >> 1) * 4
    q = (w[..., None] >> shifts) & 0xF  # nt, kq, g, r, u, j
    return q.permute(0, 3, 1, 4, 2, 5).reshape(N, K).to(torch.int32)


def pack_awq(qint: torch.Tensor) -> torch.Tensor:
    """int4 values [N, K] (0..15) -> int32 [N/16, K/128, 64, 4]; word u of lane l holds the 8
    values W[16nt + (l&15)][128kq + 32u + 8(l>>4) + j], j = 0..7, with the EVEN j in the low
    half-word and the odd j in the high one: value j at bit (16 if j odd) + 4 (j >> 1).
    Then (word >> 4d) & 0x000F000F | 0x43004300 is the bf16 pair (128 + v_2d, 128 + v_2d+1):
    two VALU ops per MFMA operand dword (gemm.hip, AWQ decode kernel)."""
    N, K = qint.shape
    assert N % 16 == 0 and K % 128 == 0
    q = qint.to(torch.int64).reshape(N // 16, 16, K // 128, 4, 4, 8)  # nt, r, kq, u, g, j
    q = q.permute(0, 2, 4, 1, 3, 5)  # nt, kq, g, r, u, j  -> lane = g*16 + r
    j = torch.arange(8, dtype=torch.int64, device=qint.device)
    shifts = (j & 1) * 16 + (j >> 1) * 4
    words = (q << shifts).sum(-1)  # [nt, kq, g, r, u]
    words = words.reshape(N // 16, K // 128, 64, 4)
    words = torch.where(words >= 2**31, words - 2**32, words)
    return words.to(torch.int32).contiguous()


def pack_awq_sz(scales: torch.Tensor, sz: torch.Tensor) -> torch.Tensor:
    """Group scales in the AWQ decode kernels' fragment order (csrc/kernels/gemm_awq_kx.hip, gemm_awq_mid.hip):
    [N/16][K/128][4 lane groups][s(4 cols), s*z(4 cols)] bf16, so the lanes of a 16-lane group load
    their 4 columns' scale AND zero term with ONE 16-B load per (tile, k-quad). Group 128 only."""
    G, N = scales.shape
    s4 = scales.t().reshape(N // 16, 4, 4, G).permute(0, 3, 1, 2)  # [nt][g][lane group][4]
    z4 = sz.t().reshape(N // 16, 4, 4, G).permute(0, 3, 1, 2)
    return torch.cat([s4, z4], dim=-1).to(torch.bfloat16).contiguous()  # [nt][g][4][8]


def row_permutation(N: int, layout: str) -> torch.Tensor | None:
    """Row order of the packed weight for a fused epilogue (None = identity).

    silu: tile t = gate rows 8t..8t+7 then up rows 8t..8t+7 (rows [gate; up] in the dense
          matrix), so one 16-row tile holds 8 SiLU pairs on lanes l, l^32 and a decode block
          can own a single tile (gemm_epilogue.h);
    qkv : per 128-wide head, tile t (t = 0..7) = rows 8t..8t+7 then their NeoX rotation
          partners 64+8t..64+8t+7, so one 16-row tile holds both halves of 8 rotation pairs
          (the GEMM epilogue exchanges them across lanes l, l^32; csrc/kernels/gemm.hip qkv_col).
    """
    if layout == "silu":
        I = N // 2
        assert I % 8 == 0
        t = torch.arange(2 * I).reshape(2, I // 8, 8).transpose(0, 1)
        return t.reshape(-1)
    if layout == "qkv":
        assert N % 128 == 0
        heads = N // 128
        tile = torch.arange(128).reshape(2, 8, 8).permute(1, 0, 2).reshape(8, 16)
        t = torch.arange(heads)[:, None, None] * 128 + tile[None]
        return t.reshape(-1)
    return None


class Linear:
    """A linear layer's weights in kernel-ready form.

    layout: "plain" | "silu" (rows [gate; up] -> out = silu(gate) * up)
            | "qkv" (rows [q; k; v], heads of 128: fused bias + RoPE + KV-cache write).
    Dense bf16 weights or AWQ int4 (``awq={"qint", "scales", "zeros", "group"}``).
    On GPU only the fragment-packed copy is kept; on CPU the dense matrix (reference path).
    """

    def __init__(self, w: torch.Tensor | None, bias: torch.Tensor | None = None, kind: str = "plain",
                 awq: dict | None = None, layout: str | None = None):
        if kind in ("silu", "qkv"):
            layout, kind = kind, "dense"
        self.layout = layout or (awq.get("layout", "plain") if awq else "plain")
        if awq is not None and awq.get("silu"):
            self.layout = "silu"
        self.kind = "awq" if awq is not None else "dense"
        self.bias = bias
        self.norm_gamma = None  # RMSNorm weight folded into the packed copy (see fold_norm)
        # decode-GEMM decomposition for M <= 16 steps (0 = the launcher's heuristic): set by the
        # model from the measured per-shape table (vgate/models/decode_plans.py)
        self.dec_waves = 0
        self.dec_splitk = 0
        self.dec_sk = None  # stream-K decode kernel: None = STREAMK_DECODE, or (waves, blocks/CU, group)
        self.dec_ntb = 0
        self.dec_path = 0  # 4: the register-stationary decode kernel (csrc/kernels/gemm_kx.h)
        # prefill (M >= 128) tile / K-slice choice per M bucket, measured at engine start-up
        # (tune_prefill); empty = the launcher's heuristic
        self.prefill_plan: dict[int, tuple[int, int]] = {}
        if self.kind == "awq":
            q = awq["qint"]
            self.N, self.K = q.shape
            self.group = awq["group"]
            dev = awq["scales"].device
            perm = row_permutation(self.N, self.layout)
            scales, zeros = awq["scales"], awq["zeros"]
            if dev.type == "cuda":
                q = q.to(dev)
                if perm is not None:
                    pd = perm.to(dev)
                    q, scales, zeros = q[pd], scales[:, pd], zeros[:, pd]
                self.wp = pack_awq(q)
                self.scales = scales.to(torch.bfloat16).contiguous()
                self.zeros = (scales.float() * zeros.float()).to(torch.bfloat16).contiguous()
                self.szp = pack_awq_sz(self.scales, self.zeros) if self.group == 128 else None
                self.w = None
            else:
                self.w = ref.awq_dequant_ref(q, scales, zeros, self.group)
                self.wp = None
            return
        self.N, self.K = w.shape
        if w.is_cuda:
            perm = row_permutation(self.N, self.layout)
            self.wp = pack_weight(w[perm.to(w.device)] if perm is not None else w)
            self.w = None
        else:
            self.wp = None
            self.w = w

    def fold_norm(self, gamma: torch.Tensor) -> bool:
        """Fold the preceding RMSNorm's weight into the packed matrix: W'[n,k] = W[n,k]*g[k].

        The fused GEMM then applies only the per-row scale rsqrt(mean(x^2)+eps) (deferred, in
        the epilogue) and streams no gamma bytes. GPU bf16 weights only; returns whether folded.
        """
        if self.kind != "dense" or self.wp is None or self.norm_gamma is not None:
            return False
        g = gamma.to(self.wp.device, torch.float32).reshape(1, self.K // 32, 4, 1, 8)
        self.wp.copy_((self.wp.float() * g).to(torch.bfloat16))
        self.norm_gamma = gamma.detach().clone()
        return True

    def _awq_dense(self) -> torch.Tensor:
        """int4 -> bf16 (v * s - s * z) in the original row order."""
        q = unpack_awq(self.wp, self.N, self.K)  # permuted row order, like scales / zeros
        g = torch.arange(self.K, device=q.device) // self.group
        w = (q.float() * self.scales.float()[g].t() - self.zeros.float()[g].t()).to(torch.bfloat16)
        perm = row_permutation(self.N, self.layout)
        if perm is not None:
            out = torch.empty_like(w)
            out[perm.to(w.device)] = w
            w = out
        return w

    @property
    def out_features(self) -> int:
        return self.N // 2 if self.layout == "silu" else self.N

    def dense_weight(self) -> torch.Tensor:
        """[N, K] in the ORIGINAL row order (references / checkpoint export)."""
        if self.w is not None:
            return self.w
        if self.kind == "awq":  # dequantised bf16 (v - z) * s in the original row order (references)
            return self._awq_dense()
        w = unpack_weight(self.wp, self.N, self.K)
        if self.norm_gamma is not None:  # un-fold (approximate: W' was rounded to bf16)
            w = (w.float() / self.norm_gamma.to(w.device, torch.float32)[None]).to(torch.bfloat16)
        perm = row_permutation(self.N, self.layout)
        if perm is not None:
            out = torch.empty_like(w)
            out[perm.to(w.device)] = w
            w = out
        return w

    def nbytes(self) -> int:
        """Bytes a decode step streams."""
        if self.kind == "awq" and self.w is None:
            n = self.wp.numel() * 4 + self.scales.numel() * 4  # int4 + (s, s*z) bf16 per group
            return n + (self.szp.numel() * 2 if getattr(self, "szp", None) is not None else 0)
        t = self.wp if self.wp is not None else self.w
        return t.numel() * t.element_size()


_WS: dict = {}


def workspace(device) -> torch.Tensor:
    """Per-device GEMM workspace: 64k split-K tickets (zeroed once) + fp32 slabs (256 MiB on a GPU:
    a K-split prefill GEMM needs slices x M x N x 4 bytes — with 32 MiB the 4-way split of Llama-3-8B
    down_proj at M = 1024 silently fell back to one slice on 64 tiles; 32 MiB on the CPU)."""
    key = _dev_key(device)
    ws = _WS.get(key)
    if ws is None:
        slab_words = (64 if torch.device(device).type == "cuda" else 8) * 2**20
        ws = torch.zeros(65536 + slab_words, dtype=torch.int32, device=device)
        _WS[key] = ws
    return ws


def linear(x: torch.Tensor, lin: Linear, out: torch.Tensor | None = None,
           residual: torch.Tensor | None = None, out_f32: bool = False, waves: int = 0, splitk: int = 0,
           norm: tuple | None = None, row_idx: torch.Tensor | None = None, qkv: dict | None = None,
           path: int = 0, norm_out: tuple | None = None, prenorm: tuple | None = None,
           ar=None, attn: dict | None = None) -> torch.Tensor:
    """out = epilogue(prologue(x) @ W^T).

    attn (with qkv, decode-only steps): dict(block_tables, context_lens, query_start, out, part_o,
    part_ml, part_size, scale) — the step's decode attention over q = this projection's output, run
    in the projection's launch when the decode kernel takes it (csrc/kernels/qkv_attn.hip), else
    launched right after it; returns q as without it.

    ar (GPU, <= 16 rows, bf16 epilogue): a :class:`vgate.parallel.custom_allreduce.CustomAllReduce`;
    the TP row-parallel GEMM then all-reduces in its epilogue: out = bf16(sum over ranks of
    x @ W^T [+ bias]) + residual, one launch and no copy-in (gemm_epilogue.h epilogue_ar).

    RMSNorm hand-off to the int4 decode kernels (GPU, <= 16 rows, TP = 1; gemm_epilogue.h):
    norm_out=(hg, ssp, gamma) on a residual GEMM also writes hg = out * gamma and per-16-column
    sums of out^2 into ssp; prenorm=(ssp, eps) on an AWQ consumer whose x IS that hg applies the
    row scale from ssp (no gamma loads or x^2 pass in the int4 kernel).

    norm=(w, eps): fused RMSNorm of x rows (deferred row scale, see gemm.hip); row_idx: gather rows of x first;
    qkv=dict(positions, slots, cos_sin, k_cache, v_cache, hq, hkv): fused bias + RoPE +
    KV write, returns q [M, hq*128] (layout "qkv" only).
    """
    M = row_idx.numel() if row_idx is not None else x.shape[0]
    silu = lin.layout == "silu"
    if qkv is not None:
        ncols = qkv["hq"] * 128
    else:
        ncols = lin.N // 2 if silu else lin.N
    if out is None:
        out = torch.empty(M, ncols, dtype=torch.float32 if out_f32 else torch.bfloat16, device=x.device)
    if not _gpu(x):
        xx = x[row_idx.long()] if row_idx is not None else x
        if norm is not None:
            xx, _ = ref.rmsnorm_ref(xx, norm[0], norm[1])
        wd = lin.dense_weight()
        if silu:
            I = lin.N // 2
            out.copy_(ref.silu_mul_linear_ref(xx, wd[:I], wd[I:]))
        elif qkv is not None:
            y = ref.linear_ref(xx, wd, lin.bias)
            ref.rope_kv_ref(y, qkv["positions"], qkv["slots"], qkv["cos_sin"], qkv["k_cache"], qkv["v_cache"],
                            qkv["hq"], qkv["hkv"], 128)
            out.copy_(y[:, :ncols])
            if attn is not None:
                _attn_after(out, qkv, attn)
        else:
            out.copy_(ref.linear_ref(xx, wd, lin.bias, residual, out_f32))
        return out
    C = native()
    epi = 3 if qkv is not None else (2 if silu else (1 if out_f32 else 0))
    awq_mid = (lin.kind == "awq" and 16 < M <= 64 and row_idx is None and waves == 0 and splitk == 0
               and path == 0 and lin.group == 128 and getattr(lin, "szp", None) is not None)
    if awq_mid:
        path = 2  # int4 medium kernel (csrc/kernels/gemm_awq_mid.hip awq_mid_kernel): no bf16 scratch
    elif lin.kind == "awq" and M >= AWQ_DEQUANT_MIN_M and row_idx is None and waves == 0 and splitk == 0:
        return _linear_awq_dequant(x, lin, out, residual, norm, qkv, epi, M)
    ntb = 0
    sk = False
    if M <= 16 and waves == 0 and splitk == 0:
        waves, splitk, ntb = lin.dec_waves, lin.dec_splitk, lin.dec_ntb
        if path == 0 and lin.kind == "dense" and row_idx is None and ar is None:
            path = getattr(lin, "dec_path", 0)
        # stream-K decode kernel (csrc/kernels/gemm_streamk.hip): per-Linear plan, else the module default
        sk = (lin.kind == "dense" and path == 0 and row_idx is None and norm_out is None and ar is None
              and (lin.dec_sk if lin.dec_sk is not None else STREAMK_DECODE))
        if sk:  # (W, blocks per CU, k-steps per register group) of the plan, 0 = the kernel's default
            path = 3
            waves, splitk, ntb = lin.dec_sk if isinstance(lin.dec_sk, tuple) else (0, 0, 0)
    elif M > 16 and waves == 0 and splitk == 0 and path == 0 and lin.prefill_plan and lin.kind == "dense":  # (AWQ: below)
        pk = _plan_kw(lin.prefill_plan.get(_plan_bucket(lin.prefill_plan, M)), M)
        ntb, splitk, path, waves = pk.get("ntb", 0), pk.get("splitk", 0), pk.get("path", 0), pk.get("waves", 0)
    kw = dict(bias=lin.bias, res=residual, ws=workspace(x.device), waves=waves, splitk=splitk, ntb=ntb, path=path)
    if M <= 16:  # stream-K slots / the decode split-K granules (zeroed, self-clearing) and the fault word
        kw.update(sk_ws=sk_workspace(x.device), fault=fault_word(x.device))
    else:  # the stream-K prefill kernel's bounded ticket poll
        kw.update(fault=fault_word(x.device))
    if norm is not None:
        if lin.norm_gamma is not None:  # gamma lives in the weights: row scale only
            kw.update(rownorm=True, eps=float(norm[1]))
        else:
            kw.update(norm_w=norm[0], eps=float(norm[1]))
    if row_idx is not None:
        kw["row_idx"] = row_idx
    if qkv is not None:
        kw.update(positions=qkv["positions"], slots=qkv["slots"], cos_sin=qkv["cos_sin"],
                  k_cache=qkv["k_cache"], v_cache=qkv["v_cache"], hq=qkv["hq"], hkv=qkv["hkv"])
    if lin.kind == "awq":
        kw.update(awq_scales=lin.scales, awq_zeros=lin.zeros, group=lin.group)
        if getattr(lin, "szp", None) is not None:
            kw["awq_szp"] = lin.szp
    if norm_out is not None:
        kw.update(hg_out=norm_out[0], ssp_out=norm_out[1], hg_gamma=norm_out[2])
    if prenorm is not None:
        kw.update(ssp_in=prenorm[0], eps=float(prenorm[1]))
    if ar is not None:
        if M > 16 or epi != 0:
            raise ValueError("fused all-reduce: decode rows (<= 16) and the bf16 epilogue only")
        kw.update(ar_bases=ar.bases, ar_rank=ar.rank, ar_fused_off=ar.fused_off)
    if attn is not None:
        if qkv is None or M > 16:
            raise ValueError("fused attention: the decode QKV projection (qkv epilogue, <= 16 rows)")
        if not FUSE_QKV_ATTN:
            C.gemm(x, lin.wp, lin.N, lin.K, out, epi, **kw)
            _attn_after(out, qkv, attn)
            return out
        kw.update(fa_block_tables=attn["block_tables"], fa_context_lens=attn["context_lens"],
                  fa_query_start=attn["query_start"], fa_out=attn["out"], fa_part_o=attn["part_o"],
                  fa_part_ml=attn["part_ml"], fa_tickets=attn_tickets(x.device), fa_sync=qa_sync(x.device),
                  fa_part_size=int(attn["part_size"]), fa_scale=float(attn["scale"]), fa_dbg_ts=attn.get("dbg_ts"))
    C.gemm(x, lin.wp, lin.N, lin.K, out, epi, **kw)
    return out


# decode-only steps: the decode attention rides in the QKV projection's launch (qkv_attn.hip); tests
# turn it off to compare against the two-launch path (the o_proj as a third role measured no faster:
# profiles/r5_qa_oproj_negative.log)
FUSE_QKV_ATTN = True
_QA_SYNC: dict = {}


def qa_sync(device) -> torch.Tensor:
    """Zeroed granule buffer of the fused QKV + attention launch (QaSync: 16 rows x N/2 x 8 B, N <= 32768;
    the consumers clear what they read)."""
    key = _dev_key(device)
    t = _QA_SYNC.get(key)
    if t is None:
        t = _QA_SYNC[key] = torch.zeros(1 << 20, dtype=torch.int32, device=device)
    return t


def _attn_after(q, qkv, attn):
    """The two-launch form of ``linear(..., attn=...)``: decode attention over the projection's q."""
    if not _gpu(q):
        attention_decode(q, q.stride(0), qkv["k_cache"], qkv["v_cache"], attn["block_tables"], attn["context_lens"],
                         attn["out"], attn["part_o"], attn["part_ml"], qkv["hq"], qkv["hkv"], int(attn["part_size"]),
                         float(attn["scale"]), query_start=attn["query_start"])
        return
    e = torch.empty(0, dtype=torch.int32, device=q.device)
    attention(q, q.stride(0), qkv["k_cache"], qkv["v_cache"], attn["block_tables"], attn["context_lens"],
              attn["query_start"], e, e, attn["out"], attn["part_o"], attn["part_ml"], qkv["hq"], qkv["hkv"],
              int(attn["part_size"]), float(attn["scale"]))


# AWQ steps of 16 < M <= 64 rows (mixed prefill + decode) run the int4 medium kernel; longer ones
# (M >= AWQ_DEQUANT_MIN_M not taken by it) dequantise to scratch + the bf16 prefill / tile kernels
AWQ_DEQUANT_MIN_M = 32
_AWQ_SCRATCH: dict = {}


def reserve_awq_scratch(device, numel: int) -> torch.Tensor:
    """The per-device bf16 scratch one dequantised AWQ matrix lives in during a long step."""
    key = _dev_key(device)
    t = _AWQ_SCRATCH.get(key)
    if t is None or t.numel() < numel:
        t = _AWQ_SCRATCH[key] = torch.empty(numel, dtype=torch.bfloat16, device=device)
    return t


def _linear_awq_dequant(x, lin: "Linear", out, residual, norm, qkv, epi, M):
    """Long AWQ step: int4 -> bf16 fragment-packed scratch (RMSNorm gamma folded in), then the
    bf16 kernels with the row-scale-only RMSNorm mode — same epilogues, no resident bf16 copy."""
    C = native()
    scratch = reserve_awq_scratch(x.device, lin.N * lin.K)[: lin.N * lin.K]
    gamma = norm[0] if norm is not None else None
    C.awq_dequant(lin.wp, lin.scales, lin.zeros, lin.N, lin.K, lin.group, scratch, gamma)
    kw = dict(bias=lin.bias, res=residual, ws=workspace(x.device))
    if norm is not None:
        kw.update(rownorm=True, eps=float(norm[1]))
    if qkv is not None:
        kw.update(positions=qkv["positions"], slots=qkv["slots"], cos_sin=qkv["cos_sin"],
                  k_cache=qkv["k_cache"], v_cache=qkv["v_cache"], hq=qkv["hq"], hkv=qkv["hkv"])
    if M > 16 and lin.prefill_plan:
        kw.update(_plan_kw(lin.prefill_plan.get(_plan_bucket(lin.prefill_plan, M)), M))
    C.gemm(x, scratch, lin.N, lin.K, out, epi, **kw)
    return out


# flash prefill: long causal ranges run as two K halves met through fp32 partials in the GEMM
# workspace (csrc/kernels/attention.hip attn_flash_kernel, two blocks per KV head); tests turn it off
FLASH_SPLIT = True


def attention(q, q_stride, k_cache, v_cache, block_tables, context_lens, query_start, tile_seq, tile_q0, out,
              part_o, part_ml, Hq: int, Hkv: int, part_size: int, scale: float, tickets=None):
    """Unified paged attention for a mixed step (decode rows + prefill tiles, one launch).
    Decode partitions of one (sequence, KV head) are merged in-launch by the last arriving
    block (``tickets``: zeroed int32 [>= S*Hkv], defaults to a per-device buffer)."""
    if tickets is None:
        tickets = attn_tickets(q.device)
    native().attention(q, q_stride, k_cache, v_cache, block_tables, context_lens, query_start, tile_seq, tile_q0,
                       out, part_o, part_ml, Hq, Hkv, part_size, scale, 0, tickets,
                       flash_ws=workspace(q.device) if FLASH_SPLIT else None, fault=fault_word(q.device))
    return out


_FAULT: dict = {}


def fault_word(device) -> torch.Tensor:
    """Per-device sticky fault word of the in-launch hand-offs (bit 1: a flash K-split waiter gave
    up, 4: a stream-K partial poll, 8: a split-K granule poll, 16: a sampler row meeting, 32: a fused
    QKV + attention granule poll, 64: a stream-K prefill ticket poll; bit 0 is reserved). Kernels only OR bits in; the step graph's last node
    copies it to the host ring (ModelRunner.kernel_fault), and a non-zero word fails the engine."""
    key = _dev_key(device)
    t = _FAULT.get(key)
    if t is None:
        t = _FAULT[key] = torch.zeros(4, dtype=torch.int32, device=device)
    return t


def reset_handoffs(device) -> None:
    """Return every in-launch hand-off buffer of ``device`` to its zeroed start state after a fault
    (the engine's recovery path; VERDICT r5 weak #9, ADVICE r5: a poll that gave up can leave a
    late producer granule behind, which a later sequence in the same row / position would accept).
    Waits for the device first, so no launch is still writing. The buffers keep their addresses:
    captured graphs stay valid."""
    key = _dev_key(device)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    for cache in (_FAULT, _QA_SYNC, _TICKETS, _SWS, _SKWS):
        t = cache.get(key)
        if t is not None:
            t.zero_()
    ws = _WS.get(key)
    if ws is not None:
        ws[:65536].zero_()  # the split-K tickets (the slabs are written before they are read)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


_TICKETS: dict = {}


def attn_tickets(device) -> torch.Tensor:
    """Self-resetting decode-partition tickets (allocated once per device, before any capture)."""
    key = _dev_key(device)
    t = _TICKETS.get(key)
    if t is None:
        t = torch.zeros(1 << 16, dtype=torch.int32, device=device)
        _TICKETS[key] = t
    return t


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """y = RMSNorm(x [+ residual]) * w; when residual is given it is updated in place to x + residual."""
    if out is None:
        out = torch.empty_like(x)
    if not _gpu(x):
        y, s = ref.rmsnorm_ref(x, w, eps, residual)
        if residual is not None:
            residual.copy_(s)
        out.copy_(y)
        return out
    native().rmsnorm(x, residual, w, out, eps)
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, out: torch.Tensor | None = None, vstart: int = 0,
              prev: torch.Tensor | None = None):
    """Row gather with vocab-shard masking (rows outside this TP rank's shard are zero).
    ids < 0 name a token the previous step sampled on the device: id = prev[-id - 1]."""
    if out is None:
        out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device)
    if not _gpu(table):
        if prev is not None and bool((ids < 0).any()):
            ids = torch.where(ids < 0, prev.to(ids.device)[(-ids - 1).clamp(min=0).long()], ids)
        out.copy_(ref.embedding_ref(ids, table, vstart))
        return out
    native().embedding(ids, table, out, vstart, prev)
    return out


def rope_kv(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq: int, Hkv: int, D: int) -> None:
    if not _gpu(qkv):
        ref.rope_kv_ref(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D)
        return
    native().rope_kv(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D)


def attention_decode(q, q_stride, k_cache, v_cache, block_tables, context_lens, out, part_o, part_ml,
                     Hq: int, Hkv: int, part_size: int, scale: float, query_start=None):
    """One query token per sequence. q rows index = sequence (or query_start[s+1]-1)."""
    if not _gpu(q):
        S = context_lens.numel()
        if query_start is None:
            qs = torch.arange(S + 1, dtype=torch.int32)
        else:
            qs = query_start
        # reference wants only the decode rows
        rows = (qs[1:] - 1).long()
        D = k_cache.shape[-1]
        qq = q.view(q.shape[0], -1)[rows, : Hq * D].reshape(S, Hq, D)
        o = ref.attention_ref(qq, k_cache, v_cache, block_tables, context_lens,
                              torch.arange(S + 1, dtype=torch.int32), Hq, Hkv, scale)
        out.view(out.shape[0], Hq, D)[rows] = o
        return out
    native().attn_decode(q, q_stride, k_cache, v_cache, block_tables, context_lens, query_start, out,
                         part_o, part_ml, Hq, Hkv, part_size, scale)
    return out


def prefill_tiles(query_lens: list[int], lead: int = 32) -> tuple[list[int], list[int]]:
    """16-query prefill tiles (sequence, first query) in the attention kernel's order: see
    :func:`tile_order`."""
    seq, q0 = [], []
    for s, ql in enumerate(query_lens):
        for t in tile_order(ql, lead):
            seq.append(s)
            q0.append(int(t))
    return seq, q0


def flash_lead(hq: int, hkv: int) -> int:
    """Queries per flash-prefill block for a head layout (attention.hip flash_cfg: 8 waves when
    G = hq / hkv divides 8, else 6; two 16-query column tiles per wave up to G = 4, one above;
    the waves are G heads x NW / G query groups)."""
    G = max(1, hq // max(hkv, 1))
    nw = 8 if 8 % G == 0 else (6 if 6 % G == 0 else 0)
    if nw == 0:
        return 16
    return 16 * (2 if G <= 4 else 1) * (nw // G)


def tile_order(qlen: int, lead: int = 32):
    """First queries of a sequence's 16-query tiles, ordered for the flash prefill kernel: the
    tiles that start a ``lead``-query group (the flash blocks that work; the others exit at once)
    first, longest causal range first, then the rest. The working blocks are then the first ones
    of the grid, spread round-robin over the 8 XCDs, and the longest start first. Correctness
    does not depend on the order (the 16-query kernel is order-free, flash blocks find their
    group from the tile), only the load balance does."""
    import numpy as _np
    t = _np.arange(0, qlen, 16, dtype=_np.int32)[::-1]
    return _np.concatenate([t[t % lead == 0], t[t % lead != 0]])


def attention_prefill(q, q_stride, k_cache, v_cache, block_tables, context_lens, query_start,
                      tile_seq, tile_q0, out, Hq: int, Hkv: int, scale: float):
    if not _gpu(q):
        D = k_cache.shape[-1]
        T = q.shape[0]
        qq = q.view(T, -1)[:, : Hq * D].reshape(T, Hq, D)
        o = ref.attention_ref(qq, k_cache, v_cache, block_tables, context_lens, query_start, Hq, Hkv, scale)
        out.view(T, Hq, D).copy_(o)
        return out
    native().attn_prefill(q, q_stride, k_cache, v_cache, block_tables, context_lens, query_start,
                          tile_seq, tile_q0, out, Hq, Hkv, scale,
                          flash_ws=workspace(q.device) if FLASH_SPLIT else None, fault=fault_word(q.device))
    return out


def sample(logits, temperature=None, top_p=None, top_k=None, seeds=None, offsets=None,
           out=None, out_logprob=None, generators=None):
    """Temperature / top-k / top-p sampling per row (csrc/kernels/sampling.hip)."""
    B = logits.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    if not _gpu(logits):
        out.copy_(ref.sample_ref(logits, temperature, top_p, top_k, generators))
        return out
    native().sample(logits, temperature, top_p, top_k, seeds, offsets, out, out_logprob, sample_workspace(logits.device),
                    fault_word(logits.device))
    return out


def _plan_bucket(plan: dict, M: int):
    """Smallest planned M >= M (a step's rows are padded up to its graph bucket), else None.
    Medium rows (M < 128) only take a medium bucket's plan (they are timed against another
    default path than the prefill buckets)."""
    keys = [k for k in plan if k >= M and (M >= 128 or k < 128)]
    return min(keys) if keys else None


# (tile code, K slices) candidates of the prefill kernels (csrc/kernels/gemm_prefill.hip
# launch_prefill_epi): 0 = the launcher's heuristic, 64 / 128 = 128 x 64 / 128 x 128 tiles,
# 256 = 256 x 128 3-deep ring, 768 / 1024 = the 4-phase 256 x 128 / 256 x 256 kernels
PREFILL_CANDIDATES = [(0, 0), (64, 0), (128, 0), (128, 2), (128, 4), (256, 0), (256, 4), (256, 6), (768, 0),
                      (768, 2), (768, 3), (768, 4), (768, 6), (1024, 0), (1024, 2), (1024, 3), (1024, 4),
                      (1024, 6), (1025, 0), (769, 0)]
# (1025 / 769: the persistent forms of the 4-phase 256 x 256 / 256 x 128 kernel — one block per CU,
# whole rounds of tiles + the last round K-split and met in-launch; gemm_prefill.hip
# gemm_prefill4sk_kernel)
# 128-row tiles on a 4-deep ring, one block per CU (128 x 128 / 128 x 64, 4 or 8 waves): timed for
# 64 < M <= 1024 only, where the grid of the 2-deep-ring tile is one or two partial rounds
# + the wide-N tiles 64 x 512 / 128 x 320 (gate_up at 320 / 448 rows: 245 / 224 blocks, 35 vs 44-64 us)
PREFILL_RING_CANDIDATES = ([(t, s) for t in (1280, 1281, 640, 641) for s in (0, 2, 3)]
                           + [(2560, 0), (2561, 0)])
# medium-M kernel (csrc/kernels/gemm_mid.hip, 16 < M <= 64) candidates, encoded as tile code
# MID_BASE - W (W tiles = waves per block) and K slices (0 = its heuristic)
MID_BASE = -10
MID_CANDIDATES = [(MID_BASE - w, s) for w in (4, 2) for s in (0, 2, 3, 4, 6, 8, 10, 12, 16)] + [(MID_BASE - 8, 0)]
_FLUSH: dict = {}


def _cold_timer(dev):
    """Event timer of one launch with the Infinity Cache flushed first: a 512 MiB read sweep evicts
    the weights a back-to-back repeat would find resident (gate_up's 55 MB fits the 256 MiB cache),
    so medium-M candidates are ranked by the cold-weight time they take inside a decode step."""
    buf = _FLUSH.get(str(dev))
    if buf is None:
        buf = _FLUSH[str(dev)] = torch.empty(512 * 2**20, dtype=torch.uint8, device=dev)
    C = native()

    def timed(run, iters):
        total = 0.0
        for _ in range(iters):
            C.prefetch(buf, 1024)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            run()
            s1.record()
            s1.synchronize()
            total += s0.elapsed_time(s1)
        return total / iters
    return timed


def _mid_code(cfg) -> int:
    """Waves per block of a medium-kernel plan entry, 0 for any other entry."""
    return MID_BASE - cfg[0] if cfg is not None and cfg[0] <= MID_BASE - 1 else 0


def _plan_kw(cfg, M: int) -> dict:
    """C.gemm keyword overrides of a plan entry (empty: the default path)."""
    if cfg is None or cfg == MEDIUM_DEFAULT or (cfg == (0, 0) and M >= 128):
        return {}
    w = _mid_code(cfg)
    if w:
        return dict(path=2, waves=w, splitk=cfg[1])
    return dict(ntb=cfg[0], splitk=cfg[1], path=1)


MEDIUM_DEFAULT = (-1, -1)  # medium-M plan entry: keep the default (decode / tile kernel) path


# bump whenever the MEANING of a stored plan changes on the Python side (the _plan_kw encoding of a
# (tile, K slices) code, MID_BASE, the tuner margin): a cached plan set is keyed on this too
PLAN_FORMAT = 3  # 3: candidates timed with the layer's folded-norm row scale
TUNE_MARGIN = 0.05
LONG_M, LONG_MARGIN = 1024, 0.02  # the margin for M >= LONG_M buckets


def tune_prefill(lins: list, ms: list[int], iters: int = 5, margin: float = TUNE_MARGIN) -> dict:
    """Start-up measurement of the prefill GEMM decomposition per (N, K) shape and M bucket.

    The launcher's tile / K-split heuristic misses by up to 1.8x at mid M, where the grid of
    one tile shape needs a second partial round on 256 CUs and another's does not (Qwen2.5-1.5B
    gate_up at M = 384: 64 us heuristic vs 35 us for 128 x 128 tiles; down at M = 512: 56 vs
    40 us, profiles/r2_prefill_tile_sweep.log). Every candidate is timed on random operands of
    the layer's shape (plain epilogue, all candidates are exact kernels of the same product);
    the heuristic is kept unless a candidate beats it by more than ``margin``. The plan is
    shared by every Linear of the same shape (AWQ layers: the plan of their bf16 dequant scratch).

    Medium buckets (16 < M < 128: the mixed steps of a serving load, one prompt chunk beside the
    decode rows) are timed against the DEFAULT path at that M too (the K-split decode kernels /
    the LDS tile kernel, which stream the weights with one or two k-step groups in flight: a
    Qwen2.5-1.5B step with a 48-token prompt took 2.77 ms against 1.24 ms for pure decode,
    profiles/r3_mixed_step.log); the entry is :data:`MEDIUM_DEFAULT` unless a prefill
    decomposition beats that path by more than ``margin``.
    Returns {(N, K): {M: (tile, slices)}}."""
    cand = [lin for lin in lins if getattr(lin, "wp", None) is not None and lin.wp.is_cuda]
    if not cand or not native_available():
        return {}
    C = native()
    dev = cand[0].wp.device
    ws = workspace(dev)
    plans: dict = {}
    for lin in cand:
        key = (lin.N, lin.K)
        if key in plans:
            lin.prefill_plan = plans[key]
            continue
        plan = {}
        g = torch.Generator(device=dev)
        g.manual_seed(lin.N + lin.K)
        # AWQ layers run their long steps on a bf16 fragment-packed dequant scratch of the same
        # shape (_linear_awq_dequant): time a random bf16 matrix in that layout
        wp = lin.wp if lin.kind == "dense" else pack_weight(
            (torch.rand(lin.N, lin.K, device=dev, generator=g) * 2 - 1).bfloat16())
        # the folded RMSNorm's row scale as in the step (qkv / gate_up: the x^2 sums ride in the K loop
        # and cost some kernels up to ~30 % more than others — 128 x 320 tiles with four wave columns:
        # Qwen2.5-1.5B qkv at 448 rows 17.7 -> 22.9 us, profiles/r6_tuner_norm_timing.log)
        nkw = dict(rownorm=True, eps=1e-6) if (lin.norm_gamma is not None
                                                or getattr(lin, "layout", "plain") in ("qkv", "silu")) else {}
        for M in ms:
            x = torch.rand(M, lin.K, device=dev, generator=g).bfloat16()
            out = torch.empty(M, lin.N, dtype=torch.bfloat16, device=dev)
            times = {}
            # (cold-weight timing for M >= 128 too was measured: it picked slower down_proj plans at
            # M = 448 and the same gate_up tile, profiles/r4_prefill_step_timeline.log)
            cold = _cold_timer(dev) if M < 128 else None
            extra = MID_CANDIDATES if 16 < M <= 64 else PREFILL_RING_CANDIDATES if 64 < M <= 1024 else []
            for bn, sk in PREFILL_CANDIDATES + extra:
                def run():
                    C.gemm(x, wp, lin.N, lin.K, out, 0, ws=ws, **_plan_kw((bn, sk), M), **nkw)
                try:
                    run()
                except RuntimeError:
                    continue
                if cold is not None:
                    times[(bn, sk)] = cold(run, iters)
                    continue
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                for _ in range(iters):
                    run()
                s1.record()
                s1.synchronize()
                times[(bn, sk)] = s0.elapsed_time(s1) / iters
            if (0, 0) not in times:
                continue
            best = min(times, key=times.get)
            if M < 128:
                # medium bucket: against the default path (M > 16 rows -> decode / tile kernels)
                def run_default():
                    C.gemm(x, wp, lin.N, lin.K, out, 0, ws=ws, **nkw)
                run_default()
                t_def = cold(run_default, iters)
                plan[M] = best if times[best] < (1.0 - margin) * t_def else MEDIUM_DEFAULT
                continue
            # long chunks: 100+ us launches time to ~1 %, so a 2 % win is kept (Llama-3-8B qkv_proj at
            # 2048 rows: split-K 6 + reduce 105 vs 111 us for the default grid sat on the 5 % edge)
            m_eff = margin if M < LONG_M else LONG_MARGIN
            plan[M] = best if times[best] < (1.0 - m_eff) * times[(0, 0)] else (0, 0)
        plans[key] = plan
        lin.prefill_plan = plan
    # the cache-flush buffer of the cold timer (512 MiB) is start-up scratch: give it back
    _FLUSH.pop(str(dev), None)
    torch.cuda.empty_cache()
    return plans


def _plan_cache_key(lins: list, ms: list[int]) -> str:
    """What a stored plan set was measured for: the device, the native build (size + mtime of the
    extension), the plan encoding (PLAN_FORMAT, TUNE_MARGIN) and every (N, K) shape x M bucket x
    candidate list — any change re-measures."""
    import hashlib
    dev = lins[0].wp.device
    props = torch.cuda.get_device_properties(dev)
    so = getattr(native(), "__file__", "") or ""
    st = os.stat(so) if so and os.path.exists(so) else None
    shapes = sorted({(lin.N, lin.K, lin.kind) for lin in lins if getattr(lin, "wp", None) is not None})
    blob = json_dumps([PLAN_FORMAT, TUNE_MARGIN, LONG_M, LONG_MARGIN, props.name, props.multi_processor_count, st.st_size if st else 0,
                       int(st.st_mtime) if st else 0, shapes, sorted(ms), PREFILL_CANDIDATES, PREFILL_RING_CANDIDATES,
                       MID_CANDIDATES])
    return hashlib.sha1(blob.encode()).hexdigest()


def json_dumps(x) -> str:
    import json
    return json.dumps(x, sort_keys=True, default=str)


def load_plan_cache(path: str, key: str) -> dict | None:
    """Plans stored by :func:`save_plan_cache` under ``key``, or None."""
    import json
    try:
        with open(os.path.expanduser(path)) as f:
            d = json.load(f).get(key)
    except (OSError, ValueError):
        return None
    if not isinstance(d, dict):
        return None
    return {tuple(int(v) for v in nk.split(",")): {int(m): tuple(c) for m, c in plan.items()} for nk, plan in d.items()}


def save_plan_cache(path: str, key: str, plans: dict) -> None:
    """Persist measured plans under ``key`` (other keys in the file are kept; best effort)."""
    import json
    path = os.path.expanduser(path)
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            d = {}
        d[key] = {f"{n},{k}": {str(m): list(c) for m, c in plan.items()} for (n, k), plan in plans.items()}
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(d, f)
        os.replace(tmp, path)
    except OSError:
        pass


def tune_prefill_cached(lins: list, ms: list[int], cache: str | None) -> tuple[dict, bool]:
    """:func:`tune_prefill` behind a per-(device, build, shapes) plan file: a restart of the same
    engine on the same device skips the start-up measurement (~3,400 cache-flush launches for
    Qwen2.5-1.5B). Returns (plans, from_cache)."""
    cand = [lin for lin in lins if getattr(lin, "wp", None) is not None and lin.wp.is_cuda]
    if not cache or not cand or not native_available():
        return tune_prefill(lins, ms), False
    key = _plan_cache_key(cand, ms)
    plans = load_plan_cache(cache, key)
    if plans is not None:
        apply_prefill_plans(lins, plans)
        return plans, True
    plans = tune_prefill(lins, ms)
    save_plan_cache(cache, key, plans)
    return plans, False


def apply_prefill_plans(lins: list, plans: dict) -> None:
    """Give every Linear the plan measured for its (N, K) shape (plans from :func:`tune_prefill`,
    e.g. broadcast from TP rank 0)."""
    for lin in lins:
        plan = (plans or {}).get((lin.N, lin.K))
        if plan is not None:
            lin.prefill_plan = dict(plan)


def host_device_copy(dst: torch.Tensor, src: torch.Tensor, nbytes: int) -> None:
    """Copy the first ``nbytes`` between a pinned host tensor and a device tensor on the current
    stream. GPU: a kernel on the compute queue (csrc/kernels/elementwise.hip copy16_kernel), so the
    step loop's metadata upload and sampled-id download take no SDMA engine hand-off; both tensors
    must hold ``nbytes`` rounded up to 16 (without the extension: a non-blocking tensor copy)."""
    if (dst.is_cuda or src.is_cuda) and native_available():
        native().kernel_copy(dst, src, int(nbytes))
        return
    d8 = dst.view(torch.uint8) if dst.dtype != torch.uint8 else dst
    s8 = src.view(torch.uint8) if src.dtype != torch.uint8 else src
    d8[:nbytes].copy_(s8[:nbytes], non_blocking=True)


_SWS: dict = {}


def sample_workspace(device) -> torch.Tensor:
    """Per-row epochs + fixed per-row granule regions of the segmented sampler (zeroed once, per
    device; launchers.h SAMPLE_WS_*)."""
    key = _dev_key(device)
    ws = _SWS.get(key)
    if ws is None:
        ws = torch.zeros(int(native().SAMPLE_WS_WORDS), dtype=torch.int32, device=device)
        _SWS[key] = ws
    return ws


# every dense decode GEMM (<= 16 rows) on the stream-K kernel: one equal share of the packed weight
# stream per CU (csrc/kernels/gemm_streamk.hip); off by default — the measured per-shape plans
# (Linear.dec_sk, vgate/models/decode_plans.py) pick it where it wins; tests turn it on
STREAMK_DECODE = False
_SKWS: dict = {}


def sk_workspace(device) -> torch.Tensor:
    """Zeroed publisher slots of the stream-K decode kernel (the owner clears what it reads, so it
    stays zero between launches): 64 MiB covers ntiles x (contributors - 1) x 3 KiB of any model."""
    key = _dev_key(device)
    t = _SKWS.get(key)
    if t is None:
        t = _SKWS[key] = torch.zeros(16 * 2**20, dtype=torch.int32, device=device)
    return t


def softmax_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)


__all__ = [
    "native", "native_available", "pack_weight", "unpack_weight", "interleave_gate_up", "pack_awq",
    "Linear", "linear", "attention", "workspace", "fault_word", "reset_handoffs",
    "row_permutation", "reserve_awq_scratch", "pack_awq_sz", "rmsnorm", "embedding", "rope_kv", "attention_decode", "attention_prefill",
    "prefill_tiles", "sample", "softmax_scale", "ref", "host_device_copy", "tune_prefill", "apply_prefill_plans",
]
