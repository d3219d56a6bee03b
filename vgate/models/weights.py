"""Weight creation / loading for :class:`vgate.models.transformer.DecoderModel`.

* ``random_init``: seeded random weights generated directly on the device in
  kernel-ready (fragment-packed) form — the benchmark path (no checkpoints
  exist on this machine). Scales keep activations O(1) so numerics are sane.
* ``load_checkpoint``: HF safetensors (bf16/fp16/fp32 or AWQ int4 GEMM format),
  sharded for the model's TP rank at load time (only this rank's slices are
  materialised on the GPU).
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import torch

from vgate import ops
from vgate.models.config import ModelArch

AWQ_ORDER = [0, 2, 4, 6, 1, 3, 5, 7]  # AutoAWQ GEMM nibble order within an int32


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def _randn(shape, std, g, device):
    return (torch.randn(shape, generator=g, device=device, dtype=torch.float32) * std).to(torch.bfloat16)


def _rand_awq(N, K, group, g, device, silu=False, layout="plain"):
    q = torch.randint(0, 16, (N, K), generator=g, device=device, dtype=torch.int32)
    target = 1.0 / math.sqrt(K)
    scales = torch.full((K // group, N), target / 4.61, device=device).to(torch.bfloat16)
    zeros = torch.full((K // group, N), 8.0, device=device).to(torch.bfloat16)
    return ops.Linear(None, awq={"qint": q, "scales": scales, "zeros": zeros, "group": group,
                                 "layout": "silu" if silu else layout})


def random_init(model, seed: int = 0) -> None:
    a: ModelArch = model.arch
    sh = model.shard
    dev = model.device
    g = _gen(dev, seed * 1000003 + sh.tp.rank)
    H, D = a.hidden_size, a.head_dim
    awq = model.quant == "awq"
    group = 128
    model.embed = _randn((sh.vocab, H), 0.02, g, dev)
    layers = []
    from vgate.models.transformer import LayerWeights
    q_out = (sh.hq + 2 * sh.hkv) * D
    for _ in range(a.num_layers):
        qkv_b = _randn((q_out,), 0.02, g, dev) if a.qkv_bias else None
        if awq and H % 128 == 0 and (sh.hq * D) % 128 == 0 and sh.inter % 128 == 0:
            qkv = _rand_awq(q_out, H, group, g, dev, layout="qkv")
            qkv.bias = qkv_b
            o = _rand_awq(H, sh.hq * D, group, g, dev)
            gu = _rand_awq(2 * sh.inter, H, group, g, dev, silu=True)
            down = _rand_awq(H, sh.inter, group, g, dev)
        else:
            qkv = ops.Linear(_randn((q_out, H), 1 / math.sqrt(H), g, dev), bias=qkv_b, layout="qkv")
            o = ops.Linear(_randn((H, sh.hq * D), 1 / math.sqrt(sh.hq * D * sh.tp.size), g, dev))
            gu = ops.Linear(_randn((2 * sh.inter, H), 1 / math.sqrt(H), g, dev), kind="silu")
            down = ops.Linear(_randn((H, sh.inter), 1 / math.sqrt(sh.inter * sh.tp.size), g, dev))
        layers.append(LayerWeights(
            in_norm=torch.ones(H, dtype=torch.bfloat16, device=dev), qkv=qkv, o=o,
            post_norm=torch.ones(H, dtype=torch.bfloat16, device=dev), gate_up=gu, down=down))
        if awq and dev.type == "cuda":
            torch.cuda.empty_cache()
    model.layers = layers
    model.final_norm = torch.ones(H, dtype=torch.bfloat16, device=dev)
    if a.tie_embeddings:
        model.lm_head = ops.Linear(model.embed)
    else:
        model.lm_head = ops.Linear(_randn((sh.vocab, H), 1 / math.sqrt(H), g, dev))


# ------------------------------------------------------------------ checkpoints
class _SafeTensorIndex:
    def __init__(self, path: Path):
        from safetensors import safe_open
        files = sorted(path.glob("*.safetensors")) if path.is_dir() else [path]
        if not files:
            raise FileNotFoundError(f"no *.safetensors under {path}")
        self._handles = {}
        self._where = {}
        for f in files:
            h = safe_open(str(f), framework="pt", device="cpu")
            self._handles[str(f)] = h
            for k in h.keys():
                self._where[k] = str(f)

    def has(self, k: str) -> bool:
        return k in self._where

    def get(self, k: str) -> torch.Tensor:
        return self._handles[self._where[k]].get_tensor(k)

    def get_slice(self, k: str):
        return self._handles[self._where[k]].get_slice(k)


def unpack_awq_int32(packed: torch.Tensor) -> torch.Tensor:
    """AutoAWQ GEMM packing: [rows, cols/8] int32 -> [rows, cols] int (0..15)."""
    rows, c8 = packed.shape
    shifts = torch.tensor([4 * i for i in range(8)], dtype=torch.int32)
    vals = (packed.unsqueeze(-1) >> shifts) & 0xF  # nibble i
    # nibble i holds logical column AWQ_ORDER[i]
    out = torch.empty_like(vals)
    out[..., AWQ_ORDER] = vals
    return out.reshape(rows, c8 * 8)


def pack_awq_int32(q: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`unpack_awq_int32` (used by tests to build AWQ fixtures)."""
    rows, cols = q.shape
    v = q.reshape(rows, cols // 8, 8).to(torch.int64)[..., AWQ_ORDER]
    shifts = torch.tensor([4 * i for i in range(8)], dtype=torch.int64)
    w = (v << shifts).sum(-1)
    w = torch.where(w >= 2**31, w - 2**32, w)
    return w.to(torch.int32)


def _rows(t: torch.Tensor, a: int, b: int) -> torch.Tensor:
    return t[a:b]


def load_checkpoint(model, path: str) -> None:
    """Load an HF Qwen2/Llama checkpoint (safetensors) for this TP rank."""
    a: ModelArch = model.arch
    sh = model.shard
    dev = model.device
    root = Path(path)
    idx = _SafeTensorIndex(root)
    D, H = a.head_dim, a.hidden_size
    qcfg = {}
    if (root / "config.json").exists():
        qcfg = json.loads((root / "config.json").read_text()).get("quantization_config", {}) or {}
    group = int(qcfg.get("group_size", 128))

    def dense(name: str) -> torch.Tensor:
        return idx.get(name).to(torch.bfloat16)

    def is_awq(prefix: str) -> bool:
        return idx.has(prefix + ".qweight")

    def awq_rows(prefix: str, row_ranges):
        """Return (qint [N, K], scales [K/g, N], zeros [K/g, N]) restricted to output rows."""
        qw = unpack_awq_int32(idx.get(prefix + ".qweight"))  # [K, N]
        qz = unpack_awq_int32(idx.get(prefix + ".qzeros"))   # [K/g, N]
        sc = idx.get(prefix + ".scales").to(torch.bfloat16)  # [K/g, N]
        cols = torch.cat([torch.arange(s, e) for s, e in row_ranges])
        return qw[:, cols].t().contiguous(), sc[:, cols].contiguous(), qz[:, cols].to(torch.bfloat16).contiguous()

    def awq_cols(prefix: str, k0: int, k1: int):
        qw = unpack_awq_int32(idx.get(prefix + ".qweight"))[k0:k1]
        qz = unpack_awq_int32(idx.get(prefix + ".qzeros"))[k0 // group:k1 // group]
        sc = idx.get(prefix + ".scales").to(torch.bfloat16)[k0 // group:k1 // group]
        return qw.t().contiguous(), sc.contiguous(), qz.to(torch.bfloat16).contiguous()

    def make_awq(t, silu=False, layout="plain"):
        q, s, z = t
        return ops.Linear(None, awq={"qint": q, "scales": s.to(dev), "zeros": z.to(dev), "group": group,
                                     "layout": "silu" if silu else layout})

    qa, qb = sh.q_head0 * D, (sh.q_head0 + sh.hq) * D
    ka, kb = a.q_size + sh.kv_head0 * D, a.q_size + (sh.kv_head0 + sh.hkv) * D
    va, vb = a.q_size + a.kv_size + sh.kv_head0 * D, a.q_size + a.kv_size + (sh.kv_head0 + sh.hkv) * D
    from vgate.models.transformer import LayerWeights
    layers = []
    for i in range(a.num_layers):
        p = f"model.layers.{i}"
        att, mlp = p + ".self_attn", p + ".mlp"
        bias = None
        if a.qkv_bias and idx.has(att + ".q_proj.bias"):
            full_b = torch.cat([dense(att + ".q_proj.bias"), dense(att + ".k_proj.bias"), dense(att + ".v_proj.bias")])
            bias = torch.cat([full_b[qa:qb], full_b[ka:kb], full_b[va:vb]]).to(dev)
        if is_awq(att + ".q_proj"):
            q = awq_rows(att + ".q_proj", [(qa, qb)])
            k = awq_rows(att + ".k_proj", [(ka - a.q_size, kb - a.q_size)])
            v = awq_rows(att + ".v_proj", [(va - a.q_size - a.kv_size, vb - a.q_size - a.kv_size)])
            qkv = make_awq((torch.cat([q[0], k[0], v[0]]), torch.cat([q[1], k[1], v[1]], 1),
                            torch.cat([q[2], k[2], v[2]], 1)), layout="qkv")
            qkv.bias = bias
            o = make_awq(awq_cols(att + ".o_proj", qa, qb))
            g_ = awq_rows(mlp + ".gate_proj", [(sh.inter0, sh.inter0 + sh.inter)])
            u_ = awq_rows(mlp + ".up_proj", [(sh.inter0, sh.inter0 + sh.inter)])
            gu = make_awq((torch.cat([g_[0], u_[0]]), torch.cat([g_[1], u_[1]], 1), torch.cat([g_[2], u_[2]], 1)),
                          silu=True)
            down = make_awq(awq_cols(mlp + ".down_proj", sh.inter0, sh.inter0 + sh.inter))
        else:
            wq = dense(att + ".q_proj.weight")[qa:qb]
            wk = dense(att + ".k_proj.weight")[ka - a.q_size: kb - a.q_size]
            wv = dense(att + ".v_proj.weight")[va - a.q_size - a.kv_size: vb - a.q_size - a.kv_size]
            qkv = ops.Linear(torch.cat([wq, wk, wv]).to(dev), bias=bias, layout="qkv")
            o = ops.Linear(dense(att + ".o_proj.weight")[:, qa:qb].contiguous().to(dev))
            wg = dense(mlp + ".gate_proj.weight")[sh.inter0: sh.inter0 + sh.inter]
            wu = dense(mlp + ".up_proj.weight")[sh.inter0: sh.inter0 + sh.inter]
            gu = ops.Linear(torch.cat([wg, wu]).to(dev), kind="silu")
            down = ops.Linear(dense(mlp + ".down_proj.weight")[:, sh.inter0: sh.inter0 + sh.inter].contiguous().to(dev))
        layers.append(LayerWeights(dense(p + ".input_layernorm.weight").to(dev), qkv, o,
                                   dense(p + ".post_attention_layernorm.weight").to(dev), gu, down))
    model.layers = layers
    emb = dense("model.embed_tokens.weight")
    pad = sh.vocab_padded - emb.shape[0]
    if pad > 0:
        emb = torch.cat([emb, torch.zeros(pad, H, dtype=emb.dtype)])
    model.embed = emb[sh.vocab0: sh.vocab0 + sh.vocab].contiguous().to(dev)
    model.final_norm = dense("model.norm.weight").to(dev)
    if a.tie_embeddings or not idx.has("lm_head.weight"):
        model.lm_head = ops.Linear(model.embed)
    else:
        lm = dense("lm_head.weight")
        if pad > 0:
            lm = torch.cat([lm, torch.zeros(pad, H, dtype=lm.dtype)])
        model.lm_head = ops.Linear(lm[sh.vocab0: sh.vocab0 + sh.vocab].contiguous().to(dev))


def save_checkpoint(model, path: str) -> None:
    """Write a TP=1 dense model as HF-layout safetensors (fast restart / tests)."""
    from safetensors.torch import save_file
    a = model.arch
    assert model.tp.size == 1
    out = {"model.embed_tokens.weight": model.embed[: a.vocab_size].cpu(), "model.norm.weight": model.final_norm.cpu()}
    for i, L in enumerate(model.layers):
        p = f"model.layers.{i}"
        w = L.qkv.dense_weight().cpu()
        out[p + ".self_attn.q_proj.weight"] = w[: a.q_size].contiguous()
        out[p + ".self_attn.k_proj.weight"] = w[a.q_size: a.q_size + a.kv_size].contiguous()
        out[p + ".self_attn.v_proj.weight"] = w[a.q_size + a.kv_size:].contiguous()
        if L.qkv.bias is not None:
            b = L.qkv.bias.cpu()
            out[p + ".self_attn.q_proj.bias"] = b[: a.q_size].contiguous()
            out[p + ".self_attn.k_proj.bias"] = b[a.q_size: a.q_size + a.kv_size].contiguous()
            out[p + ".self_attn.v_proj.bias"] = b[a.q_size + a.kv_size:].contiguous()
        out[p + ".self_attn.o_proj.weight"] = L.o.dense_weight().cpu().contiguous()
        gu = L.gate_up.dense_weight().cpu()
        I = gu.shape[0] // 2
        out[p + ".mlp.gate_proj.weight"] = gu[:I].contiguous()
        out[p + ".mlp.up_proj.weight"] = gu[I:].contiguous()
        out[p + ".mlp.down_proj.weight"] = L.down.dense_weight().cpu().contiguous()
        out[p + ".input_layernorm.weight"] = L.in_norm.cpu()
        out[p + ".post_attention_layernorm.weight"] = L.post_norm.cpu()
    if not a.tie_embeddings:
        out["lm_head.weight"] = model.lm_head.dense_weight()[: a.vocab_size].cpu().contiguous()
    Path(path).mkdir(parents=True, exist_ok=True)
    save_file(out, str(Path(path) / "model.safetensors"))
    cfg = {"model_type": a.family, "hidden_size": a.hidden_size, "num_hidden_layers": a.num_layers,
           "num_attention_heads": a.num_heads, "num_key_value_heads": a.num_kv_heads,
           "intermediate_size": a.intermediate_size, "vocab_size": a.vocab_size, "rms_norm_eps": a.rms_eps,
           "rope_theta": a.rope_theta, "tie_word_embeddings": a.tie_embeddings,
           "max_position_embeddings": a.max_position, "head_dim": a.head_dim,
           "bos_token_id": a.bos_token_id, "eos_token_id": list(a.eos_token_ids)}
    if a.rope_scaling:
        cfg["rope_scaling"] = a.rope_scaling
    (Path(path) / "config.json").write_text(json.dumps(cfg, indent=1))
