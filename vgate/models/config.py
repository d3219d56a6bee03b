"""Model architecture descriptions (Qwen2 / Llama family decoder-only transformers).

Dimensions are the public HF ``config.json`` values of each model.
A model id resolves to an :class:`ModelArch` either by a local directory holding a
``config.json`` (real checkpoint) or by a built-in preset matched on the id's
name (random-init weights, used for benchmarks: there are no checkpoints here).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace
from pathlib import Path


@dataclass(frozen=True)
class ModelArch:
    name: str
    family: str  # "qwen2" | "llama"
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int
    rms_eps: float = 1e-6
    rope_theta: float = 10000.0
    rope_scaling: dict | None = field(default=None, hash=False, compare=False)
    qkv_bias: bool = False
    tie_embeddings: bool = False
    max_position: int = 32768
    bos_token_id: int = 1
    eos_token_ids: tuple = (2,)

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        per_layer = H * (self.q_size + 2 * self.kv_size) + self.q_size * H + 3 * H * I + 2 * H
        if self.qkv_bias:
            per_layer += self.q_size + 2 * self.kv_size
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * per_layer + emb + H

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def to_dict(self) -> dict:
        return asdict(self)


PRESETS: dict[str, ModelArch] = {
    "qwen2.5-0.5b": ModelArch("qwen2.5-0.5b", "qwen2", 896, 24, 14, 2, 64, 4864, 151936, 1e-6, 1e6,
                              qkv_bias=True, tie_embeddings=True, bos_token_id=151643,
                              eos_token_ids=(151645, 151643)),
    "qwen2.5-1.5b": ModelArch("qwen2.5-1.5b", "qwen2", 1536, 28, 12, 2, 128, 8960, 151936, 1e-6, 1e6,
                              qkv_bias=True, tie_embeddings=True, bos_token_id=151643,
                              eos_token_ids=(151645, 151643)),
    "qwen2.5-7b": ModelArch("qwen2.5-7b", "qwen2", 3584, 28, 28, 4, 128, 18944, 152064, 1e-6, 1e6,
                            qkv_bias=True, tie_embeddings=False, bos_token_id=151643,
                            eos_token_ids=(151645, 151643)),
    "llama-3-8b": ModelArch("llama-3-8b", "llama", 4096, 32, 32, 8, 128, 14336, 128256, 1e-5, 5e5,
                            max_position=8192, bos_token_id=128000, eos_token_ids=(128001, 128009)),
    "llama-3.1-8b": ModelArch("llama-3.1-8b", "llama", 4096, 32, 32, 8, 128, 14336, 128256, 1e-5, 5e5,
                              rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                            "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
                              max_position=131072, bos_token_id=128000, eos_token_ids=(128001, 128009)),
    "llama-3-70b": ModelArch("llama-3-70b", "llama", 8192, 80, 64, 8, 128, 28672, 128256, 1e-5, 5e5,
                             max_position=8192, bos_token_id=128000, eos_token_ids=(128001, 128009)),
    # small configs for tests / CPU smoke (head_dim must stay 128 for the GPU kernels)
    "tiny": ModelArch("tiny", "qwen2", 256, 2, 4, 2, 128, 512, 512, 1e-6, 1e4, qkv_bias=True,
                      tie_embeddings=True, max_position=4096, bos_token_id=1, eos_token_ids=(2,)),
    "tiny-llama": ModelArch("tiny-llama", "llama", 256, 2, 4, 1, 128, 384, 1024, 1e-5, 5e5,
                            max_position=4096, bos_token_id=1, eos_token_ids=(2,)),
    # TP tests up to 8 ranks: 8 query heads, 2 KV heads (replicated at TP 4 / 8), a vocabulary
    # that is not a multiple of 16 * 8 (padded vocab shards)
    "tiny-tp8": ModelArch("tiny-tp8", "qwen2", 256, 2, 8, 2, 128, 1024, 500, 1e-6, 1e4, qkv_bias=True,
                          tie_embeddings=True, max_position=4096, bos_token_id=1, eos_token_ids=(2,)),
}

_ALIASES = [
    ("qwen2.5-0.5b", "qwen2.5-0.5b"),
    ("qwen2.5-1.5b", "qwen2.5-1.5b"),
    ("qwen2.5-7b", "qwen2.5-7b"),
    ("llama-3.1-8b", "llama-3.1-8b"),
    ("llama-3-70b", "llama-3-70b"),
    ("meta-llama-3-70b", "llama-3-70b"),
    ("llama-3-8b", "llama-3-8b"),
    ("meta-llama-3-8b", "llama-3-8b"),
    ("tiny-llama", "tiny-llama"),
    ("tiny-tp8", "tiny-tp8"),
    ("tiny", "tiny"),
]


def _from_hf_config(cfg: dict, name: str) -> ModelArch:
    mt = cfg.get("model_type", "llama")
    family = "qwen2" if mt.startswith("qwen2") else "llama"
    H = cfg["hidden_size"]
    nh = cfg["num_attention_heads"]
    eos = cfg.get("eos_token_id", 2)
    eos = tuple(eos) if isinstance(eos, list) else (eos,)
    return ModelArch(
        name=name, family=family, hidden_size=H, num_layers=cfg["num_hidden_layers"], num_heads=nh,
        num_kv_heads=cfg.get("num_key_value_heads", nh), head_dim=cfg.get("head_dim", H // nh),
        intermediate_size=cfg["intermediate_size"], vocab_size=cfg["vocab_size"],
        rms_eps=cfg.get("rms_norm_eps", 1e-6), rope_theta=cfg.get("rope_theta", 10000.0),
        rope_scaling=cfg.get("rope_scaling"), qkv_bias=(family == "qwen2") or cfg.get("attention_bias", False),
        tie_embeddings=cfg.get("tie_word_embeddings", False),
        max_position=cfg.get("max_position_embeddings", 32768),
        bos_token_id=cfg.get("bos_token_id", 1) or 1, eos_token_ids=eos)


def resolve_arch(model_id: str, overrides: dict | None = None) -> ModelArch:
    """Resolve a model id / path to its architecture."""
    p = Path(os.path.expanduser(model_id))
    arch = None
    if p.is_dir() and (p / "config.json").exists():
        arch = _from_hf_config(json.loads((p / "config.json").read_text()), p.name)
    else:
        key = model_id.lower().split("/")[-1]
        key = key.replace("-instruct", "").replace("-awq", "").replace("_", "-")
        for alias, preset in _ALIASES:
            if alias in key:
                arch = PRESETS[preset]
                break
    if arch is None:
        raise ValueError(f"unknown model '{model_id}': pass a directory with config.json or one of {sorted(PRESETS)}")
    if overrides:
        arch = replace(arch, **overrides)
    return arch
