"""Tokenizers.

* :class:`HFTokenizer` wraps the ``tokenizers`` library when a ``tokenizer.json``
  is available next to a checkpoint.
* :class:`SyntheticTokenizer` is the default for random-init models (no vocab
  files exist on this machine): UTF-8 bytes map to ids ``[OFFSET, OFFSET+256)``
  so any prompt round-trips exactly; ids outside that range (which a random
  model emits freely) decode to short deterministic pseudo-words so generated
  text has realistic length/shape for streaming and benchmarks.
"""
from __future__ import annotations

from pathlib import Path

_SYLL = ["ka", "lo", "mi", "ne", "ru", "ta", "vo", "zi", "pe", "sa", "do", "fu", "gi", "ha", "ju", "be"]


class SyntheticTokenizer:
    OFFSET = 3  # 0 pad, 1 bos, 2 eos (overridable)

    def __init__(self, vocab_size: int, bos_token_id: int = 1, eos_token_ids=(2,)):
        self.vocab_size = vocab_size
        self.bos_token_id = bos_token_id
        self.eos_token_ids = tuple(eos_token_ids)
        self._special = {bos_token_id, *self.eos_token_ids}

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = [self.OFFSET + b for b in text.encode("utf-8")]
        return ([self.bos_token_id] + ids) if add_bos else ids

    def _piece(self, t: int) -> bytes:
        if t in self._special:
            return b""
        if self.OFFSET <= t < self.OFFSET + 256:
            return bytes([t - self.OFFSET])
        h = (t * 2654435761) & 0xFFFFFFFF
        w = _SYLL[h & 15] + _SYLL[(h >> 4) & 15]
        if (h >> 8) & 1:
            w += _SYLL[(h >> 12) & 15]
        return (" " + w).encode()

    def decode(self, ids: list[int]) -> str:
        return b"".join(self._piece(t) for t in ids).decode("utf-8", errors="replace")

    def decode_bytes(self, ids: list[int]) -> bytes:
        return b"".join(self._piece(t) for t in ids)


class HFTokenizer:
    def __init__(self, path: str, bos_token_id: int | None = None, eos_token_ids=()):
        from tokenizers import Tokenizer
        p = Path(path)
        f = p / "tokenizer.json" if p.is_dir() else p
        self._tok = Tokenizer.from_file(str(f))
        self.vocab_size = self._tok.get_vocab_size()
        self.bos_token_id = bos_token_id
        self.eos_token_ids = tuple(eos_token_ids)

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = self._tok.encode(text, add_special_tokens=False).ids
        if add_bos and self.bos_token_id is not None:
            ids = [self.bos_token_id] + ids
        return ids

    def decode(self, ids: list[int]) -> str:
        return self._tok.decode(ids, skip_special_tokens=True)

    def decode_bytes(self, ids: list[int]) -> bytes:
        return self.decode(ids).encode("utf-8")


class IncrementalDecoder:
    """Emit only complete UTF-8 text deltas as tokens arrive."""

    def __init__(self, tokenizer):
        self.tok = tokenizer
        self._pending = b""
        self._ids: list[int] = []
        self._text_len = 0
        self._hf = isinstance(tokenizer, HFTokenizer)

    def push(self, token_id: int) -> str:
        if self._hf:
            self._ids.append(token_id)
            text = self.tok.decode(self._ids)
            if text.endswith("�"):
                return ""
            delta = text[self._text_len:]
            self._text_len = len(text)
            return delta
        self._pending += self.tok.decode_bytes([token_id])
        try:
            s = self._pending.decode("utf-8")
            self._pending = b""
            return s
        except UnicodeDecodeError as e:
            if e.start > 0:
                s = self._pending[: e.start].decode("utf-8")
                self._pending = self._pending[e.start:]
                return s
            if len(self._pending) > 4:  # invalid sequence: flush with replacement
                s = self._pending.decode("utf-8", errors="replace")
                self._pending = b""
                return s
            return ""

    def flush(self) -> str:
        if self._pending:
            s = self._pending.decode("utf-8", errors="replace")
            self._pending = b""
            return s
        return ""


def load_tokenizer(model_path: str | None, tokenizer_path: str | None, arch):
    for cand in (tokenizer_path, model_path):
        if cand and (Path(cand) / "tokenizer.json").exists() or (cand and str(cand).endswith(".json") and Path(cand).exists()):
            try:
                return HFTokenizer(cand, arch.bos_token_id, arch.eos_token_ids)
            except Exception:  # noqa: BLE001
                pass
    return SyntheticTokenizer(arch.vocab_size, arch.bos_token_id, arch.eos_token_ids)
