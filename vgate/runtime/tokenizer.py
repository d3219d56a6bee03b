"""Tokenizers.

* :class:`HFTokenizer` wraps the ``tokenizers`` library when a ``tokenizer.json``
  is available next to a checkpoint.
* :class:`SyntheticTokenizer` is the default for random-init models (no vocab
  files exist on this machine). It pre-tokenises like a byte-level BPE (words
  with their leading space, digit groups, punctuation runs; long words split
  into <= 6-byte pieces) and maps each multi-byte piece to a stable hashed id
  (crc32, identical in every process) in ``[OFFSET+256, vocab)``, single bytes
  to ``[OFFSET, OFFSET+256)``. Token counts therefore track a real BPE (~1.3
  tokens per English word) instead of one token per byte, so prompt/prefill
  load in benchmarks is realistic. Round-trips are exact (the piece of every
  id this process encoded is remembered; a hash collision falls back to the
  piece's bytes); ids never encoded here (a random model emits them freely)
  decode to short deterministic pseudo-words.
"""
from __future__ import annotations

import re
import zlib
from pathlib import Path

_PRETOK = re.compile(rb" ?[A-Za-z]+| ?[0-9]{1,3}| ?[^\sA-Za-z0-9]+|\s+")

_SYLL = ["ka", "lo", "mi", "ne", "ru", "ta", "vo", "zi", "pe", "sa", "do", "fu", "gi", "ha", "ju", "be"]


class SyntheticTokenizer:
    OFFSET = 3  # 0 pad, 1 bos, 2 eos (overridable)

    def __init__(self, vocab_size: int, bos_token_id: int = 1, eos_token_ids=(2,)):
        self.vocab_size = vocab_size
        self.bos_token_id = bos_token_id
        self.eos_token_ids = tuple(eos_token_ids)
        self._special = {bos_token_id, *self.eos_token_ids}
        self._lo = self.OFFSET + 256
        self._table: dict[int, bytes] = {}
        # hot-path caches (encode runs on the serving event loop, decode on the engine thread at
        # every finished request): the ids of each pre-tokenised word, and the bytes of each id
        self._word_ids: dict[bytes, tuple] = {}
        self._bytes: list = [None] * max(0, vocab_size)

    def _pieces(self, data: bytes):
        for m in _PRETOK.finditer(data):
            p = m.group()
            for i in range(0, len(p), 6):
                yield p[i: i + 6]

    def _encode_word(self, word: bytes) -> tuple:
        ids = []
        span = self.vocab_size - self._lo
        for i in range(0, len(word), 6):
            p = word[i: i + 6]
            if len(p) > 1 and span > 0:
                t = self._lo + zlib.crc32(p) % span
                if t not in self._special:
                    prev = self._table.setdefault(t, p)
                    if prev == p:
                        if t < len(self._bytes):
                            self._bytes[t] = p  # the learned piece replaces a pseudo-word
                        ids.append(t)
                        continue
            ids.extend(self.OFFSET + b for b in p)
        return tuple(ids)

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = [self.bos_token_id] if add_bos else []
        cache = self._word_ids
        for word in _PRETOK.findall(text.encode("utf-8")):
            w = cache.get(word)
            if w is None:
                w = self._encode_word(word)
                if len(cache) < 1 << 20:
                    cache[word] = w
            ids.extend(w)
        return ids

    def _piece(self, t: int) -> bytes:
        if t in self._special:
            return b""
        if self.OFFSET <= t < self._lo:
            return bytes([t - self.OFFSET])
        known = self._table.get(t)
        if known is not None:
            return known
        h = (t * 2654435761) & 0xFFFFFFFF
        w = _SYLL[h & 15] + _SYLL[(h >> 4) & 15]
        if (h >> 8) & 1:
            w += _SYLL[(h >> 12) & 15]
        return (" " + w).encode()

    def _piece_cached(self, t: int) -> bytes:
        b = self._bytes
        if 0 <= t < len(b):
            v = b[t]
            if v is None:
                v = b[t] = self._piece(t)
            return v
        return self._piece(t)

    def decode(self, ids: list[int]) -> str:
        return self.decode_bytes(ids).decode("utf-8", errors="replace")

    def decode_bytes(self, ids: list[int]) -> bytes:
        return b"".join(map(self._piece_cached, ids))


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
