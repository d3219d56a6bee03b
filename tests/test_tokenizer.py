"""Synthetic tokenizer: exact round trips, BPE-like token counts, cross-process stable ids,
incremental UTF-8 decoding."""
import subprocess
import sys

from vgate.runtime.tokenizer import IncrementalDecoder, SyntheticTokenizer

V = 151936


def test_round_trip_exact():
    t = SyntheticTokenizer(V)
    for s in ["", "a", "Hello, world!", "héllo wörld 12345 ... ok!!  \n\tx", "日本語のテキスト", "x" * 40,
              "User: Explain the concept of machine learning in one paragraph.\nAssistant:"]:
        assert t.decode(t.encode(s)) == s


def test_token_counts_are_bpe_like():
    t = SyntheticTokenizer(V)
    s = "Explain the concept of machine learning in one paragraph."
    n = len(t.encode(s))
    assert 8 <= n <= 16  # ~1-1.5 tokens per word, not one per byte (57 bytes)


def test_ids_stable_across_processes():
    s = "the quick brown fox jumps over the lazy dog"
    code = ("from vgate.runtime.tokenizer import SyntheticTokenizer as T;"
            f"print(T({V}).encode({s!r}))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout
    assert eval(out) == SyntheticTokenizer(V).encode(s)


def test_special_and_unknown_ids():
    t = SyntheticTokenizer(V, bos_token_id=1, eos_token_ids=(2,))
    assert t.encode("hi", add_bos=True)[0] == 1
    assert t.decode([2]) == ""
    w = t.decode([123457])  # never encoded: deterministic pseudo-word
    assert w and w == SyntheticTokenizer(V).decode([123457])
    assert all(1 <= i < V for i in t.encode("any text at all 0123456789"))


def test_incremental_decoder_multibyte():
    t = SyntheticTokenizer(V)
    ids = t.encode("é")  # single multi-byte char -> byte tokens
    d = IncrementalDecoder(t)
    out = "".join(d.push(i) for i in ids) + d.flush()
    assert out == "é"
