"""Engine core in its own process (vgate/runtime/engine_process.py) on CPU: the proxy
returns exactly the in-process engine's greedy tokens, streams deltas, aborts, serves
embeddings and snapshots, and fails pending requests when the core dies."""
from __future__ import annotations

import threading

import pytest

from vgate.runtime.engine import EngineConfig, LLMEngine
from vgate.runtime.engine_process import EngineProcessClient
from vgate.runtime.sampling_params import SamplingParams

PROMPTS = {f"p{i}": [5 + (i * 37 + j * 11) % 400 for j in range(6 + 5 * i)] for i in range(4)}


def _cfg():
    return EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8, max_num_batched_tokens=64,
                        num_kv_blocks=128, warmup=False, seed=0)


def _collect(eng, reqs, stream=False):
    done, deltas = {}, {}
    ev = threading.Event()

    def cb(kind, seq, payload):
        if kind == "token":
            deltas.setdefault(seq.request_id, []).append(payload)
            return
        done[seq.request_id] = (kind, list(seq.output_ids), seq.finish_reason, seq.text, payload)
        if len(done) == len(reqs):
            ev.set()

    for rid, ids, sp in reqs:
        eng.add_request(rid, params=sp, callback=cb, prompt_ids=ids, stream=stream)
    if isinstance(eng, LLMEngine):
        eng.run_until_idle()
    assert ev.wait(120)
    return done, deltas


@pytest.mark.timeout(300)
def test_engine_process_matches_in_process():
    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    reqs = [(k, v, sp) for k, v in PROMPTS.items()]
    ref, _ = _collect(LLMEngine(_cfg()), reqs)
    cli = EngineProcessClient(_cfg())
    try:
        got, _ = _collect(cli, reqs)
        assert {k: v[1] for k, v in got.items()} == {k: v[1] for k, v in ref.items()}
        assert all(v[0] == "finish" and v[2] == "length" for v in got.values())
        # streaming: deltas arrive before the finish and concatenate to the final text
        sgot, deltas = _collect(cli, [("s0", PROMPTS["p1"], sp)], stream=True)
        assert len(deltas["s0"]) >= 1 and "".join(deltas["s0"]) == sgot["s0"][3]
        # embeddings + snapshot through the pipe
        vec, n = cli.embed(prompt_ids=PROMPTS["p0"])
        assert n == len(PROMPTS["p0"]) and len(vec) > 0
        snap = cli.snapshot()
        assert "kv_usage" in snap and cli.healthy
        # abort: a long request is cut short
        long_sp = SamplingParams(temperature=0.0, max_tokens=200, ignore_eos=True)
        ev = threading.Event()
        res = {}

        def cb(kind, seq, payload):
            if kind != "token":
                res["reason"] = seq.finish_reason
                ev.set()

        cli.add_request("long", params=long_sp, callback=cb, prompt_ids=PROMPTS["p2"])
        cli.abort("long")
        assert ev.wait(60) and res["reason"] in ("abort", "length")
    finally:
        cli.stop()
    assert not cli.healthy
    # after stop, new requests fail immediately instead of hanging
    err = {}
    cli.add_request("late", params=sp, callback=lambda k, s, p: err.setdefault("kind", k), prompt_ids=[1, 2, 3])
    assert err.get("kind") == "error"
