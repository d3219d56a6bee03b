"""Tensor parallelism on CPU (gloo, world_size 2): a TP=2 engine loaded from a TP=1
checkpoint (column/row-parallel linears, vocab-parallel embedding + LM head, per-rank KV
heads, rank-0-driven step broadcast) must generate exactly the TP=1 engine's greedy
tokens. Mirrors the MI355X layout (RCCL over xGMI) with the gloo backend."""
from __future__ import annotations

import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

from vgate.models.weights import save_checkpoint
from vgate.runtime.engine import EngineConfig, LLMEngine
from vgate.runtime.sampling_params import SamplingParams

PROMPTS = {f"p{i}": [5 + (i * 37 + j * 11) % 400 for j in range(6 + 7 * i)] for i in range(4)}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(path, tp, timeout=120.0, **kw):
    return EngineConfig(model=path, device="cpu", tensor_parallel_size=tp, max_model_len=256, max_num_seqs=8,
                        max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0,
                        tp_timeout_seconds=timeout, **kw)


def _generate(eng):
    done = {}

    def cb(kind, seq, payload):
        if kind in ("finish", "error"):
            done[seq.request_id] = list(seq.output_ids)

    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    for rid, ids in PROMPTS.items():
        eng.add_request(rid, params=sp, callback=cb, prompt_ids=ids)
    eng.run_until_idle()
    return done


def _worker(rank, world, port, path, q, overlap_min=None, embed_ids=None, interval=None, inject=0.0):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if overlap_min is not None:  # row-chunked row-parallel GEMMs + per-chunk all-reduce
            from vgate.models import transformer
            transformer.TP_OVERLAP_MIN_TOKENS, transformer.TP_OVERLAP_CHUNKS = overlap_min, 3
        if inject:  # the last rank's all-reduce results are perturbed (run-time divergence guard)
            from vgate.parallel import comm
            comm._INJECT_DIVERGENCE = inject
        torch.set_num_threads(1)
        eng = LLMEngine(_cfg(path, world, **({"tp_consistency_interval": interval} if interval else {})))
        assert eng.tp.size == world and eng.tp.rank == rank
        assert eng.model.num_heads_local * world == eng.arch.num_heads
        if interval:
            if rank == 0:
                try:
                    out = {"gen": _generate(eng), "error": None}
                except Exception as e:  # noqa: BLE001 - the guard fails the step
                    out = {"gen": None, "error": f"{type(e).__name__}: {e}"}
                out.update(healthy=eng.healthy, state=eng.tp_consistency, checks=eng.tp_consistency_checks)
                eng.shutdown_followers()
                q.put(("ok", out))
            else:
                eng.follower_loop()
                q.put(("ok", None) if eng.tp_consistency_checks > 0 else ("err", "follower ran no check"))
            return
        if rank == 0:
            out = _generate(eng)
            if embed_ids is not None:  # the followers run the same hidden-states forward
                vec, n = eng.embed(prompt_ids=embed_ids)
                out = {"gen": out, "embed": vec}
            eng.shutdown_followers()
            q.put(("ok", out))
        else:
            eng.follower_loop()
            q.put(("ok", None))
    except Exception:  # noqa: BLE001
        q.put(("err", traceback.format_exc()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("overlap_min", [None, 16])
def test_tp2_matches_tp1(tmp_path, overlap_min):
    ref_eng = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8,
                                     max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0))
    path = str(tmp_path / "ckpt")
    save_checkpoint(ref_eng.model, path)
    ref = _generate(LLMEngine(_cfg(path, 1)))
    assert set(ref) == set(PROMPTS) and all(len(v) == 8 for v in ref.values())

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, q, overlap_min)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    tp_out = next(r[1] for r in results if r[1] is not None)
    assert tp_out == ref


def _run_group(world, path, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=280) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    return next(r[1] for r in results if r[1] is not None)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [4, 8])
def test_tp4_tp8_match_tp1_with_kv_replication_vocab_padding_and_embed(tmp_path, world):
    """TP 4 / 8 over gloo (one process per rank, the shared-memory step ring carrying every plan):
    2 KV heads replicated over 4 / 8 ranks, a 500-token vocabulary padded to whole 16-row
    shards per rank; greedy tokens == TP=1 and the embedding (hidden-states forward that the
    followers join) == TP=1's."""
    base = LLMEngine(EngineConfig(model="tiny-tp8", device="cpu", max_model_len=256, max_num_seqs=8,
                                  max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=3))
    path = str(tmp_path / "ckpt")
    save_checkpoint(base.model, path)
    ref_eng = LLMEngine(_cfg(path, 1))
    ref = _generate(ref_eng)
    eids = [7, 9, 11, 13, 200, 300, 499]
    ref_vec, _ = ref_eng.embed(prompt_ids=eids)
    out = _run_group(world, path, embed_ids=eids)
    assert out["gen"] == ref
    a, b = torch.tensor(out["embed"]), torch.tensor(ref_vec)
    # the row-parallel partial sums are rounded to bf16 per rank before the all-reduce
    assert torch.allclose(a, b, atol=3e-3) and torch.nn.functional.cosine_similarity(a, b, 0) > 0.999


def test_tp_group_routes_small_allreduce_to_custom_ar():
    """TPGroup.all_reduce: a tensor the custom all-reduce accepts goes to it (one-shot xGMI
    kernel, tests/test_custom_allreduce_gpu.py), anything else to torch.distributed."""
    import torch

    from vgate.parallel.comm import TPGroup

    class FakeAR:
        def __init__(self):
            self.seen = []

        def should_use(self, t):
            return t.numel() <= 16

        def all_reduce(self, t):
            self.seen.append(t.numel())
            return t.mul_(2)

    g = TPGroup(rank=0, size=2, group=None, backend="nccl", custom_ar=FakeAR())
    t = torch.ones(8)
    assert g.all_reduce(t) is t and t.tolist() == [2.0] * 8 and g.custom_ar.seen == [8]


def _failing_worker(rank, world, port, path, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    eng = LLMEngine(_cfg(path, world, timeout=20))
    if rank == 1:
        def boom(*a, **k):
            raise RuntimeError("injected follower fault")
        eng.runner.follow_step = boom
        eng.follower_loop()  # exits the process with status 1
        q.put(("returned", None))
        return
    try:
        _generate(eng)
        q.put(("rank0", "no error"))
    except Exception as e:  # noqa: BLE001 - expected: the peer is gone
        q.put(("rank0", type(e).__name__))


@pytest.mark.timeout(300)
def test_tp_follower_fault_tears_down_group(tmp_path):
    """a TP group is one failure domain — a follower fault exits that rank
    (status 1) and rank 0's next collective fails instead of hanging."""
    ref_eng = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8,
                                     max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0))
    path = str(tmp_path / "ckpt")
    save_checkpoint(ref_eng.model, path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    procs[1].join(timeout=200)
    assert procs[1].exitcode == 1
    kind, val = q.get(timeout=200)
    assert kind == "rank0" and val != "no error", (kind, val)
    procs[0].join(timeout=60)


def _idle_worker(rank, world, port, path, q, idle_s):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        torch.set_num_threads(1)
        eng = LLMEngine(_cfg(path, world, timeout=2))
        if rank != 0:
            eng.follower_loop()  # os._exit(1) if it sees no heartbeat for 2 s
            q.put(("ok", None))
            return
        import threading
        import time as _t
        eng.start()  # the serving loop: idle, waiting for requests
        _t.sleep(idle_s)
        done, ev = {}, threading.Event()

        def cb(kind, seq, payload):
            if kind in ("finish", "error"):
                done[seq.request_id] = (kind, list(seq.output_ids))
                if len(done) == len(PROMPTS):
                    ev.set()

        sp = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)
        for rid, ids in PROMPTS.items():
            eng.add_request(rid, params=sp, callback=cb, prompt_ids=ids)
        ok = ev.wait(60)
        eng.stop()
        q.put(("ok", {"finished": ok, "done": done}))
    except Exception:  # noqa: BLE001
        q.put(("err", traceback.format_exc()))


@pytest.mark.timeout(300)
def test_tp_group_survives_idle_longer_than_timeout(tmp_path):
    """ROUND-2 ADVICE (high): rank 0 must stamp the step-ring heartbeat while its serving loop
    idles, else every follower's ring wait times out after tp_timeout_seconds and the group
    tears itself down. Idle 5 s at a 2 s timeout, then serve: every request completes."""
    ref_eng = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8,
                                     max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0))
    path = str(tmp_path / "ckpt")
    save_checkpoint(ref_eng.model, path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_idle_worker, args=(r, 2, port, path, q, 5.0)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=200) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    out = next(r[1] for r in results if r[1] is not None)
    assert out["finished"], out
    assert all(kind == "finish" and len(ids) == 4 for kind, ids in out["done"].values()), out
    assert procs[1].exitcode == 0


def test_simulated_rank_runs_the_rank_shapes_without_a_group():
    """TPGroup(simulated=True): one process builds rank r's shard of a TP=4 model (no process
    group, collectives no-ops, the all-gather replicates the shard) and steps it — the per-rank
    shape bench (benchmarks/tp_rank_bench.py) on one GPU."""
    from vgate.parallel.comm import TPGroup
    from vgate.runtime.engine import EngineConfig, LLMEngine
    from vgate.runtime.sampling_params import SamplingParams

    tp = TPGroup(rank=1, size=4, simulated=True)
    eng = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=128, max_num_seqs=4,
                                 max_num_batched_tokens=64, num_kv_blocks=32, warmup=False,
                                 tensor_parallel_size=4), tp=tp)
    assert eng.model.num_heads_local * 4 == eng.arch.num_heads and eng.ring is None
    x = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    assert torch.equal(tp.all_gather_lastdim(x), torch.cat([x] * 4, -1))
    assert tp.all_reduce(x) is x
    done = {}
    eng.add_request("a", prompt_ids=[3, 4, 5, 6], callback=lambda k, s, p: done.update({s.request_id: s}),
                    params=SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))
    eng.run_until_idle()
    assert len(done["a"].output_ids) == 3


def test_decode_plan_table_applies_to_matching_shapes():
    """vgate/models/decode_plans.py: measured per-shape decode decompositions land on the Linear
    objects whose (N, K, layout, kind) match (the 70B TP=8 rank shapes), nothing else changes."""
    from types import SimpleNamespace

    from vgate.models import decode_plans

    def lin(N, K, layout="plain", kind="dense"):
        return SimpleNamespace(N=N, K=K, layout=layout, kind=kind, dec_waves=0, dec_splitk=0, dec_ntb=0)

    L = SimpleNamespace(qkv=lin(1280, 8192, "qkv"), o=lin(8192, 1024), gate_up=lin(7168, 8192, "silu"),
                        down=lin(8192, 3584))
    other = SimpleNamespace(qkv=lin(2048, 1536, "qkv"), o=lin(1536, 1536), gate_up=lin(17920, 1536, "silu"),
                            down=lin(1536, 8960))
    m = SimpleNamespace(layers=[L, other], lm_head=lin(16032, 8192))
    assert decode_plans.apply(m) == 5
    assert (L.gate_up.dec_waves, L.gate_up.dec_splitk) == (4, 1) and L.qkv.dec_splitk == 3
    assert all(getattr(other, k).dec_waves == 0 for k in ("qkv", "o", "gate_up", "down"))


@pytest.mark.timeout(300)
def test_tp_runtime_consistency_guard(tmp_path):
    """Run-time divergence guard: every 2nd step the ranks compare checksums of
    their replicated logits. Clean: tokens == TP = 1 and the checks ran on every rank. With the
    last rank's all-reduce results perturbed (as if it read a peer's partial stale): the first
    check fails the step, marks rank 0 unhealthy with the reason, on every rank."""
    ref_eng = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8,
                                     max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0))
    path = str(tmp_path / "ckpt")
    save_checkpoint(ref_eng.model, path)
    ref = _generate(LLMEngine(_cfg(path, 1)))
    clean = _run_group(2, path, interval=2)
    assert clean["error"] is None and clean["gen"] == ref
    assert clean["healthy"] and clean["state"] == "ok" and clean["checks"] >= 3
    bad = _run_group(2, path, interval=2, inject=0.25)
    assert bad["error"] is not None and bad["error"].startswith("TPDivergence"), bad
    assert not bad["healthy"] and "diverged" in bad["state"] and "ranks [1]" in bad["state"]
    assert bad["checks"] == 1


def test_checksum64_is_exact_and_position_sensitive():
    """The consistency guard's checksum: same bits -> same value whatever the reduction order (exact
    wrapping int64 adds), any single-bit or position change -> a different value, all dtypes."""
    from vgate.parallel.comm import checksum64
    torch.manual_seed(3)
    for dt in (torch.float32, torch.bfloat16, torch.int32, torch.int64):
        t = (torch.randn(37, 129) * 100).to(dt)
        a = int(checksum64(t))
        assert a == int(checksum64(t.clone().contiguous()))
        assert a == int(checksum64(t.t().contiguous().t()))  # non-contiguous view of the same values
        u = t.clone()
        flat = u.view(-1)
        flat[1000] = flat[1001] if flat[1000] != flat[1001] else flat[1000] + 1
        assert int(checksum64(u)) != a
        sw = t.clone().view(-1)
        i, j = 5, 4000
        if sw[i] != sw[j]:
            sw[i], sw[j] = sw[j].clone(), sw[i].clone()
            assert int(checksum64(sw)) != a  # a permutation changes it


def test_exchange_words_single_rank():
    from vgate.parallel.comm import TPGroup
    w = torch.tensor([1, -2, 3], dtype=torch.int64)
    out = TPGroup().exchange_words(w)
    assert out.shape == (1, 3) and torch.equal(out[0], w)
