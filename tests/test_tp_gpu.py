"""Tensor parallelism on a real MI355X: a TP=2 engine whose two ranks share the box's one
GPU must generate the TP=1 GPU engine's greedy tokens from the same checkpoint.

Both ranks run the sharded model through the gfx950 kernels (column-parallel QKV with
per-rank heads + RoPE/KV-write epilogue, row-parallel o/down, vocab-parallel embedding and
LM head). All-reduces of decode size go through the custom one-shot kernel over IPC-mapped
peer buffers (csrc/kernels/allreduce.hip, the same mapping two GPUs of a node use over
xGMI); larger ones and the logits all-gather go through a gloo group carrying GPU tensors,
since RCCL refuses two ranks on one device. On an 8-GPU node (the 70B TP=8 config) the
same code runs over RCCL. CPU twin: tests/test_tp_cpu.py.
"""
from __future__ import annotations

import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PROMPTS = {f"p{i}": [5 + (i * 37 + j * 11) % 400 for j in range(6 + 7 * i)] for i in range(4)}
# >= 256 prompt tokens: the row-parallel GEMMs run in row chunks with each chunk's all-reduce on
# the comm stream (fork / join through events) through the custom kernel
PROMPTS["long"] = [3 + (j * 29) % 500 for j in range(300)]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(path, tp, eager=False, tokens=320, **opts):
    from vgate.runtime.engine import EngineConfig

    return EngineConfig(model=path, device="cuda:0", tensor_parallel_size=tp, max_model_len=1024, max_num_seqs=8,
                        max_num_batched_tokens=tokens, num_kv_blocks=256, warmup=False, seed=0,
                        enforce_eager=eager, tp_timeout_seconds=60.0, **opts)


def _generate(eng, prompts=None):
    from vgate.runtime.sampling_params import SamplingParams

    done = {}

    def cb(kind, seq, payload):
        if kind in ("finish", "error"):
            done[seq.request_id] = list(seq.output_ids)

    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    for rid, ids in (prompts or PROMPTS).items():
        eng.add_request(rid, params=sp, callback=cb, prompt_ids=ids)
    eng.run_until_idle()
    return done


# >= 512 tokens in ONE prefill step: the row-parallel all-reduces of the chunked prefill move
# 512-token slices through the two-shot kernel (VGATE_AR_TWO_SHOT=1 forces it; at TP = 2 the size
# rule never picks it)
LONG = {"long600": [7 + (j * 13) % 450 for j in range(600)], "short": [9, 8, 7, 6, 5]}


def _worker(rank, world, port, path, q, eager=False, env=None, tokens=320, prompts=None, opts=None, inject=False,
            runs=None):
    """One TP rank. ``runs``: [(eager, opts), ...] engines built one after another in this process group
    (one spawn for several configurations: a spawn costs ~3 s of the GPU tier); rank 0 reports
    [(tokens, used_ar, graphs), ...]."""
    if runs is not None:
        try:
            os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port), **(env or {}))
            import torch.distributed as dist

            from vgate.runtime.engine import LLMEngine

            torch.cuda.set_device(0)
            dist.init_process_group("gloo", rank=rank, world_size=world)
            res = []
            for ea, op in runs:
                eng = LLMEngine(_cfg(path, world, ea, tokens, **(op or {})))
                eng.runner.defer_capture = False
                assert eng.tp_self_check == "passed", eng.tp_self_check
                if rank == 0:
                    out = _generate(eng, prompts)
                    res.append((out, eng.tp.custom_ar is not None and eng.tp.custom_ar.calls > 0,
                                len(eng.runner.graphs)))
                    eng.shutdown_followers()
                else:
                    eng.follower_loop()
                del eng
                torch.cuda.synchronize()
                dist.barrier()
            q.put(("ok", res if rank == 0 else None))
        except Exception:  # noqa: BLE001
            q.put(("err", traceback.format_exc()))
        return
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), **(env or {}))
        if inject:  # the start-up self-check of the last rank sees a corrupted all-reduce result
            from vgate.parallel import custom_allreduce
            custom_allreduce._INJECT_SELF_CHECK_FAULT = True
        import torch.distributed as dist

        from vgate.runtime.engine import LLMEngine

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        eng = LLMEngine(_cfg(path, world, eager, tokens, **(opts or {})))
        assert eng.tp.size == world and eng.tp.rank == rank and eng.tp.backend == "gloo"
        eng.runner.defer_capture = False
        assert eng.model.num_heads_local * world == eng.arch.num_heads
        if inject:
            assert eng.tp.custom_ar is None and eng.tp_self_check.startswith("failed"), eng.tp_self_check
        else:
            assert eng.tp_self_check == "passed", eng.tp_self_check
        if rank == 0:
            out = _generate(eng, prompts)
            used_ar = eng.tp.custom_ar is not None and eng.tp.custom_ar.calls > 0
            graphs = len(eng.runner.graphs)
            eng.shutdown_followers()
            q.put(("ok", (out, used_ar, graphs)))
        else:
            eng.follower_loop()
            q.put(("ok", None))
    except Exception:  # noqa: BLE001
        q.put(("err", traceback.format_exc()))


@pytest.mark.timeout(300)
def test_tp2_on_gpu_matches_tp1(tmp_path):
    """graph == eager == TP=1: with every decode collective on the IPC kernels (all-reduce and the
    logits all-gather) a gloo TP group replays captured hipGraphs for the buckets they cover.
    fused (default): the decode o_proj / down_proj all-reduce inside their GEMM epilogue
    (gemm_epilogue.h epilogue_ar); not fused: the GEMM stores its partial, the one-shot kernel reduces."""
    from vgate.models.weights import save_checkpoint
    from vgate.runtime.engine import EngineConfig, LLMEngine

    src = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8,
                                 max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0))
    path = str(tmp_path / "ckpt")
    save_checkpoint(src.model, path)
    ref_eng = LLMEngine(_cfg(path, 1, True))
    ref = _generate(ref_eng)
    assert set(ref) == set(PROMPTS) and all(len(v) == 8 for v in ref.values())
    del ref_eng
    torch.cuda.synchronize()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    cfgs = [(False, True), (True, True), (False, False)]  # (eager, fused)
    runs = [(e, {"tp_fused_allreduce": f}) for e, f in cfgs]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, q), kwargs={"runs": runs}) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    per_run = next(r[1] for r in results if r[1] is not None)
    assert len(per_run) == len(cfgs)
    for (eager, fused), (tp_out, used_ar, graphs) in zip(cfgs, per_run):
        assert used_ar, ("the custom all-reduce was not used between the two ranks", eager, fused)
        assert tp_out == ref, (eager, fused)
        assert (graphs > 0) == (not eager), (graphs, eager, fused)


@pytest.mark.timeout(300)
def test_tp2_collective_self_check_failure_falls_back_to_tp1_tokens(tmp_path):
    """Start-up self-check: one rank's check sees a wrong custom all-reduce result (test hook); the
    verdict is agreed over the group, EVERY rank drops the custom IPC collectives (RCCL / gloo for
    everything, eager steps on this gloo group) and the generation still equals TP = 1."""
    path = _ckpt(tmp_path)
    ref_eng = __import__("vgate.runtime.engine", fromlist=["LLMEngine"]).LLMEngine(_cfg(path, 1, True))
    ref = _generate(ref_eng)
    del ref_eng
    torch.cuda.synchronize()
    port = _free_port()
    _, q, procs = _spawn(2, _worker, lambda r, q: (r, 2, port, path, q, False, None, 320, None, None, True))
    try:
        results = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    tp_out, used_ar, graphs = next(r[1] for r in results if r[1] is not None)
    assert not used_ar
    assert tp_out == ref


def _ckpt(tmp_path):
    from vgate.models.weights import save_checkpoint
    from vgate.runtime.engine import EngineConfig, LLMEngine

    src = LLMEngine(EngineConfig(model="tiny", device="cpu", max_model_len=256, max_num_seqs=8,
                                 max_num_batched_tokens=64, num_kv_blocks=128, warmup=False, seed=0))
    path = str(tmp_path / "ckpt")
    save_checkpoint(src.model, path)
    return path


def _spawn(n, target, args_of):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=args_of(r, q)) for r in range(n)]
    for p in procs:
        p.start()
    return ctx, q, procs


@pytest.mark.timeout(300)
def test_tp2_two_shot_long_prefill_matches_tp1(tmp_path):
    """A 600-token prompt in one 640-token prefill step at TP = 2 with every all-reduce forced onto
    the two-shot kernel (reduce-scatter + all-gather over the peer buffers) == TP = 1."""
    path = _ckpt(tmp_path)
    ref_eng = __import__("vgate.runtime.engine", fromlist=["LLMEngine"]).LLMEngine(_cfg(path, 1, True, 640))
    ref = _generate(ref_eng, LONG)
    del ref_eng
    torch.cuda.synchronize()
    port = _free_port()
    _, q, procs = _spawn(2, _worker, lambda r, q: (r, 2, port, path, q, False, {"VGATE_AR_TWO_SHOT": "1"}, 640, LONG))
    try:
        results = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    tp_out, used_ar, _ = next(r[1] for r in results if r[1] is not None)
    assert used_ar
    assert tp_out == ref


def _timeout_worker(rank, port, path, q, go):
    import sys

    def say(*a):
        print(f"[rank {rank}]", *a, file=sys.stderr, flush=True)

    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), VGATE_AR_SPIN_LIMIT="200000")
        import torch.distributed as dist

        from vgate.runtime.engine import LLMEngine
        from vgate.runtime.sampling_params import SamplingParams

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        eng = LLMEngine(_cfg(path, 2))
        say("engine up")
        if rank != 0:
            q.put(("pid", os.getpid()))
            eng.follower_loop()
            return
        eng.runner.defer_capture = False
        first = _generate(eng, {"a": [5, 6, 7, 8]})
        assert len(first["a"]) == 8 and eng.healthy
        say("first generation ok")
        eng.start()
        q.put(("ready", None))
        go.wait(120)  # the test stopped rank 1
        say("peer stopped; submitting")
        done = {}
        import threading
        ev = threading.Event()

        def cb(kind, seq, payload):
            if kind in ("finish", "error"):
                done[seq.request_id] = (kind, payload)
                ev.set()

        eng.add_request("b", prompt_ids=[9, 10, 11], callback=cb,
                        params=SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
        ev.wait(60)
        say("request done:", done.get("b"), eng.healthy, eng.last_error)
        q.put(("ok", (done.get("b"), eng.healthy, eng.last_error)))
        q.close()
        q.join_thread()  # the queue's feeder thread must flush before the hard exit below
        os._exit(0)  # rank 1 is stopped: no orderly shutdown of the group
    except Exception:  # noqa: BLE001
        q.put(("err", traceback.format_exc()))


@pytest.mark.timeout(300)
def test_tp2_peer_stops_custom_allreduce_times_out_and_engine_fails(tmp_path):
    """Timeout path of the custom all-reduce: rank 1 is frozen (SIGSTOP) after a good generation;
    rank 0's next step waits for it at the first collective, gives up after the spin limit (set
    short here), every later collective of the step skips the wait (sticky error word), the
    step's last graph node hands the word to the host, and the engine fails the step: the request
    ends with an error and the engine reports unhealthy (its /health then answers 503)."""
    import signal

    path = _ckpt(tmp_path)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    go = ctx.Event()
    procs = [ctx.Process(target=_timeout_worker, args=(r, port, path, q, go)) for r in range(2)]
    for p in procs:
        p.start()
    pid1 = None
    try:
        got = {}
        for _ in range(2):
            kind, val = q.get(timeout=150)
            assert kind != "err", val
            got[kind] = val
        pid1 = got["pid"]
        os.kill(pid1, signal.SIGSTOP)
        go.set()
        kind, val = q.get(timeout=100)
        assert kind == "ok", val
        res, healthy, err = val
        assert res is not None and res[0] == "error", res
        assert not healthy and "custom all-reduce" in (err or ""), err
    finally:
        if pid1 is not None:
            try:
                os.kill(pid1, signal.SIGKILL)
            except ProcessLookupError:
                pass
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()


def _guard_worker(rank, port, path, q, runs):
    """TP = 2 on the one GPU; per run (fused, inject): a consistency-checked generation. Rank 0
    reports (tokens or None, error, healthy, state, checks, custom collectives left on)."""
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
        import torch.distributed as dist

        from vgate.parallel import comm
        from vgate.runtime.engine import LLMEngine

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        res = []
        for fused, inject in runs:
            comm._INJECT_DIVERGENCE = inject
            eng = LLMEngine(_cfg(path, 2, tp_fused_allreduce=fused, tp_consistency_interval=2))
            eng.runner.defer_capture = False
            if rank == 0:
                try:
                    out, err = _generate(eng), None
                except Exception as e:  # noqa: BLE001 - the guard fails the step
                    out, err = None, f"{type(e).__name__}: {e}"
                res.append((out, err, eng.healthy, eng.tp_consistency, eng.tp_consistency_checks,
                            eng.tp.custom_ar is not None))
                eng.shutdown_followers()
            else:
                eng.follower_loop()
                assert eng.tp_consistency_checks > 0
                assert (eng.tp.custom_ar is None) == bool(inject), "the fallback must be group-wide"
            del eng
            torch.cuda.synchronize()
            dist.barrier()
        q.put(("ok", res if rank == 0 else None))
    except Exception:  # noqa: BLE001
        q.put(("err", traceback.format_exc()))


@pytest.mark.timeout(300)
def test_tp2_runtime_consistency_guard(tmp_path):
    """Run-time TP divergence guard on the GPU (graph replay, custom IPC collectives): every 2nd
    step the two ranks compare checksums of the post-all-reduce residual, the logits and the
    sampled ids. Clean (fused epilogue all-reduce): tokens == TP = 1 and no false alarm. With rank
    1's all-reduce results perturbed inside the captured step (the unfused path, as a peer partial
    read stale): the first check fails the step, rank 0 goes unhealthy with the reason, and BOTH
    ranks drop the custom collectives."""
    path = _ckpt(tmp_path)
    ref_eng = __import__("vgate.runtime.engine", fromlist=["LLMEngine"]).LLMEngine(_cfg(path, 1, True))
    ref = _generate(ref_eng)
    del ref_eng
    torch.cuda.synchronize()
    port = _free_port()
    runs = [(True, 0.0), (False, 0.25)]
    _, q, procs = _spawn(2, _guard_worker, lambda r, q: (r, port, path, q, runs))
    try:
        results = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs[0]
    (out, err, healthy, state, checks, car_on), bad = next(r[1] for r in results if r[1] is not None)
    assert err is None and out == ref and healthy and state == "ok" and checks >= 3 and car_on
    out, err, healthy, state, checks, car_on = bad
    assert out is None and err.startswith("TPDivergence") and not healthy and not car_on, bad
    assert "residual" in state and checks == 1, state


_RCCL_GRAPH_SCRIPT = r"""
import torch, torch.distributed as dist
from vgate.parallel.comm import TPGroup
dist.init_process_group("nccl")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
tp = TPGroup(rank=0, size=1, group=dist.group.WORLD, backend="nccl")
x = (torch.arange(4 << 20, device=dev, dtype=torch.float32) % 977).bfloat16()  # 8 MiB: the RCCL size class
ref = x.clone()
out = torch.empty((1,) + tuple(x.shape), dtype=x.dtype, device=dev)
m = torch.tensor([7, 3], dtype=torch.int64, device=dev)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):  # RCCL's first calls (communicator set-up) outside the capture
    dist.all_reduce(x)
    dist.all_gather_into_tensor(out, x)
    dist.all_reduce(m, op=dist.ReduceOp.MIN)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    dist.all_reduce(x)
    dist.all_gather_into_tensor(out, x)
    dist.all_reduce(m, op=dist.ReduceOp.MIN)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
assert torch.equal(x, ref) and torch.equal(out[0], ref) and m.tolist() == [7, 3]
w = tp.exchange_words(torch.tensor([11, 22], dtype=torch.int64, device=dev))
assert w.tolist() == [[11, 22]]
dist.destroy_process_group()
print("rccl-graph-ok")
"""


def test_rccl_collectives_inside_a_captured_graph_single_rank(tmp_path):
    """RCCL (the `nccl` backend) on this stack, one rank on the box's one GPU: an 8 MiB bf16
    all-reduce (the size class the TP path hands to RCCL above the IPC kernels), the logits-style
    all-gather and the int64 MIN-reduce the engine's KV sizing uses, captured in a hipGraph and
    replayed, plus the consistency guard's word exchange. One rank only (RCCL refuses two on one
    device): this executes the RCCL calls and their graph capture, not a cross-device transfer."""
    import subprocess
    import sys

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _RCCL_GRAPH_SCRIPT], env=env, capture_output=True, text=True,
                       timeout=180, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "rccl-graph-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
