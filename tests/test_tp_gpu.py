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


def _cfg(path, tp, eager=False):
    from vgate.runtime.engine import EngineConfig

    return EngineConfig(model=path, device="cuda:0", tensor_parallel_size=tp, max_model_len=512, max_num_seqs=8,
                        max_num_batched_tokens=320, num_kv_blocks=256, warmup=False, seed=0,
                        enforce_eager=eager)


def _generate(eng):
    from vgate.runtime.sampling_params import SamplingParams

    done = {}

    def cb(kind, seq, payload):
        if kind in ("finish", "error"):
            done[seq.request_id] = list(seq.output_ids)

    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    for rid, ids in PROMPTS.items():
        eng.add_request(rid, params=sp, callback=cb, prompt_ids=ids)
    eng.run_until_idle()
    return done


def _worker(rank, world, port, path, q, eager=False):
    try:
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), VGATE_TP_TIMEOUT_S="60")
        import torch.distributed as dist

        from vgate.runtime.engine import LLMEngine

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        eng = LLMEngine(_cfg(path, world, eager))
        assert eng.tp.size == world and eng.tp.rank == rank and eng.tp.backend == "gloo"
        eng.runner.defer_capture = False
        assert eng.model.num_heads_local * world == eng.arch.num_heads
        if rank == 0:
            out = _generate(eng)
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
@pytest.mark.parametrize("eager", [False, True])
def test_tp2_on_gpu_matches_tp1(tmp_path, eager):
    """graph == eager == TP=1: with every decode collective on the IPC kernels (all-reduce and the
    logits all-gather) a gloo TP group replays captured hipGraphs for the buckets they cover."""
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
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, q, eager)) for r in range(2)]
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
    tp_out, used_ar, graphs = next(r[1] for r in results if r[1] is not None)
    assert used_ar, "the custom all-reduce was not used between the two ranks"
    assert tp_out == ref
    assert (graphs > 0) == (not eager), graphs
