"""Tensor-parallel process group: one process per GPU, RCCL over xGMI.

``torch.distributed`` with backend ``"nccl"`` IS RCCL on ROCm. The model calls
only two collectives per transformer layer (after the row-parallel o_proj and
down_proj) plus one all-reduce after the vocab-parallel embedding and one
all-gather of the vocab-sharded logits — the Megatron layout of SURVEY.md §2.3.1.

All-reduces up to ``CUSTOM_AR_MAX_BYTES`` (8 MiB) go to the custom xGMI kernels
(:mod:`vgate.parallel.custom_allreduce`: one-shot to 512 KiB, two-shot above) and the
logits all-gather to its IPC all-gather, when they are available (all ranks on one node
with peer access); larger messages, and every collective of a CPU (gloo) group, go
through torch.distributed.
All collectives issue on the current stream, so they are hipGraph-capturable.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


# tests: the last rank adds this to the first element of every all-reduce result it gets, as if it
# had read a peer's partial stale (a torch op after the collective: captured into the step graphs
# with it). 0 = off. tests/test_tp_cpu.py, tests/test_tp_gpu.py (the run-time divergence guard).
_INJECT_DIVERGENCE = 0.0


def checksum64(t: torch.Tensor) -> torch.Tensor:
    """Order- and position-sensitive 64-bit checksum of ``t``'s bits (int64 scalar on t's device):
    sum_i bits_i * (i * 2654435761 + 1) in wrapping int64 arithmetic — exact integer adds, so the
    same bits give the same value whatever the reduction order."""
    flat = t.contiguous().reshape(-1)
    if flat.element_size() == 4:
        bits = flat.view(torch.int32).to(torch.int64)
    elif flat.element_size() == 2:
        bits = flat.view(torch.int16).to(torch.int64)
    else:
        bits = flat.view(torch.int64) if flat.element_size() == 8 else flat.to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) * 2654435761 + 1
    return (bits * w).sum()


@dataclass
class TPGroup:
    rank: int = 0
    size: int = 1
    group: object = None
    backend: str = "none"
    custom_ar: object = None
    # one process measuring rank `rank` of a `size`-way group on one GPU (benchmarks/tp_rank_bench.py):
    # the model is sharded exactly as that rank's, every collective is a no-op (the all-gather
    # replicates the local shard), no process group exists
    simulated: bool = False

    @property
    def is_first(self) -> bool:
        return self.rank == 0

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the TP group."""
        if self.size == 1 or self.simulated:
            return t
        if self.custom_ar is not None and self.custom_ar.should_use(t):
            t = self.custom_ar.all_reduce(t)
        elif self.backend == "gloo" and t.dtype in (torch.bfloat16, torch.float16):
            f = t.float()
            dist.all_reduce(f, group=self.group)
            t.copy_(f)
        else:
            dist.all_reduce(t, group=self.group)
        if _INJECT_DIVERGENCE and self.rank == self.size - 1:
            t.view(-1)[:1] += _INJECT_DIVERGENCE
        return t

    def exchange_words(self, words: torch.Tensor) -> torch.Tensor:
        """All-gather a small int64 vector over the group -> [size, n] (host tensor); RCCL takes the
        device tensor, gloo a host copy. The run-time consistency guard's exchange (engine)."""
        if self.size == 1 or self.simulated:
            return words.reshape(1, -1).cpu()
        src = words if self.backend == "nccl" else words.cpu()
        out = torch.empty((self.size, src.numel()), dtype=src.dtype, device=src.device)
        if self.backend == "gloo":
            dist.all_gather(list(out.unbind(0)), src, group=self.group)
        else:
            dist.all_gather_into_tensor(out, src, group=self.group)
        return out.cpu()

    def all_gather_lastdim(self, t: torch.Tensor) -> torch.Tensor:
        """[..., n] per rank -> [..., n * size] concatenated in rank order."""
        if self.size == 1:
            return t
        if self.simulated:
            return t.repeat(*([1] * (t.dim() - 1)), self.size)
        t = t.contiguous()
        if self.custom_ar is not None and self.custom_ar.should_gather(t):
            out = self.custom_ar.all_gather(t)
            return out.movedim(0, -2).reshape(*t.shape[:-1], self.size * t.shape[-1])
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if self.backend == "gloo":
            parts = list(out.unbind(0))
            dist.all_gather(parts, t, group=self.group)
        else:
            dist.all_gather_into_tensor(out, t, group=self.group)
        return out.movedim(0, -2).reshape(*t.shape[:-1], self.size * t.shape[-1])

    def custom_bytes(self) -> int:
        """Largest message the IPC collectives take (0 without them)."""
        return self.custom_ar.max_bytes if self.custom_ar is not None else 0

    def broadcast_object(self, obj, src: int = 0):
        if self.size == 1 or self.simulated:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def barrier(self):
        if self.size > 1 and not self.simulated:
            dist.barrier(group=self.group)


_TP: TPGroup | None = None


def normalize_backend(name: str) -> str:
    """A default group initialised without an explicit backend reports a compound string such as
    'cpu:gloo,cuda:nccl': its GPU collectives run on RCCL, so treat it as 'nccl'."""
    name = str(name)
    if "nccl" in name:
        return "nccl"
    return "gloo" if "gloo" in name else name


CUSTOM_AR_MAX_BYTES = 8 << 20


def init_tp(tp_size: int, backend: str | None = None, timeout_s: float = 120.0, custom_allreduce: bool = True,
            fused_allreduce: bool = True) -> TPGroup:
    """Initialise (or return) the TP group from torchrun-style env vars.

    With tp_size == 1 no process group is created. With tp_size > 1 the caller
    must have launched ``tp_size`` processes (torchrun) with RANK/WORLD_SIZE/
    MASTER_ADDR/MASTER_PORT set; LOCAL_RANK selects the GPU. ``timeout_s`` bounds every
    collective of a new process group (a dead peer fails the group instead of torch's 10 min);
    ``custom_allreduce`` / ``fused_allreduce``: the IPC kernels and the GEMM-epilogue all-reduce
    (model.tp_custom_allreduce / model.tp_fused_allreduce).
    """
    global _TP
    if _TP is not None and _TP.size == tp_size:
        return _TP
    if tp_size == 1:
        _TP = TPGroup()
        return _TP
    if backend is None:
        # an already-initialised default group decides (e.g. gloo carrying GPU tensors when
        # several ranks share one GPU in tests); otherwise RCCL on GPUs, gloo on CPU
        if dist.is_initialized():
            backend = normalize_backend(dist.get_backend())
        else:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        from datetime import timedelta

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, timeout=timedelta(seconds=float(timeout_s)))
    world = dist.get_world_size()
    rank = dist.get_rank()
    if world % tp_size:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    # contiguous TP groups: ranks [k*tp, (k+1)*tp)
    grp = None
    for k in range(world // tp_size):
        ranks = list(range(k * tp_size, (k + 1) * tp_size))
        g = dist.new_group(ranks, backend=backend) if world != tp_size else dist.group.WORLD
        if rank in ranks:
            grp = g
    _TP = TPGroup(rank=rank % tp_size, size=tp_size, group=grp, backend=normalize_backend(backend))
    # the one-shot kernel maps peer buffers over IPC; the group only exchanges the handles
    if torch.cuda.is_available() and custom_allreduce:
        from vgate.parallel.custom_allreduce import maybe_create

        dev = torch.device("cuda", torch.cuda.current_device())
        _TP.custom_ar = maybe_create(grp, _TP.rank, tp_size, dev, max_bytes=CUSTOM_AR_MAX_BYTES,
                                     fused=fused_allreduce)
    return _TP


def get_tp() -> TPGroup:
    return _TP if _TP is not None else TPGroup()


def shard_range(n: int, rank: int, size: int) -> tuple[int, int]:
    assert n % size == 0, f"{n} not divisible by tp={size}"
    per = n // size
    return rank * per, (rank + 1) * per
