"""Custom one-shot / two-shot all-reduce over xGMI peer memory for decode- and chunk-sized
TP collectives.

Each rank owns one uncached device allocation (``ar_alloc``: a signal area plus two
``max_bytes`` data buffers); the ranks exchange ``hipIpcMemHandle``s once over the
process group and map every peer's buffer (``ar_open``). A call launches ONE kernel
(``csrc/kernels/allreduce.hip``): each block copies its slice of the input into the own
buffer, flags its arrival in every peer's signal area, waits for the peers' flags, and
sums that slice over all ranks straight out of the peers' memory — every xGMI link is
used at once and there is a single synchronisation, where a ring pays 2(n-1) dependent
hops. Large messages (prefill) stay on RCCL (:class:`vgate.parallel.comm.TPGroup`).

Launches take fixed addresses and keep their epoch counters on the device, so the
all-reduce is captured into the decode hipGraphs like every other kernel.

Reference parity: the reference has no GPU collectives at all; this
is the MI355X-native data plane the TP engine needs.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("vgate.parallel")

SIGNAL_BYTES = 65536  # csrc/kernels/launchers.h AR_SIGNAL_BYTES
MAX_RANKS = 8
FUSED_TILES = 1024  # launchers.h AR_FUSED_TILES: output columns <= 16 * 1024 for the fused GEMM + all-reduce
_INJECT_SELF_CHECK_FAULT = False  # tests: the last rank's self-check sees a wrong all-reduce result


class CustomAllReduce:
    """One per TP group and device. ``should_use(t)`` says whether ``t`` qualifies (bf16,
    contiguous, 16-byte multiple, <= max_bytes); ``all_reduce(t)`` reduces in place."""

    def __init__(self, group, rank: int, world: int, device: torch.device, max_bytes: int = 8 << 20):
        from vgate import ops

        if not 2 <= world <= MAX_RANKS:
            raise ValueError(f"custom all-reduce supports 2..{MAX_RANKS} ranks, got {world}")
        self.C = ops.native()
        self.rank, self.world, self.device = rank, world, device
        self.fused = True
        self.max_bytes = int(max_bytes)
        self.own, self.bases, self._opened = None, [], []
        mine = None
        try:
            with torch.cuda.device(device):
                # + the fused row-parallel GEMM region (arrival words + two parity tile buffers)
                self.fused_off = SIGNAL_BYTES + 2 * self.max_bytes
                self.own = self.C.ar_alloc(self.fused_off + int(self.C.ar_fused_bytes()))
                mine = bytes(self.C.ar_ipc_handle(self.own).numpy().tobytes())
        except Exception as e:  # noqa: BLE001 - reported through the gather, so no rank waits
            log.warning("custom all-reduce allocation failed: %s: %s", type(e).__name__, e)
        handles = [None] * world
        dist.all_gather_object(handles, mine, group=group)
        if any(h is None for h in handles):
            self.close()
            raise RuntimeError("custom all-reduce setup failed: a rank could not allocate / export its buffer")
        err = None
        try:
            with torch.cuda.device(device):
                for p, h in enumerate(handles):
                    if p == rank:
                        self.bases.append(self.own)
                    else:
                        ptr = self.C.ar_open(torch.frombuffer(bytearray(h), dtype=torch.uint8))
                        self._opened.append(ptr)
                        self.bases.append(ptr)
        except Exception as e:  # noqa: BLE001 - agreed on below, so no rank waits for a failed one
            err = f"{type(e).__name__}: {e}"
        errs = [None] * world
        dist.all_gather_object(errs, err, group=group)  # also: every rank mapped every buffer
        if any(errs):
            self.close()
            raise RuntimeError(f"custom all-reduce setup failed: {[e for e in errs if e]}")
        self.calls = 0
        # VGATE_AR_TWO_SHOT: 1 forces the two-shot kernel for every all-reduce, -1 the one-shot one,
        # 0 (default) picks by size (tests force two-shot at TP = 2, where it is never picked)
        self.force = int(os.environ.get("VGATE_AR_TWO_SHOT", "0"))

    def should_use(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.dtype == torch.bfloat16 and t.is_contiguous() and t.device == self.device and nbytes % 16 == 0
                and 0 < nbytes <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor, out: torch.Tensor | None = None, two_shot: int = 0) -> torch.Tensor:
        """Sum over the group; one-shot up to 512 KiB, two-shot (reduce-scatter + all-gather over
        the direct links) above; two_shot = 1 / -1 forces one form (tests)."""
        out = t if out is None else out
        self.C.custom_allreduce(t, out, self.bases, self.rank, self.max_bytes, two_shot or self.force)
        self.calls += 1
        return out

    def fuses(self, lin, x: torch.Tensor, out: torch.Tensor) -> bool:
        """Whether the row-parallel GEMM ``out = x @ lin^T`` can all-reduce in its epilogue
        (decode rows, bf16 output of at most AR_FUSED_TILES 16-column tiles on this device)."""
        return (self.fused and x.shape[0] <= 16 and out.dtype == torch.bfloat16 and out.device == self.device
                and lin.N // 16 <= FUSED_TILES)

    def should_gather(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return t.is_contiguous() and t.device == self.device and nbytes % 16 == 0 and 0 < nbytes <= self.max_bytes

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[...] per rank -> [world, ...] in rank order (IPC kernel, capturable)."""
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.C.custom_allgather(t, out, self.bases, self.rank, self.max_bytes)
        self.calls += 1
        return out

    def check(self) -> None:
        """Raise if a wait timed out since the last check (a peer never arrived)."""
        if self.C.ar_error(self.own):
            raise RuntimeError("custom all-reduce: a peer did not arrive within the spin limit")

    def self_check(self, group, backend: str, hidden: int, row_lin=None) -> tuple[bool, list[str]]:
        """Start-up cross-check of every custom path against ``torch.distributed`` on ``group``
        (RCCL on a node; every rank calls it at the same point, before any graph capture).

        Cases: the one-shot kernel at decode sizes (1 / 8 / 16 rows x ``hidden``), the two-shot kernel
        at chunk sizes (256 / 512 rows, within ``max_bytes``), the IPC all-gather of a logits-shaped
        fp32 block, and — when ``row_lin`` (a row-parallel Linear of the model) is given and the
        fused epilogue is on — the GEMM with the all-reduce in its epilogue against the same GEMM's
        partial reduced by torch.distributed. Sums are compared within bf16 rounding; a wait that
        gave up (the sticky error word) fails the check too. Returns (ok on EVERY rank, per-case
        failure notes of this rank); the verdict is agreed over the group, so all ranks take the
        same decision (the engine then drops the custom paths group-wide)."""
        dev = self.device
        notes: list[str] = []
        gen = torch.Generator(device=dev)
        gen.manual_seed(4242 + 7919 * self.rank)

        def ref_sum(t: torch.Tensor) -> torch.Tensor:
            r = t.float() if backend == "nccl" else t.float().cpu()
            dist.all_reduce(r, group=group)
            return r.to(dev)

        def close(a: torch.Tensor, b: torch.Tensor, what: str) -> None:
            a, b = a.float(), b.float()
            scale = float(b.abs().max()) + 1e-6
            err = float((a - b).abs().max()) / scale
            if not torch.isfinite(a).all() or err > 2e-2:
                notes.append(f"{what}: max rel err {err:.3g}")

        def rnd(*shape, dtype=torch.bfloat16):
            return torch.randn(*shape, generator=gen, device=dev).to(dtype)

        with torch.cuda.device(dev):
            for rows, form in ((1, -1), (8, -1), (16, -1), (256, 1), (512, 1)):
                if rows * hidden * 2 > self.max_bytes:
                    continue
                t = rnd(rows, hidden)
                want = ref_sum(t)
                got = self.all_reduce(t.clone(), two_shot=form)
                if _INJECT_SELF_CHECK_FAULT and self.rank == self.world - 1:
                    got[0, :8] += 64.0  # test hook: as if a peer's slice had been read stale
                close(got, want, f"{'one' if form < 0 else 'two'}-shot all-reduce {rows}x{hidden}")
            g = rnd(8, 1024, dtype=torch.float32)
            if self.should_gather(g):
                got = self.all_gather(g)
                want = [torch.empty_like(g if backend == "nccl" else g.cpu()) for _ in range(self.world)]
                dist.all_gather(want, g if backend == "nccl" else g.cpu(), group=group)
                close(got, torch.stack([w.to(dev) for w in want]), "all-gather 8x1024 f32")
            if row_lin is not None and self.fused and getattr(row_lin, "wp", None) is not None:
                from vgate import ops
                x = rnd(8, row_lin.K)
                out = torch.zeros(8, row_lin.N, dtype=torch.bfloat16, device=dev)
                if self.fuses(row_lin, x, out):
                    part = ops.linear(x, row_lin)
                    want = ref_sum(part)
                    ops.linear(x, row_lin, out=out, ar=self)
                    close(out, want, f"fused GEMM epilogue all-reduce 8x{row_lin.N}")
            torch.cuda.synchronize(dev)
            if self.C.ar_error(self.own):
                notes.append("a wait gave up (error word set)")
        verdicts = [None] * self.world
        dist.all_gather_object(verdicts, notes, group=group)
        bad = [(r, v) for r, v in enumerate(verdicts) if v]
        return not bad, [f"rank {r}: {'; '.join(v)}" for r, v in bad]

    def close(self) -> None:
        if self.own is None:
            return
        torch.cuda.synchronize(self.device)
        for ptr in self._opened:
            self.C.ar_close(ptr)
        self.C.ar_free(self.own)
        self.own, self._opened = None, []


class LoopbackFused:
    """A one-rank fused all-reduce region (world 1: every tile exchanges with itself). It prices
    the fused epilogue — partial store, arrival word, poll, re-read — on one GPU without peers
    (``benchmarks/tp_rank_bench.py --fused-ar``, the kernel tests); the standalone collectives
    stay no-ops (``should_use`` / ``should_gather`` are False)."""

    def __init__(self, device: torch.device):
        from vgate import ops

        self.C = ops.native()
        self.rank, self.world, self.device, self.max_bytes = 0, 1, device, 0
        self.fused_off = SIGNAL_BYTES
        with torch.cuda.device(device):
            self.own = self.C.ar_alloc(SIGNAL_BYTES + int(self.C.ar_fused_bytes()))
        self.bases = [self.own]
        self.calls = 0
        self.fused = True  # (CustomAllReduce.fuses reads it: the self-check can turn a real group's off)

    fuses = CustomAllReduce.fuses

    def should_use(self, t: torch.Tensor) -> bool:
        return False

    def should_gather(self, t: torch.Tensor) -> bool:
        return False

    def check(self) -> None:
        if self.C.ar_error(self.own):
            raise RuntimeError("custom all-reduce: a peer did not arrive within the spin limit")

    def close(self) -> None:
        if self.own is not None:
            torch.cuda.synchronize(self.device)
            self.C.ar_free(self.own)
            self.own = None


def maybe_create(group, rank: int, world: int, device: torch.device, max_bytes: int = 8 << 20,
                 fused: bool = True):
    """The custom all-reduce when every rank of ``group`` is a GPU of this node with peer
    access, else None (callers fall back to RCCL)."""
    if world < 2 or world > MAX_RANKS or device.type != "cuda":
        return None
    # peer access is needed only between the devices of THIS group's ranks
    devs = [None] * world
    dist.all_gather_object(devs, device.index, group=group)
    ok = all(d == device.index or torch.cuda.can_device_access_peer(device.index, d) for d in devs)
    flags = [None] * world
    dist.all_gather_object(flags, ok, group=group)
    if not all(flags):
        log.info("custom all-reduce disabled: no peer access between all ranks")
        return None
    try:
        ar = CustomAllReduce(group, rank, world, device, max_bytes)
        # model.tp_fused_allreduce=false: decode row-parallel GEMMs store their partial and the
        # separate all-reduce kernel reduces it; default: the all-reduce runs inside the GEMM's
        # epilogue (gemm_epilogue.h epilogue_ar)
        ar.fused = fused
        return ar
    except Exception as e:  # noqa: BLE001 - fall back to RCCL, loudly
        log.warning("custom all-reduce unavailable (%s: %s); using RCCL for every all-reduce", type(e).__name__, e)
        return None
