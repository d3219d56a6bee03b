"""The native LLM engine: one background thread driving schedule -> execute -> emit.

Thread model: the HTTP event loop only enqueues requests (``add_request``) and
receives results through per-request callbacks (the backend marshals them onto
its asyncio loop); the engine thread owns the scheduler, KV manager and GPU.
No executor thread is held per request — this removes the reference's
thread-pool ceiling by construction.

Tensor parallelism: TP rank 0 runs the scheduler; followers run
:meth:`LLMEngine.follower_loop`, receiving each step's metadata through a host
shared-memory ring (native ``StepRing``, csrc/runtime/step_ring.cpp) and replaying
the same hipGraph bucket, so all ranks stay in lock-step with no collective, no
device sync and no Python object traffic on the hot path; rank 0 schedules
asynchronously (step t+1 queued before step t is post-processed) under TP too.
"""
from __future__ import annotations

import collections
import logging
import os
import threading
import time
import zlib
from dataclasses import dataclass, field

import torch

from vgate import ops
from vgate.models.config import resolve_arch
from vgate.models.transformer import DecoderModel
from vgate.parallel.comm import TPGroup, init_tp
from vgate.runtime.kv_cache import BLOCK_SIZE, KVCacheManager, allocate_kv_tensors
from vgate.runtime.model_runner import ModelRunner
from vgate.runtime.sampling_params import SamplingParams
from vgate.runtime.scheduler import Scheduler
from vgate.runtime.sequence import PENDING, Sequence, SeqStatus
from vgate.runtime.tokenizer import IncrementalDecoder, load_tokenizer
from vgate.utils.profiling import range_

log = logging.getLogger("vgate.engine")


class TPDivergence(RuntimeError):
    """The TP run-time consistency guard saw ranks disagree on replicated step outputs."""


class KernelHandoffFault(RuntimeError):
    """An in-launch hand-off of a step gave up waiting (ops.fault_word): that step's results are
    invalid, but the engine can reset the hand-off state and go on (LLMEngine._recover_fault)."""


@dataclass
class EngineConfig:
    model: str = "Qwen/Qwen2.5-1.5B-Instruct"
    weights_path: str | None = None
    tokenizer: str | None = None
    quantization: str | None = None
    dtype: str = "bfloat16"
    device: str = "auto"
    tensor_parallel_size: int = 1
    max_model_len: int = 2048
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 2048
    gpu_memory_utilization: float = 0.7
    num_kv_blocks: int | None = None
    enforce_eager: bool = False
    enable_prefix_caching: bool = True
    seed: int = 0
    block_size: int = BLOCK_SIZE
    part_size: int = 0  # 0 = auto: 512-token decode partitions (one workgroup each, merged in-launch)
    async_scheduling: bool = True  # GPU, TP=1: queue step t+1 before post-processing step t
    graph_token_buckets: list[int] | None = None
    warmup: bool = True
    # start-up hipGraph capture: every token bucket <= warmup_max_tokens x every sequence bucket
    # <= warmup_max_seqs (S <= T), so the mixed prefill+decode steps of a serving load replay
    # graphs instead of running eagerly (eager steps were the p99 tail: profiles/r2_bench*.log)
    warmup_max_tokens: int = 512
    warmup_max_seqs: int = 16
    # Admission window of an IDLE engine (no sequence running, no step in flight): the first request
    # to arrive waits until no further request has arrived for `idle_batch_gap_ms` (at most
    # `idle_batch_window_ms` in all, or until max_num_seqs are queued), so requests that arrive
    # together — a closed-loop client's next wave — are prefilled in ONE step instead of one step per
    # arrival (each extra prompt step costs ~2 ms on the decode weights; bench.py
    # timed_prefill_steps). A running engine never waits: new requests join the next step.
    idle_batch_window_ms: float = 3.0
    idle_batch_gap_ms: float = 0.6
    # ...but only when a burst is expected: at least 2 requests finished within the last
    # `idle_batch_recent_ms` (a closed-loop client's wave comes back right after the previous wave
    # ended). A request reaching an engine that has been quiet longer (an interactive request) is
    # prefilled at once, with no added time to first token (round-3 ADVICE).
    idle_batch_recent_ms: float = 20.0
    # GPU: time the prefill GEMM decompositions per layer shape and token bucket >= 128 at start-up
    # (ops.tune_prefill) instead of relying on the launcher's heuristic alone
    prefill_autotune: bool = True
    # measured plans persist per (device, native build, shapes) in this JSON file ("" = off): a restart
    # skips the start-up measurement (ops.tune_prefill_cached)
    plan_cache: str = "~/.cache/vgate/gemm_plans.json"
    # tensor parallel: collective timeout of the process group and the TP step ring, the custom IPC
    # all-reduce / all-gather kernels (else RCCL for everything), the all-reduce fused into the
    # decode row-parallel GEMM epilogue, and the start-up self-check of the custom collectives
    # against torch.distributed (a mismatch turns the custom paths off group-wide)
    tp_timeout_seconds: float = 120.0
    tp_custom_allreduce: bool = True
    tp_fused_allreduce: bool = True
    tp_collective_self_check: bool = True
    tp_consistency_interval: int = 256  # run-time divergence guard: every N-th step (0 = off)
    arch_overrides: dict | None = None

    def resolve_device(self) -> torch.device:
        if self.device != "auto":
            d = torch.device(self.device)
            if d.type == "cuda" and d.index is None:
                d = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
            return d
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            return torch.device("cuda", local % max(1, torch.cuda.device_count()))
        return torch.device("cpu")


@dataclass
class EngineStats:
    steps: int = 0
    tokens_generated: int = 0
    prompt_tokens: int = 0
    prefill_tokens: int = 0
    decode_tokens: int = 0
    step_time_s: float = 0.0
    cycle_time_s: float = 0.0  # schedule + execute + output processing
    requests_finished: int = 0
    last_step_ms: float = 0.0
    max_cycle_ms: float = 0.0  # slowest schedule -> launch -> collect cycle and its (T, S) bucket
    max_cycle_bucket: tuple = (0, 0)
    batch_sizes: collections.Counter = field(default_factory=collections.Counter)
    fault_recoveries: int = 0  # kernel hand-off faults the engine recovered from (LLMEngine._recover_fault)
    idle_s: float = 0.0        # engine thread waiting for work (no step in flight, nothing queued)
    # the engine thread's wall time splits into idle_s + coalesce_s + busy_s (+ captures / loop
    # overhead): coalesce_s = the idle admission window waiting for the rest of a wave
    # (_coalesce_arrivals), busy_s = inside step() / side calls (schedule, launch, collect, process)
    coalesce_s: float = 0.0
    busy_s: float = 0.0
    prefill_steps: int = 0     # steps that carried prompt tokens (mixed or prefill-only)
    # idle -> busy transitions (engine._wave_account): sums of the three boundary phases
    waves: int = 0
    wave_first_s: float = 0.0
    wave_spread_s: float = 0.0
    wave_tail_s: float = 0.0
    wave_size: int = 0


class LLMEngine:
    def __init__(self, cfg: EngineConfig, tp: TPGroup | None = None):
        self.cfg = cfg
        self.device = cfg.resolve_device()
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.tp = tp or (init_tp(cfg.tensor_parallel_size, timeout_s=cfg.tp_timeout_seconds,
                                 custom_allreduce=cfg.tp_custom_allreduce, fused_allreduce=cfg.tp_fused_allreduce)
                         if cfg.tensor_parallel_size > 1 else TPGroup())
        weights = cfg.weights_path
        if weights is None and os.path.isdir(os.path.expanduser(cfg.model)):
            weights = os.path.expanduser(cfg.model)
        self.arch = resolve_arch(cfg.model, cfg.arch_overrides)
        t0 = time.perf_counter()
        self.model = DecoderModel(self.arch, self.device, self.tp, cfg.quantization, cfg.seed, weights,
                                  cfg.max_model_len)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        self.load_seconds = time.perf_counter() - t0
        self.num_blocks = self._size_kv()
        self.tp_self_check = "n/a"
        if self.tp.custom_ar is not None and cfg.tp_collective_self_check and not self.tp.simulated:
            self._collective_self_check()
        self.kv_caches = allocate_kv_tensors(self.arch.num_layers, self.num_blocks, self.model.num_kv_heads_local,
                                             self.arch.head_dim, self.device, block_size=cfg.block_size)
        self.kvm = KVCacheManager(self.num_blocks, cfg.block_size, cfg.enable_prefix_caching)
        self.scheduler = Scheduler(self.kvm, cfg.max_num_seqs, cfg.max_num_batched_tokens, cfg.max_model_len)
        part = cfg.part_size or 512
        part = min(1024, max(32, (part + 31) // 32 * 32))
        # a gloo group (ranks sharing one GPU in tests) runs its collectives on the host, which a
        # hipGraph cannot capture: such a group replays graphs only for the buckets whose every
        # collective fits the IPC kernels (custom all-reduce / all-gather), and runs the rest eagerly
        gloo_tp = self.tp.size > 1 and self.tp.backend != "nccl" and not self.tp.simulated
        eager = cfg.enforce_eager or (gloo_tp and self.tp.custom_ar is None)
        self.runner = ModelRunner(self.model, self.kv_caches, cfg.max_num_seqs, cfg.max_num_batched_tokens,
                                  cfg.max_model_len, cfg.block_size, eager, part,
                                  cfg.graph_token_buckets)
        self.prefill_plans: dict = {}
        self.plans_from_cache = False
        if self.device.type == "cuda" and cfg.prefill_autotune:
            t1 = time.perf_counter()
            # prefill buckets (>= 128 rows) and the medium buckets of mixed prefill + decode steps
            ms = [t for t in self.runner.t_buckets if t > 16]  # (t_buckets end at max_num_batched_tokens)
            lins = [lin for L in self.model.layers for lin in (L.qkv, L.o, L.gate_up, L.down)]
            if self.tp.size > 1:
                # rank 0 measures, every rank applies the same plans (per-rank timing noise would
                # otherwise give TP ranks different tile / K-split choices, and N x the start-up cost)
                plans = ops.tune_prefill_cached(lins, ms, cfg.plan_cache)[0] if self.tp.is_first else None
                self.prefill_plans = self.tp.broadcast_object(plans)
                ops.apply_prefill_plans(lins, self.prefill_plans)
                cached = False
            else:
                self.prefill_plans, cached = ops.tune_prefill_cached(lins, ms, cfg.plan_cache)
            self.plans_from_cache = cached
            log.info("prefill GEMM plans for %d shapes x %d buckets in %.2fs%s: %s", len(self.prefill_plans), len(ms),
                     time.perf_counter() - t1, " (plan cache)" if cached else "",
                     {f"{n}x{k}": p for (n, k), p in self.prefill_plans.items()})
        if gloo_tp and not eager:
            cap = self.tp.custom_bytes()
            H, vloc = self.arch.hidden_size, self.model.shard.vocab
            self.runner.graph_ok = lambda T, S: T * H * 2 <= cap and S * vloc * 4 <= cap
        self.tokenizer = load_tokenizer(weights, cfg.tokenizer, self.arch)
        self.stats = EngineStats()
        self._inbox: collections.deque = collections.deque()
        self._aborts: collections.deque = collections.deque()
        self._cv = threading.Condition()
        self._running = False
        self._thread: threading.Thread | None = None
        self._by_id: dict[str, Sequence] = {}
        self._seq_counter = 0
        self.healthy = True
        # TP: every rank must capture at the same step (a capture's eager warm-up runs the
        # collectives), so buckets are captured on first use there, not deferred to idle time
        self.runner.defer_capture = self.tp.size == 1
        self.capture_idle_s = 0.05
        self.async_sched = bool(cfg.async_scheduling and self.device.type == "cuda")
        self.ring = None
        self._ring_closed = False
        self._ar_check_every = 1 if self.tp.is_first else 64
        self._steps_since_check = 0
        self._ar_ms: list[float] = []
        if self.tp.size > 1 and not self.tp.simulated:
            self._init_ring()
        self._inflight = None  # (batch, handle) of the launched, not yet post-processed step
        self._finish_times: collections.deque = collections.deque(maxlen=64)  # idle admission window
        self._calls: collections.deque = collections.deque()  # (fn, future) run on the engine thread
        self.last_error: str | None = None
        self._fault_times: collections.deque = collections.deque()
        self._idle_t: float | None = None  # start of the engine thread's current idle wait
        self._launch_no = 0                # rank 0 launches (the consistency guard's step clock)
        # per idle -> busy transition: (last finish before it, idle start, first / last arrival, step
        # start), perf_counter clock (bench.py joins it with its client's send / receive times)
        self.wave_log: collections.deque = collections.deque(maxlen=4096)
        self.tp_consistent = True
        self.tp_consistency = "ok"
        self.tp_consistency_checks = 0
        self.fault_recoveries_max = 3
        self.fault_window_s = 300.0
        self.last_step_wall = time.monotonic()
        log.info("engine ready: model=%s params=%.2fB weights=%.2f GB load=%.1fs kv_blocks=%d (%.1fk tokens) device=%s tp=%d",
                 self.arch.name, self.arch.num_params() / 1e9, self.model.weight_bytes() / 1e9, self.load_seconds,
                 self.num_blocks, self.num_blocks * cfg.block_size / 1e3, self.device, self.tp.size)

    # ------------------------------------------------------------------ sizing
    def _size_kv(self) -> int:
        cfg = self.cfg
        per_block = 2 * self.arch.num_layers * self.model.num_kv_heads_local * cfg.block_size * self.arch.head_dim * 2
        max_useful = cfg.max_num_seqs * ((cfg.max_model_len + cfg.block_size - 1) // cfg.block_size) * 2 + 64
        if cfg.num_kv_blocks:
            n = cfg.num_kv_blocks
        elif self.device.type == "cuda":
            ops.workspace(self.device)  # the 256 MiB GEMM workspace is allocated before the free memory is read
            free, total = torch.cuda.mem_get_info(self.device)
            reserve = 4 * 2**30 + cfg.max_num_seqs * self.arch.vocab_size * 12
            budget = cfg.gpu_memory_utilization * total - (total - free) - reserve
            n = int(max(0, budget) // per_block)
            n = min(n, max_useful)
        else:
            n = min(max_useful, 4096)
        if self.tp.size > 1 and not self.tp.simulated:  # identical pool on every rank
            t = torch.tensor([n], device=self.device if self.tp.backend == "nccl" else "cpu")
            import torch.distributed as dist
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.tp.group)
            n = int(t.item())
        if n < (1 if cfg.num_kv_blocks else 16):
            raise RuntimeError(f"not enough memory for the KV cache ({n} blocks)")
        return n

    def _collective_self_check(self) -> None:
        """Every rank, before the first graph capture: the custom collectives (one-shot, two-shot,
        all-gather, the fused GEMM-epilogue all-reduce) against torch.distributed on the group. The
        verdict is agreed over the group; on a mismatch or a give-up every rank drops the custom
        paths (RCCL for every collective from then on), logs it and reports it (/stats
        tp_self_check, gauge vgate_engine_tp_custom_collectives)."""
        car = self.tp.custom_ar
        t0 = time.perf_counter()
        ok, notes = car.self_check(self.tp.group, self.tp.backend, self.arch.hidden_size, self.model.layers[0].o)
        if ok:
            self.tp_self_check = "passed"
            log.info("TP collective self-check passed in %.2fs (custom all-reduce / all-gather == %s)",
                     time.perf_counter() - t0, self.tp.backend)
            return
        self.tp_self_check = "failed: " + " | ".join(notes)
        log.error("TP collective self-check FAILED (%s); the custom IPC collectives are disabled on every rank "
                  "of the group, all collectives go through %s", "; ".join(notes), self.tp.backend)
        car.close()
        self.tp.custom_ar = None

    # --------------------------------------------------------------- lifecycle
    def start(self) -> None:
        if self._running:
            return
        if self.cfg.warmup and self.runner.use_graphs:
            tb = [t for t in self.runner.t_buckets if t <= self.cfg.warmup_max_tokens]
            sb = [b for b in self.runner.s_buckets if b <= self.cfg.warmup_max_seqs]
            secs = self.runner.warmup(tb, sb)
            log.info("pre-captured %d hipGraphs in %.2fs", len(self.runner.graphs), secs)
        self._running = True
        self._thread = threading.Thread(target=self._loop, name="vgate-engine", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._running = False
        with self._cv:
            self._cv.notify_all()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None

    # ------------------------------------------------------------------- input
    def add_request(self, request_id: str, prompt: str | None = None, params: SamplingParams | None = None,
                    callback=None, stream: bool = False, prompt_ids: list[int] | None = None) -> Sequence:
        params = params or SamplingParams()
        if prompt_ids is None:
            prompt_ids = self.tokenizer.encode(prompt or "")
        if not prompt_ids:
            prompt_ids = [self.arch.bos_token_id]
        if len(prompt_ids) >= self.cfg.max_model_len:
            prompt_ids = prompt_ids[-(self.cfg.max_model_len - 1):]
        seq = Sequence(request_id=request_id, prompt_ids=list(prompt_ids), params=params, callback=callback,
                       stream=stream)
        seq.seed = params.seed if params.seed is not None else \
            (self.cfg.seed * 1000003 + zlib.crc32(request_id.encode())) & 0x7FFFFFFFFFFFFFFF
        if stream:
            seq.detok = IncrementalDecoder(self.tokenizer)
        with self._cv:
            if not self.has_unfinished():  # the step watchdog measures from the first work on
                self.last_step_wall = time.monotonic()
            self._inbox.append(seq)
            self._cv.notify()
        return seq

    def abort(self, request_id: str) -> None:
        with self._cv:
            self._aborts.append(request_id)
            self._cv.notify()

    def has_unfinished(self) -> bool:
        return bool(self._inbox) or self.scheduler.has_work() or self._inflight is not None

    # -------------------------------------------------------------------- loop
    def _drain_inbox(self) -> None:
        while self._inbox:
            seq = self._inbox.popleft()
            self._by_id[seq.request_id] = seq
            self.scheduler.add(seq)
        while self._aborts:
            rid = self._aborts.popleft()
            seq = self._by_id.get(rid)
            if seq is not None and not seq.is_finished:
                self.scheduler.remove(seq)
                seq.aborted = True
                self._finish(seq, "abort", notify_sched=False)

    def _coalesce_arrivals(self) -> None:
        """Called with the condition held: when the engine has nothing running and requests just
        arrived, give the rest of an arriving burst ``idle_batch_gap_ms`` (since the latest arrival)
        to join, up to ``idle_batch_window_ms`` in all (EngineConfig)."""
        win, gap = self.cfg.idle_batch_window_ms, self.cfg.idle_batch_gap_ms
        if (win <= 0 or gap <= 0 or not self._inbox or self._inflight is not None or self._calls
                or self.scheduler.has_work() or self.ring is not None):
            return
        recent = time.perf_counter() - 1e-3 * self.cfg.idle_batch_recent_ms
        came_back = sum(1 for t in self._finish_times if t >= recent)
        if came_back < 2 and len(self._inbox) < 2:
            return  # no wave is coming back: a lone request starts now
        t0 = time.perf_counter()
        t_end = t0 + 1e-3 * win
        cap = self.cfg.max_num_seqs
        # a closed-loop client sends one new request per finished one: once as many have arrived as
        # just finished, the wave is complete and the prefill starts without waiting out the gap
        if came_back >= 2:
            cap = min(cap, came_back)
        n = len(self._inbox)
        while self._running and n < cap:
            now = time.perf_counter()
            if now >= t_end:
                break
            self._cv.wait(timeout=min(1e-3 * gap, t_end - now))
            if len(self._inbox) == n:
                break  # nobody arrived within the gap
            n = len(self._inbox)
        self.stats.coalesce_s += time.perf_counter() - t0

    def _wave_account(self, t_idle0: float) -> None:
        """Break an idle -> busy transition into (idle start -> first arrival), (first -> last
        arrival of the batch), (last arrival -> step start): the wave-boundary forensics of
        bench.py (``wave_breakdown_ms``)."""
        arr = [s.arrival for s in self._inbox]
        now = time.perf_counter()
        fin = self._finish_times[-1] if self._finish_times else t_idle0
        self.wave_log.append((fin, t_idle0, min(arr), max(arr), now))
        st = self.stats
        st.waves += 1
        st.wave_first_s += max(0.0, min(arr) - t_idle0)
        st.wave_spread_s += max(arr) - min(arr)
        st.wave_tail_s += now - max(arr)
        st.wave_size += len(arr)

    def _idle(self) -> bool:
        return (not self._inbox and not self._aborts and not self.scheduler.has_work() and self._inflight is None
                and not self._calls)

    def _loop(self) -> None:
        torch.set_grad_enabled(False)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while self._running:
            if self.ring is not None:
                self.ring.heartbeat()
            if self.runner.pending_captures and self._idle():
                # buckets first seen under load ran eagerly; capture them once the engine has
                # stayed idle for a moment (not in the microseconds between two requests of a
                # running load), one bucket at a time, re-checking for new work in between
                with self._cv:
                    self._cv.wait_for(lambda: not self._running or not self._idle(), timeout=self.capture_idle_s)
                if self._running and self._idle():
                    try:
                        self.runner.capture_pending(max_graphs=1)
                    except Exception:  # noqa: BLE001 - those buckets keep running eagerly
                        log.exception("deferred hipGraph capture failed")
                        self.runner.defer_capture_failed = True
                        self.runner.pending_captures.clear()
            with self._cv:
                t_idle0 = None
                while self._running and self._idle() and not self.runner.pending_captures:
                    if self.ring is not None:  # an idle TP group must not look dead to its followers
                        self.ring.heartbeat()
                    t_idle = self._idle_t = time.perf_counter()
                    if t_idle0 is None:
                        t_idle0 = t_idle
                    self._cv.wait(timeout=0.5)
                    self._idle_t = None
                    self.stats.idle_s += time.perf_counter() - t_idle
                if self._idle():
                    continue  # idle with captures pending: back to the capture check
                if not self._running:
                    break
                self._coalesce_arrivals()
                if t_idle0 is not None and self._inbox:
                    self._wave_account(t_idle0)
                self._drain_inbox()
            t_busy = time.perf_counter()
            if self._calls:
                self._run_calls()
            try:
                self.step()
                self.stats.busy_s += time.perf_counter() - t_busy
            except Exception as e:  # noqa: BLE001 - engine faults fail every in-flight request
                log.exception("engine step failed")
                self._inflight = None
                self.last_error = f"{type(e).__name__}: {e}"
                failed = list(self.scheduler.running) + list(self.scheduler.waiting)
                for seq in failed:
                    self.scheduler.remove(seq)
                # recover (or go unhealthy) before any client hears of the failure
                if not (isinstance(e, KernelHandoffFault) and self._recover_fault()):
                    self.healthy = False
                for seq in failed:
                    self._finish(seq, "error", notify_sched=False, error=self.last_error)
        self.shutdown_followers()

    # ------------------------------------------------------------- side calls
    def _run_calls(self) -> None:
        """Work that needs the device between steps (embeddings): drain the in-flight step
        first, since it shares the step-metadata buffers."""
        self._drain_inflight()
        while self._calls:
            fn, fut = self._calls.popleft()
            try:
                fut.set_result(fn())
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)

    def call(self, fn, timeout: float = 300.0):
        """Run ``fn`` on the engine thread (or inline when no loop is running)."""
        import concurrent.futures
        if not self._running or threading.current_thread() is self._thread:
            self._drain_inflight()
            return fn()
        fut: concurrent.futures.Future = concurrent.futures.Future()
        with self._cv:
            self._calls.append((fn, fut))
            self._cv.notify()
        return fut.result(timeout=timeout)

    def embed(self, text: str | None = None, prompt_ids: list[int] | None = None) -> tuple[list[float], int]:
        """Sentence embedding: L2-normalised mean over tokens of the final-RMSNorm hidden
        states (prefill only, through scratch KV blocks that are released afterwards).
        Returns (vector [hidden_size], prompt token count)."""
        ids = prompt_ids if prompt_ids is not None else self.tokenizer.encode(text or "")
        ids = (ids or [self.arch.bos_token_id])[: min(self.cfg.max_model_len - 1, self.cfg.max_num_batched_tokens)]

        def run():
            from vgate.runtime.scheduler import ScheduledBatch
            seq = Sequence(request_id="__embed__", prompt_ids=list(ids), params=SamplingParams(max_tokens=1))
            if not self.kvm.ensure(seq, len(ids)):
                raise RuntimeError("no free KV blocks for the embedding request")
            try:
                batch = ScheduledBatch([(seq, len(ids))], len(ids), len(ids), 0, [])
                hid = self.runner.hidden_states(batch).float()
                var = hid.pow(2).mean(-1, keepdim=True)
                xn = hid * torch.rsqrt(var + self.arch.rms_eps) * self.model.final_norm.float()
                v = xn.mean(0)
                v = v / v.norm().clamp_min(1e-12)
                return v.cpu().tolist()
            finally:
                self.kvm.free(seq)

        return self.call(run), len(ids)

    def run_until_idle(self, max_steps: int = 1_000_000) -> None:
        """Synchronous driver (tests / offline use): process everything queued."""
        self._drain_inbox()
        n = 0
        while (self.scheduler.has_work() or self._inflight is not None) and n < max_steps:
            self.step()
            self._drain_inbox()
            n += 1
        if self.async_sched:
            self._drain_inflight()
        self.runner.capture_pending()

    # -------------------------------------------------------------------- step
    def step(self) -> int:
        """One engine iteration. Synchronous mode: schedule -> execute -> post-process.
        Asynchronous mode (GPU, TP=1): schedule -> launch step t+1 -> post-process step t
        while t+1 runs (tokens of the in-flight step are PENDING placeholders that the
        device resolves from the previous sampler output)."""
        if self.async_sched:
            return self._step_async()
        tc = time.perf_counter()
        batch = self.scheduler.schedule()
        if batch.empty:
            return 0
        t0 = time.perf_counter()
        check = self._consistency_due()
        toks, samples = self.runner.execute(batch, check=check)
        if check:
            self._consistency_exchange(batch.num_tokens, len(batch.items))
        self._check_collectives()
        for seq, n in batch.items:
            seq.num_computed += n
        self._process(batch, toks, samples, t0, tc, resolve=False)
        return len(batch.items)

    def _step_async(self) -> int:
        tc = time.perf_counter()
        with range_("vgate.schedule"):
            batch = self.scheduler.schedule(no_preempt=self._inflight is not None)
            if batch.kv_pressure:  # preemption needs every placeholder resolved first
                self._drain_inflight()
                batch = self.scheduler.schedule()
        if batch.empty:
            self._drain_inflight()
            return 0
        pend = {seq.seq_id: seq.pending_slot for seq, _ in batch.items if seq.pending}
        check = self._consistency_due()
        with range_("vgate.launch"):
            h = self.runner.launch(batch, pend, check=check)
        if check:
            # synchronous: every rank must take (or not take) the group-wide fallback before its
            # next launch, so the exchange is read right here, once per interval
            self._consistency_exchange(batch.num_tokens, h.ns)
        for i, ((seq, n), smp) in enumerate(zip(batch.items, h.samples)):
            seq.num_computed += n
            if smp:
                seq.output_ids.append(PENDING)
                seq.pending.append(len(seq.output_ids) - 1)
                seq.pending_slot = i
        prev, self._inflight = self._inflight, (batch, h, tc)
        if prev is not None:
            self._complete(prev)
        return len(batch.items)

    def _drain_inflight(self) -> None:
        if self._inflight is not None:
            prev, self._inflight = self._inflight, None
            self._complete(prev)

    def _complete(self, entry) -> None:
        batch, h, tc = entry
        with range_("vgate.collect"):
            toks = self.runner.collect(h)
        self._check_collectives()
        with range_("vgate.process"):
            self._process(batch, toks, h.samples, h.t_launch, tc, resolve=True)

    def _process(self, batch, toks, samples, t0: float, tc: float, resolve: bool) -> None:
        """Post-process one executed step: append (or resolve) sampled tokens, stop checks,
        streaming deltas, prefix-cache registration, finished requests."""
        now = time.perf_counter()
        st = self.stats
        st.steps += 1
        st.step_time_s += now - t0
        st.cycle_time_s += now - tc
        st.last_step_ms = 1e3 * (now - t0)
        cyc = 1e3 * (now - tc)
        if cyc > st.max_cycle_ms:
            st.max_cycle_ms = cyc
            st.max_cycle_bucket = (batch.num_tokens, len(batch.items))
        st.prefill_tokens += batch.num_prefill_tokens
        st.prefill_steps += batch.num_prefill_tokens > 0
        st.decode_tokens += batch.num_decode
        st.batch_sizes[len(batch.items)] += 1
        self.last_step_wall = time.monotonic()
        eos = set(self.arch.eos_token_ids)
        for (seq, n), tok, smp in zip(batch.items, toks, samples):
            if not smp:
                if not seq.is_finished:
                    self.kvm.register_computed(seq)
                continue
            if resolve:
                idx = seq.pending.popleft() if seq.pending else None
                if seq.is_finished or idx is None:
                    continue  # finished (stop / abort) while this step was in flight: dropped
                seq.output_ids[idx] = tok
                nout = idx + 1
            else:
                if seq.is_finished:
                    continue
                seq.output_ids.append(tok)
                nout = len(seq.output_ids)
            self.kvm.register_computed(seq)
            st.tokens_generated += 1
            if seq.first_token_time is None:
                seq.first_token_time = now
            seq.last_token_time = now
            sp = seq.params
            reason = None
            if not sp.ignore_eos and tok in eos and nout >= sp.min_tokens:
                reason = "stop"
            elif tok in sp.stop_token_ids and nout >= sp.min_tokens:
                reason = "stop"
            elif nout >= sp.max_tokens:
                reason = "length"
            elif len(seq.prompt_ids) + nout >= self.cfg.max_model_len:
                reason = "length"
            delta = ""
            if seq.stream and seq.detok is not None:
                delta = seq.detok.push(tok) if reason != "stop" or tok not in eos else ""
                seq.text += delta
            if sp.stop and reason is None:
                text = seq.text if seq.stream else self.tokenizer.decode(seq.output_ids[:nout])
                for stop_s in sp.stop:
                    if stop_s and stop_s in text:
                        reason = "stop"
                        break
            if seq.stream and seq.callback is not None and delta:
                seq.callback("token", seq, delta)
            if reason is not None:
                if resolve:  # later in-flight samples of this sequence are discarded
                    del seq.output_ids[nout:]
                    seq.pending.clear()
                self._finish(seq, reason)

    def _finish(self, seq: Sequence, reason: str, notify_sched: bool = True, error: str | None = None) -> None:
        if notify_sched:
            self.scheduler.finish(seq, reason)
        else:
            seq.status = SeqStatus.FINISHED
            seq.finish_reason = reason
        seq.finish_time = time.perf_counter()
        self._finish_times.append(seq.finish_time)
        if seq.pending:  # abort / error with samples still in flight: drop the placeholders
            seq.output_ids = [t for t in seq.output_ids if t != PENDING]
            seq.pending.clear()
        self._by_id.pop(seq.request_id, None)
        self.stats.requests_finished += 1
        self.stats.prompt_tokens += len(seq.prompt_ids)
        if seq.stream and seq.detok is not None:
            tail = seq.detok.flush()
            if tail:
                seq.text += tail
                if seq.callback is not None:
                    seq.callback("token", seq, tail)
        elif not seq.stream:
            out = seq.output_ids
            if reason == "stop" and out and out[-1] in self.arch.eos_token_ids:
                out = out[:-1]
            seq.text = self.tokenizer.decode(out)
        if seq.callback is not None:
            seq.callback("error" if error else "finish", seq, error)

    # ----------------------------------------------------------- tensor parallel
    RING_PLAN, RING_EMBED, RING_CAPTURE, RING_STOP, RING_PLAN_CHECK = 0, 1, 2, 3, 4

    def _init_ring(self) -> None:
        """Create (rank 0) / attach (followers) the group's shared-memory step ring. Rank 0 picks
        a unique name and hands it to the group once over the process group; from then on every
        step plan travels through the ring (csrc/runtime/step_ring.cpp)."""
        from vgate import ops
        C = ops.native()
        name = None
        if self.tp.is_first:
            name = f"/vgate_ring_{os.getpid()}_{id(self) & 0xffffff:x}"
            self.ring = C.StepRing(name, True, slots=8,
                                   slot_bytes=self.runner.meta.nbytes, followers=self.tp.size - 1)
        name = self.tp.broadcast_object(name)
        if not self.tp.is_first:
            self.ring = C.StepRing(name, False)
        self.tp.barrier()  # every follower has mapped the segment
        if self.tp.is_first:
            self.ring.unlink()
        self.runner.on_plan = self._publish if self.tp.is_first else None

    def _publish(self, T: int, S: int, ns: int, nt: int, mode: int) -> None:
        """Rank 0: ship the step plan now in the runner's host metadata buffer to the followers."""
        m = self.runner.meta
        n = m.used_bytes(ns) if mode != self.RING_CAPTURE else m.used_bytes(0)
        timeout = float(self.cfg.tp_timeout_seconds)
        if not self.ring.publish(T, S, ns, nt, mode, m.host, n, timeout):
            raise RuntimeError(f"TP step ring: a follower made no progress for {timeout:.0f}s")

    def _check_collectives(self) -> None:
        """Fail the step (engine unhealthy) if the custom all-reduce gave up waiting for a peer:
        its bounded spin reduces stale peer data after a timeout, so the error word is the only
        signal. Every rank, every step, with no device sync: the step graph's last node copies the
        sticky error word (and the collective time counters) into the pinned ids ring
        (ModelRunner.collective_words), so the check is a host memory read (ROUND-2 ADVICE: the
        blocking hipMemcpy of ``ar.check()`` serialised rank 0 with its in-flight step)."""
        fault = self.runner.kernel_fault() if self.runner.gpu else 0
        if fault:
            raise KernelHandoffFault(f"an in-launch kernel hand-off gave up waiting (fault word {fault:#x}); "
                                     "the step's results are invalid")
        ar = self.tp.custom_ar
        if ar is None:
            return
        # the step graph's ids_to_host node copies the all-reduce's words into the ring slot; a CPU
        # group (gloo, no ring words) reads the error word through ar.check() below
        if self.runner.gpu and self.runner.ar_base:
            err, secs, calls = self.runner.collective_words()
            if calls and len(self._ar_ms) < 65536:
                self._ar_ms.append(1e3 * secs)
            if err:
                raise RuntimeError("custom all-reduce: a peer did not arrive within the spin limit")
            return
        self._steps_since_check += 1
        if self._steps_since_check >= self._ar_check_every:
            self._steps_since_check = 0
            ar.check()

    def _recover_fault(self) -> bool:
        """A kernel hand-off gave up (sticky fault word): the step's requests were failed; reset the
        hand-off state and keep serving instead of going unhealthy for good. One process, one GPU
        only (a TP group is one failure domain: its ranks' streams cannot be reset in lock-step).
        The prefix cache is dropped too: a faulted step may have written wrong K / V into blocks
        it published. More than ``fault_recoveries_max`` faults inside ``fault_window_s``: the
        engine goes unhealthy (something persistent is wrong; an external restart is the fix)."""
        if self.tp.size > 1:
            return False
        now = time.monotonic()
        hist = self._fault_times
        while hist and now - hist[0] > self.fault_window_s:
            hist.popleft()
        if len(hist) >= self.fault_recoveries_max:
            log.error("%d kernel faults within %.0f s: engine marked unhealthy", len(hist) + 1, self.fault_window_s)
            return False
        hist.append(now)
        try:
            ops.reset_handoffs(self.device)
            self.runner.reset_fault_ring()
            self.kvm.alloc.reset_prefix_cache()
        except Exception:  # noqa: BLE001
            log.exception("kernel fault recovery failed")
            return False
        self.stats.fault_recoveries += 1
        log.warning("kernel hand-off fault recovered (%d in the last %.0f s): hand-off buffers reset, "
                    "prefix cache dropped, in-flight requests failed", len(hist), self.fault_window_s)
        return True

    def _consistency_due(self) -> bool:
        """Rank 0: is this launch one whose result the TP group cross-checks (every
        ``tp_consistency_interval``-th launch; followers learn it from ring mode 4)?"""
        n = self.cfg.tp_consistency_interval
        if n <= 0 or self.tp.size == 1 or self.tp.simulated or not self.tp_consistent:
            return False
        self._launch_no += 1
        return self._launch_no % n == 0

    def _consistency_exchange(self, nt: int, S: int) -> None:
        """Every rank, after the same step: all-gather [checksum(logits), checksum(sampled ids)]
        and compare. They are replicated by construction (custom one-shot / fused all-reduce and
        all-gather sum and concatenate in fixed rank order), so a difference means a rank computed
        on different data, e.g. a peer partial read stale on the link — silently wrong tokens
        otherwise. On a mismatch every rank sees it: the custom IPC collectives go off group-wide
        (graphs dropped; RCCL for every collective from the next step on, buckets re-captured in
        lock-step), and rank 0 fails the step and marks the engine unhealthy with the reason."""
        words = self.tp.exchange_words(self.runner.check_words)
        self.tp_consistency_checks += 1
        if bool((words == words[0:1]).all()):
            return
        bad = [r for r in range(words.shape[0]) if not bool((words[r] == words[0]).all())]
        what = [n for i, n in enumerate(("residual", "logits", "sampled ids"))
                if any(bool(words[r][i] != words[0][i]) for r in bad)]
        reason = (f"TP ranks diverged at consistency check {self.tp_consistency_checks} "
                  f"(step {self.stats.steps}): ranks {bad} differ from rank 0 in {', '.join(what)}")
        self.tp_consistent = False
        self.tp_consistency = reason
        log.error("%s; custom collectives disabled group-wide", reason)
        car = self.tp.custom_ar
        if car is not None:
            if self.runner.gpu:
                torch.cuda.synchronize(self.device)
            self.runner.graphs.clear()
            self.runner.ar_base = 0
            self.tp.custom_ar = None
            car.close()
        if self.tp.is_first:
            self.healthy = False
            raise TPDivergence(reason)

    def follower_loop(self) -> None:
        """TP ranks > 0: execute whatever rank 0 publishes on the step ring, until it stops."""
        torch.set_grad_enabled(False)
        try:
            self._follow()
        except BaseException:  # noqa: BLE001 - a TP group is one failure domain
            # rank 0 would otherwise wait for this rank (ring back-pressure / collectives) until
            # its timeout: exit now, so the launcher (torchrun) tears the whole group down and
            # the gateway's health checks take this worker out of rotation
            log.exception("TP follower rank %d failed; exiting so the TP group is torn down", self.tp.rank)
            logging.shutdown()
            os._exit(1)

    def _follow(self) -> None:
        r = self.runner
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        f = self.tp.rank - 1
        timeout = float(self.cfg.tp_timeout_seconds)
        while True:
            buf = r.follower_host_buffer()
            T, S, ns, nt, mode, _ = self.ring.wait(f, buf, timeout)
            if mode == -2:
                raise RuntimeError(f"TP step ring: no heartbeat from rank 0 for {timeout:.0f}s")
            if mode in (-1, self.RING_STOP):
                return
            r.follow_step(T, S, ns, nt, self.RING_PLAN if mode == self.RING_PLAN_CHECK else mode,
                          check=mode == self.RING_PLAN_CHECK)
            self.last_step_wall = time.monotonic()
            if mode in (self.RING_PLAN, self.RING_PLAN_CHECK):
                self.stats.steps += 1
                self._check_collectives()
            if mode == self.RING_PLAN_CHECK:
                self._consistency_exchange(nt, ns)

    def shutdown_followers(self) -> None:
        if self.tp.size > 1 and self.tp.is_first and self.ring is not None and not self._ring_closed:
            self._ring_closed = True
            try:
                self.ring.publish(0, 0, 0, 0, self.RING_STOP, self.runner.meta.host, 0, 5.0)
            finally:
                self.ring.close()

    def drain_allreduce_times(self) -> list[float]:
        out, self._ar_ms = self._ar_ms, []
        return out

    # ------------------------------------------------------------------- stats
    def drain_step_times(self) -> list[float]:
        """Device time (ms) of every step collected since the last call (metrics loop)."""
        r = self.runner
        out, r.step_gpu_ms = r.step_gpu_ms, []
        return out

    def reset_peaks(self) -> None:
        """Restart the slowest-step trackers (a benchmark's timed region starts here)."""
        self.runner.max_gpu_ms, self.runner.max_gpu_bucket, self.runner.max_gpu_eager = 0.0, (0, 0), False
        self.stats.max_cycle_ms, self.stats.max_cycle_bucket = 0.0, (0, 0)

    def snapshot(self) -> dict:
        st = self.stats
        t_idle = self._idle_t  # an idle wait in progress counts up to now
        return {
            "model": self.arch.name, "device": str(self.device), "tp": self.tp.size,
            "running": len(self.scheduler.running), "waiting": len(self.scheduler.waiting),
            "kv_blocks_total": self.num_blocks, "kv_blocks_free": self.kvm.num_free(),
            "kv_usage": round(self.kvm.usage(), 4), "steps": st.steps, "tokens_generated": st.tokens_generated,
            "prefill_tokens": st.prefill_tokens, "decode_tokens": st.decode_tokens,
            "avg_step_ms": round(1e3 * st.step_time_s / max(1, st.steps), 3),
            "avg_cycle_ms": round(1e3 * st.cycle_time_s / max(1, st.steps), 3),
            "avg_gpu_ms": round(self.runner.gpu_ms / max(1, self.runner.gpu_steps), 3),
            "avg_host_ms": round(self.runner.host_ms / max(1, st.steps), 3),
            "idle_ms": round(1e3 * (st.idle_s + (time.perf_counter() - t_idle if t_idle is not None else 0.0)), 3),
            "prefill_steps": st.prefill_steps,
            # raw cumulative sums (bench.py differences them over its timed region): the engine
            # thread's wall = idle + coalesce + busy (+ deferred captures); collect_wait = busy time
            # blocked on the device; gpu = device time of the timed steps (every 8th)
            "coalesce_ms": round(1e3 * st.coalesce_s, 3), "busy_ms": round(1e3 * st.busy_s, 3),
            "collect_wait_ms": round(self.runner.collect_wait_ms, 3),
            "sum_step_ms": round(1e3 * st.step_time_s, 3), "sum_cycle_ms": round(1e3 * st.cycle_time_s, 3),
            "sum_gpu_ms": round(self.runner.gpu_ms, 3), "gpu_steps": self.runner.gpu_steps,
            "graphs_captured": len(self.runner.graphs), "graph_hits": self.runner.graph_hits,
            "graph_misses_eager": self.runner.graph_misses,
            "pending_captures": len(self.runner.pending_captures),
            "graph_captures": self.runner.captures,
            "graph_hit_ratio": round(self.runner.graph_hits / max(1, self.runner.graph_hits + self.runner.graph_misses), 4),
            "max_gpu_step_ms": round(self.runner.max_gpu_ms, 3),
            "max_gpu_step_bucket": list(self.runner.max_gpu_bucket),
            "max_gpu_step_eager": self.runner.max_gpu_eager,
            "max_cycle_ms": round(st.max_cycle_ms, 3),
            "max_cycle_tokens_seqs": list(st.max_cycle_bucket),
            "preemptions": self.scheduler.num_preemptions, "prefix_cache_hits": int(getattr(self.kvm.alloc, "hits", 0)),
            "healthy": self.healthy, "fault_recoveries": st.fault_recoveries,
            "tp_custom_collectives": int(self.tp.custom_ar is not None), "tp_self_check": self.tp_self_check,
            "tp_consistency": self.tp_consistency, "tp_consistency_checks": self.tp_consistency_checks,
            "waves": st.waves, "wave_sum_ms": [round(1e3 * st.wave_first_s, 3), round(1e3 * st.wave_spread_s, 3),
                                                round(1e3 * st.wave_tail_s, 3)], "wave_requests": st.wave_size,
        }
