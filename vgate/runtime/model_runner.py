"""Executes scheduled batches on the model: metadata build, hipGraph replay, sampling.

Graph strategy (MI355X-first, no tracing compiler): every step — decode-only,
prefill-only or mixed — is padded to a (token bucket T, sequence bucket S) and
replayed from a hipGraph captured on first use (``torch.cuda.graph`` records the
HIP stream: every kernel launch of the forward plus the sampler). All dynamic
inputs live in :class:`StepMeta` device buffers, so a replay costs one H2D copy,
one graph launch and one D2H copy of the sampled token ids. ``enforce_eager``
(or a CPU device) runs the same code without capture.

Asynchronous scheduling: :meth:`launch` enqueues a step and returns at once;
:meth:`collect` waits for its sampled ids. A decode token the host has not seen
yet is passed as ``-(slot + 1)`` and resolved on the device from the previous
step's sampler output (``out_tokens``), so step t+1 is queued behind step t while
the host post-processes t: the GPU never idles between steps. Host metadata and
host-side sample buffers are double-buffered for that overlap.
"""
from __future__ import annotations

import bisect
import logging
import time
from dataclasses import dataclass

import numpy as np
import torch

from vgate import ops
from vgate.runtime.scheduler import ScheduledBatch
from vgate.runtime.step_meta import StepMeta
from vgate.utils.profiling import range_

log = logging.getLogger("vgate.engine")

# (320 / 448 / 640: a wave of 8 ~50-token prompts lands on 384-448 tokens; padded to 512 its prefill
# GEMMs did 14-33 % more work, profiles/r4_prefill_ring_tiles.log)
DEFAULT_T_BUCKETS = [1, 2, 4, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 320, 384, 448, 512, 640, 768, 1024, 1536,
                     2048, 3072, 4096, 6144, 8192, 12288, 16384]
DEFAULT_S_BUCKETS = [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024]


@dataclass
class StepHandle:
    k: int                 # double-buffer index
    ns: int                # batch items
    samples: list[bool]    # item consumes its sampled token
    toks: list[int] | None  # already known (CPU path)
    t_launch: float
    bucket: tuple = (0, 0)  # (T, S) graph bucket of the step
    eager: bool = False     # ran without a captured graph (first sight of its bucket)
    timed: bool = False     # a start event was recorded (device time of sampled steps)


class ModelRunner:
    def __init__(self, model, kv_caches, max_num_seqs: int, max_num_batched_tokens: int, max_model_len: int,
                 block_size: int = 16, enforce_eager: bool = False, part_size: int = 512,
                 graph_token_buckets: list[int] | None = None):
        self.model = model
        self.kv = kv_caches
        self.device = model.device
        self.gpu = self.device.type == "cuda"
        self.block_size = block_size
        self.max_blocks = (max_model_len + block_size - 1) // block_size
        self.part_size = part_size
        tb = [b for b in (graph_token_buckets or DEFAULT_T_BUCKETS) if b < max_num_batched_tokens]
        self.t_buckets = sorted(set(tb + [max_num_batched_tokens]))
        sb = [b for b in DEFAULT_S_BUCKETS if b < max_num_seqs]
        self.s_buckets = sorted(set(sb + [max_num_seqs]))
        if self.t_buckets[-1] <= self.s_buckets[-1]:
            # a step with a prompt chunk needs a token bucket above its sequence bucket
            # (StepMeta.tile_cap): keep one above the largest
            self.t_buckets.append(self.s_buckets[-1] + 16)
        self.max_tokens = self.t_buckets[-1]
        self.max_seqs = max_num_seqs
        self.meta = StepMeta(self.max_tokens, self.max_seqs, self.max_blocks, self.device)
        self.use_graphs = self.gpu and not enforce_eager
        sh = getattr(model, "shard", None)
        self.tile_lead = ops.flash_lead(sh.hq, sh.hkv) if sh is not None else 32
        self.graph_ok = lambda T, S: True  # per-bucket veto (TP groups without capturable collectives)
        self.graphs: dict[tuple[int, int], tuple] = {}
        self.pool = None
        # rounded up to 4 ids: the sampled-id download moves 16-B pieces (ops.host_device_copy)
        self.out_tokens = torch.zeros((self.max_seqs + 3) // 4 * 4, dtype=torch.int32, device=self.device)
        self.meta.prev_tokens = self.out_tokens if self.gpu else None
        self._k = 0  # double-buffer index of the next launch
        if self.gpu:
            # pinned ring the step graph's last node writes the sampled ids into (slot = the
            # launch's double-buffer index, read by the kernel from the step metadata)
            # (+4 ints per slot: the custom all-reduce's {error, ticks, calls} words, copied by the
            # same node, so the TP collective check and its time need no host <-> device sync)
            self.out_ring = torch.zeros(2, self.out_tokens.numel() + 4, dtype=torch.int32, pin_memory=True)
            self.out_hosts = [self.out_ring[0], self.out_ring[1]]
            ar = getattr(getattr(model, "tp", None), "custom_ar", None)
            self.ar_base = int(ar.own) if ar is not None and getattr(ar, "own", None) else 0
            self._ar_last = (0, 0)  # (ticks, calls) at the last read
            self.fault = ops.fault_word(self.device)  # in-launch hand-off give-ups, read via the ring
            self._last_collected: int | None = None
            self._launches = 0
            self.stream = torch.cuda.Stream(self.device)
            # per-step device time from timing events (every 8th step is timed)
            self.started = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            self.dones = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            self.meta_copied = [torch.cuda.Event() for _ in range(2)]  # TP followers (they never collect)
            self._meta_pending = [False, False]
            self._uncollected = [False, False]  # launch() of buffer k whose step is not collected yet
        else:
            self.out_hosts = [self.out_tokens]
        self.graph_hits = 0
        self.graph_misses = 0
        self.defer_capture = True  # miss -> eager step now, capture at the next idle point
        self.pending_captures: dict[tuple[int, int], int] = {}
        self.defer_capture_failed = False  # a deferred capture raised: stop queueing more
        self.capture_seconds = 0.0
        self.gpu_ms = 0.0  # device time of every 8th step (upload -> sampled ids on host)
        self.host_ms = 0.0  # host time of execute() outside the device wait
        self.gpu_steps = 0
        self.collect_wait_ms = 0.0  # host time blocked in collect() waiting for a step's device work
        self.check_words = None  # consistency-guard words of the last step launched with check=True
        self.captures = 0  # hipGraph captures so far (start-up warm-up + deferred + on-miss)
        self.max_gpu_ms = 0.0  # slowest step's device time and its bucket (p99 forensics)
        self.max_gpu_bucket = (0, 0)
        self.max_gpu_eager = False
        self.step_gpu_ms: list[float] = []  # device time per collected step, drained by the metrics loop
        # TP rank 0: called with (T, S, ns, nt, mode) once a step's metadata is in the host buffer
        # (before the step runs) -> the engine publishes it on the shared-memory step ring
        self.on_plan = None

    # ----------------------------------------------------------------- buckets
    def _bucket(self, buckets, n):
        i = bisect.bisect_left(buckets, n)
        if i == len(buckets):
            raise ValueError(f"{n} exceeds the largest bucket {buckets[-1]}")
        return buckets[i]

    def bucket_for(self, nt: int, ns: int) -> tuple[int, int]:
        """Graph bucket (T, S) of a step with nt tokens over ns sequences. A step with a prompt
        chunk (nt > ns) gets a token bucket above its sequence bucket: buckets with T <= S carry
        no prefill tiles (StepMeta.tile_cap), so decode-only graphs launch no prefill attention."""
        T = self._bucket(self.t_buckets, nt)
        S = self._bucket(self.s_buckets, ns)
        if nt > ns and T <= S:
            T = self._bucket(self.t_buckets, S + 1)
        return T, S

    # ---------------------------------------------------------------- metadata
    def _fill(self, batch: ScheduledBatch, T: int, S: int, pending_slots: dict | None = None) -> list[bool]:
        m = self.meta
        h = m.h
        bs = self.block_size
        ids, pos, slots = h["ids"], h["positions"], h["slots"]
        qs, cl, sidx = h["query_start"], h["context_lens"], h["sample_idx"]
        temp, topp, topk, seeds, offs = h["temperature"], h["top_p"], h["top_k"], h["seeds"], h["offsets"]
        tseq, tq0 = h["tile_seq"], h["tile_q0"]
        bt = m.bt_host
        t = 0
        ntile = 0
        npre = 0
        samples = []
        qs[0] = 0
        for s, (seq, n) in enumerate(batch.items):
            c0 = seq.num_computed
            blocks = seq.blocks
            if n == 1:  # decode row: O(1) scalar writes (no per-step copy of the context)
                P = len(seq.prompt_ids)
                tok = seq.output_ids[c0 - P] if c0 >= P else seq.prompt_ids[c0]
                if pending_slots and tok < 0:  # unresolved sample of the previous step
                    tok = -(pending_slots[seq.seq_id] + 1)
                ids[t] = tok
                pos[t] = c0
                slots[t] = blocks[c0 // bs] * bs + c0 % bs
            else:
                toks = seq.ids_slice(c0, c0 + n)
                ids[t: t + n] = toks
                if pending_slots and toks[-1] < 0:
                    ids[t + n - 1] = -(pending_slots[seq.seq_id] + 1)
                p = np.arange(c0, c0 + n, dtype=np.int32)
                pos[t: t + n] = p
                slots[t: t + n] = np.asarray(blocks, dtype=np.int32)[p // bs] * bs + (p % bs)
            nb = len(blocks)
            bt[s, :nb] = blocks
            ctx = c0 + n
            cl[s] = ctx
            t += n
            qs[s + 1] = t
            sidx[s] = t - 1
            if n > 1:
                order = ops.tile_order(n, self.tile_lead)
                k = len(order)
                if ntile + k <= len(tseq):
                    tseq[ntile: ntile + k] = s
                    tq0[ntile: ntile + k] = order
                ntile += k
                npre += 1
            sp = seq.params
            temp[s] = 0.0 if sp.greedy else sp.temperature
            topp[s] = sp.top_p
            topk[s] = sp.top_k
            seeds[s] = seq.seed
            offs[s] = len(seq.output_ids)
            samples.append(ctx == seq.total_len)
        ns = len(batch.items)
        # padding (graph bucket)
        ids[t:T] = 0
        pos[t:T] = 0
        slots[t:T] = -1
        qs[ns + 1: S + 1] = t
        cl[ns:S] = 0
        sidx[ns:S] = 0
        temp[ns:S] = 0.0
        topp[ns:S] = 1.0
        topk[ns:S] = -1
        tile_cap = self.meta.tile_cap(T, S)
        if ntile > tile_cap:
            raise RuntimeError("prefill tile overflow")
        if npre > 1:
            self._order_tiles(tseq, tq0, ntile, qs, cl)
        tseq[ntile:tile_cap] = -1
        self._n_tok, self._n_seq = t, ns
        return samples

    def _order_tiles(self, tseq, tq0, ntile, qs, cl) -> None:
        """One longest-first tile order over the whole step (several prompt chunks): the flash
        kernel dispatches tiles in list order (csrc/kernels/attention.hip attn_flash_kernel, grid
        (KV heads x halves, tiles)), so every sequence's working blocks (lead-query group
        leaders) go first by causal range, then the tiles that exit at once."""
        ts, tq = tseq[:ntile].copy(), tq0[:ntile].copy()
        kv = cl[ts] - (qs[ts + 1] - qs[ts]) + tq  # context before the tile's first query
        key = np.where(tq % self.tile_lead == 0, kv, -1)
        o = np.argsort(-key, kind="stable")
        tseq[:ntile] = ts[o]
        tq0[:ntile] = tq[o]

    # ----------------------------------------------------------------- forward
    def _forward_sample(self, view):
        logits = self.model.forward(view, self.kv, self.part_size)
        ops.sample(logits, view.temperature, view.top_p, view.top_k, view.seeds, view.offsets,
                   out=self.out_tokens[: view.S])
        if self.gpu:  # last node of the step graph: sampled ids (+ fault / collective words) -> pinned ring slot
            ops.native().ids_to_host(self.out_tokens, self.out_ring, view.ring_slot, view.S, self.ar_base,
                                     fault=self.fault)
        return logits

    def _capture(self, T: int, S: int):
        with range_(f"vgate.capture T={T} S={S}"):
            return self._capture_impl(T, S)

    def _capture_impl(self, T: int, S: int):
        t0 = time.perf_counter()
        view = self.meta.view(T, S)
        # warm-up (eager) on the capture stream, then capture
        s = self.stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._forward_sample(view)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool, stream=s):
            logits = self._forward_sample(view)
        # the graph's static residual + logits tensors (the TP consistency guard reads them), owned by
        # the graph object: dropping a graph drops them with it (references kept beside a deleted
        # graph would pin blocks of its private pool, which the next capture into that pool asserts on)
        g.vg_out = (self.model.last_resid, logits)
        torch.cuda.synchronize()
        self.captures += 1
        self.capture_seconds += time.perf_counter() - t0
        log.debug("captured hipGraph T=%d S=%d in %.1f ms", T, S, 1e3 * (time.perf_counter() - t0))
        return g

    @torch.inference_mode()
    def execute(self, batch: ScheduledBatch, check: bool = False) -> tuple[list[int], list[bool]]:
        """Run one step synchronously; returns (sampled token per item, whether consumed)."""
        h = self.launch(batch, check=check)
        return self.collect(h), h.samples

    @torch.inference_mode()
    def launch(self, batch: ScheduledBatch, pending_slots: dict | None = None, check: bool = False) -> "StepHandle":
        """Enqueue one step (GPU: returns before it runs). ``pending_slots`` maps a
        sequence id to the previous step's sample slot of its unresolved last token. ``check``:
        TP followers are told to join the consistency exchange after this step (ring mode 4)."""
        if not self.gpu:
            toks, samples = self._execute_cpu(batch, check)
            return StepHandle(0, len(batch.items), samples, toks, time.perf_counter())
        ns = len(batch.items)
        nt = batch.num_tokens
        T, S = self.bucket_for(nt, ns)
        t_host = time.perf_counter()
        k = self._k
        self._k ^= 1
        if self._uncollected[k]:
            # host buffers k (metadata, sampled ids) still belong to the step two back: wait for it
            # (the engine loop collects a step before launching the one after next, so this is rare;
            # no per-step event after the upload: every event record is a marker packet in the queue)
            self.dones[k].synchronize()
        self.meta.select(k)
        samples = self._fill(batch, T, S, pending_slots)
        self.meta.h["ring_slot"][0] = k
        if self.on_plan is not None:
            self.on_plan(T, S, ns, nt, 4 if check else 0)
        # device time of every 8th step (an event record is a marker packet in the queue)
        timed = self._launches % 8 == 0
        self._launches += 1
        if timed:
            self.started[k].record()
        self.meta.upload(ns)
        self._uncollected[k] = True
        graphs = self.use_graphs and self.graph_ok(T, S)
        g = self.graphs.get((T, S)) if graphs else None
        if g is None and graphs and not self.defer_capture:
            # the capture's eager warm-up samples into out_tokens, which this step may
            # still have to read (ids < 0): keep the previous step's samples aside
            saved = self.out_tokens.clone()
            g = self.graphs[(T, S)] = self._capture(T, S)
            self.out_tokens.copy_(saved)
        eager = g is None
        if g is not None:
            self.graph_hits += 1
            g.replay()
            if check:
                self.check_words = self._words(*g.vg_out, nt, ns)
        else:
            if graphs and not self.defer_capture_failed:
                # first sight of this bucket under load: run it eagerly (a few ms of launch
                # overhead) and capture it when the engine is next idle (capture_pending) —
                # a capture (eager warm-up + record, ~0.1-0.5 s) would stall every in-flight
                # request behind this step
                self.graph_misses += 1
                self.pending_captures[(T, S)] = self.pending_captures.get((T, S), 0) + 1
            view = self.meta.view(T, S)
            view.num_tokens, view.num_seqs = nt, ns
            lg = self._forward_sample(view)
            if check:
                self.check_words = self._words(self.model.last_resid, lg, nt, ns)
        self.dones[k].record()
        self.host_ms += 1e3 * (time.perf_counter() - t_host)
        return StepHandle(k, ns, samples, None, t_host, (T, S), eager, timed)

    def collect(self, h: "StepHandle") -> list[int]:
        """Wait for a launched step and return its sampled ids (one per batch item)."""
        if h.toks is not None:
            return h.toks
        t_wait = time.perf_counter()
        self.dones[h.k].synchronize()
        self.collect_wait_ms += 1e3 * (time.perf_counter() - t_wait)
        if h.timed:
            ms = self.started[h.k].elapsed_time(self.dones[h.k])
            self.gpu_ms += ms
            self.gpu_steps += 1
            if ms > self.max_gpu_ms:
                self.max_gpu_ms, self.max_gpu_bucket, self.max_gpu_eager = ms, h.bucket, h.eager
            if len(self.step_gpu_ms) < 65536:
                self.step_gpu_ms.append(ms)
        toks = self.out_hosts[h.k][: h.ns].tolist()
        self._uncollected[h.k] = False
        self._last_collected = h.k
        return toks

    def kernel_fault(self, k: int | None = None) -> int:
        """The sticky fault word of the in-launch hand-offs (ops.fault_word) as the step graph's last
        node copied it into ring slot ``k`` (default: the last collected step); 0 = healthy. No sync."""
        if not self.gpu:
            return 0
        if k is None:
            k = self._last_collected if self._last_collected is not None else self._k ^ 1
        return int(self.out_ring[k][-1])

    def _words(self, resid, lg, nt: int, S: int) -> torch.Tensor:
        """[checksum of a step's post-all-reduce residual rows, of its logits rows, of its sampled
        ids] (int64, device; enqueued right behind the step). All three are replicated over a TP group: every rank's
        all-reduce sums the same partials in rank order, the logits all-gather concatenates in rank
        order, the sampler draws with the same seeds. The residual is the one that catches a
        collective read stale on one rank (the logits would hide it: the next all-reduce adds only
        rank 0's residual). CPU followers take argmax instead of sampling: ids count on the GPU only,
        where followers' sampled ids resolve their next step's inputs."""
        from vgate.parallel.comm import checksum64
        zero = torch.zeros((), dtype=torch.int64, device=self.device)
        a = checksum64(resid[:nt]) if resid is not None else zero
        b = checksum64(lg[:S]) if lg is not None else zero
        c = checksum64(self.out_tokens[:S]) if self.gpu else zero
        return torch.stack([a, b.to(a.device), c.to(a.device)])

    def reset_fault_ring(self) -> None:
        """After the engine's fault recovery (ops.reset_handoffs, device idle): clear the fault
        word copies in both ring slots, so the next check reads the new steps' words."""
        if self.gpu:
            self.out_ring[:, -1].zero_()

    def collective_words(self, k: int | None = None) -> tuple[int, float, int]:
        """(error, seconds, calls) of the custom all-reduce since the previous call, from the words
        the step graph's last node copied into ring slot ``k`` (default: the last launched one).
        No device sync: a slot holds a completed step's copy (or an older one; the error word is
        sticky, so a timeout is reported at most two steps late). (0, 0.0, 0) without TP."""
        if not self.gpu or not self.ar_base:
            return 0, 0.0, 0
        if k is None:  # rank 0: the step just collected; followers (never collect): the last launched
            k = self._last_collected if self._last_collected is not None else self._k ^ 1
        w = self.out_ring[k]
        err, ticks, calls = int(w[-4]), int(w[-3]) & 0xFFFFFFFF, int(w[-2]) & 0xFFFFFFFF
        t0, c0 = self._ar_last
        dc = (calls - c0) & 0xFFFFFFFF
        if dc == 0 or dc > 1 << 30:  # nothing new in this slot (or an older slot than the last read)
            return err, 0.0, 0
        self._ar_last = (ticks, calls)
        return err, ((ticks - t0) & 0xFFFFFFFF) / 1e8, dc

    @torch.inference_mode()
    def hidden_states(self, batch: ScheduledBatch) -> torch.Tensor:
        """Eager prefill of ``batch`` returning the last layer's residual stream [T, H]
        (embeddings). The caller guarantees no step is in flight (shared metadata buffers)."""
        ns, nt = len(batch.items), batch.num_tokens
        if self.gpu:
            self.meta.select(self._k)
        else:
            self.meta.select(0)
        self._fill(batch, nt, ns)
        if self.on_plan is not None:  # TP: the followers run the same hidden-states forward
            self.on_plan(nt, ns, ns, nt, 1)
        self.meta.upload(ns)
        view = self.meta.view(nt, ns)
        view.num_tokens, view.num_seqs = nt, ns
        view.prev_tokens = None
        h = self.model.forward(view, self.kv, self.part_size, return_hidden=True)
        return h[:nt]

    def _execute_cpu(self, batch, check: bool = False):
        ns, nt = len(batch.items), batch.num_tokens
        self.meta.select(0)
        samples = self._fill(batch, nt, ns)
        if self.on_plan is not None:
            self.on_plan(nt, ns, ns, nt, 4 if check else 0)
        self.meta.upload(ns)
        view = self.meta.view(nt, ns)
        view.num_tokens, view.num_seqs = nt, ns
        logits = self._cpu_sample(view, batch)
        if check:
            self.check_words = self._words(self.model.last_resid, logits, nt, ns)
        return self.out_tokens[:ns].tolist(), samples

    def _cpu_sample(self, view, batch):
        logits = self.model.forward(view, self.kv, self.part_size)
        gens = []
        for seq, _ in batch.items:
            g = torch.Generator()
            g.manual_seed((seq.seed * 1000003 + len(seq.output_ids)) & 0x7FFFFFFFFFFFFFFF)
            gens.append(g)
        self.out_tokens[: view.S] = ops.ref.sample_ref(logits, view.temperature, view.top_p, view.top_k, gens)
        return logits

    def warmup(self, token_buckets: list[int] | None = None, seq_buckets: list[int] | None = None) -> float:
        """Pre-capture graphs for the given buckets (all-padding metadata)."""
        if not self.use_graphs:
            return 0.0
        t0 = time.perf_counter()
        for T in token_buckets or []:
            for S in seq_buckets or [1]:
                if S > T or (T, S) in self.graphs or not self.graph_ok(T, S):
                    continue
                self._fill_padding(T, S)
                if self.on_plan is not None:  # TP: every rank captures the same bucket in step
                    self.on_plan(T, S, 0, 0, 2)
                self.meta.upload(0)
                self.graphs[(T, S)] = self._capture(T, S)
        return time.perf_counter() - t0

    # ------------------------------------------------------------ TP followers
    def follower_host_buffer(self):
        """The pinned host buffer the next ring entry is copied into (double-buffered like
        launch(): buffer k may still feed the H2D copy of two steps back)."""
        if not self.gpu:
            self.meta.select(0)
            return self.meta.host
        k = self._k
        if self._meta_pending[k]:
            self.meta_copied[k].synchronize()
        self.meta.select(k)
        return self.meta.host

    @torch.inference_mode()
    def follow_step(self, T: int, S: int, ns: int, nt: int, mode: int, check: bool = False):
        """Run rank 0's step from the metadata just copied into follower_host_buffer():
        mode 0 = a step (graph replay, captured on first sight exactly as rank 0 does), 1 = the
        hidden-states forward of an embedding request, 2 = capture bucket (T, S) (start-up
        warm-up). Returns nothing: followers never read their sampled tokens on the host (their
        sampler output only resolves the next step's pending ids on the device)."""
        if not self.gpu:
            view = self.meta.view(T, S)
            view.num_tokens, view.num_seqs = nt, ns
            view.prev_tokens = None
            if mode == 1:
                self.model.forward(view, self.kv, self.part_size, return_hidden=True)
            elif mode == 0:
                logits = self.model.forward(view, self.kv, self.part_size)
                self.out_tokens[:S] = logits.argmax(-1).int()
                if check:
                    self.check_words = self._words(self.model.last_resid, logits, nt, ns)
            return
        k = self._k
        if mode == 2:
            self.meta.upload(0)
            if (T, S) not in self.graphs:
                self.graphs[(T, S)] = self._capture(T, S)
            return
        self._k ^= 1
        self.meta.upload(ns)
        self.meta_copied[k].record()
        self._meta_pending[k] = True
        view = self.meta.view(T, S)
        view.num_tokens, view.num_seqs = nt, ns
        if mode == 1:
            view.prev_tokens = None
            self.model.forward(view, self.kv, self.part_size, return_hidden=True)
            return
        graphs = self.use_graphs and self.graph_ok(T, S)
        g = self.graphs.get((T, S)) if graphs else None
        if g is None and graphs:
            saved = self.out_tokens.clone()
            g = self.graphs[(T, S)] = self._capture(T, S)
            self.out_tokens.copy_(saved)
        if g is not None:
            self.graph_hits += 1
            g.replay()
            if check:
                self.check_words = self._words(*g.vg_out, nt, ns)
        else:
            lg = self._forward_sample(view)
            if check:
                self.check_words = self._words(self.model.last_resid, lg, nt, ns)

    def capture_pending(self, max_graphs: int = 64) -> int:
        """Capture the buckets that ran eagerly since the last call (most frequent first).
        Call only with no step in flight: captures reuse the step-metadata buffers."""
        if not self.use_graphs or not self.pending_captures:
            return 0
        keys = sorted(self.pending_captures, key=lambda k: -self.pending_captures[k])[:max_graphs]
        t0 = time.perf_counter()
        n = 0
        for T, S in keys:
            if (T, S) not in self.graphs:
                self._fill_padding(T, S)
                self.meta.upload(0)
                self.graphs[(T, S)] = self._capture(T, S)
                n += 1
            del self.pending_captures[(T, S)]  # removed last: present means "capture still to come"
        log.info("captured %d deferred hipGraph bucket(s) in %.2fs", n, time.perf_counter() - t0)
        return n

    def _fill_padding(self, T, S):
        h = self.meta.h
        h["ids"][:T] = 0
        h["positions"][:T] = 0
        h["slots"][:T] = -1
        h["query_start"][: S + 1] = 0
        h["context_lens"][:S] = 0
        h["sample_idx"][:S] = 0
        h["temperature"][:S] = 0
        h["top_p"][:S] = 1
        h["top_k"][:S] = -1
        h["tile_seq"][: self.meta.tile_cap(T, S)] = -1
