"""Continuous-batching scheduler with chunked prefill and recompute preemption.

Every step builds ONE flat token batch mixing decode tokens and prefill chunks
(the attention kernels split it: single-query sequences -> split-K decode kernel,
multi-token chunks -> varlen prefill kernel), so a new request's prefill never
stalls running decodes for a whole extra weight-streaming pass.

Policy per step (token budget = max_num_batched_tokens):
  1. running sequences in arrival order get their remaining tokens (1 for a
     decode, the rest of a chunked prefill), growing their KV blocks; when the
     pool is exhausted the most recently arrived running sequence is preempted
     (blocks freed, re-queued at the front, recomputed later with its outputs);
  2. waiting sequences are admitted while the budget, ``max_num_seqs`` and the
     KV pool allow (prefix-cache hits skip already-cached prompt blocks).
"""
from __future__ import annotations

import collections
from dataclasses import dataclass

from vgate.runtime.kv_cache import KVCacheManager
from vgate.runtime.sequence import Sequence, SeqStatus


@dataclass
class ScheduledBatch:
    items: list[tuple[Sequence, int]]  # (sequence, number of new tokens this step)
    num_tokens: int
    num_prefill_tokens: int
    num_decode: int
    preempted: list[Sequence]
    kv_pressure: bool = False  # no_preempt mode stopped early for lack of KV blocks

    @property
    def empty(self) -> bool:
        return not self.items


class Scheduler:
    def __init__(self, kv: KVCacheManager, max_num_seqs: int, max_num_batched_tokens: int,
                 max_model_len: int):
        self.kv = kv
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        self.num_preemptions = 0

    def add(self, seq: Sequence) -> None:
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def remove(self, seq: Sequence) -> None:
        if seq in self.running:
            self.running.remove(seq)
        try:
            self.waiting.remove(seq)
        except ValueError:
            pass
        self.kv.free(seq)

    def _preempt(self, victim: Sequence, out: list) -> None:
        self.running.remove(victim)
        self.kv.free(victim)
        victim.status = SeqStatus.WAITING
        victim.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(victim)
        out.append(victim)

    def schedule(self, no_preempt: bool = False) -> ScheduledBatch:
        """Build the next step. ``no_preempt`` (a step is in flight): stop instead of
        preempting when the KV pool runs out (the caller drains and reschedules)."""
        budget = self.max_tokens
        items: list[tuple[Sequence, int]] = []
        preempted: list[Sequence] = []
        n_prefill = 0
        n_decode = 0
        # 1. running sequences (oldest first); preempt from the newest end on KV pressure
        i = 0
        while i < len(self.running) and budget > 0:
            seq = self.running[i]
            if seq.pending and (len(seq.output_ids) >= seq.params.max_tokens
                                or seq.total_len >= self.max_model_len):
                i += 1  # its last token is in flight and will end it: nothing to compute
                continue
            n = min(seq.remaining, budget)
            if no_preempt and not self.kv.ensure(seq, n):
                return ScheduledBatch(items, sum(k for _, k in items), n_prefill, n_decode, preempted, True)
            while not self.kv.ensure(seq, n):
                victim = self.running[-1]
                self._preempt(victim, preempted)
                if victim is seq:
                    break
            if seq.status != SeqStatus.RUNNING:
                continue  # it preempted itself; do not advance i (list shrank)
            items.append((seq, n))
            budget -= n
            if seq.remaining == 1 and n == 1:
                n_decode += 1
            else:
                n_prefill += n
            i += 1
        # 2. admit waiting sequences
        while self.waiting and budget > 0 and len(self.running) < self.max_num_seqs:
            seq = self.waiting[0]
            if not seq.blocks:
                self.kv.reuse_prefix(seq)
            n = min(seq.remaining, budget)
            if not self.kv.ensure(seq, n):
                if not self.running and not items:
                    # nothing else can free memory: the request can never fit
                    if self.kv.blocks_needed(seq, n) > self.kv.num_blocks:
                        raise RuntimeError("request does not fit in the KV cache")
                break
            self.waiting.popleft()
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
            items.append((seq, n))
            budget -= n
            n_prefill += n
        total = sum(n for _, n in items)
        return ScheduledBatch(items, total, n_prefill, n_decode, preempted)

    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        if seq in self.running:
            self.running.remove(seq)
        self.kv.free(seq)
