"""Request state inside the native engine."""
from __future__ import annotations

import collections
import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Callable

from vgate.runtime.sampling_params import SamplingParams

_ids = itertools.count()


PENDING = -1  # placeholder for a token sampled by an in-flight step


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


@dataclass
class Sequence:
    request_id: str
    prompt_ids: list[int]
    params: SamplingParams
    callback: Callable | None = None
    stream: bool = False
    seq_id: int = field(default_factory=lambda: next(_ids))
    arrival: float = field(default_factory=time.perf_counter)
    output_ids: list[int] = field(default_factory=list)
    status: SeqStatus = SeqStatus.WAITING
    blocks: list[int] = field(default_factory=list)
    num_computed: int = 0
    num_cached_prefix: int = 0
    num_preemptions: int = 0
    first_token_time: float | None = None
    last_token_time: float | None = None
    finish_time: float | None = None
    finish_reason: str | None = None
    seed: int = 0
    text: str = ""
    detok: object = None
    hashed_blocks: int = 0
    block_hashes: list[int] = field(default_factory=list)
    aborted: bool = False
    # asynchronous scheduling: output_ids indices still holding PENDING (sampled on the
    # device, not yet seen by the host) and the sample slot of the newest one
    pending: collections.deque = field(default_factory=collections.deque)
    pending_slot: int = -1

    @property
    def all_ids(self) -> list[int]:
        return self.prompt_ids + self.output_ids if self.output_ids else self.prompt_ids

    def ids_slice(self, a: int, b: int) -> list[int]:
        """all_ids[a:b] without concatenating the whole prompt and output."""
        P = len(self.prompt_ids)
        if b <= P:
            return self.prompt_ids[a:b]
        if a >= P:
            return self.output_ids[a - P: b - P]
        return self.prompt_ids[a:] + self.output_ids[: b - P]

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def num_outputs_resolved(self) -> int:
        return len(self.output_ids) - len(self.pending)

    @property
    def remaining(self) -> int:
        """Tokens whose KV is not yet computed (>= 1 while running)."""
        return self.total_len - self.num_computed

    @property
    def is_finished(self) -> bool:
        return self.status == SeqStatus.FINISHED
