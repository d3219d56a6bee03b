"""Per-step metadata in ONE pinned host buffer mirrored by ONE device buffer.

Every forward pass reads its token/sequence metadata (ids, positions, KV slots,
query offsets, context lengths, block tables, prefill tiles, sampling params)
from fixed-address device views, so a captured hipGraph replays any step of its
bucket after a single H2D copy of the used prefix of the buffer. The block
table is the last field, so only the rows of live sequences are copied.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from vgate import ops


def _align(n: int, a: int = 16) -> int:
    return (n + a - 1) // a * a


@dataclass
class StepView:
    T: int
    S: int
    ids: torch.Tensor
    positions: torch.Tensor
    slots: torch.Tensor
    query_start: torch.Tensor
    context_lens: torch.Tensor
    tile_seq: torch.Tensor
    tile_q0: torch.Tensor
    sample_idx: torch.Tensor
    block_tables: torch.Tensor
    temperature: torch.Tensor
    top_p: torch.Tensor
    top_k: torch.Tensor
    seeds: torch.Tensor
    offsets: torch.Tensor
    ring_slot: torch.Tensor | None = None  # [1]: slot of the pinned ring the step's sampled ids go to
    prev_tokens: torch.Tensor | None = None  # previous step's sampled ids (ids < 0 refer into it)
    num_tokens: int = 0
    num_seqs: int = 0


class StepMeta:
    def __init__(self, max_tokens: int, max_seqs: int, max_blocks: int, device, pinned: bool = True):
        self.T = max_tokens
        self.S = max_seqs
        self.max_blocks = max_blocks
        self.tiles = max_tokens // 16 + max_seqs
        self.device = torch.device(device)
        fields = [  # (name, dtype, count) ; 8-byte fields first, block table last
            ("seeds", np.int64, self.S), ("offsets", np.int64, self.S),
            ("temperature", np.float32, self.S), ("top_p", np.float32, self.S), ("top_k", np.int32, self.S),
            ("ids", np.int32, self.T), ("positions", np.int32, self.T), ("slots", np.int32, self.T),
            ("query_start", np.int32, self.S + 1), ("context_lens", np.int32, self.S),
            ("tile_seq", np.int32, self.tiles), ("tile_q0", np.int32, self.tiles),
            ("sample_idx", np.int32, self.S), ("ring_slot", np.int32, 4),
            ("block_tables", np.int32, self.S * max_blocks),
        ]
        off = 0
        self.layout = {}
        for name, dt, n in fields:
            off = _align(off, 16)
            self.layout[name] = (off, dt, n)
            off += np.dtype(dt).itemsize * n
        self.nbytes = _align(off, 16)
        use_pin = pinned and self.device.type == "cuda"
        # two pinned host buffers: with asynchronous scheduling the next step is written
        # while the previous step's H2D copy may still be queued behind a running graph
        nhost = 2 if self.device.type == "cuda" else 1
        self.hosts = [torch.zeros(self.nbytes, dtype=torch.uint8, pin_memory=use_pin) for _ in range(nhost)]
        self.dev = torch.zeros(self.nbytes, dtype=torch.uint8, device=self.device) if self.device.type == "cuda" \
            else self.hosts[0]
        tdt = {np.int64: torch.int64, np.float32: torch.float32, np.int32: torch.int32}
        self._h = []
        for host in self.hosts:
            hnp = host.numpy()
            self._h.append({name: hnp[o: o + np.dtype(dt).itemsize * n].view(dt)
                            for name, (o, dt, n) in self.layout.items()})
        self.d = {name: self.dev[o: o + np.dtype(dt).itemsize * n].view(tdt[dt])
                  for name, (o, dt, n) in self.layout.items()}
        self.prev_tokens = None
        self.select(0)

    def select(self, k: int) -> None:
        """Make host buffer k the one _fill writes and upload() copies from."""
        self.k = k
        self.host = self.hosts[k]
        self.h = self._h[k]
        self.bt_host = self.h["block_tables"].reshape(self.S, self.max_blocks)

    def reset(self) -> None:
        self.h["tile_seq"][:] = -1
        self.h["tile_q0"][:] = 0

    def used_bytes(self, num_seqs: int) -> int:
        off, _, _ = self.layout["block_tables"]
        return off + num_seqs * self.max_blocks * 4

    def upload(self, num_seqs: int, stream=None) -> None:
        if self.dev is self.host:
            return
        # a copy kernel on the compute queue, not an SDMA copy (ops.host_device_copy); nbytes is a
        # multiple of 16, so the 16-B rounded prefix stays inside both buffers
        ops.host_device_copy(self.dev, self.host, self.used_bytes(num_seqs))

    @staticmethod
    def tile_cap(T: int, S: int) -> int:
        """Prefill tiles a (T, S) bucket carries: none when T <= S — a bucket with no more token
        slots than sequence slots serves decode-only steps (the runner sends a step with a prompt
        chunk to a token bucket above S), so its graphs launch no prefill attention at all."""
        return T // 16 + S if T > S else 0

    def view(self, T: int, S: int) -> StepView:
        d = self.d
        nt = self.tile_cap(T, S)
        return StepView(
            T=T, S=S, ids=d["ids"][:T], positions=d["positions"][:T], slots=d["slots"][:T],
            query_start=d["query_start"][: S + 1], context_lens=d["context_lens"][:S],
            tile_seq=d["tile_seq"][:nt], tile_q0=d["tile_q0"][:nt],
            sample_idx=d["sample_idx"][:S], block_tables=d["block_tables"].view(self.S, self.max_blocks)[:S],
            temperature=d["temperature"][:S], top_p=d["top_p"][:S], top_k=d["top_k"][:S],
            seeds=d["seeds"][:S], offsets=d["offsets"][:S], ring_slot=d["ring_slot"][:1],
            prev_tokens=self.prev_tokens)
