"""Paged KV-cache manager.

Device side: one ``[num_blocks, Hkv_local, 16, 128]`` bf16 tensor per layer for
K and for V, allocated once from ``gpu_memory_utilization x HBM`` (288 GB per
MI355X -> millions of cached tokens for the 1.5B-8B models).
Host side: the native :class:`vgate._C.BlockAllocator` (C++, refcounts, prefix
cache with chained content hashes and LRU eviction). A pure-Python allocator with
the same interface backs CPU-only environments where the extension is absent.
"""
from __future__ import annotations

import collections
import hashlib
import threading

import torch

from vgate.runtime.sequence import Sequence

BLOCK_SIZE = 16


class PyBlockAllocator:
    """Python twin of the native allocator (same semantics; used when _C is missing)."""

    def __init__(self, num_blocks: int, block_size: int, prefix_caching: bool = False):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self._pc = prefix_caching
        self._ref = [0] * num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))
        self._lru: collections.OrderedDict[int, None] = collections.OrderedDict()
        self._hash_of: dict[int, int] = {}
        self._block_of: dict[int, int] = {}
        self._mu = threading.Lock()
        self.hits = 0
        self.queries = 0

    def num_free(self) -> int:
        return len(self._free) + len(self._lru)

    def num_cached(self) -> int:
        return len(self._block_of)

    def can_allocate(self, n: int) -> bool:
        return self.num_free() >= n

    def _take(self) -> int:
        if self._free:
            b = self._free.pop()
        elif self._lru:
            b, _ = self._lru.popitem(last=False)
            h = self._hash_of.pop(b, None)
            if h is not None and self._block_of.get(h) == b:
                del self._block_of[h]
        else:
            raise RuntimeError("out of KV blocks")
        self._ref[b] = 1
        return b

    def allocate(self, n: int) -> list[int]:
        with self._mu:
            if self.num_free() < n:
                raise RuntimeError("out of KV blocks")
            return [self._take() for _ in range(n)]

    def free(self, blocks) -> None:
        with self._mu:
            for b in blocks:
                if self._ref[b] <= 0:
                    raise RuntimeError("double free")
                self._ref[b] -= 1
                if self._ref[b] == 0:
                    if self._pc and b in self._hash_of:
                        self._lru[b] = None
                    else:
                        self._hash_of.pop(b, None)
                        self._free.append(b)

    def incref(self, blocks) -> None:
        with self._mu:
            for b in blocks:
                self._ref[b] += 1

    def refcount(self, b: int) -> int:
        return self._ref[b]

    def lookup(self, h: int) -> int:
        with self._mu:
            if not self._pc:
                return -1
            self.queries += 1
            b = self._block_of.get(h)
            if b is None:
                return -1
            self._lru.pop(b, None)
            self._ref[b] += 1
            self.hits += 1
            return b

    def register_hash(self, b: int, h: int) -> None:
        with self._mu:
            if not self._pc or h in self._block_of:
                return
            old = self._hash_of.get(b)
            if old is not None:
                self._block_of.pop(old, None)
            self._hash_of[b] = h
            self._block_of[h] = b

    def reset_prefix_cache(self) -> None:
        with self._mu:
            for b in list(self._lru):
                self._free.append(b)
            self._lru.clear()
            self._hash_of.clear()
            self._block_of.clear()

    @staticmethod
    def hash_block(parent: int, tokens) -> int:
        m = hashlib.blake2b(digest_size=8)
        m.update(int(parent).to_bytes(8, "little", signed=False))
        for t in tokens:
            m.update(int(t).to_bytes(8, "little", signed=True))
        return int.from_bytes(m.digest(), "little")


def make_allocator(num_blocks: int, block_size: int = BLOCK_SIZE, prefix_caching: bool = False,
                   prefer_native: bool = True):
    if prefer_native:
        try:
            from vgate import ops
            C = ops.native()
            return C.BlockAllocator(num_blocks, block_size, prefix_caching)
        except Exception:  # noqa: BLE001
            pass
    return PyBlockAllocator(num_blocks, block_size, prefix_caching)


class KVCacheManager:
    def __init__(self, num_blocks: int, block_size: int = BLOCK_SIZE, prefix_caching: bool = False,
                 prefer_native: bool = True):
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.prefix_caching = prefix_caching
        self.alloc = make_allocator(num_blocks, block_size, prefix_caching, prefer_native)
        self._hash = self.alloc.hash_block

    # ------------------------------------------------------------------ queries
    def num_free(self) -> int:
        return self.alloc.num_free()

    def usage(self) -> float:
        return 1.0 - self.alloc.num_free() / max(1, self.num_blocks)

    def blocks_needed(self, seq: Sequence, n_new: int) -> int:
        need = (seq.num_computed + n_new + self.block_size - 1) // self.block_size
        return max(0, need - len(seq.blocks))

    # ------------------------------------------------------------------ updates
    def reuse_prefix(self, seq: Sequence) -> None:
        """On admission: attach cached blocks of the prompt prefix (never the final token)."""
        if not self.prefix_caching or seq.blocks:
            return
        ids = seq.all_ids
        nfull = (len(ids) - 1) // self.block_size
        parent = 0
        for i in range(nfull):
            h = self._hash(parent, ids[i * self.block_size:(i + 1) * self.block_size])
            b = self.alloc.lookup(h)
            if b < 0:
                break
            seq.blocks.append(b)
            seq.block_hashes.append(h)
            parent = h
        seq.num_computed = len(seq.blocks) * self.block_size
        seq.num_cached_prefix = seq.num_computed
        seq.hashed_blocks = len(seq.blocks)

    def ensure(self, seq: Sequence, n_new: int) -> bool:
        need = self.blocks_needed(seq, n_new)
        if need == 0:
            return True
        if not self.alloc.can_allocate(need):
            return False
        seq.blocks.extend(self.alloc.allocate(need))
        return True

    def register_computed(self, seq: Sequence) -> None:
        """Publish hashes of newly completed full blocks for prefix reuse."""
        if not self.prefix_caching:
            return
        full = seq.num_computed // self.block_size
        ids = None
        while seq.hashed_blocks < full:
            if ids is None:
                ids = seq.all_ids
            i = seq.hashed_blocks
            parent = seq.block_hashes[-1] if seq.block_hashes else 0
            h = self._hash(parent, ids[i * self.block_size:(i + 1) * self.block_size])
            self.alloc.register_hash(seq.blocks[i], h)
            seq.block_hashes.append(h)
            seq.hashed_blocks += 1

    def free(self, seq: Sequence) -> None:
        if seq.blocks:
            self.alloc.free(seq.blocks)
        seq.blocks = []
        seq.block_hashes = []
        seq.hashed_blocks = 0
        seq.num_computed = 0


def allocate_kv_tensors(num_layers: int, num_blocks: int, hkv: int, head_dim: int, device,
                        dtype=torch.bfloat16, block_size: int = BLOCK_SIZE):
    """[(K, V)] per layer, zero-initialised (stale slots are always finite)."""
    caches = []
    for _ in range(num_layers):
        k = torch.zeros(num_blocks, hkv, block_size, head_dim, dtype=dtype, device=device)
        v = torch.zeros(num_blocks, hkv, block_size, head_dim, dtype=dtype, device=device)
        caches.append((k, v))
    return caches
