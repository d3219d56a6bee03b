// Native paged-KV block allocator (host side of the engine's memory manager).
//
// The KV pool is one preallocated device tensor per layer ([num_blocks, Hkv, 16, 128]
// bf16, sized from gpu_memory_utilization x HBM); this allocator hands out block ids.
// Features:
//   * O(1) alloc/free with per-block reference counts (forked / shared prefixes)
//   * prefix caching: a full block can be registered under a chained content hash;
//     when its refcount drops to 0 it stays resident in an LRU "evictable" list and a
//     later request with the same prefix re-acquires it instead of recomputing.
//   * thread safe (the engine thread and the API thread may both query stats)
#pragma once
#include <pybind11/pybind11.h>

#include <cstdint>
#include <list>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace vgate {

class BlockAllocator {
 public:
  BlockAllocator(int64_t num_blocks, int64_t block_size, bool prefix_caching);

  int64_t num_blocks() const { return num_blocks_; }
  int64_t block_size() const { return block_size_; }
  int64_t num_free() const;           // immediately allocatable (free + evictable)
  int64_t num_cached() const;         // blocks holding a registered hash
  bool can_allocate(int64_t n) const { return num_free() >= n; }

  std::vector<int64_t> allocate(int64_t n);
  void free(const std::vector<int64_t>& blocks);
  void incref(const std::vector<int64_t>& blocks);
  int64_t refcount(int64_t block) const;

  // prefix cache
  int64_t lookup(uint64_t hash);      // -1 if absent; otherwise block with refcount+1
  void register_hash(int64_t block, uint64_t hash);
  uint64_t hits() const { return hits_; }
  uint64_t queries() const { return queries_; }
  void reset_prefix_cache();

  static uint64_t hash_block(uint64_t parent, const std::vector<int64_t>& tokens);

 private:
  int64_t take_one();  // requires lock
  int64_t num_blocks_, block_size_;
  bool prefix_caching_;
  mutable std::mutex mu_;
  std::vector<int32_t> ref_;
  std::vector<int64_t> free_;                 // never-hashed free blocks (stack)
  std::list<int64_t> lru_;                    // hashed, refcount 0, evictable (front = oldest)
  std::vector<std::list<int64_t>::iterator> lru_pos_;
  std::vector<char> in_lru_;
  std::vector<uint64_t> block_hash_;
  std::vector<char> has_hash_;
  std::unordered_map<uint64_t, int64_t> hash_to_block_;
  uint64_t hits_ = 0, queries_ = 0;
};

void bind_runtime(pybind11::module_& m);
void bind_step_ring(pybind11::module_& m);  // step_ring.cpp

}  // namespace vgate
