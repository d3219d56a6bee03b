// Native sharded LRU for the gateway's result cache (vgate/cache.py, backend "native").
//
// The reference keeps its result cache in a Python OrderedDict under an asyncio.Lock
// (reference vgate/cache.py:28-108) and plans a C++ sharded LRU for its Phase 7
// (reference ROADMAP.md:615-654). Here: keys are the 16-hex-char request keys, values
// the serialized (JSON) response bytes, so a hit is an independent copy by construction.
// The key space is split over power-of-two shards (hash -> shard), each with its own
// mutex, intrusive recency list and hash index: concurrent gateway threads (HTTP loop,
// executor threads, a second worker thread pool) contend only per shard, and every call
// drops the GIL while it holds a shard lock. Capacity is global and split evenly, so an
// eviction is always the least-recent entry of the inserting key's shard.
#pragma once
#include <cstdint>
#include <list>
#include <mutex>
#include <optional>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace vgate {

class ShardedLRU {
 public:
  ShardedLRU(int64_t capacity, int64_t shards);

  std::optional<std::string> get(const std::string& key);
  // returns the number of entries evicted by this insert (0 or 1)
  int64_t put(const std::string& key, std::string value);
  bool erase(const std::string& key);
  void clear();

  int64_t size() const;
  int64_t capacity() const { return capacity_; }
  int64_t num_shards() const { return (int64_t)shards_.size(); }
  uint64_t hits() const;
  uint64_t misses() const;
  uint64_t evictions() const;

 private:
  struct Shard {
    mutable std::mutex mu;
    std::list<std::pair<std::string, std::string>> order;  // front = most recent
    std::unordered_map<std::string, std::list<std::pair<std::string, std::string>>::iterator> index;
    int64_t cap = 0;
    uint64_t hits = 0, misses = 0, evictions = 0;
  };
  Shard& shard_of(const std::string& key);
  int64_t capacity_;
  std::vector<Shard> shards_;
};

}  // namespace vgate
