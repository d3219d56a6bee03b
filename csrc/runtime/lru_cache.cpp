// Native sharded LRU (see lru_cache.h). Pure C++: the pybind11 glue lives in bindings.cpp
// so this file also builds into the host-only sanitizer test (csrc/tests/host_test.cpp).
#include "lru_cache.h"

#include <functional>
#include <stdexcept>

namespace vgate {

ShardedLRU::ShardedLRU(int64_t capacity, int64_t shards) : capacity_(capacity) {
  if (capacity < 0) throw std::invalid_argument("ShardedLRU: capacity < 0");
  int64_t n = 1;
  while (n < shards && n < 256) n <<= 1;  // power of two, at most 256
  // never more shards than entries: each shard must hold >= 1 entry when capacity > 0
  while (n > 1 && n > capacity) n >>= 1;
  shards_ = std::vector<Shard>(n);
  for (int64_t i = 0; i < n; ++i) shards_[i].cap = capacity / n + (i < capacity % n ? 1 : 0);
}

ShardedLRU::Shard& ShardedLRU::shard_of(const std::string& key) {
  // splitmix the std::hash so short hex keys spread over the low bits
  uint64_t h = std::hash<std::string>{}(key);
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  return shards_[h & (shards_.size() - 1)];
}

std::optional<std::string> ShardedLRU::get(const std::string& key) {
  Shard& s = shard_of(key);
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.index.find(key);
  if (it == s.index.end()) {
    ++s.misses;
    return std::nullopt;
  }
  s.order.splice(s.order.begin(), s.order, it->second);
  ++s.hits;
  return it->second->second;
}

int64_t ShardedLRU::put(const std::string& key, std::string value) {
  Shard& s = shard_of(key);
  std::lock_guard<std::mutex> g(s.mu);
  if (s.cap <= 0) return 0;
  auto it = s.index.find(key);
  if (it != s.index.end()) {
    it->second->second = std::move(value);
    s.order.splice(s.order.begin(), s.order, it->second);
    return 0;
  }
  s.order.emplace_front(key, std::move(value));
  s.index.emplace(key, s.order.begin());
  int64_t ev = 0;
  while ((int64_t)s.index.size() > s.cap) {
    s.index.erase(s.order.back().first);
    s.order.pop_back();
    ++s.evictions;
    ++ev;
  }
  return ev;
}

bool ShardedLRU::erase(const std::string& key) {
  Shard& s = shard_of(key);
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.index.find(key);
  if (it == s.index.end()) return false;
  s.order.erase(it->second);
  s.index.erase(it);
  return true;
}

void ShardedLRU::clear() {
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> g(s.mu);
    s.order.clear();
    s.index.clear();
  }
}

int64_t ShardedLRU::size() const {
  int64_t n = 0;
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> g(s.mu);
    n += (int64_t)s.index.size();
  }
  return n;
}

uint64_t ShardedLRU::hits() const {
  uint64_t n = 0;
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> g(s.mu);
    n += s.hits;
  }
  return n;
}

uint64_t ShardedLRU::misses() const {
  uint64_t n = 0;
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> g(s.mu);
    n += s.misses;
  }
  return n;
}

uint64_t ShardedLRU::evictions() const {
  uint64_t n = 0;
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> g(s.mu);
    n += s.evictions;
  }
  return n;
}

}  // namespace vgate
