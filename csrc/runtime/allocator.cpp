#include "allocator.h"

#include <pybind11/stl.h>

#include <stdexcept>

namespace vgate {

BlockAllocator::BlockAllocator(int64_t num_blocks, int64_t block_size, bool prefix_caching)
    : num_blocks_(num_blocks), block_size_(block_size), prefix_caching_(prefix_caching) {
  if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("BlockAllocator: sizes must be > 0");
  ref_.assign(num_blocks, 0);
  lru_pos_.resize(num_blocks);
  in_lru_.assign(num_blocks, 0);
  block_hash_.assign(num_blocks, 0);
  has_hash_.assign(num_blocks, 0);
  free_.reserve(num_blocks);
  // hand out low block ids first (stack pops from the back)
  for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
}

int64_t BlockAllocator::num_free() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)free_.size() + (int64_t)lru_.size();
}

int64_t BlockAllocator::num_cached() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)hash_to_block_.size();
}

int64_t BlockAllocator::take_one() {
  int64_t b;
  if (!free_.empty()) {
    b = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {
    b = lru_.front();  // evict least recently freed cached block
    lru_.pop_front();
    in_lru_[b] = 0;
    if (has_hash_[b]) {
      auto it = hash_to_block_.find(block_hash_[b]);
      if (it != hash_to_block_.end() && it->second == b) hash_to_block_.erase(it);
      has_hash_[b] = 0;
    }
  } else {
    throw std::runtime_error("BlockAllocator: out of KV blocks");
  }
  ref_[b] = 1;
  return b;
}

std::vector<int64_t> BlockAllocator::allocate(int64_t n) {
  std::lock_guard<std::mutex> g(mu_);
  if ((int64_t)(free_.size() + lru_.size()) < n) throw std::runtime_error("BlockAllocator: out of KV blocks");
  std::vector<int64_t> out;
  out.reserve(n);
  for (int64_t i = 0; i < n; ++i) out.push_back(take_one());
  return out;
}

void BlockAllocator::free(const std::vector<int64_t>& blocks) {
  std::lock_guard<std::mutex> g(mu_);
  for (int64_t b : blocks) {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("BlockAllocator::free: bad block id");
    if (ref_[b] <= 0) throw std::runtime_error("BlockAllocator::free: double free");
    if (--ref_[b] == 0) {
      if (prefix_caching_ && has_hash_[b]) {
        lru_.push_back(b);
        lru_pos_[b] = std::prev(lru_.end());
        in_lru_[b] = 1;
      } else {
        has_hash_[b] = 0;
        free_.push_back(b);
      }
    }
  }
}

void BlockAllocator::incref(const std::vector<int64_t>& blocks) {
  std::lock_guard<std::mutex> g(mu_);
  for (int64_t b : blocks) {
    if (b < 0 || b >= num_blocks_ || ref_[b] <= 0) throw std::runtime_error("BlockAllocator::incref: block not live");
    ++ref_[b];
  }
}

int64_t BlockAllocator::refcount(int64_t block) const {
  std::lock_guard<std::mutex> g(mu_);
  if (block < 0 || block >= num_blocks_) throw std::out_of_range("refcount: bad block id");
  return ref_[block];
}

int64_t BlockAllocator::lookup(uint64_t hash) {
  std::lock_guard<std::mutex> g(mu_);
  if (!prefix_caching_) return -1;
  ++queries_;
  auto it = hash_to_block_.find(hash);
  if (it == hash_to_block_.end()) return -1;
  const int64_t b = it->second;
  if (in_lru_[b]) {
    lru_.erase(lru_pos_[b]);
    in_lru_[b] = 0;
  }
  ++ref_[b];
  ++hits_;
  return b;
}

void BlockAllocator::register_hash(int64_t block, uint64_t hash) {
  std::lock_guard<std::mutex> g(mu_);
  if (!prefix_caching_) return;
  if (block < 0 || block >= num_blocks_) throw std::out_of_range("register_hash: bad block id");
  if (hash_to_block_.count(hash)) return;  // an identical block is already cached
  if (has_hash_[block]) hash_to_block_.erase(block_hash_[block]);
  block_hash_[block] = hash;
  has_hash_[block] = 1;
  hash_to_block_[hash] = block;
}

void BlockAllocator::reset_prefix_cache() {
  std::lock_guard<std::mutex> g(mu_);
  for (int64_t b : lru_) {
    in_lru_[b] = 0;
    has_hash_[b] = 0;
    free_.push_back(b);
  }
  lru_.clear();
  hash_to_block_.clear();
  for (int64_t b = 0; b < num_blocks_; ++b) has_hash_[b] = 0;
}

// FNV-1a over (parent, tokens) followed by a splitmix64 finaliser.
uint64_t BlockAllocator::hash_block(uint64_t parent, const std::vector<int64_t>& tokens) {
  uint64_t h = 1469598103934665603ull ^ parent;
  auto mix = [&](uint64_t v) {
    for (int i = 0; i < 8; ++i) {
      h ^= (v >> (8 * i)) & 0xff;
      h *= 1099511628211ull;
    }
  };
  mix(parent);
  for (int64_t t : tokens) mix((uint64_t)t);
  h += 0x9e3779b97f4a7c15ull;
  h = (h ^ (h >> 30)) * 0xbf58476d1ce4e5b9ull;
  h = (h ^ (h >> 27)) * 0x94d049bb133111ebull;
  return h ^ (h >> 31);
}

void bind_runtime(pybind11::module_& m) {
  namespace py = pybind11;
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int64_t, int64_t, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = false)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks)
      .def_property_readonly("block_size", &BlockAllocator::block_size)
      .def("num_free", &BlockAllocator::num_free)
      .def("num_cached", &BlockAllocator::num_cached)
      .def("can_allocate", &BlockAllocator::can_allocate)
      .def("allocate", &BlockAllocator::allocate)
      .def("free", &BlockAllocator::free)
      .def("incref", &BlockAllocator::incref)
      .def("refcount", &BlockAllocator::refcount)
      .def("lookup", &BlockAllocator::lookup)
      .def("register_hash", &BlockAllocator::register_hash)
      .def("reset_prefix_cache", &BlockAllocator::reset_prefix_cache)
      .def_property_readonly("hits", &BlockAllocator::hits)
      .def_property_readonly("queries", &BlockAllocator::queries)
      .def_static("hash_block", &BlockAllocator::hash_block);
}

}  // namespace vgate
