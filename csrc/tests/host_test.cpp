// Host-only test of the native runtime's C++ data structures, built with
// -fsanitize=address,undefined (and separately -fsanitize=thread) by
// tests/test_native_sanitizers.py — SURVEY.md §5.2: the reference has no sanitizers at all;
// GPU sanitizers are unavailable on this pool, so the host code is checked here.
//
// Covers: BlockAllocator (alloc/free/refcounts, prefix-cache register/lookup/eviction,
// concurrent stats queries while allocating), ShardedLRU (capacity / LRU order /
// overwrite / erase, and a multi-thread get/put hammer with an exact accounting check) and the
// lock-free shared-memory StepRing (one publisher thread, several follower threads: every payload
// byte checked, back-pressure on a ring smaller than the run, close, heartbeat timeout).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../runtime/allocator.h"
#include "../runtime/lru_cache.h"
#include "../runtime/step_ring.h"

#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

static void test_allocator() {
  using vgate::BlockAllocator;
  BlockAllocator a(64, 16, true);
  CHECK(a.num_free() == 64);
  auto b = a.allocate(10);
  CHECK(b.size() == 10 && a.num_free() == 54);
  a.incref({b[0], b[1]});
  CHECK(a.refcount(b[0]) == 2);
  a.free(b);
  CHECK(a.num_free() == 62 && a.refcount(b[0]) == 1);
  a.free({b[0], b[1]});
  CHECK(a.num_free() == 64);
  // prefix cache: register, free (-> evictable), look up again, then evict under pressure
  std::vector<int64_t> toks(16);
  for (int i = 0; i < 16; ++i) toks[i] = 100 + i;
  const uint64_t h = BlockAllocator::hash_block(0, toks);
  auto c = a.allocate(1);
  a.register_hash(c[0], h);
  a.free(c);
  CHECK(a.num_free() == 64 && a.num_cached() == 1);
  CHECK(a.lookup(h) == c[0]);
  a.free(c);
  auto all = a.allocate(64);  // takes every block: the cached one is evicted
  CHECK(all.size() == 64 && a.num_free() == 0);
  CHECK(a.lookup(h) == -1);
  a.free(all);
  // stats readers racing the engine thread
  std::atomic<bool> stop{false};
  std::thread reader([&] {
    int64_t s = 0;
    while (!stop.load()) s += a.num_free() + a.num_cached();
    (void)s;
  });
  for (int it = 0; it < 2000; ++it) {
    auto x = a.allocate(1 + it % 7);
    a.free(x);
  }
  stop = true;
  reader.join();
  CHECK(a.num_free() == 64);
}

static void test_lru_basic() {
  vgate::ShardedLRU c(4, 1);
  CHECK(c.num_shards() == 1);
  c.put("a", "1");
  c.put("b", "2");
  c.put("c", "3");
  c.put("d", "4");
  CHECK(c.get("a").value() == "1");  // a is now most recent
  CHECK(c.put("e", "5") == 1);       // evicts b
  CHECK(!c.get("b").has_value());
  CHECK(c.get("a") && c.get("c") && c.get("d") && c.get("e"));
  c.put("a", "one");  // overwrite keeps size
  CHECK(c.size() == 4 && c.get("a").value() == "one");
  CHECK(c.erase("a") && !c.erase("a") && c.size() == 3);
  c.clear();
  CHECK(c.size() == 0);
  vgate::ShardedLRU z(0, 8);
  CHECK(z.put("k", "v") == 0 && z.size() == 0);
  vgate::ShardedLRU s(3, 16);  // never more shards than entries
  CHECK(s.num_shards() <= 3);
}

static void test_lru_threads() {
  vgate::ShardedLRU c(512, 16);
  const int T = 8, N = 20000;
  std::atomic<uint64_t> gets{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < N; ++i) {
        const std::string k = "k" + std::to_string((i * 7 + t * 13) % 2048);
        if (i % 3 == 0) {
          c.put(k, std::string(32 + i % 64, 'x'));
        } else {
          auto v = c.get(k);
          if (v) CHECK(v->size() >= 32);
          gets.fetch_add(1);
        }
      }
    });
  for (auto& x : th) x.join();
  CHECK(c.size() <= 512);
  CHECK(c.hits() + c.misses() == gets.load());
}

static void test_step_ring() {
  using vgate::StepRingCore;
  const std::string name = "/vgate_host_test_" + std::to_string((long)getpid());
  const int steps = 3000, followers = 3;
  StepRingCore leader(name, true, /*slots=*/4, /*slot_bytes=*/4096, followers);
  std::vector<std::thread> ts;
  std::atomic<int> bad{0};
  for (int f = 0; f < followers; ++f) {
    ts.emplace_back([&, f] {
      StepRingCore me(name, false, 0, 0, 0);
      std::vector<unsigned char> buf(4096);
      for (int i = 1; i <= steps; ++i) {
        auto st = me.wait(f, buf.data(), buf.size(), 5.0);
        if (st.mode != i % 3 || st.T != i || st.nbytes != (i * 37) % 4096) {
          ++bad;
          return;
        }
        for (int64_t b = 0; b < st.nbytes; ++b)
          if (buf[b] != (unsigned char)(i + b)) {
            ++bad;
            return;
          }
      }
      auto end = me.wait(f, buf.data(), buf.size(), 5.0);
      if (end.mode != -1) ++bad;  // closed
    });
  }
  std::vector<unsigned char> payload(4096);
  for (int i = 1; i <= steps; ++i) {
    const int n = (i * 37) % 4096;
    for (int b = 0; b < n; ++b) payload[b] = (unsigned char)(i + b);
    CHECK(leader.publish(i, 0, 0, 0, i % 3, payload.data(), (size_t)n, 5.0));
  }
  leader.close_ring();
  for (auto& t : ts) t.join();
  CHECK(bad.load() == 0);
  CHECK(leader.published() == steps);
  // a follower of a ring whose leader stopped stamping its heartbeat gives up (mode -2)
  {
    const std::string n2 = name + "_hb";
    StepRingCore l2(n2, true, 2, 64, 1);
    StepRingCore f2(n2, false, 0, 0, 0);
    unsigned char b[64];
    auto st = f2.wait(0, b, sizeof(b), 0.05);
    CHECK(st.mode == -2);
  }
}

int main() {
  test_allocator();
  test_lru_basic();
  test_lru_threads();
  test_step_ring();
  std::printf("host_test: ok\n");
  return 0;
}
