// Host shared-memory ring that carries each engine step's plan from TP rank 0 to its follower
// ranks: one POSIX shm segment per TP group, rank 0 the only writer.
//
// Why not a collective: a per-step RCCL broadcast of the metadata costs a device round trip and
// the followers a host sync on the header (engine.py round 1); the plan is host data that rank 0
// already holds, and the TP ranks of an MI355X node share the host. Here rank 0 memcpy's the
// used prefix of its pinned step-metadata buffer into the next slot and release-stores the step
// number; a follower acquire-loads it, copies the slot into ITS pinned buffer and replays the
// same hipGraph — no Python objects, no collective, no device sync on the hot path.
//
// Layout: [Header (one cache line per field)] [slots x (SlotHeader + payload)].
// Back-pressure: rank 0 never runs more than `slots` steps ahead of the slowest follower
// (per-follower ack words). Liveness: rank 0 stamps a heartbeat (steady clock, ns) on every
// publish and from its idle loop; a follower whose wait sees no new step AND a stale heartbeat
// gives up (returns a timeout) instead of spinning forever on a dead leader.
#pragma once
// Torch-free core (tested under ASan / TSan by csrc/tests/host_test.cpp); step_ring.cpp binds it.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace vgate {

namespace ring_detail {

constexpr int kMaxFollowers = 15;
constexpr uint64_t kMagic = 0x76676174655f7231ull;  // "vgate_r1"

struct alignas(64) Line64 {
  std::atomic<uint64_t> v;
  char pad[56];
};

struct RingHeader {
  uint64_t magic;
  uint32_t slots, slot_bytes, followers, pad0;
  char pad[40];
  Line64 seq;                     // last published step (0 = none)
  Line64 heartbeat_ns;            // leader liveness stamp
  Line64 closed;                  // 1 = leader shut down
  Line64 ack[kMaxFollowers];      // last step consumed by each follower
};

struct SlotHeader {
  uint64_t seq;
  int32_t T, S, ns, nt, mode, pad;
  uint64_t nbytes;
};

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// spin briefly (a decode step arrives every few ms), then back off with sleeps
void backoff(uint64_t& spins) {
  ++spins;
  if (spins < 2000) return;
  if (spins < 4000) {
    std::this_thread::yield();
    return;
  }
  struct timespec ts{0, spins < 20000 ? 20000 : 200000};  // 20 us, then 200 us
  nanosleep(&ts, nullptr);
}

}  // namespace ring_detail
using namespace ring_detail;

class StepRingCore {
 public:
  // create=true: the leader (TP rank 0) creates (and later unlinks) the segment
  StepRingCore(const std::string& name, bool create, int64_t slots, int64_t slot_bytes, int64_t followers)
      : name_(name), owner_(create) {
    if (create) {
      if (slots < 2 || slot_bytes < 64 || followers < 1 || followers > kMaxFollowers)
        throw std::invalid_argument("StepRing: slots >= 2, slot_bytes >= 64, 1..15 followers");
      shm_unlink(name.c_str());
      fd_ = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("StepRing: shm_open(create) failed for " + name);
      stride_ = (sizeof(SlotHeader) + (size_t)slot_bytes + 63) / 64 * 64;
      bytes_ = sizeof(RingHeader) + stride_ * (size_t)slots;
      if (ftruncate(fd_, (off_t)bytes_) != 0) throw std::runtime_error("StepRing: ftruncate failed");
      map();
      std::memset(base_, 0, sizeof(RingHeader));
      hdr_->slots = (uint32_t)slots;
      hdr_->slot_bytes = (uint32_t)slot_bytes;
      hdr_->followers = (uint32_t)followers;
      hdr_->heartbeat_ns.v.store(now_ns(), std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = kMagic;
    } else {
      fd_ = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd_ < 0) throw std::runtime_error("StepRing: shm_open(attach) failed for " + name);
      struct stat st;
      if (fstat(fd_, &st) != 0 || (size_t)st.st_size < sizeof(RingHeader))
        throw std::runtime_error("StepRing: segment too small");
      bytes_ = (size_t)st.st_size;
      map();
      if (hdr_->magic != kMagic) throw std::runtime_error("StepRing: not initialised");
      stride_ = (sizeof(SlotHeader) + (size_t)hdr_->slot_bytes + 63) / 64 * 64;
    }
  }

  ~StepRingCore() {
    if (base_ != nullptr) munmap(base_, bytes_);
    if (fd_ >= 0) close(fd_);
    if (owner_) shm_unlink(name_.c_str());
  }

  // Leader: publish one step. Waits while the ring is full; returns false if a follower made no
  // progress within timeout_s (the group is broken). The caller releases the GIL around it.
  bool publish(int64_t T, int64_t S, int64_t ns, int64_t nt, int64_t mode, const void* data, size_t nbytes,
               double timeout_s) {
    if (nbytes > hdr_->slot_bytes) throw std::invalid_argument("StepRing.publish: payload larger than a slot");
    const uint64_t next = hdr_->seq.v.load(std::memory_order_relaxed) + 1;
    {
      const uint64_t t0 = now_ns();
      uint64_t spins = 0;
      while (next - min_ack() > hdr_->slots) {  // slot `next % slots` still unread by someone
        hdr_->heartbeat_ns.v.store(now_ns(), std::memory_order_relaxed);
        if (timeout_s > 0 && (double)(now_ns() - t0) * 1e-9 > timeout_s) return false;
        backoff(spins);
      }
    }
    char* slot = slot_ptr(next);
    SlotHeader sh{next, (int32_t)T, (int32_t)S, (int32_t)ns, (int32_t)nt, (int32_t)mode, 0, (uint64_t)nbytes};
    std::memcpy(slot, &sh, sizeof(sh));
    if (nbytes > 0) std::memcpy(slot + sizeof(SlotHeader), data, nbytes);
    hdr_->heartbeat_ns.v.store(now_ns(), std::memory_order_relaxed);
    hdr_->seq.v.store(next, std::memory_order_release);
    return true;
  }

  // Follower `f`: wait for the step after the last one it consumed, copy its payload into `out`
  // (capacity `cap` bytes). Returns the slot header; mode = -1: the leader closed the ring; -2:
  // timeout (no new step and the leader's heartbeat older than timeout_s).
  struct Step {
    int32_t T, S, ns, nt, mode;
    int64_t nbytes;
  };
  Step wait(int64_t f, void* out, size_t cap, double timeout_s) {
    if (f < 0 || f >= (int64_t)hdr_->followers) throw std::invalid_argument("StepRing.wait: follower index");
    const uint64_t want = hdr_->ack[f].v.load(std::memory_order_relaxed) + 1;
    SlotHeader sh{};
    int mode = 0;
    uint64_t spins = 0;
    for (;;) {
      if (hdr_->seq.v.load(std::memory_order_acquire) >= want) break;
      if (hdr_->closed.v.load(std::memory_order_acquire)) {
        mode = -1;
        break;
      }
      if (timeout_s > 0 && spins % 64 == 0) {
        const uint64_t hb = hdr_->heartbeat_ns.v.load(std::memory_order_relaxed);
        const uint64_t t = now_ns();
        if (t > hb && (double)(t - hb) * 1e-9 > timeout_s) {
          mode = -2;
          break;
        }
      }
      backoff(spins);
    }
    if (mode != 0) return Step{0, 0, 0, 0, mode, 0};
    const char* slot = slot_ptr(want);
    std::memcpy(&sh, slot, sizeof(sh));
    if (sh.seq != want) throw std::runtime_error("StepRing: slot overwritten before it was read");
    if (sh.nbytes > cap) throw std::runtime_error("StepRing: payload larger than buffer");
    if (sh.nbytes > 0) std::memcpy(out, slot + sizeof(SlotHeader), sh.nbytes);
    hdr_->ack[f].v.store(want, std::memory_order_release);
    return Step{sh.T, sh.S, sh.ns, sh.nt, sh.mode, (int64_t)sh.nbytes};
  }

  void heartbeat() { hdr_->heartbeat_ns.v.store(now_ns(), std::memory_order_relaxed); }
  // drop the segment's name once every follower has mapped it: the mappings stay valid and no
  // /dev/shm entry outlives the group, however its processes end
  void unlink() {
    if (owner_) {
      shm_unlink(name_.c_str());
      owner_ = false;
    }
  }
  void close_ring() { hdr_->closed.v.store(1, std::memory_order_release); }
  int64_t published() const { return (int64_t)hdr_->seq.v.load(std::memory_order_acquire); }
  int64_t acked(int64_t f) const { return (int64_t)hdr_->ack[f].v.load(std::memory_order_acquire); }
  int64_t slots() const { return hdr_->slots; }
  int64_t slot_bytes() const { return hdr_->slot_bytes; }
  const std::string& name() const { return name_; }

 private:
  void map() {
    base_ = static_cast<char*>(mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0));
    if (base_ == MAP_FAILED) {
      base_ = nullptr;
      throw std::runtime_error("StepRing: mmap failed");
    }
    hdr_ = reinterpret_cast<RingHeader*>(base_);
  }
  uint64_t min_ack() const {
    uint64_t m = UINT64_MAX;
    for (uint32_t i = 0; i < hdr_->followers; ++i) {
      const uint64_t a = hdr_->ack[i].v.load(std::memory_order_acquire);
      m = a < m ? a : m;
    }
    return m;
  }
  char* slot_ptr(uint64_t seq) const {
    return base_ + sizeof(RingHeader) + stride_ * (size_t)(seq % hdr_->slots);
  }

  std::string name_;
  bool owner_;
  int fd_ = -1;
  char* base_ = nullptr;
  RingHeader* hdr_ = nullptr;
  size_t bytes_ = 0, stride_ = 0;
};

}  // namespace vgate
