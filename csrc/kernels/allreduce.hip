// Custom one-shot all-reduce over xGMI peer memory (tensor-parallel decode collectives).
//
// Why: a decode step of a TP-sharded model all-reduces [B, H] bf16 twice per layer
// (70B at TP=8, B=64: 1 MiB, 160x per step). Those messages are latency-bound; a ring
// (RCCL) pays 2(n-1) link hops of latency and uses one xGMI link per direction. On the
// MI355X node every GPU has a direct link to each of its 7 peers, so here every rank reads
// the other ranks' inputs directly over all 7 links at once and reduces locally: ONE
// synchronisation, no intermediate hops.
//
// Above 512 KiB (and > 2 ranks) the two-shot variant below moves 2 (n-1)/n of the message per
// rank (reduce-scatter + all-gather, two synchronisations) instead of the one-shot's n-1 copies.
//
// Memory (per rank, one hipExtMallocWithFlags(hipDeviceMallocUncached) allocation, shared
// with the peers through hipIpcGetMemHandle): [0, 64 KiB) signal area — flags[AR_BLOCKS]
// [AR_MAX_RANKS] u32 written BY PEERS, then epochs[AR_BLOCKS] u32 private to the owner —
// followed by two data buffers of max_bytes (call parity). Uncached memory keeps remote
// reads and flag polls coherent without cache maintenance.
//
// Protocol, per block b (blocks own the same contiguous slice on every rank):
//   e = ++epoch[b]; copy my input slice b -> my data[e & 1] slice b; fence (system);
//   store e into flags[b][me] of EVERY peer; wait until my flags[b][p] >= e for all p;
//   sum slice b of data[e & 1] over all peers (own slice from the input) -> out.
// Block b of peer p having arrived means p's slice b is in p's buffer. A peer can run at
// most one call ahead (its next arrival needs my next flag), and that call writes the
// other parity buffer, so no closing barrier is needed. Every wait is bounded
// (AR_SPIN_LIMIT polls): on timeout the block records an error word and exits, so the
// grid always drains; the host checks the word (custom_allreduce.py).
//
// hipGraph-capturable: all addresses are fixed kernel arguments, the epoch lives in
// device memory.
#include <cstddef>
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace vgate {

constexpr int AR_BLOCKS = 128;  // signal-area capacity; a launch uses ar_blocks() of them
constexpr int AR_MAX_RANKS = 8;
constexpr int AR_THREADS = 512;
constexpr unsigned AR_SPIN_LIMIT = 1u << 22;  // ~4M uncached polls: seconds, not minutes

struct ArSignal {
  uint32_t flags[AR_BLOCKS][AR_MAX_RANKS];
  uint32_t epoch[AR_BLOCKS];
  uint32_t error;
  // collective time accounting (metrics: vgate_engine_allreduce_seconds): block 0 of every call
  // adds its entry -> exit span in 100 MHz s_memrealtime ticks (wraps; the host takes deltas)
  // and bumps the call count; the step graph's last node copies both to the host with the ids
  uint32_t ticks;
  uint32_t calls;
  uint32_t pad[AR_BLOCKS - 3];
  uint32_t flags2[AR_BLOCKS][AR_MAX_RANKS];  // two-shot: "my reduced slice is in my buffer"
  uint32_t flags3[AR_BLOCKS][AR_MAX_RANKS];  // all-gather: "my input slice is in my buffer"
};
static_assert(sizeof(ArSignal) <= AR_SIGNAL_BYTES, "signal area");

struct ArPeers {
  char* base[AR_MAX_RANKS];  // every rank's mapped allocation (own one included)
};

// block 0, thread 0: the call's span (entry -> exit, peers' waits included) into the own signal area
struct ArClock {
  ArSignal* me;
  unsigned long long t0;
  __device__ __forceinline__ explicit ArClock(ArSignal* s) : me(s), t0(0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) t0 = __builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ ~ArClock() {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
      __hip_atomic_fetch_add(&me->ticks, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&me->calls, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
};

// blocks per call: VGATE_AR_BLOCKS (16..128, read once per process, so every rank of a group
// launched with the same environment agrees; benchmarks/allreduce_bench.py sweeps it), default 64
// polls before a wait gives up: VGATE_AR_SPIN_LIMIT (default AR_SPIN_LIMIT; tests shorten it to
// exercise the timeout path in milliseconds), read once per process
static uint32_t ar_spin_limit() {
  static const uint32_t n = [] {
    const char* e = getenv("VGATE_AR_SPIN_LIMIT");
    const long v = e ? atol(e) : (long)AR_SPIN_LIMIT;
    return (uint32_t)(v < 1000 ? 1000 : v);
  }();
  return n;
}

static int ar_blocks() {
  static const int n = [] {
    const char* e = getenv("VGATE_AR_BLOCKS");
    int v = e ? atoi(e) : 64;
    if (v < 8) v = 8;
    if (v > AR_BLOCKS) v = AR_BLOCKS;
    return v;
  }();
  return n;
}

// wait until every peer arrived at epoch e in `flags` (one lane per peer). A timed-out wait sets
// the sticky error word and gives up; once it is set, later calls do not wait at all (the group is
// one failure domain: the engine reads the word after the step and fails it), so a dead peer costs
// one spin limit, not one per collective of the step.
__device__ __forceinline__ void ar_wait_all(uint32_t (*flags)[AR_MAX_RANKS], int b, int world, uint32_t e,
                                            ArSignal* me, uint32_t spin_limit) {
  const int tid = threadIdx.x;
  if (tid < world && __hip_atomic_load(&me->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    unsigned spins = 0;
    while ((int32_t)(__hip_atomic_load(&flags[b][tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++spins > spin_limit) {
        __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(AR_THREADS) void ar_one_shot_kernel(const uint4* in, uint4* out,  // may alias
                                                               ArPeers peers, int rank, int world,
                                                               int64_t n16, int64_t max_bytes, uint32_t spin_limit) {
  const int b = blockIdx.x, tid = threadIdx.x, nblk = gridDim.x;
  ArSignal* me = reinterpret_cast<ArSignal*>(peers.base[rank]);
  const ArClock clk(me);
  __shared__ uint32_t s_epoch;
  if (tid == 0) s_epoch = me->epoch[b] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  const int64_t par_off = AR_SIGNAL_BYTES + (int64_t)(e & 1) * max_bytes;
  // this block's slice of 16-byte vectors
  const int64_t per = (n16 + nblk - 1) / nblk;
  const int64_t i0 = (int64_t)b * per, i1 = min(n16, i0 + per);
  uint4* mine = reinterpret_cast<uint4*>(peers.base[rank] + par_off);
  for (int64_t i = i0 + tid; i < i1; i += AR_THREADS) mine[i] = in[i];
  __threadfence_system();
  __syncthreads();
  // arrive at every peer, then wait for every peer's arrival
  if (tid < world) {
    ArSignal* peer = reinterpret_cast<ArSignal*>(peers.base[tid]);
    __hip_atomic_store(&peer->flags[b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  ar_wait_all(me->flags, b, world, e, me, spin_limit);
  // reduce slice b over the ranks (fp32 accumulation, fixed rank order on every rank)
  // every peer's vector is loaded before the first is summed (a runtime-trip loop would wait
  // one xGMI round trip per peer); slots past `world` re-read rank 0 and are masked
  for (int64_t i = i0 + tid; i < i1; i += AR_THREADS) {
    uint4 v[AR_MAX_RANKS];
#pragma unroll
    for (int p = 0; p < AR_MAX_RANKS; ++p) {
      const int q = p < world ? p : 0;
      v[p] = q == rank ? in[i] : ld_nt16(reinterpret_cast<const uint4*>(peers.base[q] + par_off) + i);
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < AR_MAX_RANKS; ++p) {
      if (p < world) {
        float f[8];
        unpack8(v[p], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
    }
    out[i] = pack8(acc);
  }
  if (tid == 0) me->epoch[b] = e;
}

// Two-shot all-reduce for the 0.5-8 MiB range (TP prefill chunks, 70B decode at large batch):
// reduce-scatter then all-gather, each rank moving 2 (n-1)/n of the message over its n-1
// direct xGMI links instead of the one-shot's (n-1) full copies. Block b owns sub-range b of
// every rank's slice (slice r = elements [r n/w, (r+1) n/w)):
//   1. copy my input's sub-ranges b into my buffer (parity e & 1); arrive (flags) at every peer;
//   2. wait for every peer's arrival; sum sub-range b of MY slice over all peers' buffers (fixed
//      rank order: bit-identical on every rank); write it to out and back into my buffer;
//   3. arrive (flags2) at every peer; wait for theirs; copy sub-range b of every OTHER slice
//      from its owner's buffer into out.
// Safety of the parity buffers is the one-shot's argument: a peer cannot pass phase 1 of call
// e+1 (writing the other parity) before I arrive there, i.e. before I finished reading call e.
__global__ __launch_bounds__(AR_THREADS) void ar_two_shot_kernel(const uint4* in, uint4* out, ArPeers peers,
                                                               int rank, int world, int64_t n16, int64_t max_bytes,
                                                               uint32_t spin_limit) {
  const int b = blockIdx.x, tid = threadIdx.x, nblk = gridDim.x;
  ArSignal* me = reinterpret_cast<ArSignal*>(peers.base[rank]);
  const ArClock clk(me);
  __shared__ uint32_t s_epoch;
  if (tid == 0) s_epoch = me->epoch[b] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  const int64_t par_off = AR_SIGNAL_BYTES + (int64_t)(e & 1) * max_bytes;
  auto slice = [&](int r, int64_t& a, int64_t& z) {  // sub-range b of rank r's slice
    const int64_t s0 = n16 * r / world, s1 = n16 * (r + 1) / world;
    const int64_t per = (s1 - s0 + nblk - 1) / nblk;
    a = min(s1, s0 + (int64_t)b * per);
    z = min(s1, a + per);
  };
  uint4* mine = reinterpret_cast<uint4*>(peers.base[rank] + par_off);
  for (int r = 0; r < world; ++r) {
    int64_t a, z;
    slice(r, a, z);
    for (int64_t i = a + tid; i < z; i += AR_THREADS) mine[i] = in[i];
  }
  __threadfence_system();
  __syncthreads();
  if (tid < world) {
    ArSignal* peer = reinterpret_cast<ArSignal*>(peers.base[tid]);
    __hip_atomic_store(&peer->flags[b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  ar_wait_all(me->flags, b, world, e, me, spin_limit);
  {
    int64_t a, z;
    slice(rank, a, z);
    for (int64_t i = a + tid; i < z; i += AR_THREADS) {
      uint4 v[AR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < AR_MAX_RANKS; ++p) {
        const int q = p < world ? p : 0;
        v[p] = q == rank ? mine[i] : ld_nt16(reinterpret_cast<const uint4*>(peers.base[q] + par_off) + i);
      }
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < AR_MAX_RANKS; ++p) {
        if (p < world) {
          float f[8];
          unpack8(v[p], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += f[j];
        }
      }
      const uint4 r4 = pack8(acc);
      mine[i] = r4;
      out[i] = r4;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (tid < world) {
    ArSignal* peer = reinterpret_cast<ArSignal*>(peers.base[tid]);
    __hip_atomic_store(&peer->flags2[b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  ar_wait_all(me->flags2, b, world, e, me, spin_limit);
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    int64_t a, z;
    slice(r, a, z);
    const uint4* src = reinterpret_cast<const uint4*>(peers.base[r] + par_off);
    for (int64_t i = a + tid; i < z; i += AR_THREADS) out[i] = ld_nt16(src + i);
  }
  if (tid == 0) me->epoch[b] = e;
}

// All-gather over the same peer buffers (the vocab-sharded logits of a TP decode step, C2):
// every rank copies its input into its buffer (block b: slice b), arrives at every peer, waits
// for every peer, then reads slice b of every rank's input into out[rank-major]. Same epoch /
// parity / bounded-wait protocol as the all-reduces, so the three kinds interleave freely and
// the call is captured into the TP decode hipGraphs (a gloo or RCCL all-gather is not needed).
__global__ __launch_bounds__(AR_THREADS) void ar_all_gather_kernel(const uint4* in, uint4* out, ArPeers peers,
                                                                 int rank, int world, int64_t n16, int64_t max_bytes,
                                                                 uint32_t spin_limit) {
  const int b = blockIdx.x, tid = threadIdx.x, nblk = gridDim.x;
  ArSignal* me = reinterpret_cast<ArSignal*>(peers.base[rank]);
  const ArClock clk(me);
  __shared__ uint32_t s_epoch;
  if (tid == 0) s_epoch = me->epoch[b] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  const int64_t par_off = AR_SIGNAL_BYTES + (int64_t)(e & 1) * max_bytes;
  const int64_t per = (n16 + nblk - 1) / nblk;
  const int64_t i0 = min(n16, (int64_t)b * per), i1 = min(n16, i0 + per);
  uint4* mine = reinterpret_cast<uint4*>(peers.base[rank] + par_off);
  for (int64_t i = i0 + tid; i < i1; i += AR_THREADS) mine[i] = in[i];
  __threadfence_system();
  __syncthreads();
  if (tid < world) {
    ArSignal* peer = reinterpret_cast<ArSignal*>(peers.base[tid]);
    __hip_atomic_store(&peer->flags3[b][rank], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  ar_wait_all(me->flags3, b, world, e, me, spin_limit);
  for (int p = 0; p < world; ++p) {
    const uint4* src = p == rank ? in : reinterpret_cast<const uint4*>(peers.base[p] + par_off);
    for (int64_t i = i0 + tid; i < i1; i += AR_THREADS) out[(int64_t)p * n16 + i] = p == rank ? src[i] : ld_nt16(src + i);
  }
  if (tid == 0) me->epoch[b] = e;
}

int64_t ar_error_offset() { return (int64_t)offsetof(ArSignal, error); }
uint32_t ar_spin() { return ar_spin_limit(); }
int64_t ar_blocks_used() { return ar_blocks(); }
static_assert(offsetof(ArSignal, ticks) == offsetof(ArSignal, error) + 4 && offsetof(ArSignal, calls) == offsetof(ArSignal, error) + 8,
              "ids_to_host copies {error, ticks, calls} as consecutive words");

void launch_custom_allgather(const void* in, void* out, int64_t nbytes, char* const* bases, int rank, int world,
                             int64_t max_bytes, hipStream_t st) {
  ArPeers peers{};
  for (int p = 0; p < world && p < AR_MAX_RANKS; ++p) peers.base[p] = bases[p];
  hipLaunchKernelGGL(ar_all_gather_kernel, dim3(ar_blocks()), dim3(AR_THREADS), 0, st,
                     reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), peers, rank, world,
                     nbytes / 16, max_bytes, ar_spin_limit());
}

void launch_custom_allreduce(const void* in, void* out, int64_t nbytes, char* const* bases, int rank, int world,
                             int64_t max_bytes, hipStream_t st, int two_shot) {
  ArPeers peers{};
  for (int p = 0; p < world && p < AR_MAX_RANKS; ++p) peers.base[p] = bases[p];
  // one-shot up to 512 KiB (one synchronisation, latency-bound messages), two-shot above
  // (bandwidth: 2 (n-1)/n of the message per rank instead of n-1 copies); two_shot < 0 forces
  // one-shot, > 0 forces two-shot (tests)
  const bool two = two_shot > 0 || (two_shot == 0 && world > 2 && nbytes > (512 << 10));
  if (two)
    hipLaunchKernelGGL(ar_two_shot_kernel, dim3(ar_blocks()), dim3(AR_THREADS), 0, st,
                       reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), peers, rank, world,
                       nbytes / 16, max_bytes, ar_spin_limit());
  else
    hipLaunchKernelGGL(ar_one_shot_kernel, dim3(ar_blocks()), dim3(AR_THREADS), 0, st,
                       reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), peers, rank, world,
                       nbytes / 16, max_bytes, ar_spin_limit());
}

}  // namespace vgate
