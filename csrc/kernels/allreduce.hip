// Custom one-shot all-reduce over xGMI peer memory (tensor-parallel decode collectives).
//
// Why: a decode step of a TP-sharded model all-reduces [B, H] bf16 twice per layer
// (70B at TP=8, B=64: 1 MiB, 160x per step). Those messages are latency-bound; a ring
// (RCCL) pays 2(n-1) link hops of latency and uses one xGMI link per direction. On the
// MI355X node every GPU has a direct link to each of its 7 peers, so here every rank reads
// the other ranks' inputs directly over all 7 links at once and reduces locally: ONE
// synchronisation, no intermediate hops.
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
#include "common.h"
#include "launchers.h"

namespace vgate {

constexpr int AR_BLOCKS = 64;
constexpr int AR_MAX_RANKS = 8;
constexpr int AR_THREADS = 512;
constexpr unsigned AR_SPIN_LIMIT = 1u << 22;  // ~4M uncached polls: seconds, not minutes

struct ArSignal {
  uint32_t flags[AR_BLOCKS][AR_MAX_RANKS];
  uint32_t epoch[AR_BLOCKS];
  uint32_t error;
};
static_assert(sizeof(ArSignal) <= AR_SIGNAL_BYTES, "signal area");

struct ArPeers {
  char* base[AR_MAX_RANKS];  // every rank's mapped allocation (own one included)
};

__global__ __launch_bounds__(AR_THREADS) void ar_one_shot_kernel(const uint4* in, uint4* out,  // may alias
                                                               ArPeers peers, int rank, int world,
                                                               int64_t n16, int64_t max_bytes) {
  const int b = blockIdx.x, tid = threadIdx.x;
  ArSignal* me = reinterpret_cast<ArSignal*>(peers.base[rank]);
  __shared__ uint32_t s_epoch;
  if (tid == 0) s_epoch = me->epoch[b] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  const int64_t par_off = AR_SIGNAL_BYTES + (int64_t)(e & 1) * max_bytes;
  // this block's slice of 16-byte vectors
  const int64_t per = (n16 + AR_BLOCKS - 1) / AR_BLOCKS;
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
  if (tid < world) {
    unsigned spins = 0;
    while ((int32_t)(__hip_atomic_load(&me->flags[b][tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (++spins > AR_SPIN_LIMIT) {
        __hip_atomic_store(&me->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // reduce slice b over the ranks (fp32 accumulation, fixed rank order on every rank)
  for (int64_t i = i0 + tid; i < i1; i += AR_THREADS) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      const uint4 v = p == rank ? in[i] : ld_nt16(reinterpret_cast<const uint4*>(peers.base[p] + par_off) + i);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    out[i] = pack8(acc);
  }
  if (tid == 0) me->epoch[b] = e;
}

void launch_custom_allreduce(const void* in, void* out, int64_t nbytes, char* const* bases, int rank, int world,
                             int64_t max_bytes, hipStream_t st) {
  ArPeers peers{};
  for (int p = 0; p < world && p < AR_MAX_RANKS; ++p) peers.base[p] = bases[p];
  hipLaunchKernelGGL(ar_one_shot_kernel, dim3(AR_BLOCKS), dim3(AR_THREADS), 0, st,
                     reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), peers, rank, world,
                     nbytes / 16, max_bytes);
}

}  // namespace vgate
