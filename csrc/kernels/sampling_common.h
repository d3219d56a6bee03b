// Sampling math of the sampler (sampling.hip): Philox4x32-10 uniforms, the (max, Z, argmax,
// Gumbel key) accumulator and its merges.
#pragma once
#include "common.h"

namespace vgate {

__device__ __forceinline__ void philox_round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c[0] = hi1 ^ c[1] ^ k[0];
  c[1] = lo1;
  c[2] = hi0 ^ c[3] ^ k[1];
  c[3] = lo0;
}

// Four uniforms in (0, 1) for counter (i4, offset, round).
__device__ __forceinline__ void philox4(uint64_t seed, uint64_t offset, uint32_t i4, uint32_t round,
                                        float (&u)[4]) {
  uint32_t c[4] = {i4, (uint32_t)offset, round, (uint32_t)(offset >> 32) ^ 0x9E3779B9u};
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k);
    k[0] += 0x9E3779B9u;
    k[1] += 0xBB67AE85u;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = ((float)(c[j] >> 9) + 0.5f) * (1.0f / 8388608.0f);  // (0,1): 1-2^-24 max is exact
}

constexpr int SAMPLE_THREADS = 256;
// B * NSEG bound: one block per CU, all co-resident (more segments per row measured slower:
// nseg 16 / 32 / 64 / 128 -> 38.7 / 35.2 / 55.8 / 143 us for 8 rows at top-p 0.9,
// profiles/r2_sampler_nseg_sweep.log)
constexpr int SAMPLE_MAX_BLOCKS = 256;
constexpr int SAMPLE_MAX_ROUNDS = 60;  // rejection rounds before the row keeps its last candidate / argmax
constexpr float LOG2E_S = 1.4426950408889634f;

struct Acc {  // POD (lives in LDS too); start from acc_init()
  float mx, z;
  int amx;
  float gk;
  int gi;
  float cnt, q;
};

__device__ __forceinline__ Acc acc_init() { return Acc{-INFINITY, 0.f, 0x7fffffff, -INFINITY, -1, 0.f, 0.f}; }

__device__ __forceinline__ void merge_mz(float& mx, float& z, int& amx, float om, float oz, int oi, float c) {
  const float nm = fmaxf(mx, om);
  const float zz = (mx == -INFINITY ? 0.f : z * exp2f((mx - nm) * c)) + (om == -INFINITY ? 0.f : oz * exp2f((om - nm) * c));
  if (om > mx || (om == mx && oi < amx)) amx = oi;
  mx = nm;
  z = zz;
}

__device__ __forceinline__ void merge_g(float& gk, int& gi, float ok, int oi) {
  if (oi >= 0 && (ok > gk || (ok == gk && (gi < 0 || oi < gi)))) {
    gk = ok;
    gi = oi;
  }
}

}  // namespace vgate
