// Per-row token sampling over the full vocabulary (V ~ 128k-152k) on gfx950:
// temperature -> top-k -> top-p -> categorical, or argmax when temperature == 0.
//
// Exact top-k/top-p WITHOUT sorting or histogram atomics (rejection sampling):
//   1. one pass: running max m and Z = sum exp((x - m)/T)
//   2. draw token j by inverse CDF over {i : x_i > pivot} (thread-major order:
//      any fixed order is a valid CDF order, so every load stays coalesced)
//   3. one pass: c = #{x_i > x_j}, q = sum_{x_i > x_j} e_i
//      accept j iff c < top_k and q < top_p * Z (j is inside both prefix sets);
//      otherwise every token <= x_j is outside the nucleus too: pivot = x_j,
//      the remaining mass is exactly q, repeat.
// Accepted samples are distributed exactly as the renormalised filtered
// distribution. Typical cost: 3-5 L2-resident passes over the row.
// RNG: Philox4x32-10 keyed by the per-row seed, countered by (offset, round).
#include "common.h"
#include "launchers.h"

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

__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t offset, uint32_t round) {
  uint32_t c[4] = {(uint32_t)offset, (uint32_t)(offset >> 32), round, 0x9E3779B9u};
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k);
    k[0] += 0x9E3779B9u;
    k[1] += 0xBB67AE85u;
  }
  return (float)(c[0] >> 8) * (1.0f / 16777216.0f);
}

constexpr int SAMPLE_THREADS = 1024;
constexpr float LOG2E_S = 1.4426950408889634f;

// Block-wide exclusive scan of one float per thread (1024 threads, 16 waves).
__device__ __forceinline__ float block_excl_scan(float v, float* sw, float& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  __syncthreads();
  if (lane == 63) sw[wid] = inc;
  __syncthreads();
  float base = 0.f;
  total = 0.f;
  const int nw = blockDim.x >> 6;
  for (int w = 0; w < nw; ++w) {
    const float t = sw[w];
    if (w < wid) base += t;
    total += t;
  }
  return base + inc - v;
}

// Row sweep helper: every thread visits float4 vectors v = tid + k*nt (k ascending),
// U vectors in flight per iteration (latency hiding: a 1024-thread block on one CU
// needs many bytes in flight to stream a 600 KB row at L2/HBM rate).
#define ROW_SWEEP(BODY)                                                        \
  for (int v0 = tid; v0 < V4; v0 += nt * 8) {                                  \
    float4 q_[8];                                                              \
    /* clamped, unconditional loads: no per-element branch/vmcnt(0) (guide §5 trap c) */ \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_) {                         \
      const int vi_ = v0 + u_ * nt;                                            \
      q_[u_] = x4[vi_ < V4 ? vi_ : V4 - 1];                                    \
    }                                                                          \
    _Pragma("unroll") for (int u_ = 0; u_ < 8; ++u_) {                         \
      const int vi_ = v0 + u_ * nt;                                            \
      const bool ok_ = vi_ < V4;                                               \
      const float e_[4] = {q_[u_].x, q_[u_].y, q_[u_].z, q_[u_].w};            \
      _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_) {                       \
        const float v = ok_ ? e_[j_] : -INFINITY;                              \
        const int i = 4 * vi_ + j_;                                            \
        (void)i;                                                               \
        BODY                                                                   \
      }                                                                        \
    }                                                                          \
  }

__global__ __launch_bounds__(SAMPLE_THREADS) void sample_kernel(SampleArgs a) {
  __shared__ float red[64];
  __shared__ int ridx[16];
  __shared__ float sw[16];
  __shared__ int sel;
  const int row = blockIdx.x;
  const int V4 = a.V >> 2;  // host guarantees V % 4 == 0 and 16-B aligned rows
  const float* x = a.logits + (size_t)row * a.ldl;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  const float T = a.temperature ? a.temperature[row] : 0.f;
  const bool greedy = !(T > 1e-5f);
  const float c = greedy ? LOG2E_S : LOG2E_S / T;

  // ---- pass 1: online (max, argmax, Z) in one sweep ----
  float mx = -INFINITY, z = 0.f;
  int amx = 0x7fffffff;
  ROW_SWEEP({
    if (v > mx) {
      z = (mx == -INFINITY ? 0.f : z * exp2f((mx - v) * c)) + 1.f;
      mx = v;
      amx = i;
    } else if (v > -INFINITY) {
      z += exp2f((v - mx) * c);
    }
  })
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const float oz = __shfl_xor(z, o, 64);
    const int oi = __shfl_xor(amx, o, 64);
    const float nm = fmaxf(mx, om);
    const float zz = (mx == -INFINITY ? 0.f : z * exp2f((mx - nm) * c)) +
                     (om == -INFINITY ? 0.f : oz * exp2f((om - nm) * c));
    if (om > mx || (om == mx && oi < amx)) amx = oi;
    mx = nm;
    z = zz;
  }
  if (lane == 0) { red[wid] = mx; red[16 + wid] = z; ridx[wid] = amx; }
  __syncthreads();
  if (tid == 0) {
    float bm = red[0], bz = red[16];
    int bi = ridx[0];
    for (int w = 1; w < nw; ++w) {
      const float om = red[w], oz = red[16 + w];
      const float nm = fmaxf(bm, om);
      bz = (bm == -INFINITY ? 0.f : bz * exp2f((bm - nm) * c)) + (om == -INFINITY ? 0.f : oz * exp2f((om - nm) * c));
      if (om > bm || (om == bm && ridx[w] < bi)) bi = ridx[w];
      bm = nm;
    }
    red[32] = bm;
    red[33] = bz;
    sel = bi;
  }
  __syncthreads();
  mx = red[32];
  z = red[33];
  amx = sel;
  __syncthreads();

  int chosen = amx;
  if (!greedy) {
    const int topk = a.top_k ? a.top_k[row] : -1;
    const float topp = a.top_p ? a.top_p[row] : 1.f;
    const bool use_k = topk > 0 && topk < a.V;
    const bool use_p = topp < 1.f;
    const float pmass = topp * z;
    const uint64_t seed = a.seeds ? a.seeds[row] : 0ull;
    const uint64_t off = a.offsets ? (uint64_t)a.offsets[row] : 0ull;
    float pivot = -INFINITY;
    chosen = -1;
    for (int round = 0; round < 64; ++round) {
      const float u = philox_uniform(seed, off, (uint32_t)round);
      float ls = 0.f;
      ROW_SWEEP({ if (v > pivot) ls += exp2f((v - mx) * c); })
      float total;
      const float excl = block_excl_scan(ls, sw, total);
      const float target = u * total;
      if (tid == 0) sel = -1;
      __syncthreads();
      const bool own = (ls > 0.f) && (target >= excl) && (target < excl + ls || excl + ls >= total);
      if (own) {
        float run = excl;
        int pick = -1, last = -1;
        for (int vi = tid; vi < V4 && pick < 0; vi += nt) {
          const float4 q = x4[vi];
          const float e[4] = {q.x, q.y, q.z, q.w};
          for (int j = 0; j < 4; ++j) {
            if (e[j] > pivot) {
              last = 4 * vi + j;
              run += exp2f((e[j] - mx) * c);
              if (run > target) { pick = 4 * vi + j; break; }
            }
          }
        }
        if (pick < 0) pick = last;
        atomicMax(&sel, pick);
      }
      __syncthreads();
      const int j = sel;
      __syncthreads();
      if (j < 0) break;
      if (!use_k && !use_p) { chosen = j; break; }
      const float xj = x[j];
      float cnt = 0.f, q = 0.f;
      ROW_SWEEP({ if (v > xj) { cnt += 1.f; q += exp2f((v - mx) * c); } })
      cnt = block_reduce_sum(cnt, red);
      q = block_reduce_sum(q, red);
      const bool ok_k = !use_k || cnt < (float)topk;
      const bool ok_p = !use_p || q < pmass;
      if (ok_k && ok_p) { chosen = j; break; }
      pivot = xj;
    }
    if (chosen < 0) chosen = amx;
  }
  if (tid == 0) {
    a.out[row] = chosen;
    if (a.out_logprob) a.out_logprob[row] = ((x[chosen] - mx) * c - log2f(z)) / LOG2E_S;
  }
}

void launch_sample(const SampleArgs& s, hipStream_t st) {
  if (s.B <= 0) return;
  hipLaunchKernelGGL(sample_kernel, dim3(s.B), dim3(SAMPLE_THREADS), 0, st, s);
}

}  // namespace vgate
