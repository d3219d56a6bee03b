// Per-row token sampling over the full vocabulary (V ~ 128k-152k) on gfx950:
// temperature -> top-k -> top-p -> categorical, or argmax when temperature == 0.
//
// Parallel layout: each row is split into NSEG segments, one 256-thread block per
// (segment, row), so a batch-8 step spreads its 8 x 600 KB of logits over 256 CUs
// instead of 8. After each pass the blocks of a row exchange tagged partials (sample_gran_kernel:
// NSEG is chosen on the host so that B * NSEG <= 256 blocks, all co-resident, and every wait has a
// give-up bound). With NSEG == 1 (large batches) a row is one block (sample_row_kernel).
//
// Exact sampling, no sort, no histogram atomics:
//   pass 0: per segment (max, Z = sum e^{(x-max)/T}, argmax) and the Gumbel-max draw
//           argmax_i (x_i / T + G_i) — an exact sample of the tempered distribution.
//   Without top-k/top-p the Gumbel winner is the answer (one pass).
//   With them, rejection on the pivot: candidate j is accepted iff
//     #{x_i > x_j} < top_k  and  sum_{x_i > x_j} e_i < top_p * Z
//   (j is inside both prefix sets). Every pass computes those two counts for the
//   current candidate AND, speculatively, the next candidate = Gumbel-max restricted
//   to {x_i > x_j} with fresh noise (if j is rejected, every token <= x_j is outside
//   the nucleus too). So each rejection round costs one parallel pass; accepted
//   samples are distributed exactly as the renormalised filtered distribution.
// RNG: Philox4x32-10 keyed by the per-row seed, counter (float4 index, offset, round),
// so results are reproducible for a given (seed, offset) and independent of NSEG.
// Merges read the segments' partials in a fixed order: bit-reproducible.
#include <algorithm>
#include <cstdlib>

#include "launchers.h"
#include "sampling_common.h"

namespace vgate {

// Lane exchange on the VALU (no LDS round trip per step, unlike __shfl_xor's ds_bpermute): DPP
// quad permutes for partners 1 and 2, row rotations by 4 and 8 (after the quad steps every lane of
// a quad holds the quad's merge, so rotations complete the 16-lane row), permlane swaps for 16 / 32.
template <int K>
__device__ __forceinline__ uint32_t lane_x(uint32_t v) {
  if constexpr (K == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  else if constexpr (K == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
  else if constexpr (K == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
  else if constexpr (K == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  else if constexpr (K == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? r[0] : r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? r[0] : r[1];
  }
}
template <int K>
__device__ __forceinline__ void acc_step(Acc& a, float c) {
  const float om = __uint_as_float(lane_x<K>(__float_as_uint(a.mx)));
  const float oz = __uint_as_float(lane_x<K>(__float_as_uint(a.z)));
  const int oi = (int)lane_x<K>((uint32_t)a.amx);
  const float ok = __uint_as_float(lane_x<K>(__float_as_uint(a.gk)));
  const int ogi = (int)lane_x<K>((uint32_t)a.gi);
  const float ocnt = __uint_as_float(lane_x<K>(__float_as_uint(a.cnt)));
  const float oq = __uint_as_float(lane_x<K>(__float_as_uint(a.q)));
  merge_mz(a.mx, a.z, a.amx, om, oz, oi, c);
  merge_g(a.gk, a.gi, ok, ogi);
  a.cnt += ocnt;
  a.q += oq;
}

// Block-wide reduction of an Acc into LDS slot `out` (thread 0 holds the result).
__device__ __forceinline__ void block_reduce_acc(Acc& a, float c, Acc* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();  // `red` may still be read by thread 0 from a previous reduction
  acc_step<1>(a, c);
  acc_step<2>(a, c);
  acc_step<4>(a, c);
  acc_step<8>(a, c);
  acc_step<16>(a, c);
  acc_step<32>(a, c);
  if (lane == 0) red[wid] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc r = red[0];
    for (int w = 1; w < nw; ++w) {
      merge_mz(r.mx, r.z, r.amx, red[w].mx, red[w].z, red[w].amx, c);
      merge_g(r.gk, r.gi, red[w].gk, red[w].gi);
      r.cnt += red[w].cnt;
      r.q += red[w].q;
    }
    a = r;
  }
}

// Per-row sampling parameters (row-uniform).
struct RowParams {
  float T, c, cn, topp;
  bool greedy, use_k, use_p;
  int topk;
  uint64_t seed, off;
};

__device__ __forceinline__ RowParams row_params(const SampleArgs& a, int row) {
  RowParams r;
  r.T = a.temperature ? a.temperature[row] : 0.f;
  r.greedy = !(r.T > 1e-5f);
  r.c = r.greedy ? LOG2E_S : LOG2E_S / r.T;  // log2-domain scale
  r.cn = r.greedy ? 1.f : 1.f / r.T;         // natural-domain scale (Gumbel keys)
  r.seed = a.seeds ? a.seeds[row] : 0ull;
  r.off = a.offsets ? (uint64_t)a.offsets[row] : 0ull;
  r.topk = a.top_k ? a.top_k[row] : -1;
  r.topp = a.top_p ? a.top_p[row] : 1.f;
  r.use_k = r.topk > 0 && r.topk < a.V;
  r.use_p = r.topp < 1.f;
  return r;
}

// One element's contribution to a pass (shared by the memory sweep and the register-resident
// rounds below, so both produce the same bits): mode 0 (max / Z / argmax + Gumbel key), mode 1
// (count and mass above xj + the key restricted to x > xj). L = logf(fmaxf(-logf(u), 1e-30f)) of
// this element's uniform for the pass's round (key = v / T - L: a Gumbel draw).
__device__ __forceinline__ void accum_elem(int mode, float v, int i, float L, float xj, float rmx, const RowParams& rp,
                                           Acc& acc) {
  if (mode == 0) {
    if (v > acc.mx) {
      acc.z = (acc.mx == -INFINITY ? 0.f : acc.z * exp2f((acc.mx - v) * rp.c)) + 1.f;
      acc.mx = v;
      acc.amx = i;
    } else if (v > -INFINITY) {
      acc.z += exp2f((v - acc.mx) * rp.c);
    }
  } else if (v > xj) {
    acc.cnt += 1.f;
    acc.q += exp2f((v - rmx) * rp.c);
  }
  if (!rp.greedy && (mode == 0 || v > xj) && v > -INFINITY) {
    const float g = v * rp.cn - L;
    if (g > acc.gk) { acc.gk = g; acc.gi = i; }
  }
}

// accurate logs: a fast log rounding -log(u) to 0 near u = 1 would make an infinite key
__device__ __forceinline__ float gumbel_log(float u) { return logf(fmaxf(-logf(u), 1e-30f)); }

// One sweep of float4 range [v_lo, v_hi) of a row by this block (8 float4 loads in flight per
// thread). mode 0: max / Z / argmax + Gumbel keys; mode 1: acceptance statistics of candidate
// value xj (count and mass of x > xj, mass relative to the row max rmx) + Gumbel keys restricted
// to x > xj with the noise of `round`.
__device__ __forceinline__ void sweep_range(const float4* x4, int v_lo, int v_hi, int mode, float xj, float rmx,
                                            uint32_t round, const RowParams& rp, Acc& acc) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int v0 = v_lo + tid; v0 < v_hi; v0 += nt * 8) {
    // lanes past the range load nothing (a clamped re-read of the last float4 cost a wave load
    // per lane: ~40 % of a 32-segment pass's loads at V = 152k)
    float4 q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int vi = v0 + u * nt;
      q[u] = vi < v_hi ? x4[vi] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int vi = v0 + u * nt;
      if (vi >= v_hi) break;
      const float e[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
      float uu[4] = {0.5f, 0.5f, 0.5f, 0.5f};
      if (!rp.greedy) philox4(rp.seed, rp.off, (uint32_t)vi, round, uu);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = e[j];
        const float L = (!rp.greedy && (mode == 0 || v > xj) && v > -INFINITY) ? gumbel_log(uu[j]) : 0.f;
        accum_elem(mode, v, 4 * vi + j, L, xj, rmx, rp, acc);
      }
    }
  }
}

__device__ __forceinline__ void finish_row(const SampleArgs& a, int row, int chosen, float mx, float z, float c) {
  a.out[row] = chosen;
  if (a.out_logprob) a.out_logprob[row] = ((a.logits[(size_t)row * a.ldl + chosen] - mx) * c - log2f(z)) / LOG2E_S;
}

// ---- one block per row (NSEG == 1: batches above SAMPLE_MAX_BLOCKS / 2 rows, or no workspace) ----
// Every pass sweeps the whole row and ends at a block barrier; same passes, noise and acceptance
// tests as the segmented kernel below.
__global__ __launch_bounds__(SAMPLE_THREADS) void sample_row_kernel(SampleArgs a) {
  TLScope tl_scope(a.tl);
  __shared__ Acc red[SAMPLE_THREADS / 64];
  __shared__ Acc merged;
  const int row = blockIdx.y, tid = threadIdx.x;
  const int V4 = a.V >> 2;  // host guarantees V % 4 == 0 and 16-B aligned rows
  const float* x = a.logits + (size_t)row * a.ldl;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const RowParams rp = row_params(a, row);
  const float c = rp.c;
  auto pass = [&](int mode, float xj, float rmx, uint32_t round) {
    Acc acc = acc_init();
    sweep_range(x4, 0, V4, mode, xj, rmx, round, rp, acc);
    block_reduce_acc(acc, c, red);
    if (tid == 0) merged = acc;
    __syncthreads();
  };
  pass(0, 0.f, 0.f, 0u);
  const float mx = merged.mx, z = merged.z;
  int chosen = merged.amx, j = merged.gi;
  if (!rp.greedy) {
    if (rp.use_k || rp.use_p) {
      const float pmass = rp.topp * z;
      for (uint32_t round = 1; round <= SAMPLE_MAX_ROUNDS && j >= 0; ++round) {
        pass(1, x[j], mx, round);
        const bool ok_k = !rp.use_k || merged.cnt < (float)rp.topk;
        const bool ok_p = !rp.use_p || merged.q < pmass;
        if (ok_k && ok_p) break;
        j = merged.gi;  // next candidate, drawn from {x > x_j}
      }
    }
    if (j >= 0) chosen = j;
  }
  if (tid == 0) finish_row(a, row, chosen, mx, z, c);
}

// ---- single launch: tagged granules instead of tickets / counters ----
// The pass kernels' meetings cost a launch boundary per pass, the in-launch ones a serialised
// atomic per arriving block (~0.5 us each, 32 per row). Here every block of a row publishes its
// pass partial as two 16-B granules {.., tag} (device-coherent sc1 stores, one transaction each),
// and EVERY block of the row gathers all of the row's granules itself (lane s polls segment s
// until both tags carry this pass's tag), merges them in the same fixed lane order and takes the
// same accept / reject decision — no counter, no merger block, one memory round trip after the
// last partial lands. Tags = (row epoch << 6) | pass: the epoch advances once per launch (one store
// by the row's segment 0 at its exit, see the end of the kernel), so a granule of an earlier launch
// never matches; granules alternate two buffers by pass parity (a block reaches pass g + 2,
// rewriting parity g, only after every block of the row published g + 1, i.e. finished reading g).
// Each row owns a FIXED granule region of SAMPLE_GRAN_SEGS segments whatever the launch's (B, nseg):
// a slot is only ever written by its own row, under that row's monotonic epoch. (A layout that moved
// with nseg let row r read row r' < r's leftovers from a launch of another batch size whose tag
// happened to equal r's current one — round-4 ADVICE.)
// Every wait is bounded: a give-up sets fault bit 16 (the engine fails the step) and the row
// falls back to its argmax. B x nseg <= 256 blocks: all co-resident.
__device__ __forceinline__ void gran_publish(uint4* g, const Acc& a, int mode, uint32_t tag) {
  // mode 0 (pass 0): {mx, z, amx} + {gk, gi}; mode 1 (rounds): {cnt, q, gk} + {gi}
  const f32x4 g0 = mode == 0 ? f32x4{a.mx, a.z, __int_as_float(a.amx), __uint_as_float(tag)}
                             : f32x4{a.cnt, a.q, a.gk, __uint_as_float(tag)};
  const f32x4 g1 = mode == 0 ? f32x4{a.gk, __int_as_float(a.gi), 0.f, __uint_as_float(tag)}
                             : f32x4{__int_as_float(a.gi), 0.f, 0.f, __uint_as_float(tag)};
  st_sc1_x4(reinterpret_cast<float*>(g), 0u, g0);
  st_sc1_x4(reinterpret_cast<float*>(g), 16u, g1);
}

// wave 0: gather the nseg granule pairs of (row, parity) and merge them in lane order; lane 0 ends
// with the merge. Returns false if a wait gave up.
__device__ __forceinline__ bool gran_gather(const uint4* gbase, int nseg, int mode, uint32_t tag, float c, Acc& out,
                                            uint32_t* fault) {
  const int lane = threadIdx.x & 63;
  Acc a = acc_init();
  bool ok = true;
  if (lane < nseg) {
    const float* gp = reinterpret_cast<const float*>(gbase + 2 * lane);
    f32x4 g0, g1;
    uint32_t spins = 0;
    while (true) {
      g0 = ld_sc1_x4(gp, 0u);
      g1 = ld_sc1_x4(gp, 16u);
      if (__float_as_uint(g0[3]) == tag && __float_as_uint(g1[3]) == tag) break;
      if (++spins > (1u << 22)) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (ok) {
      if (mode == 0) {
        a.mx = g0[0]; a.z = g0[1]; a.amx = __float_as_int(g0[2]); a.gk = g1[0]; a.gi = __float_as_int(g1[1]);
      } else {
        a.cnt = g0[0]; a.q = g0[1]; a.gk = g0[2]; a.gi = __float_as_int(g1[0]);
      }
    }
  }
  const bool all_ok = __all(ok);
  if (!all_ok && lane == 0 && fault != nullptr) atomicOr(fault, 16u);
  acc_step<1>(a, c);
  acc_step<2>(a, c);
  acc_step<4>(a, c);
  acc_step<8>(a, c);
  acc_step<16>(a, c);
  acc_step<32>(a, c);
  out = a;
  return all_ok;
}

template <int NT>
__global__ __launch_bounds__(NT) void sample_gran_kernel(SampleArgs a) {
  TLScope tl_scope(a.tl);
  __shared__ Acc red[NT / 64];
  __shared__ Acc merged;
  __shared__ int s_ok;
  const int seg = blockIdx.x, nseg = gridDim.x, row = blockIdx.y, tid = threadIdx.x;
  const int V4 = a.V >> 2;
  const int v_lo = (int)(((long long)V4 * seg) / nseg), v_hi = (int)(((long long)V4 * (seg + 1)) / nseg);
  const float* x = a.logits + (size_t)row * a.ldl;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const RowParams rp = row_params(a, row);
  const float c = rp.c;
  const uint32_t ep = __builtin_amdgcn_readfirstlane(__float_as_uint(ld_sc1(reinterpret_cast<const float*>(a.epoch + row))));
  uint4* rowg = reinterpret_cast<uint4*>(a.gran) + (size_t)row * SAMPLE_GRAN_ROW;  // [parity][SEGS][2]
  // one pass: sweep, block merge, publish, gather every segment's granules, share the row merge
  auto pass = [&](int mode, float xj, float rmx, uint32_t round, uint32_t gen) -> bool {
    Acc acc = acc_init();
    sweep_range(x4, v_lo, v_hi, mode, xj, rmx, round, rp, acc);
    block_reduce_acc(acc, c, red);
    const uint32_t tag = (ep << 6) | gen;
    uint4* pg = rowg + (size_t)(gen & 1) * SAMPLE_GRAN_SEGS * 2;
    if (tid == 0) {
      gran_publish(pg + 2 * seg, acc, mode, tag);
    }
    if (tid < 64) {
      Acc r;
      const bool ok = gran_gather(pg, nseg, mode, tag, c, r, a.fault);
      if (tid == 0) {
        merged = r;
        s_ok = ok;
      }
    }
    __syncthreads();
    return s_ok != 0;
  };
  uint32_t gen = 1;
  bool ok = pass(0, 0.f, 0.f, 0u, gen);
  const float mx = merged.mx, z = merged.z;
  int chosen = merged.amx, j = merged.gi;
  if (ok && !rp.greedy) {
    if (rp.use_k || rp.use_p) {
      const float pmass = rp.topp * z;
      for (uint32_t round = 1; round <= SAMPLE_MAX_ROUNDS && j >= 0; ++round) {
        ok = pass(1, x[j], mx, round, ++gen);
        if (!ok) { j = -1; break; }
        const bool ok_k = !rp.use_k || merged.cnt < (float)rp.topk;
        const bool ok_p = !rp.use_p || merged.q < pmass;
        if (ok_k && ok_p) break;
        j = merged.gi;  // next candidate, drawn from {x > x_j}
      }
    }
    if (j >= 0) chosen = j;
  }
  if (tid == 0 && seg == 0) {
    finish_row(a, row, chosen, mx, z, c);
    // advance the row's epoch for the next launch: one store by segment 0, no exit ticket (32 device-scope
    // atomics or same-word stores per row serialise at the memory side). Safe: no block gets here before
    // it gathered pass 1 from EVERY block of its row, i.e. after every block read the epoch
    st_sc1(reinterpret_cast<float*>(a.epoch + row), __uint_as_float((ep + 1u) & 0x03ffffffu));
  }
}

int g_sample_nseg = SAMPLE_GRAN_SEGS;  // segments per row cap (set_sample_nseg; benchmarks/sampler_stress.py)
void set_sample_nseg(int n) { g_sample_nseg = n < 1 ? 1 : (n > SAMPLE_GRAN_SEGS ? SAMPLE_GRAN_SEGS : n); }

int sample_segments(int B, int V) {
  const int V4 = V >> 2;
  int nseg = SAMPLE_MAX_BLOCKS / (B > 0 ? B : 1);
  if (nseg > g_sample_nseg) nseg = g_sample_nseg;
  const int cap = V4 / 256;  // >= 1024 logits per segment
  if (nseg > cap) nseg = cap;
  return nseg < 1 ? 1 : nseg;
}

void launch_sample(const SampleArgs& s, hipStream_t st) {
  if (s.B <= 0) return;
  const int nseg = sample_segments(s.B, s.V);
  SampleArgs a = s;
  if (nseg > 1 && s.gran != nullptr && s.epoch != nullptr && s.B <= SAMPLE_GRAN_ROWS) {
    a.tl = tl_take("sample_gran", nseg * s.B);
    // 256 threads per block: 512 / 1024 measured no faster / slower (profiles/r4_sampler_single_launch.log)
    hipLaunchKernelGGL(sample_gran_kernel<256>, dim3(nseg, s.B), dim3(256), 0, st, a);
    return;
  }
  a.tl = tl_take("sample", s.B);
  hipLaunchKernelGGL(sample_row_kernel, dim3(1, s.B), dim3(SAMPLE_THREADS), 0, st, a);
}

}  // namespace vgate
