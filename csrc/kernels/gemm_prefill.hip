// LDS-tiled MFMA GEMM for prefill / long steps (M >= 128) on gfx950 — the hand-written
// replacement of the hipBLASLt path, on the SAME fragment-packed weights the decode kernels
// stream (no second plain copy of any weight is kept).
//
//   out[m][n] = epilogue( rowscale(m) * sum_k x[m][k] * W[n][k] )
//
// Both operands are staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction) into a 2-deep ring, BK = 64 (two 32-deep MFMA k-steps per stage):
//   * W: the packed layout Wp[nt][kt][lane][8] IS the MFMA A-fragment order, so one 1 KiB
//     piece (one 16-column tile x one k-step) lands lane-linear and every wave reads its
//     fragments back with conflict-free ds_read_b128 (lane l at +16 l) — no swizzle needed;
//   * x: each 1 KiB piece gathers the B fragments of 16 rows x 32 k (per-lane source address =
//     row m0 + (l & 15), column 8 (l >> 4)), so the LDS image is fragment-major too.
// Pipeline (cdna_hip_programming.md §5 'glds vs register staging', first row): the stage t+1
// DMA is issued before stage t's ds_reads + MFMAs, one vmcnt(0) + barrier per stage.
// Block tile BM x BN over 4 waves (2 x 2), wave tile (BM/2) x (BN/2) in 16x16x32 bf16 MFMAs,
// orientation D = W(A) . X(B): lane holds D[n = 4(l>>4)+i][m = l&15], so the epilogues of the
// decode kernels (gemm_epilogue.h: bias, residual, SiLU*mul pairs, QKV RoPE + KV write) are
// reused unchanged. The RMSNorm in front of qkv / gate_up runs as the deferred row scale
// (gamma folded into W at load time): x^2 is accumulated from the B fragments the MFMAs read.
// Grid: 1-D, XCD-aware bijective remap, m-blocks fastest so the blocks that share a weight
// column panel run back to back on one XCD (one HBM read of the panel per XCD L2).
#include <cstdlib>

#include "gemm_epilogue.h"

namespace vgate {

// x^2 of 8 bf16 (one B fragment) into acc: 4 packed dot products (v_dot2_f32_bf16), no unpack — the
// folded RMSNorm's row sums ride along the MFMA loop at a quarter of the unpack + FMA VALU cost
typedef __bf16 p4_bf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float sumsq8(uint4 v, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(p4_bf2, v.x), __builtin_bit_cast(p4_bf2, v.x), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(p4_bf2, v.y), __builtin_bit_cast(p4_bf2, v.y), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(p4_bf2, v.z), __builtin_bit_cast(p4_bf2, v.z), acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(p4_bf2, v.w), __builtin_bit_cast(p4_bf2, v.w), acc, false);
}

template <int BM, int BN, int EPI, int NORM, int NTB>
__global__ __launch_bounds__(256, 2) void gemm_prefill_kernel(GemmParams p) {
  static_assert(BM % 32 == 0 && BN % 32 == 0, "2 x 2 waves of 16-multiple tiles");
  constexpr int KS = 2;                      // 32-deep k-steps per stage (BK = 64)
  constexpr int WTN = BN / 16, XTM = BM / 16;  // 16-wide tiles per block
  constexpr int NT = WTN / 2, MT = XTM / 2;    // per wave
  constexpr int PIECES = (WTN + XTM) * KS;     // 1 KiB pieces per stage
  static_assert(PIECES % 4 == 0, "pieces split evenly over 4 waves");
  constexpr int PPW = PIECES / 4;              // per wave
  constexpr int STAGE = PIECES * 1024;
  static_assert(NT % NTB == 0, "epilogue tile groups");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int KT = p.K >> 5;
  const int nk_all = p.K >> 6;  // stages (K % 64 == 0, host-checked)
  // split-K (small tile grids): blockIdx.y = K slice; partials go to the reduce kernel
  const int z = blockIdx.y, nz = gridDim.y;
  const int kst0 = (nk_all * z) / nz, nk = (nk_all * (z + 1)) / nz - kst0;
  // XCD-aware logical block id (bijective for any grid size), then m fastest
  const int mblocks = (p.M + BM - 1) / BM;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int m0 = (wgid % mblocks) * BM;
  const int nt_blk = (wgid / mblocks) * WTN;  // first 16-column tile of the block
  // this wave's DMA pieces: piece f < WTN*KS is W tile f / KS at k-step f % KS, else x
  // m-tile (f - WTN*KS) / KS. Source addresses per lane, advanced by one stage per iteration.
  const char* src[PPW];
  int step[PPW];  // bytes per stage
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int f = wid * PPW + i;
    if (f < WTN * KS) {
      const int nt = nt_blk + f / KS, ks = f % KS;
      src[i] = reinterpret_cast<const char*>(p.wp) + (((size_t)nt * KT + 2 * kst0 + ks) * 64 + lane) * 16;
      step[i] = KS * 1024;
    } else {
      const int g = f - WTN * KS;
      const int mt = g / KS, ks = g % KS;
      int row = m0 + mt * 16 + (lane & 15);
      row = row < p.M ? row : p.M - 1;  // rows past M repeat row M-1 (never stored)
      src[i] = reinterpret_cast<const char*>(p.x + (size_t)row * p.lda + kst0 * 64 + ks * 32 + 8 * (lane >> 4));
      step[i] = 64 * 2;
    }
  }
  const uint32_t lds0 = lds_addr_of(smem);
  auto issue = [&](int stage, int buf) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int f = wid * PPW + i;  // wave-uniform LDS destination (M0): lane l lands at +16 l
      glds16(src[i] + (size_t)stage * step[i], __builtin_amdgcn_readfirstlane(lds0 + buf * STAGE + f * 1024));
    }
  };
  f32x4 acc[NT][MT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int b = 0; b < MT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int b = 0; b < MT; ++b) ss[b] = 0.f;

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) issue(t + 1, buf ^ 1);
    const char* sb = smem + buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 wa[NT], xb[MT];
#pragma unroll
      for (int a = 0; a < NT; ++a)
        wa[a] = *reinterpret_cast<const uint4*>(sb + ((wn * NT + a) * KS + ks) * 1024 + lane * 16);
#pragma unroll
      for (int b = 0; b < MT; ++b)
        xb[b] = *reinterpret_cast<const uint4*>(sb + (WTN * KS + (wm * MT + b) * KS + ks) * 1024 + lane * 16);
      if constexpr (NORM == 2) {
#pragma unroll
        for (int b = 0; b < MT; ++b) {
          ss[b] = sumsq8(xb[b], ss[b]);
        }
      }
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int b = 0; b < MT; ++b) acc[a][b] = mfma16(as_bf16x8(wa[a]), as_bf16x8(xb[b]), acc[a][b]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nz > 1) {
    // fp32 partial of this K slice -> slabs [z][M][N] (row-major, the lane's 4 columns as one
    // 16-B store) and its rows' partial sums of squares -> [z][M] after the tiles; the reduce
    // kernel sums the slices in a fixed order (bit-reproducible) and runs the epilogue
    float* part = p.slabs + (size_t)z * p.M * p.N;
    float* ssq = p.slabs + (size_t)nz * p.M * p.N + (size_t)z * p.M;
#pragma unroll
    for (int b = 0; b < MT; ++b) {
      const int m = m0 + wm * (BM / 2) + b * 16 + (lane & 15);
      if constexpr (NORM == 2) {
        float s2 = ss[b];
        s2 += xor16(s2);
        s2 += xor32(s2);
        if (wn == 0 && lane < 16 && m < p.M) ssq[m] = s2;
      }
      if (m < p.M) {
#pragma unroll
        for (int a = 0; a < NT; ++a) {
          const int n = (nt_blk + wn * NT + a) * 16 + 4 * (lane >> 4);
          __builtin_nontemporal_store(acc[a][b], reinterpret_cast<f32x4*>(part + (size_t)m * p.N + n));
        }
      }
    }
    return;
  }
  // epilogue straight from the accumulators: row m = m0 + wm*(BM/2) + 16 b + (l & 15)
#pragma unroll
  for (int b = 0; b < MT; ++b) {
    const int m = m0 + wm * (BM / 2) + b * 16 + (lane & 15);
    float sc = 1.f;
    if constexpr (NORM == 2) {
      float s2 = ss[b];
      s2 += xor16(s2);
      s2 += xor32(s2);
      sc = rsqrtf(s2 / (float)p.K + p.eps);
    }
#pragma unroll
    for (int a = 0; a < NT; a += NTB) {
      f32x4 v[NTB];
#pragma unroll
      for (int j = 0; j < NTB; ++j) v[j] = acc[a + j][b] * sc;
      epilogue<NTB, EPI, false>(p, v, m, nt_blk + wn * NT + a, 4 * (lane >> 4), EpiPre<NTB>{}, m < p.M);
    }
  }
}

// ---- v2: deeper pipeline, bigger block tile ----
// Same operand staging (LDS-DMA of fragment-major 1 KiB pieces, conflict-free ds_read_b128),
// epilogues and split-K contract as gemm_prefill_kernel, but
//   * an NS-deep stage ring: stage t + NS - 1 is issued before stage t is consumed, with ONE
//     counted vmcnt wait + s_barrier per stage (no vmcnt(0): the NS-2 younger stages stay in
//     flight). The 2-deep ring waited for the stage it had just issued every 64 k, so each
//     stage paid a full L2 / HBM round trip (~0.5-1 us) against ~0.4 us of MFMA work;
//   * WM x WN waves (8: 512 threads) on a BM x BN = 256 x 128 tile, wave tile 64 x 64: twice the
//     MFMA work per staged byte of the 128 x 128 tile and one block per CU (144 KiB ring).
// Past the last stage the ring keeps issuing (clamped duplicate loads into buffers that are never
// read again), so every wait count is a compile-time constant.
// SCHED (k-loop schedule): 0 = the stage's DMA issued before its reads + MFMAs; 1 = + MFMAs at raised
// wave priority (s_setprio 1: the MFMA-issuing wave wins the SIMD's arbitration over the other wave's
// LDS reads / DMA issue); 2 = 1 + the stage's DMA issue split in two, half in front of each k-step
template <int BM, int BN, int WM, int WN, int NS, int EPI, int NORM, int NTB, int SCHED = 0, int KS = 2>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_prefill2_kernel(GemmParams p) {
  constexpr int NW = WM * WN;
  // KS: 32-deep k-steps per stage (BK = 32 KS)
  constexpr int WTN = BN / 16, XTM = BM / 16;  // 16-wide tiles per block
  constexpr int NT = WTN / WN, MT = XTM / WM;  // per wave
  constexpr int PIECES = (WTN + XTM) * KS;     // 1 KiB pieces per stage
  static_assert(PIECES % NW == 0, "pieces split evenly over the waves");
  constexpr int PPW = PIECES / NW;
  constexpr int STAGE = PIECES * 1024;
  static_assert(NT % NTB == 0 && NS >= 2 && NS <= 4, "tile groups / ring depth");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int KT = p.K >> 5;
  const int nk_all = KT / KS;
  const int z = blockIdx.y, nz = gridDim.y;
  const int kst0 = (nk_all * z) / nz, nk = (nk_all * (z + 1)) / nz - kst0;
  const int mblocks = (p.M + BM - 1) / BM;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int m0 = (wgid % mblocks) * BM;
  const int nt_blk = (wgid / mblocks) * WTN;
  const char* src[PPW];
  int step[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int f = wid * PPW + i;
    if (f < WTN * KS) {
      const int nt = nt_blk + f / KS, ks = f % KS;
      src[i] = reinterpret_cast<const char*>(p.wp) + (((size_t)nt * KT + KS * kst0 + ks) * 64 + lane) * 16;
      step[i] = KS * 1024;
    } else {
      const int g = f - WTN * KS;
      const int mt = g / KS, ks = g % KS;
      int row = m0 + mt * 16 + (lane & 15);
      row = row < p.M ? row : p.M - 1;
      src[i] = reinterpret_cast<const char*>(p.x + (size_t)row * p.lda + kst0 * 32 * KS + ks * 32 + 8 * (lane >> 4));
      step[i] = 32 * KS * 2;
    }
  }
  const uint32_t lds0 = lds_addr_of(smem);
  auto issue_part = [&](int stage, int buf, int i0, int i1) {
    const int st = stage < nk ? stage : nk - 1;  // past the end: a clamped duplicate, never read
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      if (i < i0 || i >= i1) continue;  // compile-time after unrolling
      const int f = wid * PPW + i;
      glds16(src[i] + (size_t)st * step[i], __builtin_amdgcn_readfirstlane(lds0 + buf * STAGE + f * 1024));
    }
  };
  auto issue = [&](int stage, int buf) { issue_part(stage, buf, 0, PPW); };
  f32x4 acc[NT][MT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int b = 0; b < MT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int b = 0; b < MT; ++b) ss[b] = 0.f;

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0) issue(s0, s0);
  for (int t = 0; t < nk; ++t) {
    // stage t landed (this wave's pieces; the NS-2 younger stages may still be in flight), then
    // every wave's pieces (barrier) — which also retires the reads of the buffer refilled next
    if constexpr (NS == 2) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * PPW) : "memory");
    if constexpr (SCHED < 2) issue(t + NS - 1, (t + NS - 1) % NS);
    else issue_part(t + NS - 1, (t + NS - 1) % NS, 0, PPW / 2);
    const char* sb = smem + (t % NS) * STAGE;
    // every fragment of the stage read up front (both k-steps): the second k-step's reads are in
    // flight under the first one's MFMAs instead of exposing the LDS latency per k-step
    uint4 wall[KS][NT], xall[KS][MT];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int a = 0; a < NT; ++a)
        wall[ks][a] = *reinterpret_cast<const uint4*>(sb + ((wn * NT + a) * KS + ks) * 1024 + lane * 16);
#pragma unroll
      for (int b = 0; b < MT; ++b)
        xall[ks][b] = *reinterpret_cast<const uint4*>(sb + (WTN * KS + (wm * MT + b) * KS + ks) * 1024 + lane * 16);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint4 (&wa)[NT] = wall[ks];
      const uint4 (&xb)[MT] = xall[ks];
      if constexpr (NORM == 2) {
#pragma unroll
        for (int b = 0; b < MT; ++b) {
          ss[b] = sumsq8(xb[b], ss[b]);
        }
      }
      if constexpr (SCHED == 2)
        if (ks == 1) issue_part(t + NS - 1, (t + NS - 1) % NS, PPW / 2, PPW);
      if constexpr (SCHED >= 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int b = 0; b < MT; ++b) acc[a][b] = mfma16(as_bf16x8(wa[a]), as_bf16x8(xb[b]), acc[a][b]);
      if constexpr (SCHED >= 1) __builtin_amdgcn_s_setprio(0);
    }
    // the next iteration's barrier orders these ds_reads before the buffer is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing duplicate DMAs
  if (nz > 1) {
    float* part = p.slabs + (size_t)z * p.M * p.N;
    float* ssq = p.slabs + (size_t)nz * p.M * p.N + (size_t)z * p.M;
#pragma unroll
    for (int b = 0; b < MT; ++b) {
      const int m = m0 + wm * (BM / WM) + b * 16 + (lane & 15);
      if constexpr (NORM == 2) {
        float s2 = ss[b];
        s2 += xor16(s2);
        s2 += xor32(s2);
        if (wn == 0 && lane < 16 && m < p.M) ssq[m] = s2;
      }
      if (m < p.M) {
#pragma unroll
        for (int a = 0; a < NT; ++a) {
          const int n = (nt_blk + wn * NT + a) * 16 + 4 * (lane >> 4);
          __builtin_nontemporal_store(acc[a][b], reinterpret_cast<f32x4*>(part + (size_t)m * p.N + n));
        }
      }
    }
    return;
  }
#pragma unroll
  for (int b = 0; b < MT; ++b) {
    const int m = m0 + wm * (BM / WM) + b * 16 + (lane & 15);
    float sc = 1.f;
    if constexpr (NORM == 2) {
      float s2 = ss[b];
      s2 += xor16(s2);
      s2 += xor32(s2);
      sc = rsqrtf(s2 / (float)p.K + p.eps);
    }
#pragma unroll
    for (int a = 0; a < NT; a += NTB) {
      f32x4 v[NTB];
#pragma unroll
      for (int j = 0; j < NTB; ++j) v[j] = acc[a + j][b] * sc;
      epilogue<NTB, EPI, false>(p, v, m, nt_blk + wn * NT + a, 4 * (lane >> 4), EpiPre<NTB>{}, m < p.M);
    }
  }
}

// ---- v4: 256 x 256 tile in four phases per K-tile ----
// 8 waves, wave (wr = wid >> 2, wc = wid & 3) owns n-tiles 8 wr .. 8 wr + 7 (two halves n0 / n1 of 4)
// x m-tiles 4 wc .. 4 wc + 3 (halves m0 / m1 of 2). A K-tile (BK = 64, 64 KiB: 16 W + 16 x tiles x
// 2 k-steps) is consumed in four phases, one 64 x 32 output quadrant x K = 64 (16 MFMAs) each, in
// the order (n0, m0) (n0, m1) (n1, m1) (n1, m0): phase 0 first needs W n0 + x m0, phase 1 x m1,
// phase 2 W n1, phase 3 nothing new (x m0 kept in registers). The next K-tile's LDS-DMA is issued
// in the same three groups, group g in phase g (into the other buffer, free since the previous
// K-tile's phase-0 barrier), so every piece has a whole K-tile (four phases) to land and each
// phase waits with a compile-time counted vmcnt (pieces issued after its group) + raw s_barrier —
// never vmcnt(0) in the loop (cdna_hip_programming.md §5 'The 256² 8-phase template').
// Group sizes per wave: 4 / 2 / 2 pieces -> the waits of phases 0 / 1 / 2: vmcnt(4) / (6) / (6).
// BN = 128: the same schedule on a 256 x 128 tile (wave 64 n x 64 m, 8 MFMAs per phase, 96 KiB;
// groups 3 / 2 / 1 pieces per wave -> vmcnt(3) / (4) / (5)).
template <int BN>
struct P4 {  // geometry of the 4-phase 256 x BN kernel
  static constexpr int BM = 256, KS = 2;
  static constexpr int WTN = BN / 16, XTM = BM / 16;  // W + x tiles per block (16 / 8 + 16)
  static constexpr int NWN = WTN / 2, NH = NWN / 2;   // n-tiles per wave, per n-half
  static constexpr int STAGE = (WTN + XTM) * KS * 1024;
  static constexpr int G0 = 4 * NH + 16, G1 = 16, G2 = 4 * NH;  // pieces per group (block)
  static constexpr int P0 = G0 / 8, P1 = G1 / 8, P2 = G2 / 8;  // per wave
  static constexpr int PPW = P0 + P1 + P2;
  static_assert(G0 % 8 == 0 && G2 % 8 == 0 && (BN == 256 || BN == 128), "pieces split over 8 waves");
};

// The K loop of the 4-phase kernel over K-tiles [kst0, kst0 + nk) of the block tile (m0, nt_blk),
// accumulated into acc / ss (zeroed by the caller). Ends with every DMA of this wave landed (the
// trailing clamped duplicates included); a caller that runs it again on the same LDS barriers first.
template <int BN, int NORM>
__device__ __forceinline__ void p4_kloop(const GemmParams& p, char* smem, int wid, int lane, int m0, int nt_blk,
                                         int kst0, int nk, f32x4 (&acc)[BN / 32][4], float (&ss)[4]) {
  using G = P4<BN>;
  constexpr int KS = G::KS, WTN = G::WTN, NWN = G::NWN, NH = G::NH, STAGE = G::STAGE;
  constexpr int P0 = G::P0, P1 = G::P1, P2 = G::P2, PPW = G::PPW;
  const int wr = wid >> 2, wc = wid & 3;
  const int KT = p.K >> 5;
  // this wave's pieces: entries of the group lists (block-local tile, k-step; W or x)
  //   group 0: the n0 W tiles of both wave rows, then x tiles {4c, 4c + 1}, x 2 k-steps
  //   group 1: x tiles {4c + 2, 4c + 3} x 2
  //   group 2: the n1 W tiles x 2
  const char* src[PPW];
  int step[PPW];
  uint32_t dst[PPW];
  const uint32_t lds0 = lds_addr_of(smem);
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    int e, isw, t;
    if (i < P0) {
      e = wid * P0 + i;
      if (e < 4 * NH) {
        isw = 1;
        const int tw = e >> 1;
        t = (tw / NH) * NWN + tw % NH;
      } else {
        isw = 0;
        const int tile8 = (e - 4 * NH) >> 1;
        t = 4 * (tile8 >> 1) + (tile8 & 1);
      }
    } else if (i < P0 + P1) {
      e = wid * P1 + (i - P0);
      isw = 0;
      const int tile8 = e >> 1;
      t = 4 * (tile8 >> 1) + 2 + (tile8 & 1);
    } else {
      e = wid * P2 + (i - P0 - P1);
      isw = 1;
      const int tw = e >> 1;
      t = (tw / NH) * NWN + NH + tw % NH;
    }
    const int ks = e & 1;
    if (isw) {
      src[i] = reinterpret_cast<const char*>(p.wp) + (((size_t)(nt_blk + t) * KT + 2 * kst0 + ks) * 64 + lane) * 16;
      step[i] = KS * 1024;
      dst[i] = (uint32_t)((t * KS + ks) * 1024);
    } else {
      int row = m0 + t * 16 + (lane & 15);
      row = row < p.M ? row : p.M - 1;
      src[i] = reinterpret_cast<const char*>(p.x + (size_t)row * p.lda + kst0 * 64 + ks * 32 + 8 * (lane >> 4));
      step[i] = 64 * 2;
      dst[i] = (uint32_t)((WTN * KS + t * KS + ks) * 1024);
    }
  }
  auto issue_group = [&](int g, int stage, int buf) {
    const int st = stage < nk ? stage : nk - 1;  // past the end: clamped duplicates, never read
    const int i0 = g == 0 ? 0 : g == 1 ? P0 : P0 + P1, i1 = g == 0 ? P0 : g == 1 ? P0 + P1 : PPW;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      if (i < i0 || i >= i1) continue;
      glds16(src[i] + (size_t)st * step[i], __builtin_amdgcn_readfirstlane(lds0 + buf * STAGE + dst[i]));
    }
  };
  uint4 wf[KS][NH], x0[KS][2], x1[KS][2];
  auto read_w = [&](const char* sb, int half) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < NH; ++a)
        wf[ks][a] = *reinterpret_cast<const uint4*>(sb + ((wr * NWN + half * NH + a) * KS + ks) * 1024 + lane * 16);
  };
  auto read_x = [&](const char* sb, int half, uint4 (&xf)[KS][2]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        xf[ks][b] = *reinterpret_cast<const uint4*>(sb + (WTN * KS + (wc * 4 + half * 2 + b) * KS + ks) * 1024 + lane * 16);
    // folded RMSNorm: x^2 of the rows in packed bf16 dot products (v_dot2_f32_bf16: one op per 2
    // elements, no unpack), and only in wave row 0 — wave row 1 reads the same x tiles; the row
    // sums reach it through LDS in p4_finish. (The unpack + FMA form in both wave rows cost the
    // folded-norm GEMMs ~20 % against the same tile without the norm: Llama-3-8B gate_up at
    // 2048 rows 472 vs 399 us.)
    if constexpr (NORM == 2) {
      if (wr == 0) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int b = 0; b < 2; ++b) ss[half * 2 + b] = sumsq8(xf[ks][b], ss[half * 2 + b]);
      }
    }
  };
  auto quadrant = [&](int nh, int mh, const uint4 (&xf)[KS][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < NH; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[nh * NH + a][mh * 2 + b] = mfma16(as_bf16x8(wf[ks][a]), as_bf16x8(xf[ks][b]), acc[nh * NH + a][mh * 2 + b]);
    __builtin_amdgcn_s_setprio(0);
  };
  issue_group(0, 0, 0);
  issue_group(1, 0, 0);
  issue_group(2, 0, 0);
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const char* sb = smem + buf * STAGE;
    // phase 0: (n0, m0) — group 0 of this K-tile (groups 1, 2 issued after it)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P1 + P2) : "memory");
    read_w(sb, 0);
    read_x(sb, 0, x0);
    issue_group(0, t + 1, buf ^ 1);
    quadrant(0, 0, x0);
    // phase 1: (n0, m1) — group 1 (issued after it: group 2 of this tile, group 0 of the next)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P2 + P0) : "memory");
    read_x(sb, 1, x1);
    issue_group(1, t + 1, buf ^ 1);
    quadrant(0, 1, x1);
    // phase 2: (n1, m1) — group 2 (issued after it: groups 0, 1 of the next tile)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P0 + P1) : "memory");
    read_w(sb, 1);
    issue_group(2, t + 1, buf ^ 1);
    quadrant(1, 1, x1);
    // phase 3: (n1, m0) from registers
    quadrant(1, 0, x0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing duplicate DMAs
}

// the epilogue of a finished 256 x BN block tile straight from the accumulators (deferred row scale)
// (NORM == 2: the row sums of squares are in wave row 0's ss; wave row 1 gets them through the 1 KiB
// LDS area P4_ROWSS past the ring — block-uniform call, one barrier)
constexpr int P4_ROWSS = 16;  // byte offset past the 2-stage ring
template <int BN, int EPI, int NORM, int NTB>
__device__ __forceinline__ void p4_finish(const GemmParams& p, char* smem, int wid, int lane, int m0, int nt_blk,
                                          f32x4 (&acc)[BN / 32][4], const float (&ss)[4]) {
  constexpr int NWN = P4<BN>::NWN;
  const int wr = wid >> 2, wc = wid & 3;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (NORM == 2) {
    float* rows = reinterpret_cast<float*>(smem + 2 * P4<BN>::STAGE + P4_ROWSS);
    if (wr == 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float s2 = ss[b];
        s2 += xor16(s2);
        s2 += xor32(s2);
        rs[b] = s2;
        if (lane < 16) rows[wc * 64 + b * 16 + lane] = s2;
      }
    }
    lds_barrier();
    if (wr != 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) rs[b] = rows[wc * 64 + b * 16 + (lane & 15)];
    }
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wc * 64 + b * 16 + (lane & 15);
    float sc = 1.f;
    if constexpr (NORM == 2) sc = rsqrtf(rs[b] / (float)p.K + p.eps);
#pragma unroll
    for (int a = 0; a < NWN; a += NTB) {
      f32x4 v[NTB];
#pragma unroll
      for (int j = 0; j < NTB; ++j) v[j] = acc[a + j][b] * sc;
      epilogue<NTB, EPI, false>(p, v, m, nt_blk + wr * NWN + a, 4 * (lane >> 4), EpiPre<NTB>{}, m < p.M);
    }
  }
}

template <int BN, int EPI, int NORM, int NTB>
__global__ __launch_bounds__(512, 1) void gemm_prefill4_kernel(GemmParams p) {
  using G = P4<BN>;
  constexpr int BM = G::BM, WTN = G::WTN, NWN = G::NWN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int nk_all = p.K >> 6;
  const int z = blockIdx.y, nz = gridDim.y;
  const int kst0 = (nk_all * z) / nz, nk = (nk_all * (z + 1)) / nz - kst0;
  const int mblocks = (p.M + BM - 1) / BM;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int m0 = (wgid % mblocks) * BM;
  const int nt_blk = (wgid / mblocks) * WTN;
  f32x4 acc[NWN][4];
#pragma unroll
  for (int a = 0; a < NWN; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[4] = {0.f, 0.f, 0.f, 0.f};
  p4_kloop<BN, NORM>(p, smem, wid, lane, m0, nt_blk, kst0, nk, acc, ss);
  if (nz > 1) {
    float* part = p.slabs + (size_t)z * p.M * p.N;
    float* ssq = p.slabs + (size_t)nz * p.M * p.N + (size_t)z * p.M;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = m0 + wc * 64 + b * 16 + (lane & 15);
      if constexpr (NORM == 2) {
        float s2 = ss[b];
        s2 += xor16(s2);
        s2 += xor32(s2);
        if (wr == 0 && lane < 16 && m < p.M) ssq[m] = s2;
      }
      if (m < p.M) {
#pragma unroll
        for (int a = 0; a < NWN; ++a) {
          const int n = (nt_blk + wr * NWN + a) * 16 + 4 * (lane >> 4);
          __builtin_nontemporal_store(acc[a][b], reinterpret_cast<f32x4*>(part + (size_t)m * p.N + n));
        }
      }
    }
    return;
  }
  p4_finish<BN, EPI, NORM, NTB>(p, smem, wid, lane, m0, nt_blk, acc, ss);
}

// ---- persistent form of the 4-phase kernel: whole rounds + a K-split last round, one launch ----
// A tile grid of T tiles on G CUs takes ceil(T / G) rounds and the last one runs R = T mod G tiles
// on a fraction of the chip (Llama-3-8B gate_up at 2048 rows: 896 tiles = 3 rounds + 128 tiles; o /
// down: 128 tiles = half the chip). Here G = #CU resident blocks (one per CU: the LDS ring) run the
// T - R tiles of the whole rounds in order — block g takes tile r * G + g in round r, so each XCD
// keeps working on 4 weight panels x all m-blocks at the same K position, as the tile grid does
// (the L2 reuse a free (tile, K-tile) stream-K split loses: its blocks sit at unrelated K offsets
// and it measured 1.3x SLOWER than the tile grid, profiles/r6_prefill_stream_k.log) — and then
// the R tail tiles as S K slices each: unit u = (S - 1 - c) * R + j is slice c of tail tile j, block
// g takes units g, g + G, ... (the launcher's S keeps R S <= G, one round: Llama-3-8B gate_up / down /
// o_proj at 2048 rows, S = 2; a forced larger S runs several rounds), so the blocks of one XCD
// again share panels and K positions.
// Slices c > 0 publish their fp32 partial (+ the x sums of squares of the folded RMSNorm) to the
// unit's slot with device-coherent stores and count in on the tile's ticket; slice 0 (the owner)
// waits for the S - 1 tickets, adds the partials in slice order (bit-reproducible), runs the epilogue
// and clears the ticket. Every block takes its units in order and all of the later slices come
// before the owners, so a slice never waits: an owner's partials are either done or being computed
// by a resident block that needs nothing from anyone; the poll is bounded all the same (give-up:
// bit 64 of the fault word, garbage, never a hang).
constexpr int P4SK_SPIN = 1 << 20;

template <int BN>
__host__ __device__ constexpr int p4sk_slot_floats() {
  return (P4<BN>::NWN * 4 + 1) * 512 * 4;  // 512 threads x (NWN x 4 accumulators + the row sums) f32x4
}

// slot traffic: lane part in ONE VGPR (tid * 16), the accumulator index in the scalar offset (a
// per-index VGPR offset is loop-invariant, gets hoisted over the K loop and spills the 256-wide tile)
__device__ __forceinline__ void p4sk_st(float* slot, int tid, int j, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc_of(slot), (uint32_t)tid * 16, j * 8192, 16 /* sc1 */);
}
__device__ __forceinline__ f32x4 p4sk_ld(const float* slot, int tid, int j) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(slot), (uint32_t)tid * 16, j * 8192, 16 /* sc1 */);
}

template <int BN, int EPI, int NORM, int NTB>
__global__ __launch_bounds__(512, 1) void gemm_prefill4sk_kernel(GemmParams p0, int tiles, int S) {
  using G = P4<BN>;
  constexpr int BM = G::BM, WTN = G::WTN, NWN = G::NWN, NACC = NWN * 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p0.dbg_ts);
  const int KT = p0.K >> 6;
  const int mblocks = (p0.M + BM - 1) / BM;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  // XCD-aware: consecutive g (tiles of one weight column panel, m-blocks fastest) on one XCD
  const int g = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int full = tiles / nwg, R = tiles - full * nwg;
  const int RS = R * S, nseg = full + (g < RS ? (RS - g + nwg - 1) / nwg : 0);
  const auto kp0 = (const GemmParams __attribute__((address_space(4)))*)(__builtin_amdgcn_kernarg_segment_ptr());
  for (int i = 0; i < nseg; ++i) {  // block-uniform
    if (i > 0) __builtin_amdgcn_s_barrier();  // the previous tile's LDS reads + DMAs are done
    // the parameters re-read from the kernel-argument segment per tile: hoisted out of this loop,
    // the epilogue's pointers would sit in SGPRs across the K loop (SGPR spills into VGPR lanes);
    // thread ids laundered likewise (no lane-derived epilogue / slot address stays live across it)
    auto kp = kp0;
    asm volatile("" : "+s"(kp));
    const GemmParams& p = *(const GemmParams*)kp;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int tile = i * nwg + g, k0 = 0, k1 = KT, c = -1, j = 0, u = 0;
    if (i >= full) {  // tail unit u: slice c of tail tile j, the later slices first (the owners last)
      u = g + (i - full) * nwg;
      j = u % R;
      c = S - 1 - u / R;
      tile = full * nwg + j;
      k0 = (KT * c) / S;
      k1 = (KT * (c + 1)) / S;
    }
    const int m0 = (tile % mblocks) * BM, nt_blk = (tile / mblocks) * WTN;
    f32x4 acc[NWN][4];
#pragma unroll
    for (int a = 0; a < NWN; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss[4] = {0.f, 0.f, 0.f, 0.f};
    if (c > 0) {  // a later K slice of a tail tile: publish, count in (its own copy of the K loop: with
                  // one copy shared by this path and the owner's the allocator spills the accumulators)
      p4_kloop<BN, NORM>(p, smem, wid, lane, m0, nt_blk, k0, k1 - k0, acc, ss);
      float* slot = p.slabs + (size_t)u * p4sk_slot_floats<BN>();  // u < R (S - 1): one slot per unit
#pragma unroll
      for (int e = 0; e < NACC; ++e) p4sk_st(slot, tid, e, acc[e >> 2][e & 3]);
      if constexpr (NORM == 2) p4sk_st(slot, tid, NACC, f32x4{ss[0], ss[1], ss[2], ss[3]});
      drain_stores();
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(p.counters + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    p4_kloop<BN, NORM>(p, smem, wid, lane, m0, nt_blk, k0, k1 - k0, acc, ss);
    if (c == 0 && S > 1) {  // the owner of a split tail tile: wait for slices 1 .. S - 1, add in order
      if (tid == 0) {
        int spins = 0;
        while (__hip_atomic_load(p.counters + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)(S - 1)) {
          if (++spins > P4SK_SPIN) {
            if (p.fault != nullptr) atomicOr(p.fault, 64u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      for (int cc = 1; cc < S; ++cc) {
        const float* slot = p.slabs + (size_t)((S - 1 - cc) * R + j) * p4sk_slot_floats<BN>();
        // a quarter of the accumulators per round trip (the loads' registers: 32 / 16 per lane)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          f32x4 v[NACC / 4];
#pragma unroll
          for (int e = 0; e < NACC / 4; ++e) v[e] = p4sk_ld(slot, tid, h * NACC / 4 + e);
#pragma unroll
          for (int e = 0; e < NACC / 4; ++e) acc[(h * NACC / 4 + e) >> 2][(h * NACC / 4 + e) & 3] += v[e];
          asm volatile("" ::: "memory");
        }
        if constexpr (NORM == 2) {
          const f32x4 s4 = p4sk_ld(slot, tid, NACC);
          ss[0] += s4[0]; ss[1] += s4[1]; ss[2] += s4[2]; ss[3] += s4[3];
        }
      }
      if (tid == 0) __hip_atomic_store(p.counters + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    p4_finish<BN, EPI, NORM, NTB>(p, smem, wid, lane, m0, nt_blk, acc, ss);
  }
}

// Split-K combine: one wave per (16 rows, NTB tiles): the slices' partials summed in slice
// order, the row scale from the summed slice sums of squares, then the shared epilogue. The
// slices' loads go out in groups of ZG (clamped index, masked add) so a combine costs one memory
// round trip per ZG slices instead of one per slice.
template <int EPI, int NORM, int NTB>
__global__ __launch_bounds__(256) void prefill_reduce_kernel(GemmParams p, int nz) {
  constexpr int ZG = 8;
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63;
  const int grp = blockIdx.x * 4 + (threadIdx.x >> 6);  // (row block, tile group), tile group fastest
  const int ngrp = p.N / (16 * NTB);
  if (grp >= ((p.M + 15) / 16) * ngrp) return;  // wave-uniform
  const int m = (grp / ngrp) * 16 + (lane & 15);
  const int nt0 = (grp % ngrp) * NTB;
  const int nsub = 4 * (lane >> 4);
  const int mm = m < p.M ? m : p.M - 1;
  f32x4 v[NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s2 = 0.f;
  for (int z0 = 0; z0 < nz; z0 += ZG) {
    f32x4 r[ZG][NTB];
    float q[ZG];
#pragma unroll
    for (int u = 0; u < ZG; ++u) {
      const int z = min(z0 + u, nz - 1);
      const float* part = p.slabs + (size_t)z * p.M * p.N + (size_t)mm * p.N;
#pragma unroll
      for (int j = 0; j < NTB; ++j) r[u][j] = *reinterpret_cast<const f32x4*>(part + (nt0 + j) * 16 + nsub);
      q[u] = NORM == 2 ? p.slabs[(size_t)nz * p.M * p.N + (size_t)z * p.M + mm] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < ZG; ++u) {
      if (z0 + u < nz) {
#pragma unroll
        for (int j = 0; j < NTB; ++j) v[j] += r[u][j];
        if constexpr (NORM == 2) s2 += q[u];
      }
    }
  }
  if constexpr (NORM == 2) {
    const float sc = rsqrtf(s2 / (float)p.K + p.eps);
#pragma unroll
    for (int j = 0; j < NTB; ++j) v[j] *= sc;
  }
  epilogue<NTB, EPI, false>(p, v, m, nt0, nsub, EpiPre<NTB>{}, m < p.M);
}

// the combine launch for p.splitk-free callers (gemm_mid.hip)
template <int EPI, int NORM, int NTB>
void launch_prefill_reduce(const GemmParams& p, int nz, hipStream_t st) {
  const int groups = ((p.M + 15) / 16) * (p.N / (16 * NTB));
  GemmParams r = p;
  r.dbg_ts = tl_take("prefill_reduce", (groups + 3) / 4);
  hipLaunchKernelGGL((prefill_reduce_kernel<EPI, NORM, NTB>), dim3((groups + 3) / 4), dim3(256), 0, st, r, nz);
}
#define VG_RED_INST(E)                                                                  \
  template void launch_prefill_reduce<E, 0, 1>(const GemmParams&, int, hipStream_t);   \
  template void launch_prefill_reduce<E, 2, 1>(const GemmParams&, int, hipStream_t);
VG_RED_INST(EPI_BF16)
VG_RED_INST(EPI_F32)
VG_RED_INST(EPI_SILU)
VG_RED_INST(EPI_QKV)
#undef VG_RED_INST

template <int EPI, int NORM, int NTB, int BM = 256, int BN = 128, int WM = 4, int WN = 2, int NS = 3, int SCHED = 0,
          int KS = 2>
static void launch_prefill2_one(const GemmParams& p, int nz, hipStream_t st) {
  constexpr int STAGE = (BN / 16 + BM / 16) * KS * 1024;
  const int blocks = ((p.M + BM - 1) / BM) * (p.N / BN);
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("gemm_prefill2", blocks * nz);
  auto kern = gemm_prefill2_kernel<BM, BN, WM, WN, NS, EPI, NORM, NTB, SCHED, KS>;
  static bool attr = [&] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               NS * STAGE) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(blocks, nz), dim3(64 * WM * WN), NS * STAGE, st, q);
  if (nz > 1) {
    const int groups = ((p.M + 15) / 16) * (p.N / (16 * NTB));
    GemmParams r = p;
    r.dbg_ts = tl_take("prefill_reduce", (groups + 3) / 4);
    hipLaunchKernelGGL((prefill_reduce_kernel<EPI, NORM, NTB>), dim3((groups + 3) / 4), dim3(256), 0, st, r, nz);
  }
}

template <int EPI, int NORM, int NTB, int BM = 256, int BN = 128, int WM = 4, int WN = 2, int NS = 3, int KS = 2>
static void launch_prefill2_cfg(const GemmParams& p, int nz, hipStream_t st) {
  // MFMAs at raised priority (schedule 1): +5-7 % on the 256 x 256 tile, neutral on 256 x 128; the
  // split DMA issue was neutral to negative (profiles/r2_prefill_gemm_sched.log)
  launch_prefill2_one<EPI, NORM, NTB, BM, BN, WM, WN, NS, 1, KS>(p, nz, st);
}

template <int EPI, int NORM, int NTB, int BN = 256>
static void launch_prefill4_cfg(const GemmParams& p, int nz, hipStream_t st) {
  constexpr int STAGE = (BN / 16 + 16) * 2 * 1024;
  const int blocks = ((p.M + 255) / 256) * (p.N / BN);
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("gemm_prefill4", blocks * nz);
  auto kern = gemm_prefill4_kernel<BN, EPI, NORM, NTB>;
  constexpr int LDS = 2 * STAGE + P4_ROWSS + 1024;  // ring + the folded norm's row sums
  static bool attr = [&] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(blocks, nz), dim3(512), LDS, st, q);
  if (nz > 1) {
    const int groups = ((p.M + 15) / 16) * (p.N / (16 * NTB));
    GemmParams r = p;
    r.dbg_ts = tl_take("prefill_reduce", (groups + 3) / 4);
    hipLaunchKernelGGL((prefill_reduce_kernel<EPI, NORM, NTB>), dim3((groups + 3) / 4), dim3(256), 0, st, r, nz);
  }
}

static int cu_count() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      c = 0;
    return c;
  }();
  return n;
}

// persistent 4-phase kernel (whole rounds + the K-split tail), one block per CU; slices = the tail's K
// slices (0: G / R, at least 4 K-tiles each, at most 8). false = not taken (no tail to split, no
// tickets / slot room)
template <int EPI, int NORM, int NTB, int BN>
static bool launch_prefill4sk_cfg(const GemmParams& p, int slices, int max_counters, size_t slab_bytes,
                                  hipStream_t st) {
  constexpr int STAGE = (BN / 16 + 16) * 2 * 1024;
  const int tiles = ((p.M + 255) / 256) * (p.N / BN);
  const int G = cu_count();
  if (G <= 0 || p.counters == nullptr || p.slabs == nullptr) return false;
  const int R = tiles % G, KT = p.K / 64;
  if (R == 0) return false;  // whole rounds: the tile grid is the same schedule
  // S (0: the launcher's choice): the tail in ONE round, S = G / R slices (<= 8). More slices than fit
  // one round (forced, or a tuner candidate) run in several: measured slower at every shape tried but
  // Llama-3-8B qkv_proj (192 tiles x 8 slices: 115 vs 123 us, where the split-K 6 grid + reduce is 108),
  // every contributor pays the drain of its 270 KB partial (r6_prefill_persistent_tail.log)
  int S = slices > 0 ? slices : (G / R > 8 ? 8 : G / R);
  while (S > 1 && KT / S < 4) --S;
  if (S < 1 || R > max_counters || (size_t)R * (S - 1) * p4sk_slot_floats<BN>() * 4 > slab_bytes) return false;
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("gemm_prefill4sk", G);
  auto kern = gemm_prefill4sk_kernel<BN, EPI, NORM, NTB>;
  constexpr int LDS = 2 * STAGE + P4_ROWSS + 1024;  // ring + the folded norm's row sums
  static bool attr = [&] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(G), dim3(512), LDS, st, q, tiles, S);
  return true;
}

template <int BM, int BN, int EPI, int NORM, int NTB>
static void launch_prefill_cfg(const GemmParams& p, int nz, hipStream_t st) {
  constexpr int STAGE = (BN / 16 + BM / 16) * 2 * 1024;
  const int blocks = ((p.M + BM - 1) / BM) * (p.N / BN);
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("gemm_prefill", blocks * nz);
  hipLaunchKernelGGL((gemm_prefill_kernel<BM, BN, EPI, NORM, NTB>), dim3(blocks, nz), dim3(256), 2 * STAGE, st, q);
  if (nz > 1) {
    const int groups = ((p.M + 15) / 16) * (p.N / (16 * NTB));
    GemmParams r = p;
    r.dbg_ts = tl_take("prefill_reduce", (groups + 3) / 4);
    hipLaunchKernelGGL((prefill_reduce_kernel<EPI, NORM, NTB>), dim3((groups + 3) / 4), dim3(256), 0, st, r, nz);
  }
}

// Split-K partials leave with non-temporal stores: dirty fp32 slabs in L2 are written back at the
// kernel boundary and held the next launch back 2-4 us (prefill-step timeline, r4).
// Tile shape: 128 x 128 when that grid covers the chip, else 128 x 64 (narrow N: o_proj,
// down, 70B/TP shards). A grid still under ~200 blocks is split along K (>= 4 stages of 64 per
// slice, <= 8 slices, partials within the workspace) and combined by prefill_reduce_kernel.
// Returns false for shapes the kernel does not take (the caller keeps the N-split tile
// kernel): K % 64, N % 64, a row gather, the gamma-in-registers RMSNorm mode.
template <int EPI, int NORM>
static bool launch_prefill_epi(const GemmParams& p, int force_bn, int force_sk, size_t slab_bytes, int max_counters,
                               hipStream_t st) {
  constexpr int NTB = 1;  // every epilogue works on self-contained 16-column tiles
  if (p.K % 64 != 0 || p.N % 64 != 0 || p.row_idx != nullptr) return false;
  const int mb = (p.M + 127) / 128;
  bool wide = p.N % 128 == 0 && mb * (p.N / 128) >= 240;
  if (force_bn == 128) wide = p.N % 128 == 0;
  if (force_bn == 64) wide = false;
  const int blocks = mb * (p.N / (wide ? 128 : 64));
  int nz = 1;
  if (force_sk > 0) {
    nz = force_sk;
  } else if (blocks < 200) {
    nz = (256 + blocks - 1) / blocks;
    nz = nz > 8 ? 8 : nz;
  }
  const int nk = p.K / 64;
  while (nz > 1 && nk / nz < 4) --nz;
  const size_t need = ((size_t)nz * p.M * p.N + (size_t)nz * p.M) * 4;
  if (nz > 1 && (p.slabs == nullptr || need > slab_bytes)) nz = 1;
  // 256 x 256 when its grid covers ~3/4 of the chip, else v2 (256 x 128, 3-deep ring)
  // when its grid still covers the chip without split-K (profiles/r2_prefill_gemm_sched.log: the
  // 256-square tile +20-35 % at >= 192 blocks, up to -30 % at 128)
  const int blocks_v3 = ((p.M + 255) / 256) * (p.N % 256 == 0 ? p.N / 256 : 0);
  const int blocks_v2 = ((p.M + 255) / 256) * (p.N % 128 == 0 ? p.N / 128 : 0);
  if (force_bn == 0 && force_sk == 0 && blocks_v3 >= 180) {
    // the 4-phase 256 x 256 kernel (v4: +7-22 % over the same tile with one barrier per K-tile,
    // profiles/r2_prefill_gemm_v4.log)
    launch_prefill4_cfg<EPI, NORM, NTB>(p, 1, st);
    return true;
  }
  if (force_bn == 0 && force_sk == 0 && blocks_v2 >= 192) {
    // the 4-phase kernel on 256 x 128 (+0-8 % over the 3-deep-ring v2 at 192-256 blocks,
    // profiles/r2_prefill_gemm_v4.log)
    launch_prefill4_cfg<EPI, NORM, NTB, 128>(p, 1, st);
    return true;
  }
  if (force_bn == 256) {  // forced (tests / sweeps), split-K as chosen above
    if (p.N % 128 != 0) return false;
    launch_prefill2_cfg<EPI, NORM, NTB>(p, nz, st);
    return true;
  }
  if (force_bn == 512) {  // 256 x 256 block tile, 8 waves of 64 (m) x 128 (n), 2-deep ring (sweeps)
    if (p.N % 256 != 0) return false;
    launch_prefill2_cfg<EPI, NORM, NTB, 256, 256, 4, 2, 2>(p, nz, st);
    return true;
  }
  if (force_bn == 1024) {  // v4: the 4-phase 256 x 256 kernel (sweeps / tests)
    if (p.N % 256 != 0) return false;
    launch_prefill4_cfg<EPI, NORM, NTB>(p, nz, st);
    return true;
  }
  // persistent forms of the 4-phase kernel, K-split tail (start-up tuner candidates; force_sk = the
  // tail's K slices); declined -> the tile grid
  if (force_bn == 1025) {
    if (p.N % 256 != 0) return false;
    if (!launch_prefill4sk_cfg<EPI, NORM, NTB, 256>(p, force_sk, max_counters, slab_bytes, st))
      launch_prefill4_cfg<EPI, NORM, NTB>(p, 1, st);
    return true;
  }
  if (force_bn == 769) {
    if (p.N % 128 != 0) return false;
    if (!launch_prefill4sk_cfg<EPI, NORM, NTB, 128>(p, force_sk, max_counters, slab_bytes, st))
      launch_prefill4_cfg<EPI, NORM, NTB, 128>(p, 1, st);
    return true;
  }
  if (force_bn == 768) {  // v4 on a 256 x 128 tile (sweeps / tests)
    if (p.N % 128 != 0) return false;
    launch_prefill4_cfg<EPI, NORM, NTB, 128>(p, nz, st);
    return true;
  }
  // mid-M (128 < M <= 512) tuner candidates: the 128-row tiles on a 4-deep ring, one block per CU
  // (the 2-deep ring above waits vmcnt(0) per K-tile and relies on a second resident block)
  if (force_bn == 1280 || force_bn == 1281) {
    if (p.N % 128 != 0) return false;
    if (force_bn == 1280) launch_prefill2_cfg<EPI, NORM, NTB, 128, 128, 2, 2, 4>(p, nz, st);
    else launch_prefill2_cfg<EPI, NORM, NTB, 128, 128, 2, 4, 4>(p, nz, st);
    return true;
  }
  // wide-N mid-M tiles that fill the chip where the 256- / 128-row tiles leave CUs idle or waste rows
  // (gate_up at 448 rows: 256 x 256 covers 140 of 256 CUs, 128-row tiles make 280 blocks): 64 x 512
  // over 8 waves (448 rows: 7 x 35 = 245 blocks, no padded rows) and 128 x 320 over 8 waves (224)
  if (force_bn == 2560) {
    if (p.N % 512 != 0) return false;
    launch_prefill2_cfg<EPI, NORM, NTB, 64, 512, 1, 8, 2>(p, nz, st);
    return true;
  }
  if (force_bn == 2561) {
    if (p.N % 320 != 0) return false;
    launch_prefill2_cfg<EPI, NORM, NTB, 128, 320, 2, 4, 2>(p, nz, st);
    return true;
  }
  // (the same tiles with 32-deep stages on 4-deep rings measured 15-30 % slower warm and cold:
  // profiles/r5_prefill_wide_tiles_sweep.log)
  if (force_bn == 640 || force_bn == 641) {
    if (force_bn == 640) launch_prefill2_cfg<EPI, NORM, NTB, 128, 64, 2, 2, 4>(p, nz, st);
    else launch_prefill2_cfg<EPI, NORM, NTB, 128, 64, 4, 2, 4>(p, nz, st);
    return true;
  }
  if (wide) launch_prefill_cfg<128, 128, EPI, NORM, NTB>(p, nz, st);
  else launch_prefill_cfg<128, 64, EPI, NORM, NTB>(p, nz, st);
  return true;
}

bool launch_gemm_prefill(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return true;
  const int norm = g.norm_w != nullptr ? 1 : (g.rownorm ? 2 : 0);
  if (norm == 1) return false;
  GemmParams p{};
  p.x = g.x; p.lda = g.lda; p.M = g.M; p.row_idx = g.row_idx;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.norm_w = nullptr; p.eps = g.eps;
  p.bias = g.bias; p.res = g.res; p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.splitk = 1;
  p.slabs = g.slabs;
  p.counters = g.counters; p.fault = g.fault;
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.dbg_ts = g.dbg_ts;
  const int fb = g.ntb;      // reused as the forced tile width (0 = heuristic, 64 / 128)
  const int fs = g.splitk;   // forced K slices (0 = heuristic)
#define VG_PF(E)                                                                                         \
  return norm == 2 ? launch_prefill_epi<E, 2>(p, fb, fs, g.slab_bytes, g.max_counters, st)               \
                   : launch_prefill_epi<E, 0>(p, fb, fs, g.slab_bytes, g.max_counters, st)
  switch (g.epi) {
    case EPI_SILU: VG_PF(EPI_SILU);
    case EPI_QKV: VG_PF(EPI_QKV);
    case EPI_F32: VG_PF(EPI_F32);
    default: VG_PF(EPI_BF16);
  }
#undef VG_PF
}

}  // namespace vgate
