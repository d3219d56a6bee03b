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
          float f[8];
          unpack8(xb[b], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[b] += f[j] * f[j];
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
          float f[8];
          unpack8(xb[b], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[b] += f[j] * f[j];
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
template <int BN, int EPI, int NORM, int NTB>
__global__ __launch_bounds__(512, 1) void gemm_prefill4_kernel(GemmParams p) {
  constexpr int BM = 256, KS = 2;
  constexpr int WTN = BN / 16, XTM = BM / 16;  // W + x tiles per block (16 / 8 + 16)
  constexpr int NWN = WTN / 2, NH = NWN / 2;   // n-tiles per wave, per n-half
  constexpr int STAGE = (WTN + XTM) * KS * 1024;
  constexpr int G0 = 4 * NH + 16, G1 = 16, G2 = 4 * NH;  // pieces per group (block)
  constexpr int P0 = G0 / 8, P1 = G1 / 8, P2 = G2 / 8;  // per wave
  constexpr int PPW = P0 + P1 + P2;
  static_assert(G0 % 8 == 0 && G2 % 8 == 0 && (BN == 256 || BN == 128), "pieces split over 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int KT = p.K >> 5;
  const int nk_all = p.K >> 6;
  const int z = blockIdx.y, nz = gridDim.y;
  const int kst0 = (nk_all * z) / nz, nk = (nk_all * (z + 1)) / nz - kst0;
  const int mblocks = (p.M + BM - 1) / BM;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int m0 = (wgid % mblocks) * BM;
  const int nt_blk = (wgid / mblocks) * WTN;
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
  f32x4 acc[NWN][4];
#pragma unroll
  for (int a = 0; a < NWN; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[4] = {0.f, 0.f, 0.f, 0.f};
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
    if constexpr (NORM == 2) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          float f[8];
          unpack8(xf[ks][b], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[half * 2 + b] += f[j] * f[j];
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
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wc * 64 + b * 16 + (lane & 15);
    float sc = 1.f;
    if constexpr (NORM == 2) {
      float s2 = ss[b];
      s2 += xor16(s2);
      s2 += xor32(s2);
      sc = rsqrtf(s2 / (float)p.K + p.eps);
    }
#pragma unroll
    for (int a = 0; a < NWN; a += NTB) {
      f32x4 v[NTB];
#pragma unroll
      for (int j = 0; j < NTB; ++j) v[j] = acc[a + j][b] * sc;
      epilogue<NTB, EPI, false>(p, v, m, nt_blk + wr * NWN + a, 4 * (lane >> 4), EpiPre<NTB>{}, m < p.M);
    }
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
  static bool attr = [&] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               2 * STAGE) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(blocks, nz), dim3(512), 2 * STAGE, st, q);
  if (nz > 1) {
    const int groups = ((p.M + 15) / 16) * (p.N / (16 * NTB));
    GemmParams r = p;
    r.dbg_ts = tl_take("prefill_reduce", (groups + 3) / 4);
    hipLaunchKernelGGL((prefill_reduce_kernel<EPI, NORM, NTB>), dim3((groups + 3) / 4), dim3(256), 0, st, r, nz);
  }
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
static bool launch_prefill_epi(const GemmParams& p, int force_bn, int force_sk, size_t slab_bytes, hipStream_t st) {
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
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.dbg_ts = g.dbg_ts;
  const int fb = g.ntb;      // reused as the forced tile width (0 = heuristic, 64 / 128)
  const int fs = g.splitk;   // forced K slices (0 = heuristic)
#define VG_PF(E)                                                                                         \
  return norm == 2 ? launch_prefill_epi<E, 2>(p, fb, fs, g.slab_bytes, st)                               \
                   : launch_prefill_epi<E, 0>(p, fb, fs, g.slab_bytes, st)
  switch (g.epi) {
    case EPI_SILU: VG_PF(EPI_SILU);
    case EPI_QKV: VG_PF(EPI_QKV);
    case EPI_F32: VG_PF(EPI_F32);
    default: VG_PF(EPI_BF16);
  }
#undef VG_PF
}

}  // namespace vgate
