// Decode / small-M GEMM kernel templates and their launch logic, shared by the per-epilogue
// translation units (gemm_epi_*.hip) so the ~200 kernel instantiations compile in parallel.
// Design notes: gemm.hip (file comment).
#pragma once
#include <algorithm>
#include <cstdlib>

#include "gemm_epilogue.h"

namespace vgate {

// Rotate a 16-B fragment across lanes within each 16-lane DPP row: lane r <- lane (r + S) % 16.
template <int S>
__device__ __forceinline__ uint4 row_ror(uint4 v) {
  if constexpr (S == 0) {
    return v;
  } else {
    constexpr int ctrl = 0x120 + ((16 - S) & 15);  // DPP row_ror:n moves lane i - n -> lane i
    uint4 r;
    r.x = __builtin_amdgcn_mov_dpp((int)v.x, ctrl, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_mov_dpp((int)v.y, ctrl, 0xf, 0xf, false);
    r.z = __builtin_amdgcn_mov_dpp((int)v.z, ctrl, 0xf, 0xf, false);
    r.w = __builtin_amdgcn_mov_dpp((int)v.w, ctrl, 0xf, 0xf, false);
    return r;
  }
}

// keep v on lanes where m == ~0u, zero elsewhere (component-wise: no struct select)
__device__ __forceinline__ uint4 and_mask(uint4 v, uint32_t m) { return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m); }

// PIPE (decode, MB == 1): ping-pong pipelined stream, <= 8 waves per block so each wave
// may hold 256 VGPRs (two U-deep register groups in flight). Otherwise (prefill tiles):
// one group at a time, up to 16 waves per block at 128 VGPRs.
//
// XP (activation packing, decode only): with M <= 16/XP real rows, ONE 16-B activation
// load per lane covers XP k-steps (lane r of a 16-lane row loads row r % R of k-step
// r / R, R = 16/XP) and the XP B-fragments are rebuilt with DPP row rotations. Every
// vector-memory instruction a CU issues for activations is one it cannot issue for the
// weight stream (measured: benchmarks/stream_probe.hip, +75% time at 96 blocks), so the
// activation side must be as thin as the batch allows.
template <int MB, int NTB, int U, int EPI, int NORM, bool PIPE, int XP>
__global__ __launch_bounds__(PIPE ? 512 : 1024) void gemm_kernel(GemmParams p) {
  static_assert(XP == 1 || (MB == 1 && PIPE && U % XP == 0), "activation packing is a decode-kernel mode");
  constexpr int R = 16 / XP;  // real rows per packed load
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  TLScope tl_scope(p.dbg_ts);
  const int KT = p.K >> 5;
  const SplitPos sp = split_pos(p);
  const int nt0 = (int)blockIdx.x * NTB;
  const int m_base = blockIdx.y * 16 * MB;
  // this block's k-slice, then this wave's contiguous range inside it
  const int s0 = (KT * sp.slice) / sp.nsl, s1 = (KT * (sp.slice + 1)) / sp.nsl;
  const int wr = wid;
  int kbeg = s0 + ((s1 - s0) * wr) / nw;
  int kend = s0 + ((s1 - s0) * (wr + 1)) / nw;
  if constexpr (XP > 1) {  // waves take whole packs of XP k-steps (K % (32 * XP) == 0 on host)
    const int np0 = s0 / XP, np1 = s1 / XP;
    kbeg = XP * (np0 + ((np1 - np0) * wr) / nw);
    kend = XP * (np0 + ((np1 - np0) * (wr + 1)) / nw);
  }
  f32x4 acc[MB][NTB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NTB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint4* wbase[NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) wbase[j] = p.wp + ((size_t)(nt0 + j) * KT) * 64 + lane;
  // Rows >= M (the 16-row MFMA tile is padded for decode batches < 16) are zero and never
  // loaded. Under XP packing lane r loads row r % R at k-step offset r / R.
  const bf16_t* xrow[MB];
  bool xok[MB];
  float ssr[MB];
  const int r16 = lane & 15;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m_base + mb * 16 + (XP > 1 ? r16 % R : r16);
    xok[mb] = m < p.M;
    xrow[mb] = p.x + (size_t)row_of(p, m) * p.lda + 8 * (lane >> 4) + (XP > 1 ? (r16 / R) * 32 : 0);
    // NORM 3: the producer's per-tile sums of squares of row (lane & 15), issued with the first
    // weight group and used only in gemm_finish (wave 0 of slice 0 carries them)
    ssr[mb] = (NORM == 3 && wid == 0 && sp.slice == 0) ? prenorm_ss(p, m_base + mb * 16 + r16, lane >> 4) : 0.f;
  }
  const bf16_t* nw_ptr = p.norm_w ? p.norm_w + 8 * (lane >> 4) : nullptr;

  // Software-pipelined weight stream (ping-pong register groups of U k-steps): group
  // g+1's weights AND activations are issued before group g is consumed, so the wait
  // for g is a partial vmcnt that leaves g+1 in flight (issue order = wait order).
  auto load_grp = [&](uint4 (&b)[U][NTB], uint4 (&a)[U][MB], int k0) {
    // a partial last group re-reads the last k-step / pack (clamped, so the issue stays
    // unconditional); mma_grp zeroes those steps' activations
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NTB; ++j) b[u][j] = ld_nt16(wbase[j] + (size_t)min(k0 + u, kend - 1) * 64);
#pragma unroll
    for (int u = 0; u < U; u += XP)  // packed: slot u holds the raw load for k-steps u..u+XP-1
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        a[u][mb] = xok[mb] ? *reinterpret_cast<const uint4*>(xrow[mb] + min(k0 + u, kend - XP) * 32)
                           : make_uint4(0, 0, 0, 0);
  };
  auto unpack_grp = [&](uint4 (&a)[U][MB]) {
    if constexpr (XP > 1) {
      const uint32_t lom = r16 < R ? ~0u : 0u;
#pragma unroll
      for (int u = 0; u < U; u += XP) {
        // the DPP reads lanes r >= R: evaluate it with every lane active, select after
        const uint4 v = a[u][0];
        const uint4 v1 = row_ror<R>(v);
        a[u][0] = and_mask(v, lom);
        a[u + 1][0] = and_mask(v1, lom);
        if constexpr (XP == 4) {
          const uint4 v2 = row_ror<2 * R>(v), v3 = row_ror<3 * R>(v);
          a[u + 2][0] = and_mask(v2, lom);
          a[u + 3][0] = and_mask(v3, lom);
        }
      }
    }
  };
  auto mma_grp = [&](const uint4 (&b)[U][NTB], uint4 (&a)[U][MB], int k0) {
    unpack_grp(a);
#pragma unroll
    for (int u = 0; u < U; ++u)  // steps past this wave's range (partial last group) add 0
      if (k0 + u >= kend)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) a[u][mb] = make_uint4(0, 0, 0, 0);
    if constexpr (NORM == 1 || NORM == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) a[u][mb] = norm_frag<NORM>(a[u][mb], nw_ptr, min(k0 + u, kend - 1) * 32, ssr[mb]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NTB; ++j)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(as_bf16x8(b[u][j]), as_bf16x8(a[u][mb]), acc[mb][j]);
  };
  // epilogue operands of this thread's (row, 4 columns) item (decode: wave 0 runs the epilogue)
  EpiPre<NTB> pre;  // (two tiles' words: blocks of 4 tiles load theirs in the epilogue)
  constexpr bool PREF = MB == 1 && NTB <= 2;
  const bool epi_thr = PREF && threadIdx.x < 64;
  if (epi_thr) epi_pre_a<NTB, EPI>(p, pre, m_base + r16, nt0, 4 * (lane >> 4));
  bool pre_b = false;
  // Whole groups of U k-steps, the last one possibly partial: no serial tail, so a wave
  // with ngrp <= 2 waits on ONE round trip (e.g. the QKV projection: 6 steps per wave)
  int kt = kbeg;
  const int ngrp = (kend - kbeg + U - 1) / U;
  if constexpr (!PIPE) {
    for (int g = 0; g < ngrp; ++g, kt += U) {
      uint4 b[U][NTB], a[U][MB];
      load_grp(b, a, kt);
      mma_grp(b, a, kt);
    }
  } else if (ngrp > 0) {
    // group g of the wave starts at k-step gk(g)
    auto gk = [&](int g) { return kbeg + g * U; };
    uint4 b0[U][NTB], a0[U][MB], b1[U][NTB], a1[U][MB];
    load_grp(b0, a0, gk(0));
    if (epi_thr) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));  // dependent on phase A only
    pre_b = true;
    int g = 0;
    for (; g + 2 <= ngrp; g += 2) {
      load_grp(b1, a1, gk(g + 1));
      mma_grp(b0, a0, gk(g));
      if (g + 2 < ngrp) load_grp(b0, a0, gk(g + 2));
      mma_grp(b1, a1, gk(g + 1));
    }
    if (g < ngrp) mma_grp(b0, a0, gk(g));
  }
  if (epi_thr && !pre_b) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));
  gemm_finish<MB, NTB, EPI, NORM, PREF>(p, acc, ssr, smem, m_base, nt0, pre);
}

// ---- AWQ W4A16 ----
// nibble order of ops.pack_awq: value j at bit (16 if j odd) + 4 (j >> 1)
__device__ __forceinline__ bf16x8 dq8(uint32_t q, float s, float sz) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)((float)((q >> ((j & 1) * 16 + 4 * (j >> 1))) & 0xF) * s - sz);
  return r;
}

// the 8 raw values as bf16 (128 + v): the group scale is applied after the MFMA
// (sum_k x (128 + v) s - (128 s + s z) sum_k x = sum_k x (v - z) s)
__device__ __forceinline__ bf16x8 raw8(uint32_t q) {
  uint4 r;
  r.x = (q & 0x000F000Fu) | 0x43004300u;
  r.y = ((q >> 4) & 0x000F000Fu) | 0x43004300u;
  r.z = ((q >> 8) & 0x000F000Fu) | 0x43004300u;
  r.w = ((q >> 12) & 0x000F000Fu) | 0x43004300u;
  return as_bf16x8(r);
}

template <int MB, int NTB, int EPI, int NORM, int QC_ = 0>
__global__ __launch_bounds__(512) void awq_gemm_kernel(GemmParams p) {  // <= 8 waves: 256 VGPRs for the chunked loads
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int KQ = p.K >> 7;
  const int nt0 = blockIdx.x * NTB;
  const int m_base = blockIdx.y * 16 * MB;
  const int s0 = (KQ * blockIdx.z) / p.splitk, s1 = (KQ * (blockIdx.z + 1)) / p.splitk;
  const int qbeg = s0 + ((s1 - s0) * wid) / nw;
  const int qend = s0 + ((s1 - s0) * (wid + 1)) / nw;
  f32x4 acc[MB][NTB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NTB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Rows >= M (the 16-row MFMA tile is padded for decode batches < 16) are zero and never
  // loaded: on a 96-block GEMM every activation byte is a weight byte the CU cannot stream.
  const bf16_t* xrow[MB];
  bool xok[MB];
  float ssr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m_base + mb * 16 + (lane & 15);
    xok[mb] = m < p.M;
    xrow[mb] = p.x + (size_t)row_of(p, m) * p.lda + 8 * (lane >> 4);
    // NORM 3: the producer's sums of squares (wave 0 of slice 0 carries them into gemm_finish)
    ssr[mb] = (NORM == 3 && wid == 0 && blockIdx.z == 0) ? prenorm_ss(p, m, lane >> 4) : 0.f;
  }
  const bf16_t* nw_ptr = p.norm_w ? p.norm_w + 8 * (lane >> 4) : nullptr;
  // Chunks of up to QC k-quads: EVERY load of a chunk (int4 weights, activations, RMSNorm
  // gamma, group scales / zeros) is issued before any is consumed, so a wave's k-range costs
  // ceil(n / QC) memory round trips instead of one per k-quad — in the engine the
  // activations arrive cold from the previous kernel (qkv 9.8 -> see profiles/r1_awq_*).
  // QC_ > 0: the launcher's chunk size (3 when every wave owns 3 k-quads: no clamped re-load)
  constexpr int QC = QC_ > 0 ? QC_ : (MB == 1 ? 4 : (MB == 2 ? 2 : 1));
  for (int kc = qbeg; kc < qend; kc += QC) {
    uint4 w[QC][NTB];
    uint4 a[QC][4][MB];
    uint4 gm[QC][4];
    float sc[QC][NTB][4], zc[QC][NTB][4];
#pragma unroll
    for (int c = 0; c < QC; ++c) {
      const int kq = min(kc + c, qend - 1);  // clamped re-load past the end: never consumed
#pragma unroll
      for (int j = 0; j < NTB; ++j) w[c][j] = ld_nt16(p.wp + ((size_t)(nt0 + j) * KQ + kq) * 64 + lane);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          a[c][u][mb] = xok[mb] ? *reinterpret_cast<const uint4*>(xrow[mb] + (kq * 4 + u) * 32) : make_uint4(0, 0, 0, 0);
        if constexpr (NORM == 1) gm[c][u] = *reinterpret_cast<const uint4*>(nw_ptr + (kq * 4 + u) * 32);
      }
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        const int n = (nt0 + j) * 16 + (lane & 15);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int gi = ((kq * 4 + u) * 32 + 8 * (lane >> 4)) / p.group;
          sc[c][j][u] = bf2f(p.scales[(size_t)gi * p.N + n]);
          zc[c][j][u] = bf2f(p.zeros[(size_t)gi * p.N + n]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < QC; ++c) {
      if (kc + c >= qend) break;  // wave-uniform
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          if constexpr (NORM == 1 || NORM == 2) {
            float f[8], g[8];
            unpack8(a[c][u][mb], f);
#pragma unroll
            for (int j = 0; j < 8; ++j) ssr[mb] += f[j] * f[j];
            if constexpr (NORM == 1) {
              unpack8(gm[c][u], g);
#pragma unroll
              for (int j = 0; j < 8; ++j) f[j] *= g[j];
              a[c][u][mb] = pack8(f);
            }
          }
        }
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        const uint32_t wq[4] = {w[c][j].x, w[c][j].y, w[c][j].z, w[c][j].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bf16x8 wf = dq8(wq[u], sc[c][j][u], zc[c][j][u]);
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(wf, as_bf16x8(a[c][u][mb]), acc[mb][j]);
        }
      }
    }
  }
  gemm_finish<MB, NTB, EPI, NORM, false>(p, acc, ssr, smem, m_base, nt0, EpiPre<NTB>{});
}

// ---- AWQ W4A16 decode (M <= 16): every weight byte of the launch in flight at once ----
// int4 decode is pure latency x bytes-in-flight: 13.8 MB of gate_up int4 at ~2 us of HBM
// latency needs ~12 MB outstanding to run at 6 TB/s (Little's law). The previous kernel
// pipelined 2 k-quads per wave (16 KB per block, 140 blocks: 2.2 MB in flight -> 1.0 TB/s,
// profiles/r1_awq_bench_kernel_summary.txt). Here each wave owns NTW tiles x the block's
// k-slice (<= AQ_KQ k-quads) and issues ALL of its int4 fragments and packed group scales
// before the first MFMA; a launch covers every tile, so the whole matrix is requested in the
// first ~microsecond.
//
// Block = AD_WAVES waves x NTW tiles; grid.z = K slices. The activation slice is staged ONCE
// per block into LDS in MFMA B-fragment order (RMSNorm gamma applied while staging; the row sum
// of squares over the FULL row so a K-slice needs no ssq hand-off) with the per-(k-quad, row)
// activation sums X that the raw-nibble trick needs:
//   sum_k x (v - z) s = s * sum_k x (128 + v)  -  (128 s + s z) * X       (one group per k-quad)
// where (128 + v) is built as bf16 straight from the nibbles (raw8, 4 ALU per 8 weights).
// Group scales arrive fragment-packed (ops.pack_awq_sz: [nt][kq][lane group][s0..3, sz0..3]):
// ONE 16-B load per (tile, k-quad) instead of two 8-B ones. Split-K slices meet at a per-group
// ticket (sc1 slabs, last arriver sums).
constexpr int AD_WAVES = 4;
constexpr int AQ_KQ = 12;      // (k-quads per slice) x NTW held in flight: 2 x 12 uint4 per lane
constexpr int AD_SK_MAX = 16;  // split-K slices

template <int NTW, int EPI, int NORM>
__global__ __launch_bounds__(256, 1) void awq_dec_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  // profiling: phase stamps of the first and the last block after the per-block slots
  // (benchmarks/awq_sweep.py; the launcher reserves 8 extra slot pairs)
  const size_t nblk = (size_t)gridDim.x * gridDim.y * gridDim.z;
  const size_t bid = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  unsigned long long* ph = (p.dbg_ts != nullptr && threadIdx.x == 0 && (bid == 0 || bid == nblk - 1))
                               ? p.dbg_ts + 2 * nblk + (bid == 0 ? 0 : 8) : nullptr;
#define AD_PHASE(i) do { if (ph != nullptr) ph[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
  AD_PHASE(0);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int KQ = p.K >> 7;
  const int nt0 = (blockIdx.x * AD_WAVES + wid) * NTW;  // this wave's first 16-column tile
  const int q0 = (KQ * blockIdx.z) / p.splitk, q1 = (KQ * (blockIdx.z + 1)) / p.splitk;
  const int nq = q1 - q0, nst = nq * 4;  // k-quads / k-steps of the slice (nq <= AQ_KQ / NTW, host-checked)
  constexpr int GQ = AQ_KQ / NTW;        // k-quads held per wave
  uint4* xs = reinterpret_cast<uint4*>(smem);                             // [nst][64] B fragments
  float* xsum = reinterpret_cast<float*>(smem + (size_t)nst * 64 * 16);  // [nq][4 waves][16] row-sum partials
  float* ssq = xsum + nq * 64;                                            // [4 waves][16] slice sums of squares
  int* flag = reinterpret_cast<int*>(ssq + 4 * 16);
  const int m = lane & 15, nsub = 4 * (lane >> 4);
  // 1) activation slice -> registers (issued first: the staging below waits for these alone and
  //    leaves every weight load in flight). Thread t stages fragment f = i * 256 + t: lane t & 63,
  //    k-step 4i + (t >> 6).
  constexpr int XMAX = GQ;  // k-steps per thread (4 waves x XMAX = 4 GQ k-steps)
  // Loads are UNCONDITIONAL (clamped k-step, value masked after the load): a load behind a
  // runtime branch makes the compiler give up its vmcnt count and wait for EVERY outstanding
  // load — all the weights below — before the staging (measured: 6 us blocks for 48 KB).
  uint4 xr[XMAX];
  const bf16_t* xrow = p.x + (size_t)row_of(p, min(m, p.M - 1)) * p.lda + 8 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < XMAX; ++i) xr[i] = ld16(xrow + (q0 * 4 + min(4 * i + wid, nst - 1)) * 32);
  uint4 gr[NORM == 1 ? XMAX : 1];
  if constexpr (NORM == 1) {
#pragma unroll
    for (int i = 0; i < XMAX; ++i) gr[i] = ld16(p.norm_w + (q0 * 4 + min(4 * i + wid, nst - 1)) * 32 + 8 * (lane >> 4));
  }
  // x first, ALONE: issued together with the weights, every CU's x requests queue behind the
  // whole launch's weight misses and the staging starts only when the weights have landed
  // (x staged at 4.5 us of a 7 us block, benchmarks/awq_phases.py); one L2 / MALL round trip
  // up front instead lets the staging overlap the weight stream
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // 2) the wave's whole weight slice + its packed group scales, all issued now (indices past the
  //    slice re-read its last k-quad: issued unconditionally, never consumed)
  uint4 w[GQ][NTW], sz[GQ][NTW];
  const uint4* szp = reinterpret_cast<const uint4*>(p.szp);  // [N/16][KQ][4][16 B]
#pragma unroll
  for (int g = 0; g < GQ; ++g) {
    const int kq = q0 + min(g, nq - 1);
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      w[g][j] = ld_nt16(p.wp + ((size_t)(nt0 + j) * KQ + kq) * 64 + lane);
      sz[g][j] = szp[((size_t)(nt0 + j) * KQ + kq) * 4 + (lane >> 4)];
    }
  }
  // 3) the activation image (x * gamma under NORM == 1), this wave's slice sum of squares and the
  //    per-(k-quad, row) activation sums X, all from registers: k-quad i is exactly the 4 k-steps
  //    4i + wave of the four waves, so X = sum over (8 elements, 4 lane groups, 4 waves)
  float* xsw = xsum;  // [nq][4 waves][16] partial sums, folded over the waves in step 4
  const bool mok = m < p.M;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < XMAX; ++i) {
    const int t = 4 * i + wid;
    uint4 v = (mok && i < nq) ? xr[i] : make_uint4(0, 0, 0, 0);  // clamped duplicates past the slice add 0
    float a[8];
    unpack8(v, a);
    if constexpr (NORM != 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
      if constexpr (NORM == 1) {
        float g8[8];
        unpack8(gr[i], g8);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] *= g8[j];
        v = pack8(a);
        unpack8(v, a);  // X must sum the bf16 values the MFMA sees
      }
    }
    float xs8 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) xs8 += a[j];
    xs8 += xor16(xs8);
    xs8 += xor32(xs8);
    if (i < nq) {  // wave-uniform (stores only)
      xs[t * 64 + lane] = v;
      if (lane < 16) xsw[(i * 4 + wid) * 16 + lane] = xs8;
    }
  }
  if constexpr (NORM != 0) {
    ss += xor16(ss);
    ss += xor32(ss);
    if (lane < 16) ssq[wid * 16 + lane] = ss;
  }
  AD_PHASE(1);
  lds_barrier();  // LDS image visible; the weight loads stay in flight
  AD_PHASE(2);
  // 4) consume in issue order (the compiler's vmcnt waits stay partial: k-quad g needs only
  //    the loads issued before it)
  f32x4 acc[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < GQ; ++g) {
    // predicated, not `break`: a multi-exit loop is not fully unrolled at GQ = 12 and the
    // register arrays w / sz then live in scratch (400 B per lane)
    if (g < nq) {  // wave-uniform
    f32x4 pr[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) pr[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bf16x8 xb = as_bf16x8(xs[(g * 4 + u) * 64 + lane]);
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const uint32_t q = u == 0 ? w[g][j].x : u == 1 ? w[g][j].y : u == 2 ? w[g][j].z : w[g][j].w;
        pr[j] = mfma16(raw8(q), xb, pr[j]);
      }
    }
    const float X = ((xsw[(g * 4 + 0) * 16 + m] + xsw[(g * 4 + 1) * 16 + m]) + xsw[(g * 4 + 2) * 16 + m]) +
                    xsw[(g * 4 + 3) * 16 + m];  // fixed wave order
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const float s4[4] = {bf_lo(sz[g][j].x), bf_hi(sz[g][j].x), bf_lo(sz[g][j].y), bf_hi(sz[g][j].y)};
      const float z4[4] = {bf_lo(sz[g][j].z), bf_hi(sz[g][j].z), bf_lo(sz[g][j].w), bf_hi(sz[g][j].w)};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(s4[i], pr[j][i], fmaf(-fmaf(128.f, s4[i], z4[i]), X, acc[j][i]));
    }
  }
  }
  AD_PHASE(3);
  // 5) finish: lane holds D[n = 4(l>>4) + i][m = l & 15] of each tile
  float ss_slice = 0.f;  // this slice's row sum of squares (fixed wave order)
  if constexpr (NORM != 0) {
#pragma unroll
    for (int ww = 0; ww < AD_WAVES; ++ww) ss_slice += ssq[ww * 16 + m];
  }
  auto finish = [&](f32x4 (&v)[NTW], float ss_row) {
    if constexpr (NORM != 0) {
      const float rs = rsqrtf(ss_row / (float)p.K + p.eps);
#pragma unroll
      for (int j = 0; j < NTW; ++j) v[j] *= rs;
    }
    epilogue<NTW, EPI, false>(p, v, m, nt0, nsub, EpiPre<NTW>{}, m < p.M);
  };
  if (p.splitk == 1) {
    finish(acc, ss_slice);
    AD_PHASE(4);
    return;
  }
  const int grp = blockIdx.x;  // column group: AD_WAVES * NTW tiles
  constexpr int SLOTS = AD_WAVES * NTW * 64;
  constexpr int SLAB = SLOTS * 4 + 16;  // floats per (group, slice): tiles + per-row ssq
  float* slab = p.slabs + ((size_t)grp * p.splitk + blockIdx.z) * SLAB;
  const uint32_t slab_off = (uint32_t)(((size_t)grp * p.splitk + blockIdx.z) * SLAB * 4);  // bytes
#pragma unroll
  for (int j = 0; j < NTW; ++j) st_sc1_x4(p.slabs, slab_off + (uint32_t)((wid * NTW + j) * 64 + lane) * 16u, acc[j]);
  if (NORM != 0 && wid == 0 && lane < 16) st_sc1(slab + SLOTS * 4 + lane, ss_slice);
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(p.counters + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (uint32_t)(p.splitk - 1);
    if (last) __hip_atomic_store(p.counters + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  const float* all = p.slabs + (size_t)grp * p.splitk * SLAB;
  const uint32_t all_off = (uint32_t)((size_t)grp * p.splitk * SLAB * 4);
  f32x4 v[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    f32x4 r[AD_SK_MAX];
#pragma unroll
    for (int z = 0; z < AD_SK_MAX; ++z)
      r[z] = ld_sc1_x4(p.slabs, all_off + (uint32_t)(min(z, p.splitk - 1) * SLAB * 4 + ((wid * NTW + j) * 64 + lane) * 16));
    f32x4 t = r[0];
#pragma unroll
    for (int z = 1; z < AD_SK_MAX; ++z)
      if (z < p.splitk) t += r[z];
    v[j] = t;
  }
  float ss_row = 0.f;
  if constexpr (NORM != 0) {
    float sv[AD_SK_MAX];
#pragma unroll
    for (int z = 0; z < AD_SK_MAX; ++z) sv[z] = ld_sc1(all + (size_t)min(z, p.splitk - 1) * SLAB + SLOTS * 4 + m);
    ss_row = sv[0];
#pragma unroll
    for (int z = 1; z < AD_SK_MAX; ++z)
      if (z < p.splitk) ss_row += sv[z];
  }
  finish(v, ss_row);
  AD_PHASE(5);
#undef AD_PHASE
}

// ---- AWQ W4A16 decode, weight-streaming form (M <= 16) ----
// The bf16 decode kernel's decomposition applied to int4: a block = ONE 16-column tile, its
// waves split K, every wave streams its own k-quads with software-pipelined (ping-pong) groups
// of U k-quads: int4 fragment + packed (s, s*z) + its own activation fragments per k-quad, all
// issued one group ahead. No LDS staging (the staged kernel's x round trip sat on every
// block's critical path: x staged 3.6-4.5 us into a 7 us block, benchmarks/awq_phases.py), no
// per-block xsum pass: the per-(k-quad, row) activation sum X of the raw-nibble identity
//   sum_k x (v - z) s = s * sum_k x (128 + v) - (128 s + s z) * X
// comes from the fragments already in registers (8 values per lane per k-step, folded over the
// 4 lane groups with two cross-lane adds). XP activation packing (M <= 16/XP rows: one 16-B load
// covers XP k-steps) as in gemm_kernel. Cross-wave reduction, deferred RMSNorm row scale,
// split-K slabs and the epilogue are gemm_finish's.
//
// NTB > 1: a block owns NTB adjacent tiles and every wave streams its k-quads of all of them with
// ONE set of activation loads. At M = 8 a k-quad's activations (2 KiB per wave) outweigh its int4
// tile fragment (1 KiB), so one-tile blocks move twice as many activation bytes through the CU as
// weight bytes; NTB = 4 cuts that to half.
template <int U, int EPI, int NORM, int XP, bool PP, int NTB>
__global__ __launch_bounds__(512) void awq_stream_kernel(GemmParams p) {
  static_assert(NTB == 1 || (!PP && EPI != EPI_QKV), "multi-tile blocks: one-group form, tiles without partners");
  constexpr int R = 16 / XP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int KQ = p.K >> 7;
  const SplitPos sp = split_pos(p);
  const int nt0 = (int)blockIdx.x * NTB;
  const int s0 = (KQ * sp.slice) / sp.nsl, s1 = (KQ * (sp.slice + 1)) / sp.nsl;
  const int qbeg = s0 + ((s1 - s0) * wid) / nw;
  const int qend = s0 + ((s1 - s0) * (wid + 1)) / nw;
  const int r16 = lane & 15;
  const int mrow = XP > 1 ? r16 % R : r16;
  const bool xok = mrow < p.M;
  const bf16_t* xrow = p.x + (size_t)row_of(p, mrow) * p.lda + 8 * (lane >> 4) + (XP > 1 ? (r16 / R) * 32 : 0);
  const uint4* wbase = p.wp + (size_t)nt0 * KQ * 64 + lane;
  const uint4* szbase = reinterpret_cast<const uint4*>(p.szp) + (size_t)nt0 * KQ * 4 + (lane >> 4);
  // RMSNorm gamma (NORM == 1): packed exactly like the activations (it depends on the column only),
  // loaded with them one group ahead and applied before the unpack
  const bf16_t* grow = p.norm_w ? p.norm_w + 8 * (lane >> 4) + (XP > 1 ? (r16 / R) * 32 : 0) : nullptr;
  f32x4 acc[1][NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // NORM 3: the producer's sums of squares of row r16 (wave 0 of slice 0 carries them into gemm_finish)
  // (NORM 3: the producer's sums of squares are read after the stream, by wave 0 of slice 0, so
  // their loads never hold back the first weight group)
  float ssr[1] = {0.f};
  constexpr int XL = 4 / XP;  // activation loads per k-quad
  const uint32_t lom = r16 < R ? ~0u : 0u;
  constexpr int GL = NORM == 1 ? XL : 1;
  auto load_grp = [&](uint4 (&w)[U][NTB], uint4 (&sz)[U][NTB], uint4 (&xa)[U][XL], uint4 (&ga)[U][GL], int kq0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kq = min(kq0 + u, qend - 1);  // clamped: issued unconditionally, masked in mma
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        w[u][j] = ld_nt16(wbase + ((size_t)j * KQ + kq) * 64);
        sz[u][j] = szbase[((size_t)j * KQ + kq) * 4];
      }
#pragma unroll
      for (int v = 0; v < XL; ++v)
        xa[u][v] = xok ? *reinterpret_cast<const uint4*>(xrow + (kq * 4 + v * XP) * 32) : make_uint4(0, 0, 0, 0);
      if constexpr (NORM == 1) {
#pragma unroll
        for (int v = 0; v < XL; ++v) ga[u][v] = *reinterpret_cast<const uint4*>(grow + (kq * 4 + v * XP) * 32);
      }
    }
  };
  // the 4 unpacked B fragments of one k-quad from its XP-packed loads
  auto unpack4 = [&](const uint4 (&src)[XL], uint4 (&b)[4]) {
#pragma unroll
    for (int v = 0; v < XL; ++v) {
      const uint4 t = src[v];
      if constexpr (XP == 1) {
        b[v] = t;
      } else {
        b[v * XP] = and_mask(t, lom);
        b[v * XP + 1] = and_mask(row_ror<R>(t), lom);
        if constexpr (XP == 4) {
          b[v * XP + 2] = and_mask(row_ror<2 * R>(t), lom);
          b[v * XP + 3] = and_mask(row_ror<3 * R>(t), lom);
        }
      }
    }
  };
  auto mma_grp = [&](const uint4 (&w)[U][NTB], const uint4 (&sz)[U][NTB], const uint4 (&xa)[U][XL],
                     const uint4 (&ga)[U][GL], int kq0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kq = kq0 + u;
      const bool live = kq < qend;  // wave-uniform: a partial last group adds nothing
      uint4 b[4];
      if constexpr (NORM == 1) {
        // sum of squares over the RAW activations (unpacked: lane l <-> row l & 15, as
        // gemm_finish folds it), the MFMA operand is bf16(x * gamma)
        uint4 raw[4];
        unpack4(xa[u], raw);
        uint4 xg[XL];
#pragma unroll
        for (int v = 0; v < XL; ++v) {
          float f[8], g8[8];
          unpack8(xa[u][v], f);
          unpack8(ga[u][v], g8);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] *= g8[j];
          xg[v] = pack8(f);
        }
        unpack4(xg, b);
        if (live) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            float f[8];
            unpack8(raw[t], f);
#pragma unroll
            for (int j = 0; j < 8; ++j) ssr[0] += f[j] * f[j];
          }
        }
      } else {
        unpack4(xa[u], b);
      }
      if (!live) {
#pragma unroll
        for (int t = 0; t < 4; ++t) b[t] = make_uint4(0, 0, 0, 0);
      }
      float X = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float f[8];
        unpack8(b[t], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) X += f[j];
      }
      X += xor16(X);
      X += xor32(X);
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        f32x4 pr = {0.f, 0.f, 0.f, 0.f};
        pr = mfma16(raw8(w[u][j].x), as_bf16x8(b[0]), pr);
        pr = mfma16(raw8(w[u][j].y), as_bf16x8(b[1]), pr);
        pr = mfma16(raw8(w[u][j].z), as_bf16x8(b[2]), pr);
        pr = mfma16(raw8(w[u][j].w), as_bf16x8(b[3]), pr);
        const uint4 q = sz[u][j];
        const float s4[4] = {bf_lo(q.x), bf_hi(q.x), bf_lo(q.y), bf_hi(q.y)};
        const float z4[4] = {bf_lo(q.z), bf_hi(q.z), bf_lo(q.w), bf_hi(q.w)};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[0][j][i] = fmaf(s4[i], pr[i], fmaf(-fmaf(128.f, s4[i], z4[i]), X, acc[0][j][i]));
      }
    }
  };
  int kq = qbeg;
  const int ngrp = (qend - qbeg + U - 1) / U;
  // epilogue operands of wave 0's (row, 4 columns) item at launch, as gemm_kernel does: the
  // residual / bias words and the QKV position -> cos/sin chain leave with the weight stream
  // instead of adding one or two dependent round trips after the reduction
  // (EpiPre holds two tiles' words: blocks of 4 tiles load theirs in the epilogue)
  constexpr bool PREF = NTB <= 2;
  EpiPre<NTB> pre;
  const bool epi_thr = PREF && threadIdx.x < 64;
  if (epi_thr) epi_pre_a<NTB, EPI>(p, pre, r16, nt0, 4 * (lane >> 4));
  if constexpr (!PP) {
    // ONE group covering the wave's whole k-range (host-checked: <= U k-quads): every load of
    // the wave in flight at once, one memory round trip per block
    uint4 wa[U][NTB], sa[U][NTB], xa[U][XL], gaa[U][GL];
    load_grp(wa, sa, xa, gaa, kq);
    if (epi_thr) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));
    mma_grp(wa, sa, xa, gaa, kq);
  } else if (ngrp > 0) {
    uint4 wa[U][NTB], sa[U][NTB], xa[U][XL], gaa[U][GL], wb[U][NTB], sb[U][NTB], xb[U][XL], gab[U][GL];
    load_grp(wa, sa, xa, gaa, kq);
    if (epi_thr) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));
    int g = 0;
    for (; g + 2 <= ngrp; g += 2) {
      load_grp(wb, sb, xb, gab, kq + U);
      mma_grp(wa, sa, xa, gaa, kq);
      if (g + 2 < ngrp) load_grp(wa, sa, xa, gaa, kq + 2 * U);
      mma_grp(wb, sb, xb, gab, kq + U);
      kq += 2 * U;
    }
    if (g < ngrp) mma_grp(wa, sa, xa, gaa, kq);
  }
  if constexpr (PP) {
    if (ngrp <= 0 && epi_thr) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));
  }
  if constexpr (NORM == 3) {
    if (wid == 0 && sp.slice == 0) ssr[0] = prenorm_ss(p, r16, lane >> 4);
  }
  gemm_finish<1, NTB, EPI, NORM, PREF>(p, acc, ssr, smem, 0, nt0, pre);
}

// ---- prefill / medium-M tile GEMM (M > 16, bf16 weights) ----
// The decode kernels split K across the waves of a block, which is right when x is a
// few rows; once M grows, every wave would re-load x for its own k-range (the activation
// requests then outnumber the weight requests). Here the waves of a block split N
// instead and SHARE one LDS copy of x: block tile = 64 rows x (4 waves x NTW x 16) cols,
// x staged through a double-buffered LDS ring of KS k-steps (fragment-major, so each
// lane's B operand is one conflict-free ds_read_b128), weights stream straight to
// registers (each weight fragment is used by exactly one wave, for 4 m-tiles), software-
// pipelined one k-step ahead. For M > 64 the grid tiles M (the 256 MB MALL absorbs the
// repeated weight reads of a prompt-sized M).
constexpr int TG_WAVES = 4;   // waves per block
constexpr int TG_MB = 4;      // 16-row m-tiles per block (64 rows)
constexpr int TG_KS = 8;      // k-steps per LDS stage
constexpr int TG_STAGE_BYTES = TG_KS * TG_MB * 64 * 16;  // 32 KiB

template <int NTW, int EPI, int NORM>
__global__ __launch_bounds__(256) void gemm_tile_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  uint4* xs = reinterpret_cast<uint4*>(smem);  // [2][KS][MB][64] fragments
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int KT = p.K >> 5;
  // 1-D grid, XCD-aware: consecutive hardware block ids round-robin over the 8 XCDs (own L2
  // each), so give every XCD one contiguous range of logical tiles, m-chunk fastest — the
  // m-chunks that share a weight slab then run together on one XCD and read it from HBM once
  const int mchunks = (p.M + 16 * TG_MB - 1) / (16 * TG_MB);
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int nt0 = ((wgid / mchunks) * TG_WAVES + wid) * NTW;
  const int m_base = (wgid % mchunks) * 16 * TG_MB;
  const uint4* wbase[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) wbase[j] = p.wp + ((size_t)(nt0 + j) * KT) * 64 + lane;
  const bf16_t* nw_ptr = p.norm_w ? p.norm_w + 8 * (lane >> 4) : nullptr;
  f32x4 acc[TG_MB][NTW];
#pragma unroll
  for (int a = 0; a < TG_MB; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssr[TG_MB];
#pragma unroll
  for (int mb = 0; mb < TG_MB; ++mb) ssr[mb] = 0.f;

  // cooperative stage load: 256 threads x 16 B; fragment (kt, mb, l) <- x[row][col..+8]
  constexpr int STAGE_FRAGS = TG_KS * TG_MB * 64;  // 16-B pieces per stage (2048)
  // thread t always stages the same x row (fragment f = i*256 + t: lane t&63, m-tile t>>6,
  // k-step i), so its row pointer is resolved once. Loads are clamped and unconditional (a
  // guarded load makes the compiler wait vmcnt(0) on it): rows past M repeat row M-1
  // (masked in the epilogue), k-steps past K are skipped by compute()
  static_assert(STAGE_FRAGS / 256 == TG_KS && TG_MB == TG_WAVES, "stage mapping");
  const bf16_t* xrow = p.x + (size_t)row_of(p, min(m_base + wid * 16 + (lane & 15), p.M - 1)) * p.lda +
                       8 * (lane >> 4);
  auto load_stage = [&](uint4 (&r)[STAGE_FRAGS / 256], int kt0) {
#pragma unroll
    for (int i = 0; i < STAGE_FRAGS / 256; ++i)
      r[i] = ld16(xrow + min(kt0 + i, KT - 1) * 32);
  };
  auto store_stage = [&](const uint4 (&r)[STAGE_FRAGS / 256], int buf) {
#pragma unroll
    for (int i = 0; i < STAGE_FRAGS / 256; ++i) xs[buf * STAGE_FRAGS + i * 256 + threadIdx.x] = r[i];
  };
  const int nstage = (KT + TG_KS - 1) / TG_KS;
  // weights: one register group of TG_KS k-steps per x stage, ping-pong (group s+1 is in
  // flight while stage s computes); issue is unconditional (clamped k index) so the
  // compiler can keep partial vmcnt waits across the loop
  auto issue_w = [&](uint4 (&w)[TG_KS][NTW], int st) {
#pragma unroll
    for (int u = 0; u < TG_KS; ++u) {
      const int kt = min(st * TG_KS + u, KT - 1);
#pragma unroll
      for (int j = 0; j < NTW; ++j) w[u][j] = ld_nt16(wbase[j] + (size_t)kt * 64);
    }
  };
  auto compute = [&](const uint4 (&w)[TG_KS][NTW], int st) {
    const int buf = st & 1;
    const int kt0 = st * TG_KS;
#pragma unroll
    for (int ks = 0; ks < TG_KS; ++ks) {
      if (kt0 + ks < KT) {
        uint4 xa[TG_MB];
#pragma unroll
        for (int mb = 0; mb < TG_MB; ++mb) {
          xa[mb] = xs[buf * STAGE_FRAGS + (ks * TG_MB + mb) * 64 + lane];
          if constexpr (NORM) xa[mb] = norm_frag<NORM>(xa[mb], nw_ptr, (kt0 + ks) * 32, ssr[mb]);
        }
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
          for (int mb = 0; mb < TG_MB; ++mb) acc[mb][j] = mfma16(as_bf16x8(w[ks][j]), as_bf16x8(xa[mb]), acc[mb][j]);
      }
    }
  };
  {
    uint4 r[STAGE_FRAGS / 256];
    load_stage(r, 0);
    store_stage(r, 0);
  }
  uint4 wa[TG_KS][NTW], wb[TG_KS][NTW];
  issue_w(wa, 0);
  lds_barrier();
  for (int st = 0; st < nstage; st += 2) {
    {
      uint4 r[STAGE_FRAGS / 256];
      load_stage(r, (st + 1) * TG_KS);  // x stage st+1 (zeros past K)
      issue_w(wb, st + 1);
      compute(wa, st);
      store_stage(r, (st + 1) & 1);
      lds_barrier();
    }
    if (st + 1 >= nstage) break;
    {
      uint4 r[STAGE_FRAGS / 256];
      load_stage(r, (st + 2) * TG_KS);
      issue_w(wa, st + 2);
      compute(wb, st + 1);
      store_stage(r, st & 1);
      lds_barrier();
    }
  }
  // epilogue straight from registers: this wave owns rows m_base.. x its NTW tiles
#pragma unroll
  for (int mb = 0; mb < TG_MB; ++mb) {
    const int m = m_base + mb * 16 + (lane & 15);
    f32x4 v[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) v[j] = acc[mb][j];
    if constexpr (NORM) {
      float ss = ssr[mb];
      ss += xor16(ss);
      ss += xor32(ss);
      const float sc = rsqrtf(ss / (float)p.K + p.eps);
#pragma unroll
      for (int j = 0; j < NTW; ++j) v[j] *= sc;
    }
    epilogue<NTW, EPI, false>(p, v, m, nt0, 4 * (lane >> 4), EpiPre<NTW>{}, m < p.M);
  }
}

// ------------------------------------------------------------------ host side
struct Plan { int waves, splitk; };

extern int g_dec_u;       // gemm.hip: -100 = the launcher's rule; else the forced decode register group size (tests)

inline int cu_count_gemm() {
  static const int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

// Decomposition from the MI355X sweep (benchmarks/micro_gpu.py, M=8, in-graph timing;
// profiles/r1_gemm_sweep.log): 8 waves per block without split-K is best for the
// small projections (qkv 3.5 us, o_proj 3.6 us — at the ~1.8 us launch floor plus one
// HBM round trip); 4 waves for the >= 512-block GEMMs (gate_up 4.7 TB/s, LM head
// 6.7 TB/s); split-K (release/acquire + slab round trip) only pays for few tiles x very
// long K (down_proj: 96 tiles x 280 k-steps, 16 waves x 2 slices).
inline Plan plan(int nblk, int mchunks, int ksteps, int MB, int NTB, int force_w, int force_s) {
  const int blocks = nblk * mchunks;
  // >= 1024 one-tile blocks (gate_up at 1120 self-contained SiLU tiles): 2 waves, i.e. more
  // resident blocks per CU (in-engine sweep: 1291.8 vs 1348.9 us per step at 4 waves,
  // profiles/r2_decode_sweep_gate_up.log)
  int w = blocks >= 1024 && NTB == 1 ? 2 : blocks >= 512 ? 4 : 8;
  int s = 1;
  if (blocks < 256 && ksteps >= 192) {
    w = 16;
    s = 2;
  }
  while (w > 1 && ksteps / (w * s) < 2) w >>= 1;
  while (w > 1 && w * MB * NTB > 64) w >>= 1;
  if (force_s > 0) s = force_s;
  if (force_w > 0) w = force_w;
  if (s > SK_MAX) s = SK_MAX;
  while (s > 1 && ksteps / s < 1) s >>= 1;
  if (MB == 1 && w > 8) w = 8;  // pipelined decode kernel: __launch_bounds__(512)
  return {w, s};
}

// decode launch with a runtime-chosen register group size (one-tile blocks; see launch_one)
template <int MB, int NTB, int U, int EPI, int NORM, int XP>
static void launch_dec_u(int u, dim3 grid, dim3 block, size_t lds, hipStream_t st, const GemmParams& p) {
  if constexpr (NTB == 1) {
    if constexpr (XP != 4) {
      if (u == 6) { hipLaunchKernelGGL((gemm_kernel<MB, NTB, 6, EPI, NORM, true, XP>), grid, block, lds, st, p); return; }
      if (u == 10) { hipLaunchKernelGGL((gemm_kernel<MB, NTB, 10, EPI, NORM, true, XP>), grid, block, lds, st, p); return; }
    }
    if (u == 12) { hipLaunchKernelGGL((gemm_kernel<MB, NTB, 12, EPI, NORM, true, XP>), grid, block, lds, st, p); return; }
  }
  hipLaunchKernelGGL((gemm_kernel<MB, NTB, U, EPI, NORM, true, XP>), grid, block, lds, st, p);
}

template <int MB, int NTB, int EPI, int NORM, bool AWQ>
static void launch_one(GemmParams p, const GemmArgs& g, hipStream_t st) {
  const int ntiles = g.N / 16;
  const int nblk = ntiles / NTB;
  const int mchunks = (g.M + 16 * MB - 1) / (16 * MB);
  const int ksteps = AWQ ? g.K / 128 : g.K / 32;
  Plan pl = plan(nblk, mchunks, ksteps, MB, NTB, g.waves, g.splitk);
  if (AWQ && pl.waves > 8) pl.waves = 8;  // awq_gemm_kernel: __launch_bounds__(512)
  const size_t need_slab = (size_t)nblk * mchunks * pl.splitk * (MB * NTB * 64 * 16 + (NORM ? 16 * MB * 4 : 0));
  if (pl.splitk > 1 && (g.slabs == nullptr || need_slab > g.slab_bytes || nblk * mchunks > g.max_counters))
    pl.splitk = 1;  // workspace too small: fall back to one slice (still correct)
  p.splitk = pl.splitk;
  // decode, two slices: combined through granules (gemm_finish; down_proj 8.43 -> 8.22 us span). More
  // slices keep the slab + ticket combine, which issues every slice's loads at once (the granule
  // owner polls the slices one after another: int4 down_proj at 8 slices 8.6 -> 9.7 us)
  if constexpr (MB == 1 && NTB == 1) {
    const size_t need_g = (size_t)nblk * (2 * NTB + 1) * 64 * 16;
    if (pl.splitk == 2 && g.sk_pub != nullptr && need_g <= g.sk_bytes) p.gran = reinterpret_cast<uint4*>(g.sk_pub);
  }
  const size_t lds = red_bytes<MB, NTB>(pl.waves) + ssq_bytes<MB>(pl.waves) + 16;
  dim3 grid(nblk, mchunks, pl.splitk), block(64 * pl.waves);
  if (p.dbg_ts == nullptr)
    p.dbg_ts = tl_take(AWQ ? "awq_gemm" : (EPI == EPI_QKV ? "gemm_qkv" : EPI == EPI_SILU ? "gemm_gate_up"
                                            : EPI == EPI_F32 ? "gemm_f32" : "gemm"), (int)(grid.x * grid.y * grid.z));
  if constexpr (AWQ) {
    // chunks of 3 k-quads when every wave's range is exactly 3 (K = 1536 over 4 waves): a chunk of
    // 4 would re-load a clamped fourth k-quad (weights, 4 activation rows, 8 scale / zero words)
    const int KQ = g.K / 128;
    const bool qc3 = MB == 1 && KQ % (pl.splitk * pl.waves) == 0 && KQ / (pl.splitk * pl.waves) == 3;
    if (qc3) hipLaunchKernelGGL((awq_gemm_kernel<MB, NTB, EPI, NORM, MB == 1 ? 3 : 0>), grid, block, lds, st, p);
    else hipLaunchKernelGGL((awq_gemm_kernel<MB, NTB, EPI, NORM>), grid, block, lds, st, p);
  }
  else if constexpr (MB == 1) {
    constexpr int U = NTB == 1 ? 8 : 4;
    const int KT = g.K / 32;
    // One-tile blocks: the register group size U is chosen per launch so that a wave's whole
    // k-range is requested in at most TWO groups (every weight byte of the launch in flight from
    // the first microsecond: gate_up 24 k-steps per wave -> 2 x 12, down_proj 17-18 -> 2 x 10),
    // and among those the size that issues the fewest clamped re-reads of a partial last group
    // (qkv / o_proj: 6 k-steps per wave -> one group of 6). Every re-read is a 1 KiB wave load
    // the CU's address unit spends on nothing. VGATE_DEC_U forces one size (6 / 8 / 10 / 12).
    // default: the round-2 rule (-1). The all-in-two-groups rule (0) was measured SLOWER in-engine:
    // gate_up at 2 x 12 needs more VGPRs, its 1120 blocks no longer fit in one round (span 12.7 ->
    // 13.4 us), and down_proj at 2 x 10 took 9.4 vs 8.8 us (profiles/r3_dec_u_negative.log)
    const int force_u = g_dec_u != -100 ? g_dec_u : -1;
    const int kpw = (KT / pl.splitk + pl.waves - 1) / pl.waves;
    const int xp = g.M <= 4 && KT % 4 == 0 ? 4 : (g.M <= 8 && KT % 2 == 0 ? 2 : 1);
    auto slots = [&](int u) { return (kpw + u - 1) / u * u; };
    int u = 8;
    if (NTB == 1) {
      if (force_u > 0) {
        u = force_u;
      } else if (force_u < 0) {  // the round-2 rule (A/B): groups of 6 where they waste fewer re-reads than 8
        u = g.M > 4 && slots(6) < slots(8) ? 6 : 8;
      } else {
        int best = 0;
        for (int c : {6, 8, 10, 12}) {
          if (c % xp) continue;
          const bool two = 2 * c >= kpw;
          const bool best_two = best > 0 && 2 * best >= kpw;
          if (best == 0 || (two && !best_two) || (two == best_two && slots(c) < slots(best))) best = c;
        }
        u = best > 0 ? best : 8;
      }
      if (u != 6 && u != 8 && u != 10 && u != 12) u = 8;
      if (u % xp) u = 8;
    }
    if (xp == 4) launch_dec_u<MB, NTB, U, EPI, NORM, 4>(u, grid, block, lds, st, p);
    else if (xp == 2) launch_dec_u<MB, NTB, U, EPI, NORM, 2>(u, grid, block, lds, st, p);
    else launch_dec_u<MB, NTB, U, EPI, NORM, 1>(u, grid, block, lds, st, p);
  } else {
    hipLaunchKernelGGL((gemm_kernel<MB, NTB, MB == 4 ? 2 : 4, EPI, NORM, false, 1>), grid, block, lds, st, p);
  }
}

// AWQ decode (M <= 16): column groups of AD_WAVES x NTW tiles, the K slices chosen so the grid
// covers the chip and every slice fits the all-in-flight register budget (<= AQ_KQ k-quads).
// Needs the fragment-packed scales (p.zeros = ops.pack_awq_sz, group 128).
template <int NTB, int EPI, int NORM>
static bool launch_awq_dec(GemmParams p, const GemmArgs& g, hipStream_t st) {
  if constexpr (NORM == 3) return false;  // the staged kernel applies gamma while staging
  const int ntiles = g.N / 16;
  if (g.M > 16 || ntiles % (AD_WAVES * NTB) != 0 || g.waves > 0 || g.group != 128 || g.awq_szp == nullptr)
    return false;
  // narrow N x short K (qkv / o_proj: 1-1.5 MB of int4) is one round trip whichever way it is
  // cut; the K-split kernel (waves split K, no LDS staging) has the shorter block (3.1 vs 4.3 us,
  // profiles/r2_awq_sweep.log) — unless a slice count is forced
  if (g.splitk <= 0 && g.N < 8192 && g.K < 4096) return false;
  const int groups = ntiles / (AD_WAVES * NTB);
  const int KQ = g.K / 128;
  const int gq = AQ_KQ / NTB;  // k-quads a wave holds in flight
  int sk = (KQ + gq - 1) / gq;  // slices the register budget needs
  if (g.splitk > 0) sk = sk > g.splitk ? sk : g.splitk;
  else
    while (groups * sk < 128 && KQ / (2 * sk) >= 3) sk *= 2;  // narrow N: spread over more CUs
  if (sk > AD_SK_MAX || sk > KQ) return false;
  const size_t need_slab = (size_t)groups * sk * (AD_WAVES * NTB * 64 * 16 + 64);
  if (sk > 1 && (g.slabs == nullptr || need_slab > g.slab_bytes || groups > g.max_counters)) return false;
  p.splitk = sk;
  const int qmax = (KQ + sk - 1) / sk;
  const size_t lds = (size_t)qmax * 4 * 64 * 16 + (size_t)qmax * 64 * 4 + 4 * 16 * 4 + 16;
  if (p.dbg_ts == nullptr) p.dbg_ts = tl_take("awq_dec", groups * sk + 8);  // + phase stamps
  hipLaunchKernelGGL((awq_dec_kernel<NTB, EPI, NORM>), dim3(groups, 1, sk), dim3(64 * AD_WAVES), lds, st, p);
  return true;
}

// AWQ decode through awq_stream_kernel: blocks of NTB tiles, waves split K, K slices across
// blocks only when the tiles alone leave the chip under-filled. g.waves > 0 forces the wave
// count (sweeps), g.ntb = 1 / 2 / 4 the tiles per block (0: the launcher's choice); returns false
// when the packed scales are missing (group != 128).
template <int EPI, int NORM, int NTB>
static void launch_awq_stream_ntb(GemmParams p, dim3 grid, int w, bool one, bool small, size_t lds, hipStream_t st,
                                  int M) {
  // register groups: NTB x U k-quads of weights + scales in flight per wave
  constexpr int U1 = NTB == 1 ? 6 : NTB == 2 ? 4 : 3;
  // one-tile blocks whose waves own <= 3 k-quads: groups of 3 (a group of 6 would re-load 3+
  // clamped k-quads of weights, scales and activations per wave)
  const bool u3 = NTB == 1 && one && small;
#define VG_AS(XP_)                                                                                        \
  do {                                                                                                    \
    if (u3) hipLaunchKernelGGL((awq_stream_kernel<3, EPI, NORM, XP_, false, 1>), grid, dim3(64 * w), lds, st, p); \
    else if (one || NTB > 1) hipLaunchKernelGGL((awq_stream_kernel<U1, EPI, NORM, XP_, false, NTB>), grid, dim3(64 * w), lds, st, p); \
    else hipLaunchKernelGGL((awq_stream_kernel<2, EPI, NORM, XP_, true, 1>), grid, dim3(64 * w), lds, st, p);        \
  } while (0)
  if (M <= 4) VG_AS(4);
  else if (M <= 8) VG_AS(2);
  else VG_AS(1);
#undef VG_AS
}

template <int EPI, int NORM>
static bool launch_awq_stream(GemmParams p, const GemmArgs& g, hipStream_t st) {
  if (g.M > 16 || g.group != 128 || g.awq_szp == nullptr || g.ntb < 0) return false;
  // narrow N x short K (qkv / o_proj, 1-1.5 MB of int4): the K-split awq_gemm_kernel's block is
  // shortest (5.7 vs 6.1 us wall, profiles/r2_awq_sweep.log)
  if (g.splitk <= 0 && g.waves <= 0 && g.ntb <= 0 && g.N < 8192 && g.K < 4096) return false;
  const int ntiles = g.N / 16;
  const int KQ = g.K / 128;
  // tiles per block: forced, or 2 for wide N (gate_up, 17920 x 1536 at M = 8: 9.0 us span at 2
  // tiles vs 9.5 at 1 and 10.0 at 4, profiles/r2_awq_sweep_ntb.log — fewer activation bytes, but
  // 4-tile blocks leave too few waves in flight)
  int ntb = g.ntb > 0 ? g.ntb : (EPI != EPI_QKV && ntiles % 2 == 0 && ntiles / 2 >= 512 ? 2 : 1);
  if (EPI == EPI_QKV || (ntb != 1 && ntb != 2 && ntb != 4) || ntiles % ntb != 0) ntb = 1;
  const int nblk = ntiles / ntb;
  int sk = g.splitk > 0 ? g.splitk : 1;
  if (g.splitk <= 0)
    while (nblk * sk < 256 && KQ / (2 * sk) >= 12) sk *= 2;  // narrow N x deep K (down_proj)
  if (sk > SK_MAX || sk > KQ) return false;
  // waves: enough that each holds its whole k-range in one register group (<= U k-quads),
  // else (NTB == 1 only: forced wave count / very deep K) the ping-pong pipeline
  const int U1 = ntb == 1 ? 6 : ntb == 2 ? 4 : 3;
  const int qslice = (KQ + sk - 1) / sk;
  int w = g.waves > 0 ? g.waves : (qslice + U1 - 1) / U1;
  if (w > 8) w = 8;
  const bool one = (qslice + w - 1) / w <= U1;
  if (!one && ntb > 1) return false;
  const size_t need_slab = (size_t)nblk * sk * (ntb * 64 * 16 + (NORM ? 16 * 4 : 0));
  if (sk > 1 && (g.slabs == nullptr || need_slab > g.slab_bytes || nblk > g.max_counters)) return false;
  p.splitk = sk;
  if (sk == 2 && ntb == 1 && g.sk_pub != nullptr && (size_t)nblk * (2 * ntb + 1) * 64 * 16 <= g.sk_bytes)
    p.gran = reinterpret_cast<uint4*>(g.sk_pub);
  const size_t lds = (size_t)w * ntb * 64 * 16 * (w > 1) + ssq_bytes<1>(w) + 16;
  if (p.dbg_ts == nullptr) p.dbg_ts = tl_take("awq_stream", nblk * sk);
  const dim3 grid(nblk, 1, sk);
  const bool small = (qslice + w - 1) / w <= 3;
  if constexpr (EPI == EPI_QKV) {
    launch_awq_stream_ntb<EPI, NORM, 1>(p, grid, w, one, small, lds, st, g.M);
  } else {
    if (ntb == 4) launch_awq_stream_ntb<EPI, NORM, 4>(p, grid, w, one, small, lds, st, g.M);
    else if (ntb == 2) launch_awq_stream_ntb<EPI, NORM, 2>(p, grid, w, one, small, lds, st, g.M);
    else launch_awq_stream_ntb<EPI, NORM, 1>(p, grid, w, one, small, lds, st, g.M);
  }
  return true;
}

template <int NTB, int EPI, int NORM, bool AWQ>
static void launch_m(GemmParams p, const GemmArgs& g, hipStream_t st) {
  if constexpr (!AWQ && NORM == 3) {  // bf16 consumer of the RMSNorm hand-off: decode rows only (binding)
    launch_one<1, NTB, EPI, 3, false>(p, g, st);
    return;
  }
  if constexpr (AWQ) {
    // g.ntb: -1 forces the LDS-staged kernel, -2 the K-split awq_gemm_kernel (sweeps / tests)
    if constexpr (NORM != 2) {  // (the gamma-folded row-scale mode has no int4 form)
      if (g.ntb != -2 && launch_awq_stream<EPI, NORM>(p, g, st)) return;
      if (g.ntb != -2 && launch_awq_dec<NTB, EPI, NORM>(p, g, st)) return;
    }
  }
  if constexpr (!AWQ) {
    // M > 16: N-split tile kernel with a shared LDS copy of x (see gemm_tile_kernel)
    const int ntiles = g.N / 16;
    constexpr int NTW = NTB;
    const int tblocks = ntiles % (TG_WAVES * NTW) == 0
                            ? ntiles / (TG_WAVES * NTW) * ((g.M + 16 * TG_MB - 1) / (16 * TG_MB)) : 0;
    // measured crossover (benchmarks/micro_gpu.py --only prefill, profiles/r1_prefill_gemm.log):
    // the tile kernel wins once its grid covers half the chip (wide N: gate_up, LM head) or
    // M >= 128 for any shape; below that, narrow N (qkv / o / down) keeps the K-split
    // kernels, which spread one matrix over more CUs. waves = -1 forces it (tests, sweeps)
    const bool tile_wins = tblocks >= 128 || g.M >= 128;
    if (g.M > 16 && g.splitk <= 0 && tblocks > 0 && (g.waves < 0 || (g.waves == 0 && tile_wins))) {
      dim3 grid(tblocks), block(64 * TG_WAVES);
      if (p.dbg_ts == nullptr) p.dbg_ts = tl_take("gemm_tile", tblocks);
      hipLaunchKernelGGL((gemm_tile_kernel<NTW, EPI, NORM>), grid, block, 2 * TG_STAGE_BYTES, st, p);
      return;
    }
  }
  if (g.M <= 16) launch_one<1, NTB, EPI, NORM, AWQ>(p, g, st);
  else if (g.M <= 32) launch_one<2, NTB, EPI, NORM, AWQ>(p, g, st);
  else launch_one<4, NTB, EPI, NORM, AWQ>(p, g, st);
}

// One epilogue's share of the dispatch: gemm.hip switches on g.epi and calls the instantiation
// compiled in that epilogue's translation unit (gemm_epi_*.hip).
template <int EPI, bool AWQ>
void dispatch_epi(GemmParams p, const GemmArgs& g, hipStream_t st) {
  const int norm = g.norm_w != nullptr ? 1 : (g.rownorm ? 2 : (g.ssp_in != nullptr ? 3 : 0));
  const int ntiles = g.N / 16;
  const bool pair = ntiles % 2 == 0 && ntiles >= 1024;
  if constexpr (EPI == EPI_BF16_AR) {  // TP all-reduce in the epilogue: decode rows, no norm (gemm.hip)
    if constexpr (!AWQ) {
      if (g.ntb == 4 && ntiles % 4 == 0) { launch_one<1, 4, EPI, 0, AWQ>(p, g, st); return; }
    }
    if (g.ntb == 2 || (g.ntb == 0 && pair)) launch_one<1, 2, EPI, 0, AWQ>(p, g, st);
    else launch_one<1, 1, EPI, 0, AWQ>(p, g, st);
    return;
  }
#define VG_NORM(NTB_)                                                           \
  do {                                                                          \
    if (norm == 1) launch_m<NTB_, EPI, 1, AWQ>(p, g, st);                       \
    else if (norm == 2 && !AWQ) launch_m<NTB_, EPI, 2, AWQ>(p, g, st);          \
    else if (norm == 3) launch_m<NTB_, EPI, 3, AWQ>(p, g, st);                  \
    else launch_m<NTB_, EPI, 0, AWQ>(p, g, st);                                 \
  } while (0)
  if constexpr (EPI == EPI_SILU) {  // self-contained 16-column tiles (8 gate + 8 up); g.ntb 2 / 4: tiles per block (sweeps)
    if constexpr (!AWQ) {
      if (g.ntb == 4 && ntiles % 4 == 0 && g.M <= 16) { VG_NORM(4); return; }
      if (g.ntb == 2 && ntiles % 2 == 0 && g.M <= 16) { VG_NORM(2); return; }
    }
    VG_NORM(1);
  } else if constexpr (EPI == EPI_QKV) {
    VG_NORM(1);
  } else {
    if constexpr (!AWQ) {
      if (g.ntb == 4 && ntiles % 4 == 0 && g.M <= 16) { VG_NORM(4); return; }
    }
    if (g.ntb == 2 || (g.ntb == 0 && pair)) VG_NORM(2);
    else VG_NORM(1);
  }
#undef VG_NORM
}

#define VG_EXTERN_EPI(E)                                                            \
  extern template void dispatch_epi<E, false>(GemmParams, const GemmArgs&, hipStream_t); \
  extern template void dispatch_epi<E, true>(GemmParams, const GemmArgs&, hipStream_t);

}  // namespace vgate
