// Decode / small-M GEMM kernel templates and their launch logic, shared by the per-epilogue
// translation units (gemm_epi_*.hip) so the ~200 kernel instantiations compile in parallel.
// Design notes: gemm.hip (file comment).
#pragma once
#include <algorithm>
#include <cstdlib>
#include <type_traits>

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
__device__ __forceinline__ void gemm_block(const GemmParams& p) {
  static_assert(XP == 1 || (MB == 1 && PIPE && U % XP == 0), "activation packing is a decode-kernel mode");
  constexpr int R = 16 / XP;  // real rows per packed load
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform branches below
  TLScope tl_scope(p.dbg_ts);
  const int KT = p.K >> 5;
  const SplitPos sp = split_pos(p);
  const int nt0 = blk_x(p) * NTB;
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
  // Rows >= M of the 16-row MFMA tile (decode batches < 16) re-read row M - 1 (row_of clamps), and
  // under XP packing (lane r loads row r % R at k-step offset r / R) lanes r >= R of a rebuilt fragment
  // keep another k-step's values: both only reach output rows that are never stored, so the loads
  // are unconditional and unmasked. (An exec-masked load — `m < M ? load : 0` — makes the compiler
  // put a full vmcnt(0) where the branch joins: the ping-pong pipeline then drains every group.)
  const bf16_t* xrow[MB];
  float ssr[MB];
  const int r16 = lane & 15;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m_base + mb * 16 + (XP > 1 ? r16 % R : r16);
    xrow[mb] = p.x + (size_t)row_of_e<EPI>(p, m) * p.lda + 8 * (lane >> 4) + (XP > 1 ? (r16 / R) * 32 : 0);
    ssr[mb] = 0.f;
  }
  // NORM 3: the producer's per-tile sums of squares of row (lane & 15), issued before the weight
  // stream and summed after it (wave 0 of slice 0 carries them into gemm_finish)
  SsPre ssv;
  ssv.n4 = NORM == 3 && MB == 1 ? ss_pre_n4(p) : 0;  // (MB > 1: prenorm_ss after the stream)
  const bool ss_wave = NORM == 3 && wid == 0 && sp.slice == 0;
  if (ss_wave && ssv.n4 > 0) ss_pre_issue(p, ssv, m_base + r16, lane >> 4);
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
      for (int mb = 0; mb < MB; ++mb) a[u][mb] = *reinterpret_cast<const uint4*>(xrow[mb] + min(k0 + u, kend - XP) * 32);
  };
  auto unpack_grp = [&](uint4 (&a)[U][MB]) {
    if constexpr (XP > 1) {
#pragma unroll
      for (int u = 0; u < U; u += XP) {  // (lanes r >= R: don't-care rows, see above)
        const uint4 v = a[u][0];
        a[u + 1][0] = row_ror<R>(v);
        if constexpr (XP == 4) {
          a[u + 2][0] = row_ror<2 * R>(v);
          a[u + 3][0] = row_ror<3 * R>(v);
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
  const bool epi_thr = PREF && wid == 0;  // wave-uniform (a lane test would be an exec-masked branch)
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
    // steady state with unconditional loads, then the 1- or 2-group tail in its own branches: a
    // load issued under a condition leaves the two paths with different outstanding-load counts,
    // and at their join the compiler waits for the smaller count — vmcnt(0), a drained pipeline
    int g = 0;
    for (; g + 3 <= ngrp; g += 2) {
      load_grp(b1, a1, gk(g + 1));
      mma_grp(b0, a0, gk(g));
      load_grp(b0, a0, gk(g + 2));
      mma_grp(b1, a1, gk(g + 1));
    }
    if (ngrp - g == 2) {
      load_grp(b1, a1, gk(g + 1));
      mma_grp(b0, a0, gk(g));
      mma_grp(b1, a1, gk(g + 1));
    } else {
      mma_grp(b0, a0, gk(g));
    }
  }
  if (epi_thr && !pre_b) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));
  if constexpr (NORM == 3) {
    if (ss_wave) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) ssr[mb] = ss_pre_sum(p, ssv, m_base + mb * 16 + r16, lane >> 4);
    }
  }
  gemm_finish<MB, NTB, EPI, NORM, PREF>(p, acc, ssr, smem, m_base, nt0, pre);
}

template <int MB, int NTB, int U, int EPI, int NORM, bool PIPE, int XP>
__global__ __launch_bounds__(PIPE ? 512 : 1024) void gemm_kernel(GemmParams p) {
  gemm_block<MB, NTB, U, EPI, NORM, PIPE, XP>(p);
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

// Epilogue of the tile kernels (this wave: rows m_base.. x its NTW column tiles, 4 m-tiles). The
// epilogue operands of all 4 m-tiles (QKV: position, slot, bias, then cos / sin by position;
// residual GEMMs: residual + bias words) are requested together first: per m-tile inside the store
// loop they were 4 serial chains of dependent loads (the compiler cannot hoist a load above an earlier
// m-tile's stores it might alias) — ~4.5 us of the 448-row QKV projection's 21 us.
template <int NTW, int EPI, int NORM>
__device__ __forceinline__ void tile_epilogue(const GemmParams& p, f32x4 (&acc)[TG_MB][NTW], const float (&ssr)[TG_MB],
                                              int m_base, int nt0, int lane) {
  constexpr bool PREF = NTW <= 2;  // EpiPre carries two tiles' words
  const int nsub = 4 * (lane >> 4);
  EpiPre<NTW> pre[TG_MB];
  if constexpr (PREF) {
#pragma unroll
    for (int mb = 0; mb < TG_MB; ++mb) epi_pre_a<NTW, EPI>(p, pre[mb], m_base + mb * 16 + (lane & 15), nt0, nsub);
#pragma unroll
    for (int mb = 0; mb < TG_MB; ++mb) epi_pre_b<NTW, EPI>(p, pre[mb], nt0, nsub);
  }
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
    if constexpr (PREF) epilogue<NTW, EPI, true>(p, v, m, nt0, nsub, pre[mb], m < p.M);
    else epilogue<NTW, EPI, false>(p, v, m, nt0, nsub, EpiPre<NTW>{}, m < p.M);
  }
}

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
  tile_epilogue<NTW, EPI, NORM>(p, acc, ssr, m_base, nt0, lane);
}

// Same tile, grid, x layout and epilogue as gemm_tile_kernel, with the stage pipeline two stages
// deep instead of one. gemm_tile_kernel issues stage s+1 (x to registers, weights to registers)
// while it computes stage s, then stores x(s+1) into LDS — so every stage waits out a whole load
// round trip behind a compute phase of ~32 MFMAs per wave: at M = 448 the Qwen2.5-1.5B qkv / o
// projections took 23 / 15 us cold in the prefill step for 2.8 / 2.1 GFLOP (18 GB/s of L2 / HBM
// traffic per CU, profiles/r6_base_prefill_timeline.log). Here iteration s issues stage s+2 and
// stores x(s+1), loaded one iteration earlier, after computing s: each load has two iterations to
// land, 128 KB per block in flight instead of 64. Registers: 3 weight groups + 2 x groups
// (~190 VGPRs at NTW = 1; one 4-wave block per CU as before). Loads past the last stage re-read it
// (clamped, unconditional: a guarded load would put a vmcnt(0) where the branch joins).
template <int NTW, int EPI, int NORM>
__global__ __launch_bounds__(256) void gemm_tile3_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  uint4* xs = reinterpret_cast<uint4*>(smem);  // [2][KS][MB][64] fragments
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int KT = p.K >> 5;
  const int mchunks = (p.M + 16 * TG_MB - 1) / (16 * TG_MB);
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int nt0 = ((wgid / mchunks) * TG_WAVES + wid) * NTW;
  const int m_base = (wgid % mchunks) * 16 * TG_MB;
  const bf16_t* nw_ptr = p.norm_w ? p.norm_w + 8 * (lane >> 4) : nullptr;
  f32x4 acc[TG_MB][NTW];
#pragma unroll
  for (int a = 0; a < TG_MB; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssr[TG_MB];
#pragma unroll
  for (int mb = 0; mb < TG_MB; ++mb) ssr[mb] = 0.f;
  constexpr int STAGE_FRAGS = TG_KS * TG_MB * 64;
  constexpr int NX = STAGE_FRAGS / 256;
  static_assert(NX == TG_KS && TG_MB == TG_WAVES, "stage mapping");
  // buffer loads: one per-lane byte offset VGPR per operand, the k-step in the scalar offset — no
  // 64-bit address temporaries (with flat addresses the register allocator gave the last weight
  // load's destination to the next iteration's address temp: a vmcnt(0) at the loop head)
  const uint32_t xoff = (uint32_t)(((size_t)row_of(p, min(m_base + wid * 16 + (lane & 15), p.M - 1)) * p.lda +
                                    8 * (lane >> 4)) * 2);
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(p.x), wr = rsrc_of(p.wp);
  uint32_t woff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) woff[j] = (uint32_t)((((size_t)(nt0 + j) * KT) * 64 + lane) * 16);
  const int nstage = (KT + TG_KS - 1) / TG_KS;
  uint4 W[3][TG_KS][NTW];
  uint4 X[2][NX];
  auto as_u4 = [](u32x4 v) __attribute__((always_inline)) { return make_uint4(v[0], v[1], v[2], v[3]); };
  auto load_x = [&](uint4 (&rr)[NX], int st) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NX; ++i)
      rr[i] = as_u4(__builtin_amdgcn_raw_buffer_load_b128(xr, xoff, min(st * TG_KS + i, KT - 1) * 64, 0));
  };
  auto store_x = [&](const uint4 (&rr)[NX], int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NX; ++i) xs[buf * STAGE_FRAGS + i * 256 + threadIdx.x] = rr[i];
  };
  auto issue_w = [&](uint4 (&w)[TG_KS][NTW], int st) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < TG_KS; ++u) {
      const int kt = min(st * TG_KS + u, KT - 1);
#pragma unroll
      for (int j = 0; j < NTW; ++j)
        w[u][j] = as_u4(__builtin_amdgcn_raw_buffer_load_b128(wr, woff[j], kt * 1024, 2 /* nt */));
    }
  };
  // whole stages only (host: K % (32 * TG_KS) == 0): no per-k-step guard, so the stage's MFMAs are
  // one branch-free block and the compiler keeps exact partial vmcnt waits across it
  auto compute = [&](const uint4 (&w)[TG_KS][NTW], int st) __attribute__((always_inline)) {
    const int buf = st & 1;
    const int kt0 = st * TG_KS;
#pragma unroll
    for (int ks = 0; ks < TG_KS; ++ks) {
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
  };
  // iteration s (A = s % 3, B = s % 2): issue stage s+2 into the registers stage s-1 / s left,
  // compute s, store x(s+1) into the LDS buffer stage s-1 was read from, barrier
  auto iter = [&](auto A, auto B, int s) __attribute__((always_inline)) {
    constexpr int a = decltype(A)::value, b = decltype(B)::value;
    load_x(X[b], s + 2);
    issue_w(W[(a + 2) % 3], s + 2);
    compute(W[a], s);
    store_x(X[1 - b], 1 - b);
    lds_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  load_x(X[0], 0);
  issue_w(W[0], 0);
  load_x(X[1], 1);
  issue_w(W[1], 1);
  store_x(X[0], 0);
  lds_barrier();
  for (int s = 0; s < nstage; s += 6) {
    iter(I0{}, I0{}, s);
    if (s + 1 >= nstage) break;
    iter(I1{}, I1{}, s + 1);
    if (s + 2 >= nstage) break;
    iter(I2{}, I0{}, s + 2);
    if (s + 3 >= nstage) break;
    iter(I0{}, I1{}, s + 3);
    if (s + 4 >= nstage) break;
    iter(I1{}, I0{}, s + 4);
    if (s + 5 >= nstage) break;
    iter(I2{}, I1{}, s + 5);
  }
  tile_epilogue<NTW, EPI, NORM>(p, acc, ssr, m_base, nt0, lane);
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

// Fused QKV projection + decode attention (qkv_attn.hip): the decode QKV launch of a decode-only step
// with its attention blocks appended (QaSync). False: a (register group, packing, norm mode) it has no
// instantiation for, or an attention shape it does not take — the caller launches both kernels.
bool launch_qkv_attn(int u, int xp, int norm, GemmParams p, int gx, int slices, int waves, size_t lds_gemm,
                     const GemmArgs& g, hipStream_t st);

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
  auto take_tl = [&] {
    if (p.dbg_ts == nullptr)
      p.dbg_ts = tl_take(AWQ ? "awq_gemm" : (EPI == EPI_QKV ? "gemm_qkv" : EPI == EPI_SILU ? "gemm_gate_up"
                                              : EPI == EPI_F32 ? "gemm_f32" : "gemm"), (int)(grid.x * grid.y * grid.z));
  };
  if constexpr (AWQ) {
    take_tl();
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
    if constexpr (EPI == EPI_QKV && NTB == 1) {  // decode-only step: its attention in this launch
      if (g.fa != nullptr && grid.y == 1 && launch_qkv_attn(u, xp, NORM, p, (int)grid.x, (int)grid.z, pl.waves, lds, g, st)) {
        *g.fa_done = true;
        return;
      }
    }
    take_tl();
    if (xp == 4) launch_dec_u<MB, NTB, U, EPI, NORM, 4>(u, grid, block, lds, st, p);
    else if (xp == 2) launch_dec_u<MB, NTB, U, EPI, NORM, 2>(u, grid, block, lds, st, p);
    else launch_dec_u<MB, NTB, U, EPI, NORM, 1>(u, grid, block, lds, st, p);
  } else {
    take_tl();
    hipLaunchKernelGGL((gemm_kernel<MB, NTB, MB == 4 ? 2 : 4, EPI, NORM, false, 1>), grid, block, lds, st, p);
  }
}

template <int NTB, int EPI, int NORM, bool AWQ>
static void launch_m(GemmParams p, const GemmArgs& g, hipStream_t st) {
  if constexpr (!AWQ && NORM == 3) {  // bf16 consumer of the RMSNorm hand-off: decode rows only (binding)
    launch_one<1, NTB, EPI, 3, false>(p, g, st);
    return;
  }
  // (AWQ here: the K-split awq_gemm_kernel — TP ranks with the fused all-reduce, group 64, shapes the
  // register-stationary kernel declines, gemm_awq_kx.hip; g.ntb = -2 forces it)
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
      // two-deep stage pipeline (gemm_tile3_kernel) once K has >= 3 stages; waves -1 / -2 force
      // the one-deep / two-deep form (sweeps, tests)
      // (one column tile per wave only: with 2 / 4 the three weight groups spill to scratch)
      const bool deep = NTW == 1 && g.K % (32 * TG_KS) == 0 &&
                        (g.waves == -2 || (g.waves != -1 && (g.K / 32) >= 3 * TG_KS));
      if (p.dbg_ts == nullptr) p.dbg_ts = tl_take(deep ? "gemm_tile3" : "gemm_tile", tblocks);
      if constexpr (NTW == 1) {
        if (deep) {
          hipLaunchKernelGGL((gemm_tile3_kernel<NTW, EPI, NORM>), grid, block, 2 * TG_STAGE_BYTES, st, p);
          return;
        }
      }
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
