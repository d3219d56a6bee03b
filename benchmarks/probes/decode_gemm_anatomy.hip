// Anatomy of the bf16 decode GEMM (csrc/kernels/gemm_decode.h gemm_kernel) on its gate_up / down shapes
// (Qwen2.5-1.5B, M = 8): the production kernel, and a copy of it with one piece changed at a time —
// interleaved k-steps per wave (INTER), no epilogue (NOEPI), no MFMA (NOMMA), no activation loads
// (NOACT) — against the plain streaming skeleton of the same tile shape, all cold (a ring of weight
// copies > 1 GiB), timed as a hipGraph of 20 launches (us per launch incl. the boundary).
//
//   hipcc --offload-arch=gfx950 -O3 -I csrc/kernels -o build/decode_gemm_anatomy benchmarks/probes/decode_gemm_anatomy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "gemm_decode.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

namespace vgate {
// the production kernel body, copied with probe switches (FL bits: 1 INTER, 2 NOEPI, 4 NOMMA, 8 NOACT)
template <int MB, int NTB, int U, int EPI, int NORM, bool PIPE, int XP, int FL>
__global__ __launch_bounds__(PIPE ? 512 : 1024) void probe_kernel(GemmParams p) {
  constexpr bool INTER = FL & 1, NOEPI = FL & 2, NOMMA = FL & 4, NOACT = FL & 8;
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
  if constexpr (INTER) {  // same count per wave, k-step i of the wave -> s0 + wr + i * nw
    kbeg = 0;
    kend = (s1 - s0 - wr + nw - 1) / nw;
  }
  auto kmap = [&](int i) { return INTER ? s0 + wr + i * nw : i; };
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
    ssr[mb] = 0.f;
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
      for (int j = 0; j < NTB; ++j) b[u][j] = ld_nt16(wbase[j] + (size_t)kmap(min(k0 + u, kend - 1)) * 64);
#pragma unroll
    for (int u = 0; u < U; u += XP)  // packed: slot u holds the raw load for k-steps u..u+XP-1
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        a[u][mb] = (xok[mb] && !NOACT) ? *reinterpret_cast<const uint4*>(xrow[mb] + kmap(min(k0 + u, kend - XP)) * 32)
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
    if constexpr (NORM) {
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
        for (int mb = 0; mb < MB; ++mb) {
          if constexpr (NOMMA) acc[mb][j][0] += __uint_as_float(b[u][j].x ^ a[u][mb].y);
          else acc[mb][j] = mfma16(as_bf16x8(b[u][j]), as_bf16x8(a[u][mb]), acc[mb][j]);
        }
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
  if constexpr (NOEPI) {
    if (acc[0][0][0] == 1234.5f && ssr[0] == 7.f) reinterpret_cast<float*>(p.out)[threadIdx.x] = acc[0][0][1];
    return;
  }
  gemm_finish<MB, NTB, EPI, NORM, PREF>(p, acc, ssr, smem, m_base, nt0, pre);
}


// activations for the wave's whole k-range loaded before its weight stream (XP = 2 packs), weight
// groups unrolled (NGMAX) so every activation pack is a compile-time register index
template <int U, int EPI, int NORM, int NGMAX>
__global__ __launch_bounds__(512) void probe_xpre(GemmParams p) {
  constexpr int MB = 1, NTB = 1, XP = 2, R = 8, NX = NGMAX * U / XP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int KT = p.K >> 5;
  const SplitPos sp = split_pos(p);
  const int nt0 = (int)blockIdx.x * NTB;
  const int s0 = (KT * sp.slice) / sp.nsl, s1 = (KT * (sp.slice + 1)) / sp.nsl;
  const int np0 = s0 / XP, np1 = s1 / XP;
  const int kbeg = XP * (np0 + ((np1 - np0) * wid) / nw);
  const int kend = XP * (np0 + ((np1 - np0) * (wid + 1)) / nw);
  const int r16 = lane & 15;
  const int m = r16 % R;
  const bool xok = m < p.M;
  const bf16_t* xrow = p.x + (size_t)row_of(p, m) * p.lda + 8 * (lane >> 4) + (r16 / R) * 32;
  float ssr[1] = {(NORM == 3 && wid == 0 && sp.slice == 0) ? prenorm_ss(p, r16, lane >> 4) : 0.f};
  f32x4 acc[1][1] = {{f32x4{0.f, 0.f, 0.f, 0.f}}};
  const uint4* wbase = p.wp + ((size_t)nt0 * KT) * 64 + lane;
  const int n = kend - kbeg;
  uint4 xs[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i)
    xs[i] = (xok && XP * i < n) ? *reinterpret_cast<const uint4*>(xrow + (kbeg + XP * i) * 32) : make_uint4(0, 0, 0, 0);
  const int ngrp = (n + U - 1) / U;
  uint4 b[2][U];
  auto load = [&](uint4 (&bb)[U], int g) {
#pragma unroll
    for (int u = 0; u < U; ++u) bb[u] = ld_nt16(wbase + (size_t)min(kbeg + g * U + u, kend - 1) * 64);
  };
  const uint32_t lom = r16 < R ? ~0u : 0u;
  EpiPre<NTB> pre;
  const bool epi_thr = threadIdx.x < 64;
  if (epi_thr) epi_pre_a<NTB, EPI>(p, pre, r16, nt0, 4 * (lane >> 4));
  if (ngrp > 0) load(b[0], 0);
  if (epi_thr) epi_pre_b<NTB, EPI>(p, pre, nt0, 4 * (lane >> 4));
#pragma unroll
  for (int g = 0; g < NGMAX; ++g) {
    if (g < ngrp) {
      if (g + 1 < ngrp) load(b[(g + 1) & 1], g + 1);
#pragma unroll
      for (int u = 0; u < U; u += XP) {
        const uint4 v = xs[(g * U + u) / XP];
        uint4 a0 = and_mask(v, lom), a1 = and_mask(row_ror<R>(v), lom);
        if (g * U + u >= n) a0 = make_uint4(0, 0, 0, 0);
        if (g * U + u + 1 >= n) a1 = make_uint4(0, 0, 0, 0);
        if constexpr (NORM == 2) {
          a0 = norm_frag<2>(a0, nullptr, 0, ssr[0]);
          a1 = norm_frag<2>(a1, nullptr, 0, ssr[0]);
        }
        acc[0][0] = mfma16(as_bf16x8(b[g & 1][u]), as_bf16x8(a0), acc[0][0]);
        acc[0][0] = mfma16(as_bf16x8(b[g & 1][u + 1]), as_bf16x8(a1), acc[0][0]);
      }
    }
  }
  gemm_finish<MB, NTB, EPI, NORM, true>(p, acc, ssr, smem, 0, nt0, pre);
}
}  // namespace vgate

using namespace vgate;

template <typename F>
double time_graph(hipStream_t st, int R, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < R; ++r) launch(r);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 1e3 * best / R;
}

int main() {
  const size_t ring = (size_t)1400 << 20;
  char* base = nullptr;
  CK(hipMalloc(&base, ring));
  CK(hipMemset(base, 0, ring));  // zero weights: finite outputs, same bytes streamed
  const int M = 8;
  bf16_t *x = nullptr, *out = nullptr, *res = nullptr;
  CK(hipMalloc(&x, 16 * 8960 * 2));
  CK(hipMemset(x, 0, 16 * 8960 * 2));
  CK(hipMalloc(&out, 16 * 17920 * 2));
  CK(hipMalloc(&res, 16 * 17920 * 2));
  CK(hipMemset(res, 0, 16 * 17920 * 2));
  uint4* gran = nullptr;
  CK(hipMalloc(&gran, 64 << 20));
  CK(hipMemset(gran, 0, 64 << 20));
  float* ssp = nullptr;
  CK(hipMalloc(&ssp, 16 * 1024 * 4));
  CK(hipMemset(ssp, 0, 16 * 1024 * 4));
  uint32_t* fault = nullptr;
  CK(hipMalloc(&fault, 4));
  CK(hipMemset(fault, 0, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int R = 20;
  struct Shape { const char* name; int N, K, epi, nw, splitk; };
  // the production plans: gate_up 2-wave one-tile blocks (U 8, XP 2, SiLU + folded-norm row scale),
  // down 8 waves x 2 K slices (U 6, XP 2, residual add)
  const Shape shapes[] = {{"gate_up", 17920, 1536, EPI_SILU, 2, 1}, {"down", 1536, 8960, EPI_BF16, 8, 2}};
  for (const Shape& s : shapes) {
    const size_t bytes = (size_t)s.N * s.K * 2;
    const size_t stride = (bytes + 65535) / 65536 * 65536;
    const int ncopy = (int)(ring / stride);
    GemmParams p{};
    p.x = x; p.lda = s.K; p.M = M; p.N = s.N; p.K = s.K; p.eps = 1e-6f;
    p.out = out; p.ldo = s.epi == EPI_SILU ? s.N / 2 : s.N;
    p.res = s.epi == EPI_BF16 ? res : nullptr; p.ldr = s.N;
    p.splitk = s.splitk; p.gran = gran; p.fault = fault;
    p.ssp_in = ssp; p.ssn = s.K / 16;
    const dim3 grid(s.N / 16, 1, s.splitk), block(64 * s.nw);
    const size_t lds = 16384;
    auto wp_of = [&](int r) { return reinterpret_cast<const uint4*>(base + (size_t)(r % ncopy) * stride); };
#define RUNV(NAME, KERN)                                                                           \
    {                                                                                              \
      const double us = time_graph(st, R, [&](int r) {                                             \
        GemmParams q = p;                                                                          \
        q.wp = wp_of(r);                                                                           \
        hipLaunchKernelGGL(KERN, grid, block, lds, st, q);                                         \
      });                                                                                          \
      printf("{\"shape\": \"%s\", \"variant\": \"%s\", \"us_per_launch\": %.2f, \"tb_s\": %.2f}\n", s.name, NAME, us, \
             bytes / us / 1e6);                                                                    \
      fflush(stdout);                                                                              \
    }
    if (s.epi == EPI_SILU) {
      RUNV("production", (gemm_kernel<1, 1, 8, EPI_SILU, 2, true, 2>));
      RUNV("copy", (probe_kernel<1, 1, 8, EPI_SILU, 2, true, 2, 0>));
      RUNV("inter", (probe_kernel<1, 1, 8, EPI_SILU, 2, true, 2, 1>));
      RUNV("noepi", (probe_kernel<1, 1, 8, EPI_SILU, 2, true, 2, 2>));
      RUNV("nomma", (probe_kernel<1, 1, 8, EPI_SILU, 2, true, 2, 4>));
      RUNV("noact", (probe_kernel<1, 1, 8, EPI_SILU, 2, true, 2, 8>));
      RUNV("noepi_nomma_noact", (probe_kernel<1, 1, 8, EPI_SILU, 2, true, 2, 14>));
      RUNV("nonorm", (probe_kernel<1, 1, 8, EPI_SILU, 0, true, 2, 0>));
      RUNV("u4", (probe_kernel<1, 1, 4, EPI_SILU, 2, true, 2, 0>));
      RUNV("u4_inter", (probe_kernel<1, 1, 4, EPI_SILU, 2, true, 2, 1>));
      RUNV("xpre", (probe_xpre<8, EPI_SILU, 2, 3>));
      RUNV("xpre_norm3", (probe_xpre<8, EPI_SILU, 3, 3>));
      RUNV("norm3", (gemm_kernel<1, 1, 8, EPI_SILU, 3, true, 2>));
    } else {
      RUNV("production", (gemm_kernel<1, 1, 6, EPI_BF16, 0, true, 2>));
      RUNV("copy", (probe_kernel<1, 1, 6, EPI_BF16, 0, true, 2, 0>));
      RUNV("inter", (probe_kernel<1, 1, 6, EPI_BF16, 0, true, 2, 1>));
      RUNV("noepi", (probe_kernel<1, 1, 6, EPI_BF16, 0, true, 2, 2>));
      RUNV("nomma", (probe_kernel<1, 1, 6, EPI_BF16, 0, true, 2, 4>));
      RUNV("noact", (probe_kernel<1, 1, 6, EPI_BF16, 0, true, 2, 8>));
      RUNV("noepi_nomma_noact", (probe_kernel<1, 1, 6, EPI_BF16, 0, true, 2, 14>));
      RUNV("u8", (probe_kernel<1, 1, 8, EPI_BF16, 0, true, 2, 0>));
      RUNV("xpre", (probe_xpre<6, EPI_BF16, 0, 3>));
    }
    unsigned f = 0;
    CK(hipMemcpy(&f, fault, 4, hipMemcpyDeviceToHost));
    printf("{\"shape\": \"%s\", \"fault\": %u}\n", s.name, f);
  }
  return 0;
}
