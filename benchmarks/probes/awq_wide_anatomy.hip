// Anatomy of the int4 decode GEMM, wide form (csrc/kernels/gemm_awq_wide.hip awq_wide_kernel) on the
// Qwen2.5-1.5B AWQ gate_up shape (M = 8, N = 17920, K = 1536, group 128: 13.8 MB int4 + 0.9 MB of
// packed scales): the production kernel copied with one piece switched off at a time — the x DMA into
// LDS (NOX), the scale DMA (NOSZ), the MFMA / dequant loop (NOMMA), the activation-sum pass (NOXSUM) —
// against a plain read of the same int4 bytes; cold weights (a ring of copies > 1 GiB), hipGraph of 20.
//
//   hipcc --offload-arch=gfx950 -O3 -I csrc/kernels -o build/awq_wide_anatomy benchmarks/probes/awq_wide_anatomy.hip
#include <hip/hip_runtime.h>

#include <algorithm>
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
unsigned long long* tl_take(const char*, int) { return nullptr; }
__device__ __forceinline__ bf16x8 pa_raw8(uint32_t q) {  // nibble order of ops.pack_awq
  uint4 r;
  r.x = (q & 0x000F000Fu) | 0x43004300u;
  r.y = ((q >> 4) & 0x000F000Fu) | 0x43004300u;
  r.z = ((q >> 8) & 0x000F000Fu) | 0x43004300u;
  r.w = ((q >> 12) & 0x000F000Fu) | 0x43004300u;
  return as_bf16x8(r);
}

  // k-quads per tile held in registers (K <= 2048)

template <int KQM, int EPI, int NORM, int FL>
__global__ __launch_bounds__(1024) void probe_wide(GemmParams p) {
  constexpr bool NOX = FL & 1, NOSZ = FL & 2, NOMMA = FL & 4, NOXSUM = FL & 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // x [4 KQ][64][16 B] | sz [tiles][KQ][4][16 B] | X
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63, r16 = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int KQ = p.K >> 7, KT = KQ * 4;
  const int ntiles = p.N >> 4, nb = gridDim.x, b = blockIdx.x;
  const int t0 = (int)(((long long)ntiles * b) / nb), ntb = (int)(((long long)ntiles * (b + 1)) / nb) - t0;
  const bool active = wid < ntb;  // wave-uniform
  const int nt = t0 + (active ? wid : 0);
  const uint32_t lds0 = lds_addr_of(smem);
  const size_t x_bytes = (size_t)KT * 1024;
  const int sz_pieces = (ntb * KQ * 64 + 1023) / 1024;  // the block's (s, s z) records, 64 B per (tile, k-quad)
  // 1) x pieces then the scale pieces, spread over the waves
  for (int f = wid; f < KT + sz_pieces; f += nw) {
    if (f < KT) {
      if (NOX) continue;
      const int row = r16 < p.M ? r16 : p.M - 1;
      glds16(p.x + (size_t)row_of(p, row) * p.lda + (size_t)f * 32 + 8 * (lane >> 4),
             __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)f * 1024u));
    } else {
      if (NOSZ) continue;
      const int g = f - KT;
      // clamp the tail piece inside the matrix's records (bytes past the block's are never read)
      const size_t off = std::min((size_t)((size_t)t0 * KQ * 64 + (size_t)g * 1024 + lane * 16),
                                  (size_t)ntiles * KQ * 64 - 16);
      glds16(reinterpret_cast<const char*>(p.szp) + off,
             __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(x_bytes + (size_t)g * 1024)));
    }
  }
  uint4 w[KQM];
  if (active) {
    const uint4* wb = p.wp + (size_t)nt * KQ * 64 + lane;
#pragma unroll
    for (int q = 0; q < KQM; ++q) w[q] = ld_nt16(wb + (size_t)min(q, KQ - 1) * 64);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KQM) : "memory");  // the DMA pieces, issued before the weights
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // 2) X[kq][row]: the k-quad's activation sum per row (from the bf16 values the MFMAs read)
  const uint4* xs = reinterpret_cast<const uint4*>(smem);
  float* Xs = reinterpret_cast<float*>(smem + x_bytes + (size_t)sz_pieces * 1024);
  for (int q = wid; q < (NOXSUM ? 0 : KQ); q += nw) {
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float f[8];
      unpack8(xs[(4 * q + u) * 64 + lane], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[j];
    }
    s += xor16(s);
    s += xor32(s);
    if (lane < 16) Xs[q * 16 + lane] = s;
  }
  __syncthreads();
  if (!active) return;
  const uint4* szs = reinterpret_cast<const uint4*>(smem + x_bytes) + (size_t)(nt - t0) * KQ * 4 + (lane >> 4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < KQM; ++q) {
    if (q < KQ && NOMMA) {
      acc[0] += __uint_as_float((w[q].x ^ w[q].w) & 0x3f000000u);
    } else if (q < KQ) {  // wave-uniform
      f32x4 pr = {0.f, 0.f, 0.f, 0.f};
      pr = mfma16(pa_raw8(w[q].x), as_bf16x8(xs[(4 * q + 0) * 64 + lane]), pr);
      pr = mfma16(pa_raw8(w[q].y), as_bf16x8(xs[(4 * q + 1) * 64 + lane]), pr);
      pr = mfma16(pa_raw8(w[q].z), as_bf16x8(xs[(4 * q + 2) * 64 + lane]), pr);
      pr = mfma16(pa_raw8(w[q].w), as_bf16x8(xs[(4 * q + 3) * 64 + lane]), pr);
      const uint4 sz = szs[(size_t)q * 4];
      const float X = Xs[q * 16 + r16];
      const float s4[4] = {bf_lo(sz.x), bf_hi(sz.x), bf_lo(sz.y), bf_hi(sz.y)};
      const float z4[4] = {bf_lo(sz.z), bf_hi(sz.z), bf_lo(sz.w), bf_hi(sz.w)};
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = fmaf(s4[i], pr[i], fmaf(-fmaf(128.f, s4[i], z4[i]), X, acc[i]));
    }
  }
  f32x4 v[1] = {acc};
  if constexpr (NORM == 3) {
    float ss = prenorm_ss(p, r16, lane >> 4);
    ss += xor16(ss);
    ss += xor32(ss);
    v[0] *= rsqrtf(ss / (float)p.K + p.eps);
  }
  epilogue<1, EPI, false>(p, v, r16, nt, 4 * (lane >> 4), EpiPre<1>{}, r16 < p.M);
}

// Candidate redesign ("kx"): one block per CU owning whole tiles (as awq_wide), but its NW waves
// split K (KQW k-quads each) and every wave keeps ITS activations in registers (XP = 2 packed: one
// 16-B load per 2 k-steps, M <= 8 real rows only) while it streams the int4 fragments + scales of
// ALL the block's tiles for its k-range; LDS carries only the cross-wave partials. No x DMA, no
// block-wide barrier before the MFMAs, the dequant VALU work spread over NW waves.
// FL: 1 no MFMA / dequant, 2 no scale loads, 4 no activation loads.
template <int NW, int KQW, int TMAX, int FL>
__global__ __launch_bounds__(64 * NW) void probe_kx(GemmParams p) {
  constexpr bool NOMMA = FL & 1, NOSZ = FL & 2, NOXL = FL & 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x4* red = reinterpret_cast<f32x4*>(smem);  // [NW][TMAX][64]
  const int lane = threadIdx.x & 63, r16 = lane & 15, grp = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KQ = p.K >> 7, ntiles = p.N >> 4, nb = gridDim.x, b = blockIdx.x;
  const int t0 = (int)(((long long)ntiles * b) / nb), ntb = (int)(((long long)ntiles * (b + 1)) / nb) - t0;
  const int q0 = (KQ * wid) / NW, nq = (KQ * (wid + 1)) / NW - q0;
  constexpr int R = 8;
  const int mrow = r16 % R;
  const bool xok = mrow < p.M;
  const uint32_t lom = r16 < R ? ~0u : 0u;
  const bf16_t* xrow = p.x + (size_t)row_of(p, mrow) * p.lda + 8 * grp + (r16 / R) * 32;
  uint4 xa[KQW][2], w[KQW][TMAX], sz[KQW][TMAX];
#pragma unroll
  for (int q = 0; q < KQW; ++q) {
    const int kq = q0 + min(q, nq - 1);
#pragma unroll
    for (int v = 0; v < 2; ++v)
      xa[q][v] = (xok && !NOXL) ? *reinterpret_cast<const uint4*>(xrow + (kq * 4 + 2 * v) * 32) : make_uint4(0x3f803f80u, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      const size_t u = (size_t)(t0 + min(j, ntb - 1)) * KQ + kq;
      w[q][j] = ld_nt16(p.wp + u * 64 + lane);
      sz[q][j] = NOSZ ? make_uint4(0x3f803f80u, 0x3f803f80u, 0, 0) : reinterpret_cast<const uint4*>(p.szp)[u * 4 + grp];
    }
  }
  f32x4 acc[TMAX];
#pragma unroll
  for (int j = 0; j < TMAX; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < KQW; ++q) {
    if (q >= nq) break;  // wave-uniform
    if constexpr (NOMMA) {
#pragma unroll
      for (int j = 0; j < TMAX; ++j)
        acc[j][0] += __uint_as_float((w[q][j].x ^ w[q][j].w ^ sz[q][j].x ^ xa[q][0].y ^ xa[q][1].z) & 0x3f000000u);
      continue;
    }
    uint4 bf[4];
    bf[0] = and_mask(xa[q][0], lom);
    bf[1] = and_mask(row_ror<R>(xa[q][0]), lom);
    bf[2] = and_mask(xa[q][1], lom);
    bf[3] = and_mask(row_ror<R>(xa[q][1]), lom);
    float X = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float f[8];
      unpack8(bf[t], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) X += f[j];
    }
    X += xor16(X);
    X += xor32(X);
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      if (j < ntb) {
        f32x4 pr = {0.f, 0.f, 0.f, 0.f};
        pr = mfma16(pa_raw8(w[q][j].x), as_bf16x8(bf[0]), pr);
        pr = mfma16(pa_raw8(w[q][j].y), as_bf16x8(bf[1]), pr);
        pr = mfma16(pa_raw8(w[q][j].z), as_bf16x8(bf[2]), pr);
        pr = mfma16(pa_raw8(w[q][j].w), as_bf16x8(bf[3]), pr);
        const uint4 s = sz[q][j];
        const float s4[4] = {bf_lo(s.x), bf_hi(s.x), bf_lo(s.y), bf_hi(s.y)};
        const float z4[4] = {bf_lo(s.z), bf_hi(s.z), bf_lo(s.w), bf_hi(s.w)};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(s4[i], pr[i], fmaf(-fmaf(128.f, s4[i], z4[i]), X, acc[j][i]));
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TMAX; ++j)
    if (j < ntb) red[(wid * TMAX + j) * 64 + lane] = acc[j];
  __syncthreads();
  if (wid >= ntb) return;
  f32x4 v[1] = {{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int w2 = 0; w2 < NW; ++w2) v[0] += red[(w2 * TMAX + wid) * 64 + lane];
  epilogue<1, EPI_SILU, false>(p, v, r16, t0 + wid, 4 * grp, EpiPre<1>{}, r16 < p.M);
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

__global__ void sweep(const uint4* __restrict__ p, size_t n16, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    acc ^= __builtin_nontemporal_load(&p[i].x);
  if (acc == 0x9E3779B9u && sink) *sink = acc;
}

int main() {
  const int M = 8, N = 17920, K = 1536, KQ = K / 128;
  const size_t wbytes = (size_t)N * K / 2, szbytes = (size_t)(N / 16) * KQ * 64;
  const size_t stride = (wbytes + szbytes + 65535) / 65536 * 65536;
  const size_t ring = (size_t)1400 << 20;
  const int ncopy = (int)(ring / stride);
  char* base = nullptr;
  CK(hipMalloc(&base, ring));
  CK(hipMemset(base, 0, ring));
  bf16_t *x = nullptr, *out = nullptr;
  CK(hipMalloc(&x, 16 * K * 2));
  CK(hipMemset(x, 0, 16 * K * 2));
  CK(hipMalloc(&out, 16 * N * 2));
  unsigned* sink = nullptr;
  CK(hipMalloc(&sink, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int R = 20, nb = 256, ntiles = N / 16, tmax = (ntiles + nb - 1) / nb;
  const int szp = (tmax * KQ * 64 + 1023) / 1024;
  const size_t lds = (size_t)KQ * 4 * 1024 + (size_t)szp * 1024 + (size_t)KQ * 16 * 4;
  GemmParams p{};
  p.x = x; p.lda = K; p.M = M; p.N = N; p.K = K; p.eps = 1e-6f; p.out = out; p.ldo = N / 2; p.splitk = 1; p.group = 128;
  auto run = [&](const char* name, auto kern) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const double us = time_graph(st, R, [&](int r) {
      GemmParams q = p;
      q.wp = reinterpret_cast<const uint4*>(base + (size_t)(r % ncopy) * stride);
      q.szp = reinterpret_cast<const bf16_t*>(base + (size_t)(r % ncopy) * stride + wbytes);
      hipLaunchKernelGGL(kern, dim3(nb), dim3(64 * tmax), lds, st, q);
    });
    printf("{\"variant\": \"%s\", \"us_per_launch\": %.2f}\n", name, us);
    fflush(stdout);
  };
  run("production_copy", probe_wide<12, EPI_SILU, 0, 0>);
  run("nox", probe_wide<12, EPI_SILU, 0, 1>);
  run("nosz", probe_wide<12, EPI_SILU, 0, 2>);
  run("nomma", probe_wide<12, EPI_SILU, 0, 4>);
  run("noxsum", probe_wide<12, EPI_SILU, 0, 8>);
  run("nox_nosz_nomma_noxsum", probe_wide<12, EPI_SILU, 0, 15>);
  auto runkx = [&](const char* name, auto kern, int nw, int tm) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const double us = time_graph(st, R, [&](int r) {
      GemmParams q = p;
      q.wp = reinterpret_cast<const uint4*>(base + (size_t)(r % ncopy) * stride);
      q.szp = reinterpret_cast<const bf16_t*>(base + (size_t)(r % ncopy) * stride + wbytes);
      hipLaunchKernelGGL(kern, dim3(nb), dim3(64 * nw), (size_t)nw * tm * 1024, st, q);
    });
    printf("{\"variant\": \"kx %s\", \"waves\": %d, \"us_per_launch\": %.2f}\n", name, nw, us);
    fflush(stdout);
  };
  runkx("12w x 1kq", probe_kx<12, 1, 5, 0>, 12, 5);
  runkx("6w x 2kq", probe_kx<6, 2, 5, 0>, 6, 5);
  runkx("4w x 3kq", probe_kx<4, 3, 5, 0>, 4, 5);
  runkx("12w nomma", probe_kx<12, 1, 5, 1>, 12, 5);
  runkx("12w nosz", probe_kx<12, 1, 5, 2>, 12, 5);
  runkx("12w noxl", probe_kx<12, 1, 5, 4>, 12, 5);
  runkx("12w nosz noxl", probe_kx<12, 1, 5, 6>, 12, 5);
  runkx("12w nomma nosz noxl", probe_kx<12, 1, 5, 7>, 12, 5);
  runkx("6w nomma", probe_kx<6, 2, 5, 1>, 6, 5);
  for (int blocks : {256, 1024}) {
    const double us = time_graph(st, R, [&](int r) {
      hipLaunchKernelGGL(sweep, dim3(blocks), dim3(256), 0, st,
                         reinterpret_cast<const uint4*>(base + (size_t)(r % ncopy) * stride), wbytes / 16, sink);
    });
    printf("{\"variant\": \"plain read of the int4 bytes, %d blocks\", \"us_per_launch\": %.2f}\n", blocks, us);
  }
  return 0;
}
