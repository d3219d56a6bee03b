// AWQ W4A16 decode GEMM, wide form (M <= 16, N of at least one 16-column tile per CU: Qwen2.5-1.5B
// gate_up's 1120 tiles).
//
// At decode batch sizes an int4 k-quad of one tile (1 KiB) needs 8 rows x 128 k of activations
// (2 KiB) and a 64-B group-scale record, so the one-tile-per-block stream kernels move as many
// activation bytes through every CU as weight bytes (awq_stream gate_up 10.5 us for 13.8 MB of
// int4; 6.6 us with the activation and scale loads switched off, profiles/r2_awq_load_probe.log).
// Here the grid is one block per CU and a block owns WHOLE tiles ([N b / B, N (b + 1) / B): 4-5 of
// 1120), so x and the scales are fetched once per CU:
//   1. x (16-row MFMA B fragments, rows past M repeat row M - 1) and the block's packed (s, s z)
//      records are DMA'd into LDS (global_load_lds_dwordx4), then every wave issues ALL int4
//      fragments of its tile (one wave per tile, <= 16 k-quads = 16 registers of 16 B): the whole
//      launch's weights are requested in the first microsecond;
//   2. the per-(k-quad, row) activation sums X of the raw-nibble identity
//        sum_k x (v - z) s = s * sum_k x (128 + v) - (128 s + s z) * X
//      are computed once per block from the LDS image;
//   3. per k-quad four MFMAs on the bf16 (128 + v) built from the nibbles (two VALU per dword),
//      then the group scale; the deferred RMSNorm row scale of the producer's hand-off (NORM 3) or
//      none; the shared epilogue.
#include <algorithm>

#include "gemm_epilogue.h"

namespace vgate {

__device__ __forceinline__ bf16x8 awq_raw8(uint32_t q) {  // nibble order of ops.pack_awq
  uint4 r;
  r.x = (q & 0x000F000Fu) | 0x43004300u;
  r.y = ((q >> 4) & 0x000F000Fu) | 0x43004300u;
  r.z = ((q >> 8) & 0x000F000Fu) | 0x43004300u;
  r.w = ((q >> 12) & 0x000F000Fu) | 0x43004300u;
  return as_bf16x8(r);
}

constexpr int AW_KQ = 16;  // k-quads per tile held in registers (K <= 2048)

template <int KQM, int EPI, int NORM>  // KQM >= K / 128: registers of int4 fragments per wave
__global__ __launch_bounds__(1024) void awq_wide_kernel(GemmParams p) {
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
      const int row = r16 < p.M ? r16 : p.M - 1;
      glds16(p.x + (size_t)row_of(p, row) * p.lda + (size_t)f * 32 + 8 * (lane >> 4),
             __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)f * 1024u));
    } else {
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
  for (int q = wid; q < KQ; q += nw) {
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
    if (q < KQ) {  // wave-uniform
      f32x4 pr = {0.f, 0.f, 0.f, 0.f};
      pr = mfma16(awq_raw8(w[q].x), as_bf16x8(xs[(4 * q + 0) * 64 + lane]), pr);
      pr = mfma16(awq_raw8(w[q].y), as_bf16x8(xs[(4 * q + 1) * 64 + lane]), pr);
      pr = mfma16(awq_raw8(w[q].z), as_bf16x8(xs[(4 * q + 2) * 64 + lane]), pr);
      pr = mfma16(awq_raw8(w[q].w), as_bf16x8(xs[(4 * q + 3) * 64 + lane]), pr);
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

// Returns false (caller keeps the other int4 kernels) unless: M <= 16, no RMSNorm gamma in registers
// (NORM 0, or the producer's hand-off), the packed scales (group 128), K <= 2048, N >= one tile
// per CU, <= 16 tiles per block.
template <int EPI, int NORM>
static bool launch_awq_wide_epi(const GemmParams& p, hipStream_t st) {
  const int ntiles = p.N / 16, KQ = p.K / 128;
  static const int ncu = [] {
    int n = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int nb = std::min(ntiles, ncu);
  const int tmax = (ntiles + nb - 1) / nb;
  if (KQ > AW_KQ || tmax > 16 || ntiles < nb) return false;
  const int szp = (tmax * KQ * 64 + 1023) / 1024;
  const size_t lds = (size_t)KQ * 4 * 1024 + (size_t)szp * 1024 + (size_t)KQ * 16 * 4;
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("awq_wide", nb);
#define VG_AWK(Q_)                                                                                     \
  do {                                                                                                 \
    auto kern = awq_wide_kernel<Q_, EPI, NORM>;                                                        \
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                        \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==  \
                       hipSuccess;                                                                     \
    (void)attr;                                                                                        \
    hipLaunchKernelGGL(kern, dim3(nb), dim3(64 * tmax), lds, st, q);                                   \
  } while (0)
  if (KQ <= 8) VG_AWK(8);
  else if (KQ <= 12) VG_AWK(12);
  else VG_AWK(16);
#undef VG_AWK
  return true;
}

bool launch_awq_wide(const GemmArgs& g, hipStream_t st) {
  if (g.M > 16 || g.M <= 0 || g.norm_w != nullptr || g.awq_szp == nullptr || g.group != 128 || g.N % 16 != 0 ||
      g.K % 128 != 0 || g.rownorm)
    return false;
  GemmParams p{};
  p.x = g.x; p.lda = g.lda; p.M = g.M; p.row_idx = g.row_idx;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.norm_w = nullptr; p.eps = g.eps;
  p.bias = g.bias; p.res = g.res; p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.splitk = 1;
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.szp = g.awq_szp; p.group = g.group;
  p.dbg_ts = g.dbg_ts;
  p.hg = g.hg; p.hg_gamma = g.hg_gamma; p.ssp_out = g.ssp_out; p.ssp_in = g.ssp_in; p.ssn = g.ssn;
  const bool pre = g.ssp_in != nullptr;
#define VG_AW(E) return pre ? launch_awq_wide_epi<E, 3>(p, st) : launch_awq_wide_epi<E, 0>(p, st)
  switch (g.epi) {
    case EPI_SILU: VG_AW(EPI_SILU);
    case EPI_QKV: VG_AW(EPI_QKV);
    case EPI_F32: VG_AW(EPI_F32);
    default: VG_AW(EPI_BF16);
  }
#undef VG_AW
}

}  // namespace vgate
