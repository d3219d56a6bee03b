// AWQ W4A16 GEMM for mixed prefill + decode steps (16 < M <= 64 rows). (Decode batches, M <= 16:
// gemm_awq_kx.hip; longer prompts: the bf16 prefill kernel on a dequantised scratch copy, gemm.hip.)
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

// ---- AWQ W4A16 for mixed prefill + decode steps (16 < M <= 64) ----
// Without it a long int4 step dequantises every matrix into a bf16 scratch first (4 x the int4
// bytes written, then read back by the bf16 kernels: a Qwen2.5-1.5B AWQ step with a 48-token
// prompt beside 7 decode rows took 3.5 ms against 2.4 ms for bf16, profiles/r3_mixed_step.log).
// Here the int4 fragments stream straight into registers (one wave per tile, all k-quads of its
// K slice in flight) and x is staged in LDS a PAIR of m-tiles (32 rows) at a time; a block-wide
// pass over each staged pair applies the RMSNorm gamma (NORM 1: the int4 weights cannot carry it),
// accumulates the raw rows' sums of squares, and forms the per-(k-quad, row) activation sums X of
// the raw-nibble identity, so the MFMA loop is LDS reads, four MFMAs and the group scale.
// Grid: `wide` = one block per CU owning whole tiles (N >= one tile per CU: no K split), else
// (tiles / W, S) with W tiles per block and S K slices combined by prefill_reduce_kernel.
template <int MT, int KQM, int EPI, int NORM>
__global__ __launch_bounds__(512) void awq_mid_kernel(GemmParams p, int wide) {  // <= 8 waves: 256 VGPRs
  extern __shared__ __attribute__((aligned(16))) char smem[];  // x [4 nkq][PH][64][16 B] | X | ssp
  TLScope tl_scope(p.dbg_ts);
  constexpr int PH = MT == 1 ? 1 : 2;
  constexpr int NPH = (MT + PH - 1) / PH;
  const int lane = threadIdx.x & 63, r16 = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int KQ = p.K >> 7, ntiles = p.N >> 4;
  int t0, ntb, z, S;
  if (wide) {
    t0 = (int)(((long long)ntiles * blockIdx.x) / gridDim.x);
    ntb = (int)(((long long)ntiles * (blockIdx.x + 1)) / gridDim.x) - t0;
    z = 0;
    S = 1;
  } else {
    t0 = blockIdx.x * nw;
    ntb = nw;
    z = blockIdx.y;
    S = gridDim.y;
  }
  const int q0 = (KQ * z) / S, nkq = (KQ * (z + 1)) / S - q0;  // <= KQM (host-checked)
  const bool active = wid < ntb;
  const int nt = t0 + (active ? wid : 0);
  const uint32_t lds0 = lds_addr_of(smem);
  const size_t x_bytes = (size_t)nkq * 4 * PH * 1024;
  float* Xs = reinterpret_cast<float*>(smem + x_bytes);  // [nkq][PH][16]
  float* ssp = Xs + nkq * PH * 16;                        // [nkq][MT][16] (NORM 1)
  uint4* xs = reinterpret_cast<uint4*>(smem);
  auto dma_x = [&](int ph) {  // piece f = (k-step f / PH, m-tile PH ph + f % PH)
    for (int f = wid; f < 4 * nkq * PH; f += nw) {
      int row = (PH * ph + f % PH) * 16 + r16;
      row = row < p.M ? row : p.M - 1;
      glds16(p.x + (size_t)row * p.lda + (size_t)(q0 * 4 + f / PH) * 32 + 8 * (lane >> 4),
             __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)f * 1024u));
    }
  };
  dma_x(0);
  uint4 w[KQM], sz[KQM];
  if (active) {
    const uint4* wb = p.wp + ((size_t)nt * KQ + q0) * 64 + lane;
    const uint4* sb = reinterpret_cast<const uint4*>(p.szp) + ((size_t)nt * KQ + q0) * 4 + (lane >> 4);
#pragma unroll
    for (int q = 0; q < KQM; ++q) {
      const int qq = min(q, nkq - 1);
      w[q] = ld_nt16(wb + (size_t)qq * 64);
      sz[q] = sb[(size_t)qq * 4];
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * KQM) : "memory");  // the x pieces only
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ph = 0; ph < NPH; ++ph) {
    if (ph > 0) {
      __syncthreads();  // every wave is done with the previous pair
      dma_x(ph);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // block-wide pass over the staged pair: gamma (NORM 1), raw sums of squares, X per (k-quad, row)
    for (int u = wid; u < nkq * PH; u += nw) {
      const int kq = u / PH, i = u % PH;
      float xsum = 0.f, s2 = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint4* fp = xs + ((4 * kq + t) * PH + i) * 64 + lane;
        float f[8];
        unpack8(*fp, f);
        if constexpr (NORM == 1) {
          float g8[8];
          unpack8(ld16(p.norm_w + (size_t)(q0 * 4 + 4 * kq + t) * 32 + 8 * (lane >> 4)), g8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            s2 += f[j] * f[j];
            f[j] *= g8[j];
          }
          const uint4 pk = pack8(f);
          *fp = pk;
          unpack8(pk, f);  // X sums the bf16 values the MFMA reads
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) xsum += f[j];
      }
      xsum += xor16(xsum);
      xsum += xor32(xsum);
      if (lane < 16) Xs[(kq * PH + i) * 16 + lane] = xsum;
      if constexpr (NORM == 1) {
        s2 += xor16(s2);
        s2 += xor32(s2);
        if (lane < 16 && PH * ph + i < MT) ssp[(kq * MT + PH * ph + i) * 16 + lane] = s2;
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < KQM; ++q) {
        if (q < nkq) {
          const float s4[4] = {bf_lo(sz[q].x), bf_hi(sz[q].x), bf_lo(sz[q].y), bf_hi(sz[q].y)};
          const float z4[4] = {bf_lo(sz[q].z), bf_hi(sz[q].z), bf_lo(sz[q].w), bf_hi(sz[q].w)};
#pragma unroll
          for (int i = 0; i < PH; ++i) {
            if (PH * ph + i < MT) {
              const uint4* xq = xs + ((4 * q) * PH + i) * 64 + lane;
              f32x4 pr = {0.f, 0.f, 0.f, 0.f};
              pr = mfma16(awq_raw8(w[q].x), as_bf16x8(xq[0 * PH * 64]), pr);
              pr = mfma16(awq_raw8(w[q].y), as_bf16x8(xq[1 * PH * 64]), pr);
              pr = mfma16(awq_raw8(w[q].z), as_bf16x8(xq[2 * PH * 64]), pr);
              pr = mfma16(awq_raw8(w[q].w), as_bf16x8(xq[3 * PH * 64]), pr);
              const float X = Xs[(q * PH + i) * 16 + r16];
#pragma unroll
              for (int c = 0; c < 4; ++c)
                acc[PH * ph + i][c] = fmaf(s4[c], pr[c], fmaf(-fmaf(128.f, s4[c], z4[c]), X, acc[PH * ph + i][c]));
            }
          }
        }
      }
    }
  }
  if (!active) return;
  const int nsub = 4 * (lane >> 4);
  float ssr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    ssr[mt] = 0.f;
    if constexpr (NORM == 1)
      for (int kq = 0; kq < nkq; ++kq) ssr[mt] += ssp[(kq * MT + mt) * 16 + r16];  // fixed k-quad order
  }
  if constexpr (NORM == 3) {  // the producer's hand-off: x = h * gamma, rows' sums of squares in ssp_in
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float ss = prenorm_ss(p, mt * 16 + r16, lane >> 4);
      ss += xor16(ss);
      ss += xor32(ss);
      acc[mt] *= rsqrtf(ss / (float)p.K + p.eps);  // a per-row constant: exact on each K slice's partial
    }
  }
  if (S > 1) {
    float* part = p.slabs + (size_t)z * p.M * p.N;
    float* ssq = p.slabs + (size_t)S * p.M * p.N + (size_t)z * p.M;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + r16;
      if (NORM == 1 && blockIdx.x == 0 && wid == 0 && lane < 16 && m < p.M) ssq[m] = ssr[mt];
      if (m < p.M) *reinterpret_cast<f32x4*>(part + (size_t)m * p.N + nt * 16 + nsub) = acc[mt];
    }
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r16;
    f32x4 v[1] = {acc[mt]};
    if constexpr (NORM == 1) v[0] *= rsqrtf(ssr[mt] / (float)p.K + p.eps);
    epilogue<1, EPI, false>(p, v, m, nt, nsub, EpiPre<1>{}, m < p.M);
  }
}

template <int EPI, int NORM, int NTB>
void launch_prefill_reduce(const GemmParams& p, int nz, hipStream_t st);

static int cu_count_awq() {
  static const int n = [] {
    int v = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

template <int EPI, int NORM>
static bool launch_awq_mid_epi(const GemmParams& p, int force_w, int force_s, size_t slab_bytes, hipStream_t st) {
  const int ntiles = p.N / 16, KQ = p.K / 128, MT = (p.M + 15) / 16, PH = MT == 1 ? 1 : 2;
  const int ncu = cu_count_awq();
  int wide = 0, W = 0, S = 1, nb = 0;
  if (force_w == 8 || (force_w <= 0 && ntiles >= ncu && KQ <= 16 && (ntiles + ncu - 1) / ncu <= 8)) {
    wide = 1;
    nb = ncu;
    W = (ntiles + ncu - 1) / ncu;
    if (KQ > 16 || W > 8 || ntiles < ncu) return false;
  } else {
    W = force_w > 0 ? force_w : (ntiles % 4 == 0 ? 4 : ntiles % 2 == 0 ? 2 : 1);
    if (W < 1 || W > 8 || ntiles % W != 0) return false;
    S = force_s > 0 ? force_s : 1;
    if (force_s <= 0) {
      while ((KQ + S - 1) / S > 16) ++S;
      while ((ntiles / W) * S < 192 && (KQ + 2 * S - 1) / (2 * S) >= 2) S *= 2;
    }
    if (S < 1 || S > KQ || (KQ + S - 1) / S > 16) return false;
    if (S > 1 && (p.slabs == nullptr || ((size_t)S * p.M * p.N + (size_t)S * p.M) * 4 > slab_bytes)) return false;
    nb = ntiles / W;
  }
  const int nkq = (KQ + S - 1) / S;
  const size_t lds = (size_t)nkq * 4 * PH * 1024 + (size_t)nkq * PH * 16 * 4 + (size_t)nkq * MT * 16 * 4;
  if (lds > 160 * 1024) return false;
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take(wide ? "awq_mid_wide" : "awq_mid", nb * S);
  const dim3 grid(nb, S), block(64 * W);
#define VG_AM(MT_, Q_)                                                                                 \
  do {                                                                                                 \
    auto kern = awq_mid_kernel<MT_, Q_, EPI, NORM>;                                                    \
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                        \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==  \
                       hipSuccess;                                                                     \
    (void)attr;                                                                                        \
    hipLaunchKernelGGL(kern, grid, block, lds, st, q, wide);                                           \
  } while (0)
#define VG_AMQ(MT_)                     \
  do {                                  \
    if (nkq <= 4) VG_AM(MT_, 4);        \
    else if (nkq <= 8) VG_AM(MT_, 8);   \
    else if (nkq <= 12) VG_AM(MT_, 12); \
    else VG_AM(MT_, 16);                \
  } while (0)
  if (MT == 1) VG_AMQ(1);
  else if (MT == 2) VG_AMQ(2);
  else if (MT == 3) VG_AMQ(3);
  else VG_AMQ(4);
#undef VG_AMQ
#undef VG_AM
  if (S > 1) launch_prefill_reduce<EPI, NORM == 1 ? 2 : 0, 1>(p, S, st);
  return true;
}

bool launch_awq_mid(const GemmArgs& g, hipStream_t st) {
  // (decode batches too, M <= 16, when a decode plan asks for it: the hand-off consumer mode included)
  if (g.M <= 0 || g.M > 64 || g.awq_szp == nullptr || g.group != 128 || g.N % 16 != 0 || g.K % 128 != 0 ||
      g.rownorm || (g.ssp_in != nullptr && g.norm_w != nullptr) || g.row_idx != nullptr)
    return false;
  GemmParams p{};
  p.x = g.x; p.lda = g.lda; p.M = g.M; p.row_idx = nullptr;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.norm_w = g.norm_w; p.eps = g.eps;
  p.bias = g.bias; p.res = g.res; p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.splitk = 1;
  p.slabs = g.slabs;
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.szp = g.awq_szp; p.group = g.group;
  p.dbg_ts = g.dbg_ts;
  p.hg = g.hg; p.hg_gamma = g.hg_gamma; p.ssp_out = g.ssp_out; p.ssp_in = g.ssp_in; p.ssn = g.ssn;
  const bool gam = g.norm_w != nullptr, pre = g.ssp_in != nullptr;
#define VG_AMD(E)                                                                  \
  return gam ? launch_awq_mid_epi<E, 1>(p, g.waves, g.splitk, g.slab_bytes, st)    \
       : pre ? launch_awq_mid_epi<E, 3>(p, g.waves, g.splitk, g.slab_bytes, st)    \
             : launch_awq_mid_epi<E, 0>(p, g.waves, g.splitk, g.slab_bytes, st)
  switch (g.epi) {
    case EPI_SILU: VG_AMD(EPI_SILU);
    case EPI_QKV: VG_AMD(EPI_QKV);
    case EPI_F32: VG_AMD(EPI_F32);
    default: VG_AMD(EPI_BF16);
  }
#undef VG_AMD
}

}  // namespace vgate
