// Medium-M GEMM (16 < M <= 64 rows: the mixed steps of a serving load, one prompt chunk beside
// the decode rows) on the fragment-packed bf16 weights.
//
// At these M the step is still a weight stream (the weights of a layer are read once, the
// activations are a few hundred KB), but neither neighbour path streams well there: the K-split
// decode kernels re-load all M rows of x per wave (4 activation loads per weight load at M = 64)
// and keep one or two register groups in flight, and the LDS tile kernel prefetches one 8-k-step
// stage of weights: in-engine, a 48-token prompt beside 7 decode rows made a Qwen2.5-1.5B step
// 2.77 ms against 1.24 ms for pure decode, gate_up 30 us and down_proj 27 us per layer against
// 14 / 10 at M = 8 (profiles/r3_mixed_step.log).
//
// Here a block is W waves = W adjacent 16-column tiles (one per wave) over one K slice of at most
// KS k-steps:
//   1. the slice of x (MT m-tiles x KS k-steps, 1 KiB fragment-major pieces, rows past M repeat
//      row M - 1) is DMA'd into LDS (global_load_lds_dwordx4), spread over the W waves;
//   2. every wave then issues ALL KS weight fragments of its tile (non-temporal 16-B loads into
//      registers): the whole launch's weights are requested in the first microsecond;
//   3. one counted vmcnt (the x pieces only) + barrier, then per k-step MT conflict-free
//      ds_read_b128 of x and MT MFMAs 16x16x32 on the fragment as it lands (the compiler's
//      partial vmcnt waits follow issue order);
//   4. one slice (S == 1): the shared epilogue straight from the accumulators (deferred RMSNorm
//      row scale from the x^2 of the LDS image); S > 1: fp32 partial slabs [z][M][N] + per-slice
//      row sums of squares [z][M] for prefill_reduce_kernel (fixed slice order: bit-reproducible).
#include <algorithm>
#include <cstdlib>

#include "gemm_epilogue.h"

namespace vgate {

static int cu_count_mid() {
  static const int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

template <int MT, int KS, int EPI, int NORM>
__global__ __launch_bounds__(256) void gemm_mid_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [KS][MT][64][16 B]
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = blockDim.x >> 6;
  const int KT = p.K >> 5;
  const int z = blockIdx.y, S = gridDim.y;
  const int k0 = (KT * z) / S, nks = (KT * (z + 1)) / S - k0;  // nks <= KS (host-checked)
  const int nt = blockIdx.x * W + wid;
  // 1) x slice -> LDS: piece f = (k-step f / MT, m-tile f % MT); wave w takes f = w, w + W, ...
  const uint32_t lds0 = lds_addr_of(smem);
  const int npc = nks * MT;
  for (int f = wid; f < npc; f += W) {
    const int ks = f / MT, mt = f % MT;
    int row = mt * 16 + (lane & 15);
    row = row < p.M ? row : p.M - 1;
    const bf16_t* src = p.x + (size_t)row * p.lda + (size_t)(k0 + ks) * 32 + 8 * (lane >> 4);
    glds16(src, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)f * 1024u));
  }
  // 2) every weight fragment of this wave's tile slice (clamped past the slice: never consumed)
  uint4 w[KS];
  const uint4* wb = p.wp + ((size_t)nt * KT + k0) * 64 + lane;
#pragma unroll
  for (int u = 0; u < KS; ++u) w[u] = ld_nt16(wb + (size_t)min(u, nks - 1) * 64);
  // 3) the x pieces (issued before the KS weight loads) have landed in every wave
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KS) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ss[mt] = 0.f;
  const uint4* xs = reinterpret_cast<const uint4*>(smem);
#pragma unroll
  for (int u = 0; u < KS; ++u) {
    if (u < nks) {  // wave-uniform
      uint4 xb[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xb[mt] = xs[(u * MT + mt) * 64 + lane];
      if constexpr (NORM == 2) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          float f[8];
          unpack8(xb[mt], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[mt] += f[j] * f[j];
        }
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16(as_bf16x8(w[u]), as_bf16x8(xb[mt]), acc[mt]);
    }
  }
  const int nsub = 4 * (lane >> 4);
  if (S > 1) {
    float* part = p.slabs + (size_t)z * p.M * p.N;
    float* ssq = p.slabs + (size_t)S * p.M * p.N + (size_t)z * p.M;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + (lane & 15);
      if constexpr (NORM == 2) {
        float s2 = ss[mt];
        s2 += xor16(s2);
        s2 += xor32(s2);
        if (blockIdx.x == 0 && wid == 0 && lane < 16 && m < p.M) ssq[m] = s2;
      }
      if (m < p.M) *reinterpret_cast<f32x4*>(part + (size_t)m * p.N + nt * 16 + nsub) = acc[mt];
    }
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + (lane & 15);
    f32x4 v[1] = {acc[mt]};
    if constexpr (NORM == 2) {
      float s2 = ss[mt];
      s2 += xor16(s2);
      s2 += xor32(s2);
      v[0] *= rsqrtf(s2 / (float)p.K + p.eps);
    }
    epilogue<1, EPI, false>(p, v, m, nt, nsub, EpiPre<1>{}, m < p.M);
  }
}

// ---- wide N (more column tiles than CUs): one block per CU, no cross-block combine ----
// A K split over blocks costs a partial-slab round trip of slices x M x N x 4 bytes (gate_up at
// M = 64: 4.6 MB per slice) plus a reduce launch, and an x slice per wave set; with N wide
// enough every CU can own WHOLE tiles instead: block b owns tiles [N b / B, N (b + 1) / B) (4-5 of
// Qwen2.5-1.5B's 1120 gate_up tiles on 256 CUs: one round, no tail of late blocks), each tile's K
// is cut into KP parts of <= 16 k-steps, one wave per (tile, part) holding all of its weight
// fragments in registers (64 VGPRs, issued at launch: ~200 KB per CU in flight). x is shared
// through LDS, a PAIR of m-tiles (32 rows x full K, 2 KB per k-step) at a time: the weights stay
// in registers while the second pair is DMA'd in. The parts of a tile meet in LDS (fixed part
// order: bit-reproducible) and the part-0 wave runs the epilogue.
template <int MT, int EPI, int NORM>
__global__ __launch_bounds__(1024) void gemm_midw_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // x [KT][PH][64][16 B] | red, ssq
  TLScope tl_scope(p.dbg_ts);
  constexpr int PH = MT == 1 ? 1 : 2;  // m-tiles per x phase
  constexpr int NPH = (MT + PH - 1) / PH;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int KT = p.K >> 5, KP = (KT + 15) >> 4;
  const int ntiles = p.N >> 4, nb = gridDim.x, b = blockIdx.x;
  const int t0 = (int)(((long long)ntiles * b) / nb), ntb = (int)(((long long)ntiles * (b + 1)) / nb) - t0;
  const int my = wid / KP, part = wid - my * KP;
  const bool active = my < ntb;  // wave-uniform
  const int nt = t0 + (active ? my : 0);
  const int kb = part * 16, nks = min(16, KT - kb);
  uint4 w[16];
  const uint32_t lds0 = lds_addr_of(smem);
  const uint4* xs = reinterpret_cast<const uint4*>(smem);
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ss[mt] = 0.f;
#pragma unroll
  for (int ph = 0; ph < NPH; ++ph) {
    if (ph > 0) __builtin_amdgcn_s_barrier();  // every wave is done reading the previous phase's x
    // x pieces of m-tiles (PH ph ..): piece f = (k-step f / PH, m-tile PH ph + f % PH)
    for (int f = wid; f < PH * KT; f += nw) {
      int row = (PH * ph + f % PH) * 16 + (lane & 15);
      row = row < p.M ? row : p.M - 1;
      glds16(p.x + (size_t)row * p.lda + (size_t)(f / PH) * 32 + 8 * (lane >> 4),
             __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)f * 1024u));
    }
    if (ph == 0) {
      if (active) {
        const uint4* wb = p.wp + ((size_t)nt * KT + kb) * 64 + lane;
#pragma unroll
        for (int u = 0; u < 16; ++u) w[u] = ld_nt16(wb + (size_t)min(u, nks - 1) * 64);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // the x pieces, issued before the weights
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (active) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (u < nks) {
#pragma unroll
          for (int i = 0; i < PH; ++i) {
            if (PH * ph + i < MT) {
              const uint4 xv = xs[((kb + u) * PH + i) * 64 + lane];
              if constexpr (NORM == 2) {
                float f[8];
                unpack8(xv, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) ss[PH * ph + i] += f[j] * f[j];
              }
              acc[PH * ph + i] = mfma16(as_bf16x8(w[u]), as_bf16x8(xv), acc[PH * ph + i]);
            }
          }
        }
      }
    }
  }
  const int nsub = 4 * (lane >> 4);
  if (KP == 1) {  // one part per tile: the epilogue straight from the accumulators
    if (!active) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + (lane & 15);
      f32x4 v[1] = {acc[mt]};
      if constexpr (NORM == 2) {
        float s2 = ss[mt];
        s2 += xor16(s2);
        s2 += xor32(s2);
        v[0] *= rsqrtf(s2 / (float)p.K + p.eps);
      }
      epilogue<1, EPI, false>(p, v, m, nt, nsub, EpiPre<1>{}, m < p.M);
    }
    return;
  }
  // parts meet in LDS: red [wave][mt][64] f32x4, then ssq [wave][mt][16]
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  float* ssq = reinterpret_cast<float*>(smem + (size_t)nw * MT * 1024);
  if (active) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      red[(wid * MT + mt) * 64 + lane] = acc[mt];
      if constexpr (NORM == 2) {
        float s2 = ss[mt];
        s2 += xor16(s2);
        s2 += xor32(s2);
        if (lane < 16) ssq[(wid * MT + mt) * 16 + lane] = s2;
      }
    }
  }
  __syncthreads();
  if (!active || part != 0) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + (lane & 15);
    f32x4 v[1] = {red[(wid * MT + mt) * 64 + lane]};
    float s2 = NORM == 2 ? ssq[(wid * MT + mt) * 16 + (lane & 15)] : 0.f;
    for (int q = 1; q < KP; ++q) {
      v[0] += red[((wid + q) * MT + mt) * 64 + lane];
      if constexpr (NORM == 2) s2 += ssq[((wid + q) * MT + mt) * 16 + (lane & 15)];
    }
    if constexpr (NORM == 2) v[0] *= rsqrtf(s2 / (float)p.K + p.eps);
    epilogue<1, EPI, false>(p, v, m, nt, nsub, EpiPre<1>{}, m < p.M);
  }
}

// defined in gemm_prefill.hip (split-K combine + epilogue, shared with the prefill kernels)
template <int EPI, int NORM, int NTB>
void launch_prefill_reduce(const GemmParams& p, int nz, hipStream_t st);

template <int MT, int EPI, int NORM>
static void launch_mid_mt(const GemmParams& p, int W, int S, int ks, hipStream_t st) {
  const dim3 grid(p.N / 16 / W, S), block(64 * W);
  const size_t lds = (size_t)ks * MT * 1024;
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("gemm_mid", (int)(grid.x * grid.y));
#define VG_MID(K_)                                                                         \
  do {                                                                                     \
    auto kern = gemm_mid_kernel<MT, K_, EPI, NORM>;                                        \
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),            \
                                           hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                           K_ * MT * 1024) == hipSuccess;                  \
    (void)attr;                                                                            \
    hipLaunchKernelGGL(kern, grid, block, lds, st, q);                                     \
  } while (0)
  if (ks <= 8) VG_MID(8);
  else if (ks <= 12) VG_MID(12);
  else if (ks <= 16) VG_MID(16);
  else if (ks <= 24) VG_MID(24);
  else VG_MID(32);
#undef VG_MID
  if (S > 1) launch_prefill_reduce<EPI, NORM, 1>(p, S, st);
}

// Heuristic decomposition (force_w / force_s: the start-up tuner's plan): W = 4 tiles per block
// when N allows, then the fewest K slices (<= 32 k-steps each, LDS <= 128 KiB) that put >= 192
// blocks on the chip.
template <int EPI, int NORM>
static bool launch_mid_epi(const GemmParams& p, int force_w, int force_s, size_t slab_bytes, hipStream_t st) {
  const int ntiles = p.N / 16, KT = p.K / 32;
  const int MT = (p.M + 15) / 16;
  int W = force_w > 0 ? force_w : (ntiles % 4 == 0 ? 4 : ntiles % 2 == 0 ? 2 : 1);
  if (W < 1 || W > 4 || ntiles % W != 0) return false;
  const int groups = ntiles / W;
  int S = force_s > 0 ? force_s : 1;
  if (force_s <= 0) {
    while ((KT + S - 1) / S > 32) ++S;
    while (groups * S < 192 && (KT + 2 * S - 1) / (2 * S) >= 4) S *= 2;
  }
  const int ks = (KT + S - 1) / S;
  if (S < 1 || S > KT || ks > 32) return false;
  if (S > 1 && (p.slabs == nullptr || ((size_t)S * p.M * p.N + (size_t)S * p.M) * 4 > slab_bytes)) return false;
  if (MT <= 2) launch_mid_mt<2, EPI, NORM>(p, W, S, ks, st);
  else if (MT == 3) launch_mid_mt<3, EPI, NORM>(p, W, S, ks, st);
  else launch_mid_mt<4, EPI, NORM>(p, W, S, ks, st);
  return true;
}

// the wide form (g.waves == 8 selects it): N of at least one tile per CU, (tiles per block) x
// (16-k-step parts per tile) <= 16 waves, K <= 64 k-steps (the pair image fits 128 KiB of LDS)
template <int EPI, int NORM>
static bool launch_midw_epi(const GemmParams& p, hipStream_t st) {
  const int ntiles = p.N / 16, KT = p.K / 32, KP = (KT + 15) / 16;
  const int nb = std::min(ntiles, cu_count_mid());
  const int tmax = (ntiles + nb - 1) / nb;
  if (KT > 64 || KP * tmax > 16 || ntiles < nb) return false;
  const int MT = (p.M + 15) / 16;
  const dim3 grid(nb), block(64 * KP * tmax);
  const size_t lds = std::max<size_t>((size_t)KT * (MT == 1 ? 1 : 2) * 1024, (size_t)KP * tmax * MT * (1024 + 64));
  GemmParams q = p;
  if (q.dbg_ts == nullptr) q.dbg_ts = tl_take("gemm_midw", nb);
#define VG_MW(P_)                                                                                      \
  do {                                                                                                 \
    auto kern = gemm_midw_kernel<P_, EPI, NORM>;                                                       \
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                        \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==  \
                       hipSuccess;                                                                     \
    (void)attr;                                                                                        \
    hipLaunchKernelGGL(kern, grid, block, lds, st, q);                                                 \
  } while (0)
  if (MT == 1) VG_MW(1);
  else if (MT == 2) VG_MW(2);
  else if (MT == 3) VG_MW(3);
  else VG_MW(4);
#undef VG_MW
  return true;
}

bool launch_gemm_mid(const GemmArgs& g, hipStream_t st) {
  // (the wide form also takes decode batches, M <= 16: one m-tile, one x phase)
  if ((g.M <= 16 && g.waves != 8) || g.M > 64 || g.row_idx != nullptr || g.norm_w != nullptr || g.N % 16 != 0 ||
      g.K % 32 != 0)
    return false;
  GemmParams p{};
  p.x = g.x; p.lda = g.lda; p.M = g.M; p.row_idx = nullptr;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.norm_w = nullptr; p.eps = g.eps;
  p.bias = g.bias; p.res = g.res; p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.splitk = 1;
  p.slabs = g.slabs;
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.dbg_ts = g.dbg_ts;
  const int norm = g.rownorm ? 2 : 0;
#define VG_MD(E)                                                                             \
  if (g.waves == 8) return norm == 2 ? launch_midw_epi<E, 2>(p, st) : launch_midw_epi<E, 0>(p, st); \
  return norm == 2 ? launch_mid_epi<E, 2>(p, g.waves, g.splitk, g.slab_bytes, st)           \
                   : launch_mid_epi<E, 0>(p, g.waves, g.splitk, g.slab_bytes, st)
  switch (g.epi) {
    case EPI_SILU: VG_MD(EPI_SILU);
    case EPI_QKV: VG_MD(EPI_QKV);
    case EPI_F32: VG_MD(EPI_F32);
    default: VG_MD(EPI_BF16);
  }
#undef VG_MD
}

}  // namespace vgate
