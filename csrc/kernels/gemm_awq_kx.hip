// AWQ W4A16 decode GEMM (M <= 16), register-stationary activations ("kx").
//
// An int4 k-quad of one 16-column tile is 1 KiB of weights, but at M = 8 the k-quad's activations are
// 2 KiB and its (s, s z) record is fetched as a 1 KiB lane load: a kernel that pairs every weight
// fragment with its own activation and scale loads spends most of the CU's vector-memory requests on
// bytes that are not weights. And once the bytes are in, the nibble -> bf16 unpack (MFMA A operand)
// and the group scale cost ~45 VALU instructions per (tile, k-quad) — for Qwen2.5-1.5B gate_up
// (1120 tiles x 12 k-quads over 256 CUs) ~0.9 us of VALU time per SIMD, as long as a third of the
// HBM stream. The earlier int4 kernels serialised that work behind the stream (one wave per tile:
// awq_wide 9.85 us) or behind LDS staging of x (benchmarks/probes/awq_wide_anatomy.hip).
//
// Here the waves of a block split K and every wave keeps ITS activation fragments in registers
// (XP-packed: one 16-B load covers XP k-steps of M <= 16 / XP real rows) while it streams the int4
// fragments and packed scales of ALL the block's tiles over its k-range: the activation loads are
// amortised over the block's tiles, no LDS staging or block barrier precedes the MFMAs, and the
// unpack / scale VALU work is spread over 12-16 waves (3-4 per SIMD: MFMA, VALU and the weight stream
// of different waves overlap). Every load of a wave is issued before its first MFMA.
//
//   raw-nibble identity: sum_k x (v - z) s = s * sum_k x (128 + v) - (128 s + s z) * X,
//   X = the k-quad's activation sum per row (v_dot2 with (1, 1) over the B fragments).
//   bf16(128 + v) = (nibbles & 0x000F000F) | 0x43004300: one v_and_or_b32 per 2 values (+ a shift).
//
// Two grid forms:
//   WIDE  (N >= one tile per CU, gate_up): one block per CU owning whole tiles [t0, t0 + ntb),
//         ntb <= TMAX; the waves' partials meet in LDS and wave j finishes tile t0 + j.
//   TILE  (narrow N: qkv, o_proj, down_proj): one tile per block, gridDim.z K slices; the waves'
//         partials, the slices (granules / slabs) and the epilogue are gemm_finish's, with the
//         epilogue operands (residual, bias, RoPE position / cos-sin) prefetched at launch.
// NORM: 0 none; 1 RMSNorm gamma in registers (x * gamma in bf16, raw x^2 summed; layer 0 of the
// hand-off chain); 3 the producer's hand-off (x = h * gamma, row sums of squares in ssp_in).
#include "gemm_decode.h"

namespace vgate {

// bf16 (128 + v) of the 8 nibbles of one dword (ops.pack_awq order: element j of k-step u at bits
// 16 (j & 1) + 4 (j >> 1)): 3 shifts + 4 v_and_or_b32 (the compiler emits and + or: 11 VALU). The
// results feed MFMA A operands, and the hazard recognizer does not see through inline asm: the block
// ends with the 2 wait states a VALU-written VGPR needs before an MFMA reads it.
__device__ __forceinline__ bf16x8 kx_raw8(uint32_t q, uint32_t m, uint32_t o) {
  uint32_t r0, r1, r2, r3;
  asm("v_lshrrev_b32 %1, 4, %4\n\t"
      "v_lshrrev_b32 %2, 8, %4\n\t"
      "v_lshrrev_b32 %3, 12, %4\n\t"
      "v_and_or_b32 %0, %4, %5, %6\n\t"
      "v_and_or_b32 %1, %1, %5, %6\n\t"
      "v_and_or_b32 %2, %2, %5, %6\n\t"
      "v_and_or_b32 %3, %3, %5, %6\n\t"
      "s_nop 1"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(q), "v"(m), "v"(o));
  return as_bf16x8(make_uint4(r0, r1, r2, r3));
}

typedef __bf16 kx_bf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float kx_sum8(uint4 v, float acc) {  // acc + the 8 bf16 of v
  const kx_bf2 one = __builtin_bit_cast(kx_bf2, 0x3f803f80u);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(kx_bf2, v.x), one, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(kx_bf2, v.y), one, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(kx_bf2, v.z), one, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(kx_bf2, v.w), one, acc, false);
  return acc;
}

constexpr int KX_SSL = 8;  // NORM 3 prefetch: f32x4 loads per lane (ssn <= 128, ssn % 16 == 0)

// the producer's per-tile sums of squares of row m, this lane's quarter, loaded at launch (NORM 3)
struct KxSs {
  f32x4 r[KX_SSL];
  int n4;  // 0: prenorm_ss after the stream (ssn not in the prefetch form)
};
__device__ __forceinline__ void kx_ss_issue(const GemmParams& p, KxSs& s, int m, int quarter) {
  s.n4 = (p.ssn & 15) == 0 && p.ssn <= 16 * KX_SSL && m < p.M ? p.ssn >> 4 : 0;
  const f32x4* src = reinterpret_cast<const f32x4*>(p.ssp_in + (size_t)(m < p.M ? m : 0) * p.ssn + quarter * (p.ssn >> 2));
#pragma unroll
  for (int u = 0; u < KX_SSL; ++u)
    if (u < s.n4) s.r[u] = src[u];
}
__device__ __forceinline__ float kx_ss_sum(const GemmParams& p, const KxSs& s, int m, int quarter) {
  if (s.n4 == 0) return prenorm_ss(p, m, quarter);
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < KX_SSL; ++u)
    if (u < s.n4) acc += (s.r[u][0] + s.r[u][1]) + (s.r[u][2] + s.r[u][3]);
  return acc;
}

// XP: k-steps per activation load (2: M <= 8, 1: M <= 16); KQW: k-quads per wave (host: >= the
// wave's range); TMAX: tiles per block (WIDE) or 1 (TILE). Registers of loads in flight per lane:
// kx_regs; up to 64 the block may hold 16 waves (128 VGPRs each), else 8.
template <int XP, int KQW, int TMAX, int NORM>
__host__ __device__ constexpr int kx_regs() { return 4 * KQW * ((4 / XP) * (NORM == 1 ? 2 : 1) + 2 * TMAX); }
template <int XP, int KQW, int TMAX, int NORM>
__host__ __device__ constexpr int kx_max_threads() { return kx_regs<XP, KQW, TMAX, NORM>() <= 64 ? 1024 : 512; }

template <int XP, int KQW, int TMAX, int EPI, int NORM, bool WIDE>
__global__ __launch_bounds__((kx_max_threads<XP, KQW, TMAX, NORM>())) void awq_kx_kernel(GemmParams p) {
  static_assert(WIDE || TMAX == 1, "TILE form: one tile per block");
  static_assert(!WIDE || EPI != EPI_QKV, "QKV tiles finish through gemm_finish (prefetched RoPE operands)");
  constexpr int R = 16 / XP;   // real rows one load covers
  constexpr int XL = 4 / XP;   // activation loads per k-quad
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63, r16 = lane & 15, grp = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int KQ = p.K >> 7, ntiles = p.N >> 4;
  int t0, ntb, s0, s1;
  if constexpr (WIDE) {
    t0 = (int)(((long long)ntiles * blockIdx.x) / gridDim.x);
    ntb = (int)(((long long)ntiles * (blockIdx.x + 1)) / gridDim.x) - t0;
    s0 = 0;
    s1 = KQ;
  } else {
    t0 = blockIdx.x;
    ntb = 1;
    s0 = (KQ * (int)blockIdx.z) / p.splitk;
    s1 = (KQ * ((int)blockIdx.z + 1)) / p.splitk;
  }
  const int q0 = s0 + ((s1 - s0) * wid) / nw;
  const int nq = s0 + ((s1 - s0) * (wid + 1)) / nw - q0;  // <= KQW (host-checked), may be 0
  // NORM 3: the row's sums of squares, issued first (consumed after the stream without waiting on it)
  KxSs ssv;
  ssv.n4 = 0;
  const bool ss_wave = WIDE ? wid < ntb : (wid == 0 && blockIdx.z == 0);
  if constexpr (NORM == 3) {
    if (ss_wave) kx_ss_issue(p, ssv, r16, grp);
  }
  // TILE form: the epilogue operands of wave 0's (row, 4 columns) item at launch
  EpiPre<1> pre;
  const bool epi_thr = !WIDE && threadIdx.x < 64;
  if (epi_thr) epi_pre_a<1, EPI>(p, pre, r16, t0, 4 * grp);
  // activations: lane (r16, grp) loads row r16 % R of k-step r16 / R (+ XP v) of each load
  const int mrow = r16 % R;
  const bool xok = mrow < p.M;
  const bf16_t* xrow = p.x + (size_t)row_of(p, mrow) * p.lda + 8 * grp + (XP > 1 ? (r16 / R) * 32 : 0);
  const bf16_t* grow = NORM == 1 ? p.norm_w + 8 * grp + (XP > 1 ? (r16 / R) * 32 : 0) : nullptr;
  const uint4* wbase = p.wp + (size_t)t0 * KQ * 64 + lane;
  const uint4* szbase = reinterpret_cast<const uint4*>(p.szp) + (size_t)t0 * KQ * 4 + grp;
  constexpr int GL = NORM == 1 ? XL : 1;
  uint4 xa[KQW][XL], ga[KQW][GL], w[KQW][TMAX], sz[KQW][TMAX];
#pragma unroll
  for (int q = 0; q < KQW; ++q) {
    const int kq = q0 + min(q, max(nq - 1, 0));
    if (q < nq) {  // wave-uniform
#pragma unroll
      for (int v = 0; v < XL; ++v)
        xa[q][v] = xok ? *reinterpret_cast<const uint4*>(xrow + (size_t)(kq * 4 + v * XP) * 32) : make_uint4(0, 0, 0, 0);
      if constexpr (NORM == 1) {
#pragma unroll
        for (int v = 0; v < XL; ++v) ga[q][v] = *reinterpret_cast<const uint4*>(grow + (size_t)(kq * 4 + v * XP) * 32);
      }
#pragma unroll
      for (int j = 0; j < TMAX; ++j) {
        const size_t u = (size_t)min(j, ntb - 1) * KQ + kq;
        w[q][j] = ld_nt16(wbase + u * 64);
        sz[q][j] = szbase[u * 4];
      }
    }
  }
  asm volatile("" ::: "memory");  // every load of the wave is in flight before the first MFMA
  if (epi_thr) epi_pre_b<1, EPI>(p, pre, t0, 4 * grp);
  const uint32_t lom = r16 < R ? ~0u : 0u;
  const uint32_t nib_m = 0x000F000Fu, nib_o = 0x43004300u;
  f32x4 acc[TMAX];
#pragma unroll
  for (int j = 0; j < TMAX; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssr = 0.f;  // NORM 1: this wave's raw x^2 of row r16 (lane quarter)
#pragma unroll
  for (int q = 0; q < KQW; ++q) {
    if (q >= nq) break;  // wave-uniform
    // the 4 B fragments of a k-quad from its XP-packed loads (lane r16 < R <- row r16 of each k-step)
    auto unpack = [&](const uint4 (&src)[XL], uint4 (&b)[4]) {
#pragma unroll
      for (int v = 0; v < XL; ++v) {
        if constexpr (XP == 1) {
          b[v] = src[v];
        } else {
          b[v * XP] = and_mask(src[v], lom);
          b[v * XP + 1] = and_mask(row_ror<R>(src[v]), lom);
          if constexpr (XP == 4) {
            b[v * XP + 2] = and_mask(row_ror<2 * R>(src[v]), lom);
            b[v * XP + 3] = and_mask(row_ror<3 * R>(src[v]), lom);
          }
        }
      }
    };
    uint4 src[XL], b[4];
    if constexpr (NORM == 1) {
      // sum of squares over the RAW activations, unpacked (lane <-> row r16, as gemm_finish folds
      // it); the MFMA operand is bf16(x * gamma), gamma packed like x
      uint4 raw[4];
      unpack(xa[q], raw);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float f[8];
        unpack8(raw[t], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) ssr += f[j] * f[j];
      }
#pragma unroll
      for (int v = 0; v < XL; ++v) {
        float f[8], g8[8];
        unpack8(xa[q][v], f);
        unpack8(ga[q][v], g8);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= g8[j];
        src[v] = pack8(f);
      }
    } else {
#pragma unroll
      for (int v = 0; v < XL; ++v) src[v] = xa[q][v];
    }
    unpack(src, b);
    float X = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) X = kx_sum8(b[t], X);
    X += xor16(X);
    X += xor32(X);
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      if (j < ntb) {
        f32x4 pr = {0.f, 0.f, 0.f, 0.f};
        pr = mfma16(kx_raw8(w[q][j].x, nib_m, nib_o), as_bf16x8(b[0]), pr);
        pr = mfma16(kx_raw8(w[q][j].y, nib_m, nib_o), as_bf16x8(b[1]), pr);
        pr = mfma16(kx_raw8(w[q][j].z, nib_m, nib_o), as_bf16x8(b[2]), pr);
        pr = mfma16(kx_raw8(w[q][j].w, nib_m, nib_o), as_bf16x8(b[3]), pr);
        const uint4 s = sz[q][j];
        const float s4[4] = {bf_lo(s.x), bf_hi(s.x), bf_lo(s.y), bf_hi(s.y)};
        const float z4[4] = {bf_lo(s.z), bf_hi(s.z), bf_lo(s.w), bf_hi(s.w)};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(s4[i], pr[i], fmaf(-fmaf(128.f, s4[i], z4[i]), X, acc[j][i]));
      }
    }
  }
  if constexpr (!WIDE) {
    f32x4 a1[1][1] = {{acc[0]}};
    float sr[1] = {0.f};
    if constexpr (NORM == 1) sr[0] = ssr;
    if constexpr (NORM == 3) {
      if (ss_wave) sr[0] = kx_ss_sum(p, ssv, r16, grp);
    }
    gemm_finish<1, 1, EPI, NORM, true>(p, a1, sr, smem, 0, t0, pre);
  } else {
    // the waves' partials of every tile (rows < M only) and, NORM 1, their x^2 rows -> LDS
    f32x4* red = reinterpret_cast<f32x4*>(smem);                      // [nw][TMAX][64]
    float* ssq = reinterpret_cast<float*>(smem + (size_t)nw * TMAX * 1024);  // [nw][16]
    const bool row_ok = r16 < p.M;
#pragma unroll
    for (int j = 0; j < TMAX; ++j)
      if (j < ntb && row_ok) red[(wid * TMAX + j) * 64 + lane] = acc[j];
    if constexpr (NORM == 1) {
      ssr += xor16(ssr);
      ssr += xor32(ssr);
      if (lane < 16) ssq[wid * 16 + lane] = ssr;
    }
    __syncthreads();
    if (wid >= ntb) return;
    f32x4 v[1] = {{0.f, 0.f, 0.f, 0.f}};
    if (row_ok)
      for (int w2 = 0; w2 < nw; ++w2) v[0] += red[(w2 * TMAX + wid) * 64 + lane];
    if constexpr (NORM == 1) {
      float ss = 0.f;
      for (int w2 = 0; w2 < nw; ++w2) ss += ssq[w2 * 16 + r16];
      v[0] *= rsqrtf(ss / (float)p.K + p.eps);
    }
    if constexpr (NORM == 3) {
      float ss = kx_ss_sum(p, ssv, r16, grp);
      ss += xor16(ss);
      ss += xor32(ss);
      v[0] *= rsqrtf(ss / (float)p.K + p.eps);
    }
    epilogue<1, EPI, false>(p, v, r16, t0 + wid, 4 * grp, EpiPre<1>{}, row_ok);
  }
}

static int kx_cus() {
  static const int n = [] {
    int v = 0, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

template <int XP, int KQW, int TMAX, int EPI, int NORM, bool WIDE>
static bool kx_go(const GemmParams& p, dim3 grid, int nw, hipStream_t st) {
  if (64 * nw > kx_max_threads<XP, KQW, TMAX, NORM>()) return false;
  const size_t lds = WIDE ? (size_t)nw * TMAX * 1024 + (size_t)nw * 16 * 4 : red_bytes<1, 1>(nw) + ssq_bytes<1>(nw) + 16;
  if (lds > 160 * 1024) return false;
  auto kern = awq_kx_kernel<XP, KQW, TMAX, EPI, NORM, WIDE>;
  if (lds > 64 * 1024) {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
  }
  hipLaunchKernelGGL(kern, grid, dim3(64 * nw), lds, st, p);
  return true;
}

// Grid choice. WIDE when N has at least one tile per CU (and no slices are forced): one block per CU,
// min(16, K / 128) waves. Otherwise TILE: one tile per block, K slices while the grid still fits the
// CUs and every slice keeps >= 16 k-quads (down_proj: 96 tiles x 2 slices of 35), min(16, slice)
// waves. g.waves / g.splitk force the wave / slice counts (sweeps, tests).
template <int XP, int EPI, int NORM>
static bool kx_launch_xp(GemmParams p, const GemmArgs& g, hipStream_t st) {
  const int ntiles = g.N / 16, KQ = g.K / 128, ncu = kx_cus();
  if constexpr (EPI != EPI_QKV) {
    if (ntiles >= ncu && g.splitk <= 1) {
    const int nb = ncu, tneed = (ntiles + nb - 1) / nb;
    const int nw = g.waves > 0 ? g.waves : std::min(16, KQ);
    if (nw > 16) return false;
    const int kqw = (KQ + nw - 1) / nw;
    if (p.dbg_ts == nullptr) p.dbg_ts = tl_take("awq_kx_wide", nb);
    p.splitk = 1;
    const dim3 grid(nb);
    if (tneed <= 2 && kqw == 1) return kx_go<XP, 1, 2, EPI, NORM, true>(p, grid, nw, st);
    if (tneed <= 5 && kqw == 1) return kx_go<XP, 1, 5, EPI, NORM, true>(p, grid, nw, st);
    if (tneed <= 5 && kqw == 2) return kx_go<XP, 2, 5, EPI, NORM, true>(p, grid, nw, st);
    if (tneed <= 8 && kqw == 1) return kx_go<XP, 1, 8, EPI, NORM, true>(p, grid, nw, st);
    return false;
    }
  }
  int S = g.splitk > 0 ? g.splitk : 1;
  if (g.splitk <= 0)
    while (ntiles * (S + 1) <= ncu && KQ / (S + 1) >= 16) ++S;
  if (S > SK_MAX || S > KQ) return false;
  const int kqs = (KQ + S - 1) / S;
  int nw = g.waves > 0 ? g.waves : std::min(16, kqs);
  int kqw = (kqs + nw - 1) / nw;
  if (kqw > 4 && g.waves <= 0) {  // the 6-deep form holds 8 waves at most
    nw = std::min(8, kqs);
    kqw = (kqs + nw - 1) / nw;
  }
  if (nw > 16 || kqw > 6) return false;
  p.splitk = S;
  if (S > 1) {
    const size_t need_slab = (size_t)ntiles * S * (64 * 16 + (NORM ? 16 * 4 : 0));
    const size_t need_g = (size_t)ntiles * 3 * 64 * 16;
    if (S == 2 && g.sk_pub != nullptr && need_g <= g.sk_bytes) p.gran = reinterpret_cast<uint4*>(g.sk_pub);
    else if (g.slabs == nullptr || need_slab > g.slab_bytes || ntiles > g.max_counters) return false;
  }
  if (p.dbg_ts == nullptr) p.dbg_ts = tl_take("awq_kx", ntiles * S);
  const dim3 grid(ntiles, 1, S);
  switch (kqw) {
    case 1: return kx_go<XP, 1, 1, EPI, NORM, false>(p, grid, nw, st);
    case 2: return kx_go<XP, 2, 1, EPI, NORM, false>(p, grid, nw, st);
    case 3: return kx_go<XP, 3, 1, EPI, NORM, false>(p, grid, nw, st);
    case 4: return kx_go<XP, 4, 1, EPI, NORM, false>(p, grid, nw, st);
    default: return kx_go<XP, 6, 1, EPI, NORM, false>(p, grid, nw, st);
  }
}

template <int EPI, int NORM>
static bool kx_launch(const GemmParams& p, const GemmArgs& g, hipStream_t st) {
  return g.M <= 8 ? kx_launch_xp<2, EPI, NORM>(p, g, st) : kx_launch_xp<1, EPI, NORM>(p, g, st);
}

bool launch_awq_kx(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.M > 16 || g.awq_szp == nullptr || g.group != 128 || g.N % 16 != 0 || g.K % 128 != 0 ||
      g.rownorm || g.ar_world > 0 || (g.ssp_in != nullptr && g.norm_w != nullptr) || g.epi == EPI_F32)
    return false;
  GemmParams p{};
  p.x = g.x; p.lda = g.lda; p.M = g.M; p.row_idx = g.row_idx;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.norm_w = g.norm_w; p.eps = g.eps;
  p.bias = g.bias; p.res = g.res; p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.splitk = 1; p.slabs = g.slabs; p.counters = g.counters;
  p.gran = nullptr; p.fault = g.fault;
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.szp = g.awq_szp; p.group = g.group;
  p.dbg_ts = g.dbg_ts;
  p.hg = g.hg; p.hg_gamma = g.hg_gamma; p.ssp_out = g.ssp_out; p.ssp_in = g.ssp_in; p.ssn = g.ssn;
  const int norm = g.norm_w != nullptr ? 1 : g.ssp_in != nullptr ? 3 : 0;
#define VG_KX(E)                                            \
  return norm == 1 ? kx_launch<E, 1>(p, g, st)              \
       : norm == 3 ? kx_launch<E, 3>(p, g, st)              \
                   : kx_launch<E, 0>(p, g, st)
  switch (g.epi) {
    case EPI_SILU: VG_KX(EPI_SILU);
    case EPI_QKV: VG_KX(EPI_QKV);
    default: VG_KX(EPI_BF16);
  }
#undef VG_KX
}

}  // namespace vgate
