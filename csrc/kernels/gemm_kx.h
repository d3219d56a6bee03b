// Decode GEMM (M <= 16) with register-stationary activations ("kx"): AWQ W4A16 (gemm_kx_q4.hip) and
// bf16 (gemm_kx_bf16.hip) instantiations of one kernel template.
//
// An int4 k-quad of one 16-column tile is 1 KiB of weights, but at M = 8 the k-quad's activations are
// 2 KiB and its (s, s z) record is fetched as a 1 KiB lane load: a kernel that pairs every weight
// fragment with its own activation and scale loads spends most of the CU's vector-memory requests on
// bytes that are not weights. And once the bytes are in, the nibble -> bf16 unpack (MFMA A operand)
// and the group scale cost ~45 VALU instructions per (tile, k-quad) — for Qwen2.5-1.5B gate_up
// (1120 tiles x 12 k-quads over 256 CUs) ~0.9 us of VALU time per SIMD, as long as a third of the
// HBM stream. The round-2..4 int4 kernels serialised that work behind the stream (one wave per tile:
// 9.85 us for gate_up) or behind LDS staging of x (benchmarks/probes/awq_wide_anatomy.hip keeps a copy
// of that design; profiles/r5_awq_wide_anatomy_and_kx_probe.log).
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
//   GROUP (narrow N: qkv, o_proj, down_proj): TMAX = 1, 2 or 4 adjacent tiles per block, gridDim.z
//         K slices; the waves' partials, the slices (granules / slabs) and the epilogue are
//         gemm_finish's, with the epilogue operands (residual, bias, RoPE position / cos-sin) of
//         1-2 tile blocks prefetched at launch. More tiles per block = fewer activation bytes per
//         weight byte (deep K: down_proj), one tile = the shortest block (qkv / o_proj).
// NORM: 0 none; 1 RMSNorm gamma in registers (x * gamma in bf16, raw x^2 summed; layer 0 of the
// hand-off chain); 3 the producer's hand-off (x = h * gamma, row sums of squares in ssp_in).
#pragma once
#include "gemm_decode.h"
#include "attn_decode.h"

namespace vgate {

// bf16 (128 + v) of the 8 nibbles of one dword (ops.pack_awq order: element j of k-step u at bits
// 16 (j & 1) + 4 (j >> 1), i.e. output dword i holds the low (i even) / high (i odd) nibbles of bytes
// i/2 and i/2 + 2). The nibbles are isolated into bytes (lo = q & 0x0F0F0F0F, hi = (q >> 4) & ...)
// and each output dword is one v_perm_b32 of two of those bytes with two 0x43 bytes: 7 VALU per 8
// values, all compiler-visible (an inline-asm v_and_or_b32 form needed three register moves per
// dword to build the MFMA operand tuple plus a manual MFMA hazard wait).
__device__ __forceinline__ bf16x8 kx_raw8(uint32_t q, uint32_t c43) {
  const uint32_t lo = q & 0x0F0F0F0Fu, hi = (q >> 4) & 0x0F0F0F0Fu;
  uint4 r;
  r.x = __builtin_amdgcn_perm(c43, lo, 0x04020400u);  // [lo.b0, 0x43, lo.b2, 0x43]
  r.y = __builtin_amdgcn_perm(c43, hi, 0x04020400u);
  r.z = __builtin_amdgcn_perm(c43, lo, 0x04030401u);  // [lo.b1, 0x43, lo.b3, 0x43]
  r.w = __builtin_amdgcn_perm(c43, hi, 0x04030401u);
  return as_bf16x8(r);
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

// Q4: int4 weights + packed scales (else bf16 fragment-packed weights: 4 loads per k-quad and tile, no
// scales, no dequant — the same grid forms for the dense decode GEMMs). XP: k-steps per activation load
// (2: M <= 8, 1: M <= 16); KQW: k-quads per wave (host: >= the wave's range); TMAX: tiles per block
// (WIDE: at most, GROUP: exactly). Registers of loads in flight per lane: kx_regs (+ the NORM 3
// prefetch); up to 80 the block may hold 16 waves (128 VGPRs each), up to 120 12 waves, else 8.
template <bool Q4, int XP, int KQW, int TMAX, int NORM>
__host__ __device__ constexpr int kx_regs() {
  return 4 * KQW * ((4 / XP) * (NORM == 1 ? 2 : 1) + (Q4 ? 2 : 4) * TMAX) + (NORM == 3 ? 4 * SS_PRE : 0);
}
template <bool Q4, int XP, int KQW, int TMAX, int NORM>
__host__ __device__ constexpr int kx_max_threads() {
  return kx_regs<Q4, XP, KQW, TMAX, NORM>() <= 80 ? 1024 : kx_regs<Q4, XP, KQW, TMAX, NORM>() <= 120 ? 768 : 512;
}

template <bool Q4, int XP, int KQW, int TMAX, int EPI, int NORM, bool WIDE>
__device__ __forceinline__ void kx_block(const GemmParams& p) {
  static_assert(EPI != EPI_QKV || (!WIDE && TMAX == 1), "QKV: one-tile GROUP blocks (prefetched RoPE operands)");
  static_assert(Q4 ? NORM != 2 : NORM != 1, "int4: gamma in registers or the hand-off; bf16: gamma folded into W");
  constexpr bool PRE = !WIDE && TMAX <= 2;  // GROUP blocks of 1-2 tiles: epilogue operands at launch
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
    t0 = (int)(((long long)ntiles * blk_x(p)) / grid_x(p));
    ntb = (int)(((long long)ntiles * (blk_x(p) + 1)) / grid_x(p)) - t0;
    s0 = 0;
    s1 = KQ;
  } else {
    t0 = blk_x(p) * TMAX;
    ntb = TMAX;
    s0 = (KQ * blk_z(p)) / p.splitk;
    s1 = (KQ * (blk_z(p) + 1)) / p.splitk;
  }
  const int q0 = s0 + ((s1 - s0) * wid) / nw;
  const int nq = s0 + ((s1 - s0) * (wid + 1)) / nw - q0;  // <= KQW (host-checked), may be 0
  // NORM 3: the row's sums of squares, issued first (consumed after the stream without waiting on it)
  SsPre ssv;
  ssv.n4 = NORM == 3 ? ss_pre_n4(p) : 0;
  const bool ss_wave = WIDE ? wid < ntb : (wid == 0 && blk_z(p) == 0);  // wave-uniform
  if constexpr (NORM == 3) {
    if (ss_wave && ssv.n4 > 0) ss_pre_issue(p, ssv, r16, grp);
  }
  // GROUP form: the epilogue operands of wave 0's (row, 4 columns) items at launch
  EpiPre<TMAX> pre;
  // wave 0 runs the epilogue. Its operand loads sit under a wave-uniform branch (a lane test would be
  // an exec-masked one), except QKV's: the RoPE cos/sin loads depend on the position load and go out
  // after the weight stream, and a branch there would leave every later wait at vmcnt(0) — so every
  // wave issues them (a few L2-resident words) and only wave 0's are used
  const bool epi_thr = PRE && (EPI == EPI_QKV || wid == 0);
  if (epi_thr) epi_pre_a<TMAX, EPI>(p, pre, r16, t0, 4 * grp);
  // activations: lane (r16, grp) loads row r16 % R of k-step r16 / R (+ XP v) of each load. Rows
  // past M re-read row M - 1 (row_of clamps) and lanes r16 >= R of a rebuilt fragment keep another
  // k-step's values: both only feed output rows that are never stored (no masks, no exec-masked loads)
  const int mrow = r16 % R;
  const bf16_t* xrow = p.x + (size_t)row_of_e<EPI>(p, mrow) * p.lda + 8 * grp + (XP > 1 ? (r16 / R) * 32 : 0);
  const bf16_t* grow = NORM == 1 ? p.norm_w + 8 * grp + (XP > 1 ? (r16 / R) * 32 : 0) : nullptr;
  constexpr int WL = Q4 ? 1 : 4;  // weight loads per (k-quad, tile)
  const int KT = KQ * 4;
  const uint4* wbase = p.wp + (size_t)t0 * (Q4 ? KQ : KT) * 64 + lane;
  const uint4* szbase = reinterpret_cast<const uint4*>(p.szp) + (size_t)t0 * KQ * 4 + grp;
  constexpr int GL = NORM == 1 ? XL : 1;
  uint4 xa[KQW][XL], ga[KQW][GL], w[KQW][TMAX][WL], sz[KQW][TMAX];
  // every load unconditional (clamped re-reads past the wave's range are never consumed): a load
  // under a branch leaves the paths with different outstanding counts, and the compiler's waits
  // after the join then cover loads issued later (the weight stream) as well
#pragma unroll
  for (int q = 0; q < KQW; ++q) {
    const int kq = min(q0 + min(q, max(nq - 1, 0)), KQ - 1);
#pragma unroll
    for (int v = 0; v < XL; ++v)
      xa[q][v] = *reinterpret_cast<const uint4*>(xrow + (size_t)(kq * 4 + v * XP) * 32);
    if constexpr (NORM == 1) {
#pragma unroll
      for (int v = 0; v < XL; ++v) ga[q][v] = *reinterpret_cast<const uint4*>(grow + (size_t)(kq * 4 + v * XP) * 32);
    }
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      const size_t tj = (size_t)min(j, ntb - 1);
      if constexpr (Q4) {
        const size_t u = tj * KQ + kq;
        w[q][j][0] = ld_nt16(wbase + u * 64);
        sz[q][j] = szbase[u * 4];
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) w[q][j][t] = ld_nt16(wbase + (tj * KT + kq * 4 + t) * 64);
      }
    }
  }
  asm volatile("" ::: "memory");  // every load of the wave is in flight before the first MFMA
  if (epi_thr) epi_pre_b<TMAX, EPI>(p, pre, t0, 4 * grp);
  const uint32_t c43 = 0x43434343u;
  f32x4 acc[TMAX];
#pragma unroll
  for (int j = 0; j < TMAX; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ssr = 0.f;  // NORM 1 / 2: this wave's raw x^2 of row r16 (lane quarter)
#pragma unroll
  for (int q = 0; q < KQW; ++q) {
    if (q >= nq) break;  // wave-uniform
    // the 4 B fragments of a k-quad from its XP-packed loads (lane r16 < R <- row r16 of each k-step;
    // lanes r16 >= R: don't-care rows)
    auto unpack = [&](const uint4 (&src)[XL], uint4 (&b)[4]) {
#pragma unroll
      for (int v = 0; v < XL; ++v) {
        if constexpr (XP == 1) {
          b[v] = src[v];
        } else {
          b[v * XP] = src[v];
          b[v * XP + 1] = row_ror<R>(src[v]);
          if constexpr (XP == 4) {
            b[v * XP + 2] = row_ror<2 * R>(src[v]);
            b[v * XP + 3] = row_ror<3 * R>(src[v]);
          }
        }
      }
    };
    uint4 src[XL], b[4];
    if constexpr (NORM == 2) {  // bf16, gamma folded into W: the raw rows' sum of squares only
#pragma unroll
      for (int v = 0; v < XL; ++v) src[v] = xa[q][v];
      unpack(src, b);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float f[8];
        unpack8(b[t], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) ssr += f[j] * f[j];
      }
    } else if constexpr (NORM == 1) {
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
    if constexpr (NORM != 2) unpack(src, b);
    if constexpr (!Q4) {
#pragma unroll
      for (int j = 0; j < TMAX; ++j) {
        if (j < ntb) {
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[j] = mfma16(as_bf16x8(w[q][j][t]), as_bf16x8(b[t]), acc[j]);
        }
      }
      continue;
    }
    float X = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) X = kx_sum8(b[t], X);
    X += xor16(X);
    X += xor32(X);
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      if (j < ntb) {
        f32x4 pr = {0.f, 0.f, 0.f, 0.f};
        pr = mfma16(kx_raw8(w[q][j][0].x, c43), as_bf16x8(b[0]), pr);
        pr = mfma16(kx_raw8(w[q][j][0].y, c43), as_bf16x8(b[1]), pr);
        pr = mfma16(kx_raw8(w[q][j][0].z, c43), as_bf16x8(b[2]), pr);
        pr = mfma16(kx_raw8(w[q][j][0].w, c43), as_bf16x8(b[3]), pr);
        const uint4 s = sz[q][j];
        const float s4[4] = {bf_lo(s.x), bf_hi(s.x), bf_lo(s.y), bf_hi(s.y)};
        const float z4[4] = {bf_lo(s.z), bf_hi(s.z), bf_lo(s.w), bf_hi(s.w)};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = fmaf(s4[i], pr[i], fmaf(-fmaf(128.f, s4[i], z4[i]), X, acc[j][i]));
      }
    }
  }
  if constexpr (!WIDE) {
    f32x4 a1[1][TMAX];
#pragma unroll
    for (int j = 0; j < TMAX; ++j) a1[0][j] = acc[j];
    float sr[1] = {0.f};
    if constexpr (NORM == 1 || NORM == 2) sr[0] = ssr;
    if constexpr (NORM == 3) {
      if (ss_wave) sr[0] = ss_pre_sum(p, ssv, r16, grp);
    }
    gemm_finish<1, TMAX, EPI, NORM, PRE>(p, a1, sr, smem, 0, t0, pre);
  } else {
    // the waves' partials of every tile (rows < M only) and, NORM 1, their x^2 rows -> LDS
    f32x4* red = reinterpret_cast<f32x4*>(smem);                      // [nw][TMAX][64]
    float* ssq = reinterpret_cast<float*>(smem + (size_t)nw * TMAX * 1024);  // [nw][16]
    const bool row_ok = r16 < p.M;
#pragma unroll
    for (int j = 0; j < TMAX; ++j)
      if (j < ntb && row_ok) red[(wid * TMAX + j) * 64 + lane] = acc[j];
    if constexpr (NORM == 1 || NORM == 2) {
      ssr += xor16(ssr);
      ssr += xor32(ssr);
      if (lane < 16) ssq[wid * 16 + lane] = ssr;
    }
    __syncthreads();
    if (wid >= ntb) return;
    f32x4 v[1] = {{0.f, 0.f, 0.f, 0.f}};
    if (row_ok)
      for (int w2 = 0; w2 < nw; ++w2) v[0] += red[(w2 * TMAX + wid) * 64 + lane];
    if constexpr (NORM == 1 || NORM == 2) {
      float ss = 0.f;
      for (int w2 = 0; w2 < nw; ++w2) ss += ssq[w2 * 16 + r16];
      v[0] *= rsqrtf(ss / (float)p.K + p.eps);
    }
    if constexpr (NORM == 3) {
      float ss = ss_pre_sum(p, ssv, r16, grp);
      ss += xor16(ss);
      ss += xor32(ss);
      v[0] *= rsqrtf(ss / (float)p.K + p.eps);
    }
    epilogue<1, EPI, false>(p, v, r16, t0 + wid, 4 * grp, EpiPre<1>{}, row_ok);
  }
}

template <bool Q4, int XP, int KQW, int TMAX, int EPI, int NORM, bool WIDE>
__global__ __launch_bounds__((kx_max_threads<Q4, XP, KQW, TMAX, NORM>())) void kx_kernel(GemmParams p) {
  kx_block<Q4, XP, KQW, TMAX, EPI, NORM, WIDE>(p);
}

// The fused QKV projection + decode attention launch on this kernel (design: qkv_attn.hip): GROUP
// one-tile blocks of <= 8 waves (z-major in the 1-D grid), then the attention blocks
template <bool Q4, int XP, int KQW, int NORM>
__global__ __launch_bounds__(512) void kx_qa_kernel(GemmParams p, AttnArgs a, QaSync q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < q.nprod) {
    kx_block<Q4, XP, KQW, 1, EPI_QKV, NORM, false>(p);
    return;
  }
  TLScope tl_scope(p.dbg_ts);
  const int r = (int)blockIdx.x - q.nprod;  // (KV head, partition, sequence), sequence fastest
  decode_block<false, true>(a, r % a.S, r / (a.S * a.num_parts), (r / a.S) % a.num_parts, smem, &q);
}

template <bool Q4, int XP, int NORM>
static bool kx_qa(GemmParams p, const GemmArgs& g, int groups, int S, int kqs, hipStream_t st) {
  if constexpr (NORM == 0) {
    return false;
  } else {
    const int nw = g.waves > 0 ? g.waves : std::min(8, kqs);
    const int kqw = (kqs + nw - 1) / nw;
    if (kqw > 3 || 64 * nw > 512) return false;
    AttnArgs a;
    QaSync q;
    size_t lds;
    if (!qa_setup(p, g, groups, S, nw, red_bytes<1, 1>(nw) + ssq_bytes<1>(nw) + 16, a, q, lds)) return false;
    if (p.dbg_ts == nullptr) p.dbg_ts = tl_take(Q4 ? "awq_kx_qa" : "kx_qa", q.nprod + a.S * a.num_parts * a.Hkv);
    if (kqw == 1) qa_launch(kx_qa_kernel<Q4, XP, 1, NORM>, p, a, q, nw, lds, st);
    else if (kqw == 2) qa_launch(kx_qa_kernel<Q4, XP, 2, NORM>, p, a, q, nw, lds, st);
    else qa_launch(kx_qa_kernel<Q4, XP, 3, NORM>, p, a, q, nw, lds, st);
    *g.fa_done = true;
    return true;
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

template <bool Q4, int XP, int KQW, int TMAX, int EPI, int NORM, bool WIDE>
static bool kx_go(const GemmParams& p, dim3 grid, int nw, hipStream_t st) {
  if (64 * nw > kx_max_threads<Q4, XP, KQW, TMAX, NORM>()) return false;
  const size_t lds = WIDE ? (size_t)nw * TMAX * 1024 + (size_t)nw * 16 * 4 : red_bytes<1, TMAX>(nw) + ssq_bytes<1>(nw) + 16;
  if (lds > 160 * 1024) return false;
  auto kern = kx_kernel<Q4, XP, KQW, TMAX, EPI, NORM, WIDE>;
  if (lds > 64 * 1024) {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
  }
  hipLaunchKernelGGL(kern, grid, dim3(64 * nw), lds, st, p);
  return true;
}

// Grid choice. WIDE when N has at least one tile per CU (and no slices are forced): one block per CU,
// min(16, K / 128) waves. Otherwise GROUP: TB tiles per block (g.ntb -12 / -13 / -14 force 1 / 2 / 4;
// default 1), K slices while the grid still fits the CUs and every slice keeps >= 16 k-quads
// (down_proj: 96 tiles x 2 slices of 35), min(16, slice) waves. g.waves / g.splitk force the wave /
// slice counts (sweeps, tests).
template <bool Q4, int XP, int TB, int EPI, int NORM>
static bool kx_group(GemmParams p, const GemmArgs& g, hipStream_t st) {
  const int ntiles = g.N / 16, KQ = g.K / 128, ncu = kx_cus();
  if (ntiles % TB) return false;
  const int groups = ntiles / TB;
  int S = g.splitk > 0 ? g.splitk : 1;
  if (g.splitk <= 0)
    while (groups * (S + 1) <= ncu && KQ / (S + 1) >= 16) ++S;
  if (S > SK_MAX || S > KQ) return false;
  const int kqs = (KQ + S - 1) / S;
  int nw = g.waves > 0 ? g.waves : std::min(16, kqs);
  int kqw = (kqs + nw - 1) / nw;
  if (kqw > 5 && g.waves <= 0) {  // the 6-deep form holds 8 waves at most
    nw = std::min(8, kqs);
    kqw = (kqs + nw - 1) / nw;
  }
  if (nw > 16 || kqw > 6) return false;
  p.splitk = S;
  if (S > 1) {
    const size_t need_slab = (size_t)groups * S * (TB * 64 * 16 + (NORM ? 16 * 4 : 0));
    const size_t need_g = (size_t)groups * 3 * 64 * 16;
    if (TB == 1 && S == 2 && g.sk_pub != nullptr && need_g <= g.sk_bytes) p.gran = reinterpret_cast<uint4*>(g.sk_pub);
    else if (g.slabs == nullptr || need_slab > g.slab_bytes || groups > g.max_counters) return false;
  }
  if constexpr (EPI == EPI_QKV && TB == 1) {  // decode-only step: its attention in this launch
    if (g.fa != nullptr && kx_qa<Q4, XP, NORM>(p, g, groups, S, kqs, st)) return true;
  }
  if (p.dbg_ts == nullptr) p.dbg_ts = tl_take(Q4 ? "awq_kx" : "kx", groups * S);
  const dim3 grid(groups, 1, S);
  if constexpr (TB == 1) {
    switch (kqw) {
      case 1: return kx_go<Q4, XP, 1, 1, EPI, NORM, false>(p, grid, nw, st);
      case 2: return kx_go<Q4, XP, 2, 1, EPI, NORM, false>(p, grid, nw, st);
      case 3: return kx_go<Q4, XP, 3, 1, EPI, NORM, false>(p, grid, nw, st);
      case 4: return kx_go<Q4, XP, 4, 1, EPI, NORM, false>(p, grid, nw, st);
      case 5: return kx_go<Q4, XP, 5, 1, EPI, NORM, false>(p, grid, nw, st);
      default: return kx_go<Q4, XP, 6, 1, EPI, NORM, false>(p, grid, nw, st);
    }
  } else if constexpr (TB == 2) {
    switch (kqw) {
      case 1: return kx_go<Q4, XP, 1, 2, EPI, NORM, false>(p, grid, nw, st);
      case 2: return kx_go<Q4, XP, 2, 2, EPI, NORM, false>(p, grid, nw, st);
      case 3: return kx_go<Q4, XP, 3, 2, EPI, NORM, false>(p, grid, nw, st);
      default: return false;
    }
  } else {
    switch (kqw) {
      case 1: return kx_go<Q4, XP, 1, 4, EPI, NORM, false>(p, grid, nw, st);
      case 2: return kx_go<Q4, XP, 2, 4, EPI, NORM, false>(p, grid, nw, st);
      default: return false;
    }
  }
}

template <bool Q4, int XP, int EPI, int NORM>
static bool kx_launch_xp(GemmParams p, const GemmArgs& g, hipStream_t st) {
  const int ntiles = g.N / 16, KQ = g.K / 128, ncu = kx_cus();
  if constexpr (EPI != EPI_QKV) {
    if (ntiles >= ncu && g.splitk <= 1 && g.ntb != -13 && g.ntb != -14) {
      const int nb = ncu, tneed = (ntiles + nb - 1) / nb;
      const int nw = g.waves > 0 ? g.waves : std::min(16, KQ);
      if (nw > 16) return false;
      const int kqw = (KQ + nw - 1) / nw;
      if (p.dbg_ts == nullptr) p.dbg_ts = tl_take(Q4 ? "awq_kx_wide" : "kx_wide", nb);
      p.splitk = 1;
      const dim3 grid(nb);
      if (tneed <= 2 && kqw == 1) return kx_go<Q4, XP, 1, 2, EPI, NORM, true>(p, grid, nw, st);
      if (tneed <= 5 && kqw == 1) return kx_go<Q4, XP, 1, 5, EPI, NORM, true>(p, grid, nw, st);
      if (tneed <= 5 && kqw == 2) return kx_go<Q4, XP, 2, 5, EPI, NORM, true>(p, grid, nw, st);
      if (tneed <= 8 && kqw == 1) return kx_go<Q4, XP, 1, 8, EPI, NORM, true>(p, grid, nw, st);
      return false;
    }
    if constexpr (NORM == 0) {  // multi-tile GROUP blocks: the plain / residual (+ hand-off producer) GEMMs
      if (g.ntb == -13) return kx_group<Q4, XP, 2, EPI, NORM>(p, g, st);
      if (g.ntb == -14) return kx_group<Q4, XP, 4, EPI, NORM>(p, g, st);
    }
  }
  return kx_group<Q4, XP, 1, EPI, NORM>(p, g, st);
}

template <bool Q4, int EPI, int NORM>
static bool kx_launch(const GemmParams& p, const GemmArgs& g, hipStream_t st) {
  return g.M <= 8 ? kx_launch_xp<Q4, 2, EPI, NORM>(p, g, st) : kx_launch_xp<Q4, 1, EPI, NORM>(p, g, st);
}

static GemmParams kx_params(const GemmArgs& g) {
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
  return p;
}

}  // namespace vgate
