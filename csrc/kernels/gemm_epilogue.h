// Shared pieces of the fragment-packed GEMM family (gemm.hip: decode / tile kernels,
// gemm_prefill.hip: the LDS-tiled prefill kernel): launch parameters, the per-row epilogue
// (bias, residual, SiLU*mul, f32 logits, QKV bias + NeoX RoPE + paged-KV write) and its
// launch-time operand prefetch. Every kernel produces D = W x X^T with the MFMA orientation
// "lane holds D[n = 4(l>>4)+i][m = l&15]", so one epilogue serves all of them.
#pragma once
#include "common.h"
#include "launchers.h"

namespace vgate {

// EPI_BF16_AR: EPI_BF16 with the TP all-reduce in the epilogue (epilogue_ar); its own instantiations
// (gemm_epi_bf16ar.hip), so the TP = 1 kernels carry none of its code or registers
enum GemmEpi : int { EPI_BF16 = 0, EPI_F32 = 1, EPI_SILU = 2, EPI_QKV = 3, EPI_BF16_AR = 4 };
constexpr int SK_MAX = 8;  // split-K slices per tile (the combine issues all slices' loads at once)

// TP row-parallel decode GEMM: the all-reduce runs in the epilogue (epilogue_ar) when world >= 1
struct ArFused {
  char* base[8];   // every rank's fused region (launchers.h AR_FUSED_*), own one included
  uint32_t* err;   // own sticky all-reduce error word (allreduce.hip ArSignal::error)
  int rank, world;
  uint32_t spin;   // polls before a wait gives up
};

struct GemmParams {
  const bf16_t* x; int lda; int M; const int32_t* row_idx;
  const uint4* wp; int N; int K;
  const bf16_t* norm_w; float eps;  // norm_w null under NORM = gamma folded into W (row scale only)
  const bf16_t* bias; const bf16_t* res; int ldr;
  void* out; int ldo;
  int splitk; float* slabs; uint32_t* counters;
  // decode split-K (MB = 1) by data-carrying granules instead of slabs + ticket: slices below the last
  // publish {value, tag} pairs, the last slice's block (dispatched after every other slice: z-major
  // order) collects, adds in slice order and clears; zeroed once (ops.sk_workspace), or null
  uint4* gran; uint32_t* fault;
  const int32_t* positions; const int32_t* slots; const float* cos_sin;
  bf16_t* k_cache; bf16_t* v_cache; int hq; int hkv; int bs;
  const bf16_t* scales; const bf16_t* zeros; int group;
  const bf16_t* szp;  // AWQ decode: fragment-packed (scale, scale * zero) [N/16][K/128][4][8]
  // RMSNorm hand-off for the int4 consumers (decode, TP = 1). Producer (EPI_BF16 residual GEMMs:
  // o_proj, down_proj): hg = bf16(h * gamma) of the output rows h it stores, and per-(row, 16-column
  // tile) sums of squares of h -> ssp_out [M][N/16]. Consumer (NORM == 3): x = hg (gamma already
  // applied; int4) or x = h with gamma folded into the bf16 weights (hg null), row scale
  // rsqrt(sum of ssp_in[m][0..ssn) / K + eps) — no gamma loads, no x^2 pass.
  bf16_t* hg; const bf16_t* hg_gamma; float* ssp_out; const float* ssp_in; int ssn;
  unsigned long long* dbg_ts;  // per-block [start, end] realtime stamps (profiling), or null
  ArFused ar;                  // world 0: no fused all-reduce
  uint4* qa_gran;              // EPI_QKV: also write q / K / V as tagged granules (qkv_attn.hip), or null
  int vgx;                     // > 0: a 1-D launch carries the (vgx, 1, slices) grid z-major (qkv_attn.hip)
};

// (column-tile block, K slice, slices) of this block: the grid decomposition of gemm_finish's hand-off
struct SplitPos {
  int tile, slice, nsl;
};
__device__ __forceinline__ int grid_x(const GemmParams& p) { return p.vgx > 0 ? p.vgx : (int)gridDim.x; }
__device__ __forceinline__ int blk_x(const GemmParams& p) {
  return p.vgx > 0 ? (int)blockIdx.x % p.vgx : (int)blockIdx.x;
}
__device__ __forceinline__ int blk_z(const GemmParams& p) {
  return p.vgx > 0 ? (int)blockIdx.x / p.vgx : (int)blockIdx.z;
}
__device__ __forceinline__ SplitPos split_pos(const GemmParams& p) {
  return SplitPos{(int)blockIdx.y * grid_x(p) + blk_x(p), blk_z(p), p.splitk};
}

__device__ __forceinline__ int row_of(const GemmParams& p, int m) {
  m = m < p.M ? m : p.M - 1;  // clamp: duplicated rows are computed but never stored
  return p.row_idx ? p.row_idx[m] : m;
}
// Row gathers serve the LM head only (f32 logits of the sampled rows): every other epilogue reads
// rows in place, and its kernels carry no conditional row-index load (a load under a branch that
// joins before the weight stream costs the stream a wait on it, see gemm_kernel)
template <int EPI>
__device__ __forceinline__ int row_of_e(const GemmParams& p, int m) {
  if constexpr (EPI == EPI_F32) return row_of(p, m);
  return m < p.M ? m : p.M - 1;
}

// LDS carve (one dynamic array; Guideline 17): [reduce | ssq[nw][16*MB] | flag]
template <int MB, int NTB>
__host__ __device__ constexpr int red_bytes(int nw) { return nw > 1 ? nw * MB * NTB * 64 * 16 : 0; }
template <int MB>
__host__ __device__ constexpr int ssq_bytes(int nw) { return nw * MB * 16 * 4; }

// NORM: one A fragment (8 elements of row m at column k0): accumulate x^2 for the
// deferred row scale and return bf16(x * w) for the MFMA. With gamma folded into the
// packed weight at load time (w == null) the fragment passes through unchanged and no
// gamma bytes are fetched (they would double the per-k-step vector-memory requests).
template <int MODE>  // 1: gamma in registers, 2: gamma folded into W (row scale only)
__device__ __forceinline__ uint4 norm_frag(uint4 a, const bf16_t* w, int k0, float& ss) {
  float f[8];
  unpack8(a, f);
#pragma unroll
  for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
  if constexpr (MODE == 2) {
    return a;
  } else {
    const uint4 wv = *reinterpret_cast<const uint4*>(w + k0);
    float g[8];
    unpack8(wv, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= g[j];
    return pack8(f);
  }
}

// ---- epilogue operands that do not depend on the GEMM result ----
// The decode kernel loads them at launch (phase A: row / bias / residual words, phase B:
// the RoPE cos/sin row of the position, issued once the first weight group is in flight),
// so the epilogue after the reduction is pure ALU + stores instead of a dependent
// positions -> cos_sin load chain behind the whole GEMM (benchmarks/qkv_probe.py).
// QKV tile layout (ops.row_permutation "qkv"): tile t of head h (16 columns) holds the head's
// columns 8t..8t+7 (lane groups 0, 1) and their NeoX rotation partners 64+8t..64+8t+7 (groups
// 2, 3), so a rotation pair sits on lanes l and l ^ 32 of ONE tile (exchanged by permlane32).
// qkv_rot: rotation index (0..63) of the lane's first column; qkv_col: that column in [q|k|v].
__device__ __forceinline__ int qkv_rot(int nt, int nsub) { return 8 * (nt & 7) + (nsub & 4); }
__device__ __forceinline__ int qkv_col(int nt, int nsub) {
  return (nt >> 3) * 128 + (nsub >= 8 ? 64 : 0) + qkv_rot(nt, nsub);
}

// (plain scalar members: an array member keeps the whole struct in scratch)
template <int NTB>
struct EpiPre {
  uint2 r0, r1;  // EPI_BF16: residual words of tile 0 / 1 (4 bf16 each)
  uint2 b0, b1;  // EPI_BF16 / EPI_F32: bias words of tile 0 / 1; EPI_QKV: bias of the lane's 4 columns
  float4 cs, sn;
  int pos, slot;
};

// The loads are unconditional: a missing bias / residual reads the packed weights instead (always
// mapped, N x K >= any offset here) and the epilogue's own `if (p.bias)` / `if (p.res)` ignores the
// words. A load under a branch costs more than the bytes: the compiler's merge copy at the join
// waits for it there, i.e. before the weight stream is requested.
template <int NTB, int EPI>
__device__ __forceinline__ void epi_pre_a(const GemmParams& p, EpiPre<NTB>& e, int m, int nt0, int nsub) {
  m = m < p.M ? m : p.M - 1;
  const bf16_t* safe = reinterpret_cast<const bf16_t*>(p.wp);
  const bf16_t* bias = p.bias ? p.bias : safe;
  if constexpr (EPI == EPI_QKV) {
    e.pos = p.positions[m];
    e.slot = p.slots[m];
    e.b0 = *reinterpret_cast<const uint2*>(bias + qkv_col(nt0, nsub));
  } else if constexpr (EPI == EPI_BF16 || EPI == EPI_BF16_AR || EPI == EPI_F32) {
    // (no residual: row 0 of the packed weights — in bounds for any m; m * N is not once the tile
    // kernels prefetch with M up to the prefill bucket: a TP follower's row-parallel GEMMs carry no
    // residual, and their 448-row steps read past the matrix)
    const bf16_t* res = p.res ? p.res + (size_t)m * p.ldr : safe;
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      const int n = (nt0 + j) * 16 + nsub;
      const uint2 b = *reinterpret_cast<const uint2*>(bias + n);
      uint2 r = make_uint2(0, 0);
      if constexpr (EPI != EPI_F32) r = *reinterpret_cast<const uint2*>(res + n);
      if (j == 0) { e.b0 = b; e.r0 = r; } else { e.b1 = b; e.r1 = r; }
    }
  }
}

// (called once the weight stream is issued: the volatile asm with a memory clobber keeps every earlier
// load above it and is the first reader of the position, so the wait for the position load lands
// here — left alone, the compiler hoists the address arithmetic and the wait above the weight loads)
template <int NTB, int EPI>
__device__ __forceinline__ void epi_pre_b(const GemmParams& p, EpiPre<NTB>& e, int nt0, int nsub) {
  if constexpr (EPI == EPI_QKV) {
    const int d = qkv_rot(nt0, nsub);
    int pos = e.pos;
    asm volatile("" : "+v"(pos)::"memory");
    const float* cs = p.cos_sin + (size_t)pos * 128;
    e.cs = *reinterpret_cast<const float4*>(cs + d);
    e.sn = *reinterpret_cast<const float4*>(cs + 64 + d);
  }
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// EPI_BF16 with the RMSNorm hand-off (p.ssp_out): out = bf16(bf16(acc) + bias + res) as the plain
// epilogue, plus the tile's sum of out^2 (lane groups folded, group 0 stores ssp_out[m][tile]) and,
// for int4 consumers (p.hg), hg = bf16(out * gamma).
template <int NTB, bool have>
__device__ __forceinline__ void epilogue_norm_out(const GemmParams& p, const f32x4 (&v)[NTB], int m, int nt0, int nsub,
                                                  const EpiPre<NTB> e, bool valid) {
#pragma unroll
  for (int j = 0; j < NTB; ++j) {
    const int n = (nt0 + j) * 16 + nsub;
    float o[4] = {v[j][0], v[j][1], v[j][2], v[j][3]};
    float s2 = 0.f;
    if (valid) {
      if (p.bias) {
        uint2 b;
        if constexpr (have) b = j == 0 ? e.b0 : e.b1;
        else b = *reinterpret_cast<const uint2*>(p.bias + n);
        o[0] += bf_lo(b.x); o[1] += bf_hi(b.x);
        o[2] += bf_lo(b.y); o[3] += bf_hi(b.y);
      }
      if (p.res) {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = bf2f(f2bf(o[i]));  // torch: (x@W).bf16() + res
        uint2 r;
        if constexpr (have) r = j == 0 ? e.r0 : e.r1;
        else r = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.ldr + n);
        o[0] += bf_lo(r.x); o[1] += bf_hi(r.x);
        o[2] += bf_lo(r.y); o[3] += bf_hi(r.y);
      }
      uint2 pk;
      pk.x = pack_bf2(o[0], o[1]);
      pk.y = pack_bf2(o[2], o[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + n) = pk;
      const float h4[4] = {bf_lo(pk.x), bf_hi(pk.x), bf_lo(pk.y), bf_hi(pk.y)};  // the stored values
      if (p.hg != nullptr) {  // int4 consumers read h * gamma; bf16 ones fold gamma into W (ss only)
        const uint2 g = *reinterpret_cast<const uint2*>(p.hg_gamma + n);
        const float g4[4] = {bf_lo(g.x), bf_hi(g.x), bf_lo(g.y), bf_hi(g.y)};
        uint2 hk;
        hk.x = pack_bf2(h4[0] * g4[0], h4[1] * g4[1]);
        hk.y = pack_bf2(h4[2] * g4[2], h4[3] * g4[3]);
        *reinterpret_cast<uint2*>(p.hg + (size_t)m * p.ldo + n) = hk;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) s2 += h4[i] * h4[i];
    }
    s2 += xor16(s2);
    s2 += xor32(s2);
    if (valid && nsub == 0) p.ssp_out[(size_t)m * (p.N >> 4) + nt0 + j] = s2;
  }
}

// NORM == 3 consumer: this lane's share of the producer's per-tile sums of squares of row m (the
// lanes l, l^16, l^32, l^48 of a row each sum a quarter; gemm_finish folds them like the x^2 partials).
__device__ __forceinline__ float prenorm_ss(const GemmParams& p, int m, int quarter) {
  if (m >= p.M) return 0.f;
  const float* s = p.ssp_in + (size_t)m * p.ssn;
  const int q0 = (p.ssn * quarter) >> 2, q1 = (p.ssn * (quarter + 1)) >> 2;
  float acc = 0.f;
  if ((p.ssn & 15) == 0) {
    // 16-B loads (a quarter is a multiple of 4 values, 16-B aligned): at K = 1536 six per lane,
    // all in flight together
    const f32x4* s4 = reinterpret_cast<const f32x4*>(s + q0);
    const int n4 = (q1 - q0) >> 2;
    for (int t0 = 0; t0 < n4; t0 += 8) {
      f32x4 r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) r[u] = s4[min(t0 + u, n4 - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (t0 + u < n4) acc += (r[u][0] + r[u][1]) + (r[u][2] + r[u][3]);
    }
    return acc;
  }
  // every load of a 32-value chunk in flight together: one round trip per chunk (8-value steps
  // cost three dependent round trips at K = 1536)
  for (int t0 = q0; t0 < q1; t0 += 32) {
    float r[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) r[u] = s[min(t0 + u, q1 - 1)];
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (t0 + u < q1) acc += r[u];
  }
  return acc;
}

// NORM 3 consumers: the producer's sums issued at launch, summed after the weight stream (prefetch
// form: ssn <= 128 = K <= 2048, ssn % 16 == 0; else prenorm_ss after the stream)
constexpr int SS_PRE = 8;  // f32x4 loads per lane

// The producer's per-tile sums of squares of row m, this lane's quarter, loaded at launch (NORM 3).
// n4 is wave-uniform and the loads are unconditional inside (rows past M re-read row M - 1, their sum
// is never used): an exec-masked load makes the compiler wait for it — and for everything issued
// before it — right where the branch joins, i.e. before the weight stream is even requested.
struct SsPre {
  f32x4 r[SS_PRE];
  int n4;  // 0: prenorm_ss after the stream (ssn not in the prefetch form)
};
__device__ __forceinline__ int ss_pre_n4(const GemmParams& p) {
  return (p.ssn & 15) == 0 && p.ssn <= 16 * SS_PRE ? p.ssn >> 4 : 0;
}
__device__ __forceinline__ void ss_pre_issue(const GemmParams& p, SsPre& s, int m, int quarter) {
  const f32x4* src = reinterpret_cast<const f32x4*>(p.ssp_in + (size_t)min(m, p.M - 1) * p.ssn + quarter * (p.ssn >> 2));
#pragma unroll
  for (int u = 0; u < SS_PRE; ++u) s.r[u] = src[min(u, s.n4 - 1)];
}
// (call it after the weight stream is issued: the empty volatile asm pins the first use of the loaded
// registers there — left alone, the compiler hoists this pure-register sum right behind its loads
// and the wave waits a whole memory round trip before it requests a single weight)
__device__ __forceinline__ float ss_pre_sum(const GemmParams& p, const SsPre& s, int m, int quarter) {
  if (s.n4 == 0) return prenorm_ss(p, m, quarter);
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < SS_PRE; ++u) {
    f32x4 r = s.r[u];
    asm volatile("" : "+v"(r));
    if (u < s.n4) acc += (r[0] + r[1]) + (r[2] + r[3]);
  }
  return acc;
}


// ---- TP row-parallel decode GEMM (o_proj / down_proj): the all-reduce inside the epilogue ----
// Under tensor parallelism every rank's GEMM yields a partial sum of the output. Instead of storing
// it and launching the custom all-reduce (allreduce.hip: copy-in, signal, reduce, a launch and a
// copy per collective), the wave that finishes output tile t (M <= 16 rows x 16 columns, lane ->
// (row m, 4 columns)) publishes its fp32 partial into its own IPC-shared buffer, raises tile t's
// arrival word at every peer, waits for every peer's arrival on tile t, sums the peers' partials
// in rank order (bit-identical on every rank, so the replicated residual stream stays identical)
// and stores bf16(sum) + residual. Per-tile epochs (the owner's own arrival word in its own
// region: only it writes that slot), parity buffers by epoch, bounded waits on the all-reduce's
// sticky error word: the one-shot kernel's safety argument, per tile (a peer re-uses a parity
// buffer of tile t only after my next arrival on t, which follows my reads). Every lane of the
// wave calls in (wave-wide poll). Decode launchers only (gemm.hip routes ar_world >= 1 to the
// EPI_BF16_AR instantiations of the one-wave-per-tile decode kernels).
template <int NTB, bool have>
__device__ __forceinline__ void epilogue_ar(const GemmParams& p, const f32x4 (&v)[NTB], int m, int nt0, int nsub,
                                            const EpiPre<NTB> e, bool valid) {
  // The regions are uncached device memory (hipDeviceMallocUncached, mapped by the peers): no L2
  // holds their lines, so the hand-off needs ORDER, not cache maintenance — a system-scope release
  // / acquire would write back / drop the whole L2 (buffer_wbl2 / buffer_inv) once per tile and
  // cost the launch its weights. Partial -> sc0 sc1 vector stores, s_waitcnt vmcnt(0), relaxed
  // arrival word; relaxed polls; sc0 sc1 vector loads of the peers' partials after the poll.
  constexpr int SYS = 17;  // cache policy sc0 | sc1: system-coherent, bypasses every cache level
  const ArFused& a = p.ar;
  const int lane = threadIdx.x & 63;
  const int piece = (m & 15) | ((nsub >> 2) << 4);  // this lane's 16-B piece of a tile slot
  char* const mine = a.base[a.rank];
  uint32_t* const my_flags = reinterpret_cast<uint32_t*>(mine);
  uint32_t ep[NTB];
  f32x4 o[NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) {
    const int t = nt0 + j;
    ep[j] = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&my_flags[t * 8 + a.rank], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u);
    o[j] = v[j];
    if (p.bias) {
      uint2 b;
      if constexpr (have) b = j == 0 ? e.b0 : e.b1;
      else b = *reinterpret_cast<const uint2*>(p.bias + t * 16 + nsub);
      o[j][0] += bf_lo(b.x); o[j][1] += bf_hi(b.x);
      o[j][2] += bf_lo(b.y); o[j][3] += bf_hi(b.y);
    }
    const char* slot = mine + AR_FUSED_FLAG_BYTES + (int64_t)(ep[j] & 1) * AR_FUSED_DATA + (int64_t)t * 1024;
    __builtin_amdgcn_raw_buffer_store_b128(o[j], rsrc_of(slot), (uint32_t)piece * 16u, 0, SYS);
  }
  drain_stores();
  if (lane < a.world) {  // arrive at every peer (own region included: that word is my epoch)
    uint32_t* pf = reinterpret_cast<uint32_t*>(a.base[lane]);
#pragma unroll
    for (int j = 0; j < NTB; ++j)
      __hip_atomic_store(&pf[(nt0 + j) * 8 + a.rank], ep[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    uint32_t spins = 0;
    while (true) {
      bool ok = true;
      if (lane < a.world) {
#pragma unroll
        for (int j = 0; j < NTB; ++j)
          ok = ok && (int32_t)(__hip_atomic_load(&my_flags[(nt0 + j) * 8 + lane], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM) - ep[j]) >= 0;
      }
      if (__all(ok)) break;
      if (++spins > a.spin) {  // a peer never arrived: sticky error, the host fails the step
        if (lane == 0) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  asm volatile("" ::: "memory");  // the partial loads stay behind the poll
#pragma unroll
  for (int j = 0; j < NTB; ++j) {
    const int t = nt0 + j;
    const int64_t off = AR_FUSED_FLAG_BYTES + (int64_t)(ep[j] & 1) * AR_FUSED_DATA + (int64_t)t * 1024;
    // every peer's piece in flight before the first is summed; slots past world re-read rank 0
    f32x4 r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int src = q < a.world ? q : 0;
      r[q] = src == a.rank ? o[j]
                           : __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(a.base[src] + off), (uint32_t)piece * 16u, 0, SYS);
    }
    f32x4 s = r[0];
#pragma unroll
    for (int q = 1; q < 8; ++q)
      if (q < a.world) s += r[q];
    if (!valid) continue;
    const int n = t * 16 + nsub;
    float y[4] = {s[0], s[1], s[2], s[3]};
    if (p.res) {
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = bf2f(f2bf(y[i]));  // torch: all_reduce(x@W).bf16() + res
      uint2 rr;
      if constexpr (have) rr = j == 0 ? e.r0 : e.r1;
      else rr = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.ldr + n);
      y[0] += bf_lo(rr.x); y[1] += bf_hi(rr.x);
      y[2] += bf_lo(rr.y); y[3] += bf_hi(rr.y);
    }
    uint2 pk;
    pk.x = pack_bf2(y[0], y[1]);
    pk.y = pack_bf2(y[2], y[3]);
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + n) = pk;
  }
}

// ---- epilogue for one (row m, 4 columns) group; v[j] are the NTB reduced tiles ----
// `e` = operands prefetched at launch (decode kernel) when `have`, else loaded here.
// `have` is a compile-time choice: a runtime select between a prefetched register value
// and a load becomes a select of ADDRESSES that puts the prefetch struct in scratch.
// `valid`: row m < M. Every lane of the wave calls in (the QKV pair exchange is a cross-lane
// op); only valid rows store.
template <int NTB, int EPI, bool have>
__device__ __forceinline__ void epilogue(const GemmParams& p, const f32x4 (&v)[NTB], int m, int nt0, int nsub,
                                         const EpiPre<NTB> e, bool valid) {
  if constexpr (EPI == EPI_BF16_AR) {  // every lane calls in: wave-wide arrival poll
    epilogue_ar<NTB, have>(p, v, m, nt0, nsub, e, valid);
    return;
  }
  if constexpr (EPI == EPI_BF16) {
    if (p.ssp_out != nullptr) {  // every lane calls in: the tile's sum of squares is a cross-lane fold
      epilogue_norm_out<NTB, have>(p, v, m, nt0, nsub, e, valid);
      return;
    }
  }
  if constexpr (EPI != EPI_QKV && EPI != EPI_SILU) {
    if (!valid) return;
  }
  if constexpr (EPI == EPI_SILU) {
    // SiLU tile layout (ops.row_permutation "silu"): tile t holds gate columns 8t..8t+7 (lane
    // groups 0, 1) and their up partners (groups 2, 3), so a pair sits on lanes l and l ^ 32 of
    // ONE tile: every tile is self-contained and a decode block can own a single tile.
    const bool gate = nsub < 8;
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float up = xor32(v[j][i]);  // all 64 lanes active
        o[i] = silu(v[j][i]) * up;
      }
      if (valid && gate) {
        uint2 pk;
        pk.x = pack_bf2(o[0], o[1]);
        pk.y = pack_bf2(o[2], o[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + (nt0 + j) * 8 + nsub) = pk;
      }
    }
  } else if constexpr (EPI == EPI_QKV) {
    static_assert(NTB == 1, "QKV tiles carry their rotation partners (see qkv_col)");
    const int head = nt0 >> 3;
    const int d = qkv_rot(nt0, nsub);  // rotation index of this lane's 4 columns
    const bool upper = nsub >= 8;      // partner half (d + 64)
    uint2 w;
    float4 cs, sn;
    int slot, pos;
    if constexpr (have) {
      w = p.bias ? e.b0 : make_uint2(0, 0);  // (epi_pre_a read the weights when there is no bias)
      cs = e.cs; sn = e.sn; slot = e.slot; pos = e.pos;
    } else {
      const int mm = m < p.M ? m : p.M - 1;
      w = p.bias ? *reinterpret_cast<const uint2*>(p.bias + qkv_col(nt0, nsub)) : make_uint2(0, 0);
      pos = p.positions[mm];
      const float* cp = p.cos_sin + (size_t)pos * 128;
      cs = *reinterpret_cast<const float4*>(cp + d);
      sn = *reinterpret_cast<const float4*>(cp + 64 + d);
      slot = p.slots[mm];
    }
    const float b[4] = {bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)};
    float x[4], xp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = bf2f(f2bf(v[0][i] + b[i]));  // qkv is bf16 in the reference: round before rotating
#pragma unroll
    for (int i = 0; i < 4; ++i) xp[i] = xor32(x[i]);  // the partner column's value (all 64 lanes active)
    if (head < p.hq + p.hkv) {  // q or k: NeoX rotation
      const float cc[4] = {cs.x, cs.y, cs.z, cs.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = upper ? x[i] * cc[i] + xp[i] * ss[i] : x[i] * cc[i] - xp[i] * ss[i];
    }
    if (!valid) return;
    uint2 pk;
    pk.x = pack_bf2(x[0], x[1]);
    pk.y = pack_bf2(x[2], x[3]);
    const int dcol = (upper ? 64 : 0) + d;  // column inside the head
    bf16_t* dst = nullptr;
    if (head < p.hq) {
      dst = reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + head * 128 + dcol;
    } else if (slot >= 0) {
      const bool is_k = head < p.hq + p.hkv;
      const int kh = is_k ? head - p.hq : head - p.hq - p.hkv;
      dst = (is_k ? p.k_cache : p.v_cache) + (((size_t)(slot / p.bs) * p.hkv + kh) * p.bs + (slot % p.bs)) * 128 + dcol;
    }
    if (dst != nullptr) *reinterpret_cast<uint2*>(dst) = pk;
    if (p.qa_gran != nullptr && slot >= 0) {  // read in this launch by the fused attention blocks
      const uint32_t pair = (uint32_t)m * (uint32_t)(p.N >> 1) + (uint32_t)((head * 128 + dcol) >> 1);
      const uint32_t tag = (uint32_t)pos + 1u;
      st_sc1_x4(reinterpret_cast<float*>(p.qa_gran), pair * 8u,
                __builtin_bit_cast(f32x4, make_uint4(pk.x, tag, pk.y, tag)));
    }
  } else {
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      const int n = (nt0 + j) * 16 + nsub;
      float o[4] = {v[j][0], v[j][1], v[j][2], v[j][3]};
      if (p.bias) {
        uint2 b;
        if constexpr (have) b = j == 0 ? e.b0 : e.b1;
        else b = *reinterpret_cast<const uint2*>(p.bias + n);
        o[0] += bf_lo(b.x); o[1] += bf_hi(b.x);
        o[2] += bf_lo(b.y); o[3] += bf_hi(b.y);
      }
      if constexpr (EPI == EPI_F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + (size_t)m * p.ldo + n) =
            make_float4(o[0], o[1], o[2], o[3]);
      } else {
        if (p.res) {
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = bf2f(f2bf(o[i]));  // torch: (x@W).bf16() + res
          uint2 r;
          if constexpr (have) r = j == 0 ? e.r0 : e.r1;
          else r = *reinterpret_cast<const uint2*>(p.res + (size_t)m * p.ldr + n);
          o[0] += bf_lo(r.x); o[1] += bf_hi(r.x);
          o[2] += bf_lo(r.y); o[3] += bf_hi(r.y);
        }
        uint2 pk;
        pk.x = pack_bf2(o[0], o[1]);
        pk.y = pack_bf2(o[2], o[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out) + (size_t)m * p.ldo + n) = pk;
      }
    }
  }
}

// ---- cross-wave reduction, optional in-launch split-K combine, epilogue ----
// Row scale of the deferred RMSNorm: the waves' partial sums of squares (LDS, fixed
// summation order -> bit-reproducible) -> rsqrt(mean + eps).
template <int MB>
__device__ __forceinline__ float row_scale(const GemmParams& p, const float* ssqw, int r) {
  const int nw = blockDim.x >> 6;
  float ss = 0.f;
  for (int w = 0; w < nw; ++w) ss += ssqw[w * 16 * MB + r];
  return rsqrtf(ss / (float)p.K + p.eps);
}

// PRE: the epilogue thread of item s = threadIdx.x (MB == 1 decode: wave 0, one item each)
// prefetched its operands at launch (EpiPre)
template <int MB, int NTB, int EPI, int NORM, bool PRE>
__device__ __forceinline__ void gemm_finish(const GemmParams& p, f32x4 (&acc)[MB][NTB], const float (&ssr)[MB],
                                            char* smem, int m_base, int nt0, const EpiPre<NTB> pre) {
  static_assert(!PRE || MB == 1, "prefetched epilogue operands are a decode-kernel mode");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  constexpr int SLOTS = MB * NTB * 64;  // f32x4 slots per block tile
  f32x4* red4 = reinterpret_cast<f32x4*>(smem);
  float* ssqw = reinterpret_cast<float*>(smem + red_bytes<MB, NTB>(nw));
  int* flag = reinterpret_cast<int*>(smem + red_bytes<MB, NTB>(nw) + ssq_bytes<MB>(nw));
  if constexpr (NORM) {
    // lanes l, l^16, l^32, l^48 hold the same row: fold them, publish one value per row
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float v = ssr[mb];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) ssqw[wid * 16 * MB + mb * 16 + lane] = v;
    }
    if (nw == 1) __syncthreads();
  }
  if (nw > 1) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int j = 0; j < NTB; ++j) red4[wid * SLOTS + (mb * NTB + j) * 64 + lane] = acc[mb][j];
    __syncthreads();
  }
  const SplitPos sp = split_pos(p);
  const int tile = sp.tile;
  if constexpr (MB == 1 && NTB == 1) {  // (one-tile decode blocks: the path's registers would cost the
                                         // multi-tile LM-head blocks their occupancy)
    if (sp.nsl > 1 && p.gran != nullptr) {
      // wave 0, lane l: the block's partial of (row l & 15, 4 columns) per tile + the slice's row sum
      // of squares. Granule slot (tile, z < nsl - 1): [NTB][64][2] uint4 values + [64] uint4 sums.
      if (threadIdx.x >= 64) return;
      const int l = threadIdx.x;
      f32x4 v[NTB];
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        if (nw > 1) {
          f32x4 t = {0.f, 0.f, 0.f, 0.f};
          for (int w = 0; w < nw; ++w) t += red4[w * SLOTS + j * 64 + l];
          v[j] = t;
        } else {
          v[j] = acc[0][j];
        }
      }
      float ss = 0.f;
      if constexpr (NORM) {
        for (int w = 0; w < nw; ++w) ss += ssqw[w * 16 + (l & 15)];
      }
      constexpr int GW = (2 * NTB + 1) * 64;  // uint4 per slot
      constexpr uint32_t TAG = 1u;
      const size_t slot0 = (size_t)tile * (p.splitk - 1);
      if (sp.slice < sp.nsl - 1) {
        const uint32_t off = (uint32_t)(((slot0 + sp.slice) * GW) * 16);
#pragma unroll
        for (int j = 0; j < NTB; ++j) {
          st_sc1_x4(reinterpret_cast<float*>(p.gran), off + (uint32_t)((j * 64 + l) * 2) * 16u,
                    __builtin_bit_cast(f32x4, make_uint4(__float_as_uint(v[j][0]), TAG, __float_as_uint(v[j][1]), TAG)));
          st_sc1_x4(reinterpret_cast<float*>(p.gran), off + (uint32_t)((j * 64 + l) * 2 + 1) * 16u,
                    __builtin_bit_cast(f32x4, make_uint4(__float_as_uint(v[j][2]), TAG, __float_as_uint(v[j][3]), TAG)));
        }
        st_sc1_x4(reinterpret_cast<float*>(p.gran), off + (uint32_t)(NTB * 128 + l) * 16u,
                  __builtin_bit_cast(f32x4, make_uint4(__float_as_uint(ss), TAG, 0u, 0u)));
        return;
      }
      // the last slice: every other slice's granules, in slice order (bit-reproducible)
      for (int z = 0; z < sp.nsl - 1; ++z) {
        const uint32_t off = (uint32_t)(((slot0 + z) * GW) * 16);
        uint4 g[NTB][2], gs;
        int spins = 0;
        while (true) {
          bool ok = true;
#pragma unroll
          for (int j = 0; j < NTB; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              g[j][h] = __builtin_bit_cast(uint4, ld_sc1_x4(reinterpret_cast<const float*>(p.gran),
                                                             off + (uint32_t)((j * 64 + l) * 2 + h) * 16u));
              ok = ok && g[j][h].y == TAG && g[j][h].w == TAG;
            }
          gs = __builtin_bit_cast(uint4, ld_sc1_x4(reinterpret_cast<const float*>(p.gran), off + (uint32_t)(NTB * 128 + l) * 16u));
          ok = ok && gs.y == TAG;
          if (__all(ok)) break;
          if (++spins > (1 << 20)) {  // bounded: the step fails loudly (fault word), never hangs
            if (l == 0 && p.fault != nullptr) atomicOr(p.fault, 8u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int j = 0; j < NTB; ++j)
          v[j] += f32x4{__uint_as_float(g[j][0].x), __uint_as_float(g[j][0].z), __uint_as_float(g[j][1].x),
                        __uint_as_float(g[j][1].z)};
        ss += __uint_as_float(gs.x);
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NTB; ++j) {
          st_sc1_x4(reinterpret_cast<float*>(p.gran), off + (uint32_t)((j * 64 + l) * 2) * 16u, zero);
          st_sc1_x4(reinterpret_cast<float*>(p.gran), off + (uint32_t)((j * 64 + l) * 2 + 1) * 16u, zero);
        }
        st_sc1_x4(reinterpret_cast<float*>(p.gran), off + (uint32_t)(NTB * 128 + l) * 16u, zero);
      }
      if constexpr (NORM) {  // (ssqw rows are already folded over the row's four lanes)
        const float sc = rsqrtf(ss / (float)p.K + p.eps);
#pragma unroll
        for (int j = 0; j < NTB; ++j) v[j] *= sc;
      }
      epilogue<NTB, EPI, PRE>(p, v, m_base + (l & 15), nt0, 4 * (l >> 4), pre, m_base + (l & 15) < p.M);
      return;
    }
  }
  if (sp.nsl > 1) {
    // 1) this slice's partial tile -> fp32 slab [tile][slice][SLOTS]; under NORM also the
    //    slice's per-row partial sum of squares -> [tile][slice][16*MB] after all slabs
    //    (the row scale is applied to the summed tile: y = rsqrt(sum ss / K + eps) * sum acc)
    const uint32_t slab_off = (uint32_t)(((size_t)tile * p.splitk + sp.slice) * SLOTS * 16);  // bytes
    float* ssq_all = p.slabs + (size_t)grid_x(p) * gridDim.y * p.splitk * SLOTS * 4;
    if constexpr (NORM) {
      if (threadIdx.x < 16 * MB) {
        float ss = 0.f;
        for (int w = 0; w < nw; ++w) ss += ssqw[w * 16 * MB + threadIdx.x];
        st_sc1(ssq_all + ((size_t)tile * p.splitk + sp.slice) * 16 * MB + threadIdx.x, ss);
      }
    }
    for (int s = threadIdx.x; s < SLOTS; s += blockDim.x) {
      f32x4 t;
      if (nw > 1) {
        t = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int w = 0; w < nw; ++w) t += red4[w * SLOTS + s];
      } else {
        const int mb = s / (NTB * 64), j = (s / 64) % NTB;
        t = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < MB; ++a)
#pragma unroll
          for (int b = 0; b < NTB; ++b)
            if (a == mb && b == j) t = acc[a][b];
      }
      st_sc1_x4(p.slabs, slab_off + (uint32_t)s * 16u, t);
    }
    // 2) publish: every wave drains its sc1 stores, then one ticket (no cache-wide fence)
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t old = __hip_atomic_fetch_add(p.counters + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (old == (uint32_t)(sp.nsl - 1));
      if (last) __hip_atomic_store(p.counters + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // 3) the last arriver sums every slice's slab (device-coherent 16-B sc1 loads). All
    //    slices' loads are issued before the first is consumed (indices clamped, surplus
    //    masked): a runtime-trip loop of dependent loads costs one memory round trip per slice.
    const uint32_t all_off = (uint32_t)((size_t)tile * p.splitk * SLOTS * 16);
    for (int s = threadIdx.x; s < MB * 64; s += blockDim.x) {
      const int mb = s >> 6, l = s & 63;
      const int m = m_base + mb * 16 + (l & 15);
      f32x4 v[NTB];
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        f32x4 r[SK_MAX];
#pragma unroll
        for (int z = 0; z < SK_MAX; ++z)
          r[z] = ld_sc1_x4(p.slabs, all_off + (uint32_t)(((min(z, sp.nsl - 1)) * SLOTS + (mb * NTB + j) * 64 + l) * 16));
        f32x4 t = r[0];
#pragma unroll
        for (int z = 1; z < SK_MAX; ++z)
          if (z < sp.nsl) t += r[z];
        v[j] = t;
      }
      if constexpr (NORM) {
        float sv[SK_MAX];
#pragma unroll
        for (int z = 0; z < SK_MAX; ++z)
          sv[z] = ld_sc1(ssq_all + ((size_t)tile * p.splitk + min(z, sp.nsl - 1)) * 16 * MB + mb * 16 + (l & 15));
        float ss = sv[0];  // fixed slice order: bit-reproducible
#pragma unroll
        for (int z = 1; z < SK_MAX; ++z)
          if (z < sp.nsl) ss += sv[z];
        const float sc = rsqrtf(ss / (float)p.K + p.eps);
#pragma unroll
        for (int j = 0; j < NTB; ++j) v[j] *= sc;
      }
      epilogue<NTB, EPI, PRE>(p, v, m, nt0, 4 * (l >> 4), pre, m < p.M);
    }
    return;
  }
  for (int s = threadIdx.x; s < MB * 64; s += blockDim.x) {
    const int mb = s >> 6, l = s & 63;
    const int m = m_base + mb * 16 + (l & 15);
    f32x4 v[NTB];
    if (nw > 1) {
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        f32x4 t = {0.f, 0.f, 0.f, 0.f};
        for (int w = 0; w < nw; ++w) t += red4[w * SLOTS + (mb * NTB + j) * 64 + l];
        v[j] = t;
      }
    } else {
#pragma unroll
      for (int mm = 0; mm < MB; ++mm)
        if (mm == mb)
#pragma unroll
          for (int j = 0; j < NTB; ++j) v[j] = acc[mm][j];
    }
    if constexpr (NORM) {
      const float sc = row_scale<MB>(p, ssqw, mb * 16 + (l & 15));
#pragma unroll
      for (int j = 0; j < NTB; ++j) v[j] *= sc;
    }
    epilogue<NTB, EPI, PRE>(p, v, m, nt0, 4 * (l >> 4), pre, m < p.M);
  }
}

}  // namespace vgate
