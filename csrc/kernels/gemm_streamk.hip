// Stream-K decode GEMM for gfx950 (M <= 16 rows, bf16 fragment-packed weights).
//
// Why: the tile-per-block decode kernel (gemm_decode.h) gives every 16-column tile to whole
// blocks, so the per-CU byte streams are as uneven as the tile count allows: Qwen2.5-1.5B
// down_proj = 96 tiles -> 192 blocks (2 K slices) on 256 CUs, gate_up = 1120 tiles -> 4 or 5 per
// CU, Llama-3-70B TP=8 qkv = 80 tiles x 256 k-steps -> 160 blocks. At decode every CU streams
// at a per-CU rate (~20 GB/s, MI355X_MICROARCH.md), so the launch lasts as long as its busiest CU.
// Here the packed weight matrix is ONE linear stream of (tile, k-step) fragments — exactly its
// memory order, Wp[nt][kt][lane][8] — cut into G = #CU equal contiguous ranges, one block each.
//
// A block's range = [lead | body]: the lead is the tail of a tile that started in an earlier
// block (a partial), the body is whole tiles plus possibly the head of a tile that continues in
// later blocks. Every wave takes 1/W of the lead FIRST, then 1/W of the body (at most two body
// tiles per wave: accumulators A / B, parked in registers at the boundaries). Then:
//   * the lead partial leaves early: the last wave to finish its lead share (LDS counter) adds
//     the W partials in wave order and publishes them to the tile's owner (the block holding the
//     tile's first k-step) as data-carrying granules: {value, tag} 8-byte pairs in 16-B
//     device-coherent (sc1) stores — the data is its own flag (cdna_hip_programming.md Guideline
//     16 R2), no drain, fence or counter on the publisher — while the body loads stream on;
//   * the waves meet in LDS (fixed wave order); whole body tiles -> the epilogue directly (bias /
//     residual / SiLU*mul / QKV+RoPE+KV, the decode kernels' epilogue code, deferred RMSNorm row
//     scale from the same x fragments);
//   * the owner of the last body tile, once its own range is done, polls the later blocks'
//     granules (published at the start of their ranges: normally there already), adds them in
//     block order (bit-reproducible), runs the epilogue and clears the slots for the next launch
//     (kernel boundary in between).
// Every global load of the stream is issued unconditionally (buffer loads; a slot past the wave's
// range is an offset beyond the resource: zeros, no memory traffic), so the compiler's vmcnt
// bookkeeping stays exact (no vmcnt(0) at branch joins). Polls are bounded: a give-up sets bit 2
// of the fault word (ModelRunner fails the engine) and leaves garbage, never a hang. All G blocks
// are resident together (one per CU), which the owner's wait relies on.
#include "gemm_decode.h"

namespace vgate {

struct SkParams {
  int KT;             // k-steps per tile (K / 32)
  int Lp;             // packs (XP k-steps) in the whole matrix: ntiles * KT / XP
  int cmax;           // contributors per tile bound (host-checked); slots per tile = cmax - 1
  uint4* pub;         // [ntiles][cmax - 1][64 lanes][3] uint4 granules, zeroed once, cleared by the owner
  uint32_t* fault;    // sticky fault word (bit 2: a partial poll gave up), or null
};

namespace {

constexpr uint32_t SK_OOB = 0x80000000u;  // past rsrc_of's range: the load returns 0, no memory access
constexpr int SK_AUX_NT = 2;              // non-temporal: once-read weights
constexpr uint32_t SK_TAG = 1u;
constexpr int SK_SPIN = 1 << 20;          // poll passes before giving up

template <int AUX>
__device__ __forceinline__ uint4 skld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void skst(uint4* base, uint32_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v), rsrc_of(base), off, 0, 16 /* sc1 */);
}

// first pack of block b (32-bit: the launcher checks Lp * G < 2^31)
__device__ __host__ __forceinline__ int sk_start(int b, int Lp, int G) { return (Lp * b) / G; }
// the block whose range holds pack X: max b with sk_start(b) <= X
__device__ __host__ __forceinline__ int sk_owner(int X, int Lp, int G) { return ((X + 1) * G + Lp - 1) / Lp - 1; }


}  // namespace

template <int W, int UA, int NGA, int EPI, int NORM, int XP>
__global__ __launch_bounds__(64 * W) void gemm_sk_kernel(GemmParams p, SkParams s) {
  constexpr int R = 16 / XP;    // real rows per packed activation load
  constexpr int UP = UA / XP;   // packs per register group
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(p.dbg_ts);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int G = gridDim.x, b = blockIdx.x;
  const int KP = s.KT / XP, Lp = s.Lp;
  const int qa = sk_start(b, Lp, G), qb = sk_start(b + 1, Lp, G);
  const int t0 = qa / KP;
  const int le = (qa % KP) ? min(qb, (t0 + 1) * KP) : qa;  // lead = [qa, le), body = [le, qb)
  const int nlead = le - qa, nbody = qb - le;
  // every wave takes 1/W of the lead, then 1/W of the body: the lead partial is complete after the
  // first few packs of every wave and leaves early (its owner waits on it at the END of its range)
  const int la = qa + (nlead * w) / W, nl = qa + (nlead * (w + 1)) / W - la;
  const int ba = le + (nbody * w) / W, nb = le + (nbody * (w + 1)) / W - ba;
  const int n = nl + nb;
  const int lpos0 = la - t0 * KP;           // lead: pack index inside tile t0
  const int tA = ba / KP, bpos0 = ba - tA * KP;
  const int bnd = (tA + 1) * KP;            // body packs >= bnd: the wave's second body tile

  // LDS: lead partials [W][64] f32x4 + [W][16] sums + arrival counter | body [W][2] accumulators,
  // [W][2][16] sums, [W][2] tile ids
  f32x4* slead = reinterpret_cast<f32x4*>(smem);
  float* ssl = reinterpret_cast<float*>(smem + W * 64 * 16);
  int* lcnt = reinterpret_cast<int*>(smem + W * 64 * 16 + W * 16 * 4);
  char* body = smem + W * 64 * 16 + W * 16 * 4 + 16;
  f32x4* sacc = reinterpret_cast<f32x4*>(body);
  float* sss = reinterpret_cast<float*>(body + W * 2 * 64 * 16);
  int* stile = reinterpret_cast<int*>(body + W * 2 * 64 * 16 + W * 2 * 16 * 4);
  if (threadIdx.x == 0) *lcnt = 0;
  __syncthreads();
  // epilogue operands of this wave's first body tile (tiles tb0 + w, tb0 + w + W, ...), loaded at
  // launch beside the weight stream: residual / bias words, the QKV position -> cos/sin chain
  const int tb0 = le / KP, tb1 = nbody > 0 ? (qb - 1) / KP : tb0 - 1;
  const int tpre = tb0 + w;
  EpiPre<1> pre;
  if (tpre <= tb1) epi_pre_a<1, EPI>(p, pre, r16, tpre, 4 * g4);

  const __amdgpu_buffer_rsrc_t rW = rsrc_of(p.wp), rX = rsrc_of(p.x);
  const int mrow = XP > 1 ? r16 % R : r16;
  const bool xok = mrow < p.M;
  const uint32_t xbase = (uint32_t)(((size_t)mrow * p.lda + 8 * g4 + (XP > 1 ? (r16 / R) * 32 : 0)) * 2);
  auto load = [&](uint4 (&wv)[UA], uint4 (&xv)[UP], int g) {
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const int i = g * UP + u;
      const bool inl = i < nl, ok = i < n;
      const int P = inl ? la + i : ba + (i - nl);
      int pos = inl ? lpos0 + i : bpos0 + (i - nl);  // pack index inside its tile (one crossing at most)
      pos = pos >= KP ? pos - KP : pos;
#pragma unroll
      for (int v = 0; v < XP; ++v)
        wv[u * XP + v] = skld<SK_AUX_NT>(rW, ok ? (uint32_t)(P * XP + v) * 1024u + (uint32_t)lane * 16u : SK_OOB);
      xv[u] = skld<0>(rX, ok && xok ? xbase + (uint32_t)pos * (uint32_t)(XP * 64) : SK_OOB);
    }
  };
  // the lead partial leaves as data-carrying granules to its owner's slot (t0, j - 1): the last of
  // the W waves to arrive (LDS counter) adds their partials in wave order and publishes
  auto lead_arrive = [&](const f32x4& a, float sq) {
    if (nlead <= 0) return;  // block-uniform
    float q = sq;
    if constexpr (NORM) {
      q += xor16(q);
      q += xor32(q);
    }
    slead[w * 64 + lane] = a;
    if (lane < 16) ssl[w * 16 + lane] = q;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) last = __hip_atomic_fetch_add(lcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == W - 1;
    last = __builtin_amdgcn_readfirstlane(last);
    if (!last) return;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    float t = 0.f;
    for (int ww = 0; ww < W; ++ww) {
      v += slead[ww * 64 + lane];
      t += ssl[ww * 16 + r16];
    }
    const int j = b - sk_owner(t0 * KP, Lp, G);  // >= 1: the tile started in an earlier block
    const uint32_t off = (uint32_t)((((size_t)t0 * (s.cmax - 1) + (j - 1)) * 64 + lane) * 3 * 16);
    skst(s.pub, off, make_uint4(__float_as_uint(v[0]), SK_TAG, __float_as_uint(v[1]), SK_TAG));
    skst(s.pub, off + 16, make_uint4(__float_as_uint(v[2]), SK_TAG, __float_as_uint(v[3]), SK_TAG));
    skst(s.pub, off + 32, make_uint4(__float_as_uint(t), SK_TAG, 0u, 0u));
  };
  // one running accumulator, parked at the lead -> body switch (pack nl: the lead partial leaves)
  // and at the body's tile boundary (accA). Packs past the range were loaded as zeros and add
  // nothing: the MFMAs run unconditionally (a branch around them made the compiler re-issue loads
  // under it and drain vmcnt).
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accL = {0.f, 0.f, 0.f, 0.f}, accA = {0.f, 0.f, 0.f, 0.f},
        accB = {0.f, 0.f, 0.f, 0.f};
  float ss = 0.f, ssL = 0.f, ssA = 0.f, ssB = 0.f;
  const uint32_t lom = r16 < R ? ~0u : 0u;
  auto mma = [&](const uint4 (&wv)[UA], const uint4 (&xv)[UP], int g) {
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const int i = g * UP + u;
      uint4 a[XP];
      if constexpr (XP == 1) {
        a[0] = xv[u];
      } else {  // DPP with every lane active, select after
        a[0] = and_mask(xv[u], lom);
        a[1] = and_mask(row_ror<R>(xv[u]), lom);
        if constexpr (XP == 4) {
          a[2] = and_mask(row_ror<2 * R>(xv[u]), lom);
          a[3] = and_mask(row_ror<3 * R>(xv[u]), lom);
        }
      }
      if (i == nl) {  // wave-uniform: the lead share is done (register moves; it leaves at the group's end)
        accL = acc;
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        ssL = ss;
        ss = 0.f;
      }
      if (i > nl && ba + (i - nl) == bnd && i < n) {  // the body's tile boundary: register moves only
        accA = acc;
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        ssA = ss;
        ss = 0.f;
      }
#pragma unroll
      for (int v = 0; v < XP; ++v) {
        if constexpr (NORM) {
          float f[8];
          unpack8(a[v], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
        }
        acc = mfma16(as_bf16x8(wv[u * XP + v]), as_bf16x8(a[v]), acc);
      }
    }
  };
  // (sched_barrier: keep every issued group's loads ahead of the MFMAs that do not need them —
  // the scheduler otherwise sinks the second group below the first group's MFMAs)
  uint4 w0[UA], w1[UA], x0[UP], x1[UP];
  load(w0, x0, 0);
  if constexpr (NGA > 1) load(w1, x1, 1);
  if (tpre <= tb1) epi_pre_b<1, EPI>(p, pre, tpre, 4 * g4);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < NGA; ++g) {
    if (g & 1) {
      mma(w1, x1, g);
      if (g + 2 < NGA) load(w1, x1, g + 2);
    } else {
      mma(w0, x0, g);
      if (g + 2 < NGA) load(w0, x0, g + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    // the group in which the lead share ended (a wave without one arrives after group 0)
    if (nl < (g + 1) * UP && (nl >= g * UP || g == 0)) lead_arrive(accL, ssL);
  }
  if (nl >= NGA * UP) {  // (a lead share filling every register group: parked nowhere yet)
    lead_arrive(acc, ss);
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    ss = 0.f;
  }
  if (ba + nb > bnd && nb > 0) {
    accB = acc;
    ssB = ss;
  } else {
    accA = acc;
    ssA = ss;
  }
  if constexpr (NORM) {  // lanes l, l^16, l^32, l^48 hold row r16: fold them
    ssA += xor16(ssA);
    ssA += xor32(ssA);
    ssB += xor16(ssB);
    ssB += xor32(ssB);
  }

  // ---- the body waves meet in LDS ----
  sacc[(w * 2) * 64 + lane] = accA;
  sacc[(w * 2 + 1) * 64 + lane] = accB;
  if (lane < 16) {
    sss[(w * 2) * 16 + lane] = ssA;
    sss[(w * 2 + 1) * 16 + lane] = ssB;
  }
  if (lane == 0) {
    stile[w * 2] = nb > 0 ? tA : -1;
    stile[w * 2 + 1] = ba + nb > bnd && nb > 0 ? tA + 1 : -1;
  }
  __syncthreads();

  // the body tiles, wave w takes tiles w, w + W, ...: whole tiles -> epilogue; the last one, if it
  // continues in later blocks, first adds their published lead partials (block order)
  for (int t = tb0 + w; t <= tb1; t += W) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    float sq = 0.f;
    for (int ww = 0; ww < W; ++ww) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (stile[ww * 2 + k] == t) {
          v += sacc[(ww * 2 + k) * 64 + lane];
          sq += sss[(ww * 2 + k) * 16 + r16];
        }
      }
    }
    if ((t + 1) * KP > qb) {
      const int tend = (t + 1) * KP;
      for (int j = 1; j < s.cmax && sk_start(b + j, Lp, G) < tend; ++j) {
        const uint32_t off = (uint32_t)((((size_t)t * (s.cmax - 1) + (j - 1)) * 64 + lane) * 3 * 16);
        uint4 g0, g1, g2;
        int spins = 0;
        while (true) {
          g0 = __builtin_bit_cast(uint4, ld_sc1_x4(reinterpret_cast<const float*>(s.pub), off));
          g1 = __builtin_bit_cast(uint4, ld_sc1_x4(reinterpret_cast<const float*>(s.pub), off + 16));
          g2 = __builtin_bit_cast(uint4, ld_sc1_x4(reinterpret_cast<const float*>(s.pub), off + 32));
          const bool ok = g0.y == SK_TAG && g0.w == SK_TAG && g1.y == SK_TAG && g1.w == SK_TAG && g2.y == SK_TAG;
          if (__all(ok)) break;
          if (++spins > SK_SPIN) {
            if (lane == 0 && s.fault != nullptr) atomicOr(s.fault, 4u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        v += f32x4{__uint_as_float(g0.x), __uint_as_float(g0.z), __uint_as_float(g1.x), __uint_as_float(g1.z)};
        sq += __uint_as_float(g2.x);
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
        skst(s.pub, off, z);
        skst(s.pub, off + 16, z);
        skst(s.pub, off + 32, z);
      }
    }
    if constexpr (NORM) v *= rsqrtf(sq / (float)p.K + p.eps);
    f32x4 vv[1] = {v};
    if (t == tpre) epilogue<1, EPI, true>(p, vv, r16, t, 4 * g4, pre, r16 < p.M);
    else epilogue<1, EPI, false>(p, vv, r16, t, 4 * g4, EpiPre<1>{}, r16 < p.M);
  }
}

// ------------------------------------------------------------------ host side
namespace {

struct SkPlan {
  int XP, NGA, cmax;
  bool ok;
};

// the same arithmetic as the kernel, over every block: the longest wave range (register groups),
// the one-boundary-per-wave bound, and the contributors per tile (publisher slots)
SkPlan sk_plan(int ntiles, int KT, int M, int G, int W, int UA) {
  SkPlan pl{1, 1, 1, false};
  pl.XP = M <= 4 && KT % 4 == 0 ? 4 : (M <= 8 && KT % 2 == 0 ? 2 : 1);
  const int XP = pl.XP, KP = KT / XP;
  const long long Lp64 = (long long)ntiles * KP;
  if (Lp64 * (G + 1) >= (1ll << 31) || Lp64 * XP * 1024 >= (1ll << 31) || Lp64 < G) return pl;
  const int Lp = (int)Lp64;
  int maxn = 0;
  for (int b = 0; b < G; ++b) {
    const int qa = sk_start(b, Lp, G), qb = sk_start(b + 1, Lp, G);
    const int t0 = qa / KP;
    const int le = (qa % KP) ? std::min(qb, (t0 + 1) * KP) : qa;
    const int nlead = le - qa, nbody = qb - le;
    const int nlw = (nlead + W - 1) / W, nbw = (nbody + W - 1) / W;
    if (nbw > KP) return pl;  // a body share would cross two tile boundaries
    maxn = std::max(maxn, nlw + nbw);
  }
  // contributors per tile: blocks overlapping [t KP, (t + 1) KP)
  int cmax = 1;
  for (int t = 0; t < ntiles; ++t) {
    const int o = sk_owner(t * KP, Lp, G), last = sk_owner((t + 1) * KP - 1, Lp, G);
    cmax = std::max(cmax, last - o + 1);
  }
  const int UP = UA / XP;
  const int nga = (maxn + UP - 1) / UP;
  pl.NGA = nga <= 1 ? 1 : nga <= 2 ? 2 : nga <= 4 ? 4 : nga <= 8 ? 8 : 0;
  pl.cmax = cmax;
  pl.ok = pl.NGA > 0;
  return pl;
}

// The LDS request pins the blocks per CU: the equal shares only balance the chip if no CU takes
// two of them while another idles (the dispatcher packs workgroups onto a CU while its registers
// and LDS allow). 1 per CU: > 80 KiB of the 160 KiB; 2 per CU: > 160 / 3 KiB.
//
// The owners of a tile wait for granules of blocks dispatched after them, so all G blocks must be
// resident at once: the launcher asks the runtime how many blocks of this kernel fit per CU at this
// LDS request (VGPRs included) and declines the launch when G do not (the caller then runs the tile
// kernels). It cannot see CUs held by kernels of OTHER streams: this path assumes the engine's decode
// step owns the device (no concurrent compute stream), which the engine guarantees; the waits are
// bounded all the same (fault bit 4) so a violation fails the step instead of hanging the GPU.
template <typename K>
bool sk_fits(K kern, int threads, size_t lds, int G) {
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(kern), threads, lds) !=
      hipSuccess)
    return false;
  return (long long)per * cu_count_gemm() >= G;
}

template <int W, int UA, int EPI, int NORM, int XP>
bool sk_launch_cfg(const GemmParams& p, const SkParams& s, int nga, int G, int per_cu, hipStream_t st) {
  constexpr size_t need = W * 64 * 16 + W * 16 * 4 + 16 + W * 2 * 64 * 16 + W * 2 * 16 * 4 + W * 2 * 4;
  const size_t lds = std::max(need, per_cu == 1 ? (size_t)82 * 1024 : (size_t)54 * 1024);
#define VG_SK(N)                                                                                              \
  do {                                                                                                        \
    auto kern = gemm_sk_kernel<W, UA, N, EPI, NORM, XP>;                                                      \
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                        \
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess; \
    (void)attr;                                                                                               \
    static int fits[3] = {-1, -1, -1}; /* per blocks-per-CU setting (lds and G follow from it) */            \
    if (fits[per_cu] < 0) fits[per_cu] = sk_fits(kern, 64 * W, lds, G) ? 1 : 0;                               \
    if (!fits[per_cu]) return false;                                                                          \
    hipLaunchKernelGGL(kern, dim3(G), dim3(64 * W), lds, st, p, s);                                           \
  } while (0)
  if (nga == 1) VG_SK(1);
  else if (nga == 2) VG_SK(2);
  else if (nga == 4) VG_SK(4);
  else VG_SK(8);
#undef VG_SK
  return true;
}

// (W, UA): 8 waves x groups of 8 k-steps (default), 4 x 8, 8 x 4 (sweeps: GemmArgs waves / ntb)
template <int EPI, int NORM, int XP>
bool sk_launch_xp(const GemmParams& p, const SkParams& s, int w, int ua, int nga, int G, int per_cu, hipStream_t st) {
  if (w == 4) return sk_launch_cfg<4, 8, EPI, NORM, XP>(p, s, nga, G, per_cu, st);
  if (ua == 4) return sk_launch_cfg<8, 4, EPI, NORM, XP>(p, s, nga, G, per_cu, st);
  return sk_launch_cfg<8, 8, EPI, NORM, XP>(p, s, nga, G, per_cu, st);
}

template <int EPI, int NORM>
bool sk_launch(const GemmParams& p, const SkParams& s, int xp, int w, int ua, int nga, int G, int per_cu,
               hipStream_t st) {
  if (xp == 4) return sk_launch_xp<EPI, NORM, 4>(p, s, w, ua, nga, G, per_cu, st);
  if (xp == 2) return sk_launch_xp<EPI, NORM, 2>(p, s, w, ua, nga, G, per_cu, st);
  return sk_launch_xp<EPI, NORM, 1>(p, s, w, ua, nga, G, per_cu, st);
}

}  // namespace

bool launch_gemm_sk(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return true;
  if (g.M > 16 || g.row_idx != nullptr || g.norm_w != nullptr || g.ssp_out != nullptr || g.ssp_in != nullptr ||
      g.sk_pub == nullptr || g.K % 32 != 0)
    return false;
  if (g.epi == EPI_QKV && (g.N / 16) % 2 != 0) return false;
  const int norm = g.rownorm ? 2 : 0;
  // instantiated pairs: plain / f32 without a norm, SiLU / QKV with the folded-gamma row scale
  if ((norm == 2) != (g.epi == EPI_SILU || g.epi == EPI_QKV)) return false;
  // sweeps: g.waves 4 = 4 waves per block, g.ntb 4 = groups of 4 k-steps, g.splitk 2 = 2 blocks per CU
  const int W = g.waves == 4 ? 4 : 8, UA = (g.ntb == 4 && W == 8) ? 4 : 8;
  const int per_cu = g.splitk == 2 ? 2 : 1;
  const int G = cu_count_gemm() * per_cu;
  const int ntiles = g.N / 16, KT = g.K / 32;
  const SkPlan pl = sk_plan(ntiles, KT, g.M, G, W, UA);
  if (!pl.ok) return false;
  if ((size_t)ntiles * (pl.cmax - 1) * 64 * 3 * 16 > g.sk_bytes) return false;
  GemmParams p{};
  p.x = reinterpret_cast<const bf16_t*>(g.x); p.lda = g.lda; p.M = g.M;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.eps = g.eps;
  p.bias = reinterpret_cast<const bf16_t*>(g.bias); p.res = reinterpret_cast<const bf16_t*>(g.res); p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.splitk = 1;
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = reinterpret_cast<bf16_t*>(g.k_cache); p.v_cache = reinterpret_cast<bf16_t*>(g.v_cache);
  p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  // timeline names by role (benchmarks/timeline.py groups launches by name)
  const char* tl_name = g.epi == EPI_QKV ? "gemm_sk_qkv" : g.epi == EPI_SILU ? "gemm_sk_gate_up"
                        : g.epi == EPI_F32 ? "gemm_sk_f32" : (g.K > g.N ? "gemm_sk_down" : "gemm_sk_o");
  p.dbg_ts = g.dbg_ts != nullptr ? g.dbg_ts : tl_take(tl_name, G);
  SkParams s{KT, ntiles * KT / pl.XP, pl.cmax, reinterpret_cast<uint4*>(g.sk_pub), g.fault};
#define VG_SKE(E, NORM_) sk_launch<E, NORM_>(p, s, pl.XP, W, UA, pl.NGA, G, per_cu, st)
  switch (g.epi) {
    case EPI_SILU: return VG_SKE(EPI_SILU, 2);
    case EPI_QKV: return VG_SKE(EPI_QKV, 2);
    case EPI_F32: return VG_SKE(EPI_F32, 0);
    default: return VG_SKE(EPI_BF16, 0);
  }
#undef VG_SKE
}

}  // namespace vgate
