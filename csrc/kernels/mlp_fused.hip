// Fused decode MLP for gfx950: resid = resid + down(silu(gate(x)) * up(x)), x = RMSNorm(resid),
// ONE launch for the two weight streams of a decoder layer's MLP (M <= 16 rows).
//
// Why one launch: at decode batch sizes both GEMMs are pure weight streams (Qwen2.5-1.5B: 55 MB
// gate_up + 27.5 MB down per layer), and as two launches the down stream cannot start before the
// last gate_up block has finished — the chip idles through gate_up's tail, the launch boundary and
// down_proj's ramp (r3 timeline: 12.7 + 1.5 + 8.8 + 1.6 us per layer for 82.5 MB). Here every CU
// streams ONE contiguous share of both matrices: it issues its down_proj weight loads while its last
// gate_up group is still in flight (they do not depend on h), so the HBM pipe of each CU runs from
// the first to the last byte; only the activations wait for the gate_up -> down dependency
// (MI355X_MICROARCH.md price list: prefetch-credit, engine-vs-launches; cdna_hip_programming.md
// §5.6: the decode MLP pair is the case where one launch wins).
//
// Decomposition (G = one workgroup per CU, resident together; S h-slices, G / S workgroups per slice):
//   h = silu(gate) * up is cut into S column slices. Slice s = the SiLU tiles [s T_s, (s+1) T_s)
//   (8 h columns per tile) and the down_proj K range of the same columns. Workgroup b works on slice
//   s = b % S (under round-robin XCD dealing all of a slice lands on one XCD: speed only).
//   Phase A: the slice's SiLU tiles split over its workgroups by whole tiles; inside a workgroup the
//            (tile, k-step) pairs are cut into W contiguous wave ranges (a range spans <= 2 tiles, the
//            partial tiles meet in LDS in wave order). x (= the residual rows, RMSNorm gamma folded
//            into the packed gate_up weights) is staged once per workgroup into LDS in MFMA-fragment
//            order; the per-row sums of squares come from the same pass (deferred row scale).
//            h leaves as 8-byte {bf16 x 2, tag} granules (tag = per-forward epoch, layer): the data is
//            its own flag (Guideline 16 R2), so no drain / fence / counter sits between a workgroup's
//            gate_up stream and its down_proj stream.
//   Phase B: the slice's down_proj pairs (n-tile, k-step within the slice) are handed out so that
//            every workgroup of the slice streams the SAME number of weight bytes over both phases
//            (gate_up tiles come in 4s and 5s: the down shares even them out). The weights of a wave's
//            down range are loaded into registers as soon as its last gate_up group is issued; the
//            wave then stages the slice's h into LDS by polling the granules and runs its MFMAs.
//            Partial [16 x 16] tiles go to fp32 slabs (sc1, drained, agent-scope ticket per n-tile);
//            the last arriving piece of an n-tile sums all S x pieces slabs in fixed (slice, piece)
//            order and runs the residual epilogue: bit-reproducible, no second launch.
// Requirements (checked by the launcher): every workgroup of the grid resident at once (one per CU:
// the LDS request pins that), spins bounded (give-up -> sticky error word, no hang).
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace vgate {

namespace {

constexpr int MLP_KMAX = 4;      // down pieces of one n-tile per slice (workgroups sharing it)
constexpr int MLP_SMAX = 16;     // h slices
constexpr int MLP_SPIN = 400000;  // poll passes before giving up (~0.5 s)

struct MlpParams {
  const bf16_t* x; int ldx; int M;
  const uint4* wgu; const uint4* wd; int H; int I;
  bf16_t* out; int ldo; const bf16_t* res; int ldr;
  float eps;
  float* hbuf;              // granules: row m, column pair c -> 8 B {bf16 pair, tag}; [16][I/2]
  float* slabs;             // [H/16][S][KMAX][64 lanes][4] f32
  uint32_t* tickets;        // [H/16], zeroed once, self-resetting
  uint32_t* err;            // sticky give-up word
  const uint32_t* epoch;    // per-forward counter (bumped by the embedding kernel)
  int layer;
  int S;
  unsigned long long* tl;
  unsigned long long* dbg;  // profiling: per-workgroup phase stamps [G][8] (wave 0), or null
};

constexpr uint32_t OOB_OFF = 0x80000000u;  // past rsrc_of's range: the load returns 0, no memory access
constexpr int AUX_NT = 2;                  // buffer-load cache policy: non-temporal (once-read weights)

template <int AUX>
__device__ __forceinline__ uint4 bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ f32x4 as_f4(uint4 v) { return __builtin_bit_cast(f32x4, v); }
__device__ __forceinline__ uint4 as_u4(f32x4 v) { return __builtin_bit_cast(uint4, v); }

// slice-local work split, identical in every workgroup (pure functions of the shape)
// (32-bit arithmetic: the launcher checks BPS * QT < 2^31; a 64-bit divide is a long software sequence)
struct Split {
  int TPS, KT1, KS2, NT2, BPS;
  int QT;
  __device__ __forceinline__ int tA(int j) const { return (j * TPS) / BPS; }
  __device__ __forceinline__ int pB(int j) const { return (j * QT) / BPS - tA(j) * KT1; }
  // workgroup (of the slice) whose down range holds pair q
  __device__ __forceinline__ int owner(int q) const {
    int j = 0;
    while (j + 1 < BPS && pB(j + 1) <= q) ++j;
    return j;
  }
};

template <int W, int UA, int NGA, int NB, int XPW, int HPW, bool BEARLY, bool XWAIT>
__global__ __launch_bounds__(64 * W) void mlp_decode_kernel(MlpParams a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(a.tl);
#define MLP_STAMP(i)                                                                          \
  do {                                                                                        \
    if (a.dbg != nullptr && lane == 0) a.dbg[blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  // the wave index through readfirstlane: every range / branch below derived from it is then a
  // scalar (SCC) branch — as threadIdx.x >> 6 the compiler treats them as divergent, masks EXEC around
  // every load and drains vmcnt at the joins, which serialises the weight stream
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int S = a.S, b = blockIdx.x;
  if (w == 0) MLP_STAMP(0);
  const int s = b % S, j = b / S;
  Split sp;
  sp.KT1 = a.H >> 5;
  sp.TPS = (a.I >> 3) / S;
  sp.KS2 = (a.I >> 5) / S;
  sp.NT2 = a.H >> 4;
  sp.BPS = gridDim.x / S;
  sp.QT = sp.TPS * sp.KT1 + sp.NT2 * sp.KS2;
  const int KT1 = sp.KT1, KS2 = sp.KS2, KT2 = a.I >> 5;
  const int tl0 = sp.tA(j), tl1 = sp.tA(j + 1);     // this workgroup's SiLU tiles (slice-local)
  const int t0 = s * sp.TPS + tl0;                  // first global SiLU tile
  const int PA = (tl1 - tl0) * KT1;
  const int pb0 = sp.pB(j), pb1 = sp.pB(j + 1);     // this workgroup's down pairs (slice-local)
  const uint32_t tag = *a.epoch * 128u + (uint32_t)a.layer + 1u;

  // LDS: [xf / hf: max(KT1, KS2) x 1 KiB fragments][ssw: W x 16 f32][red: W x 2 x 1 KiB]
  const int XF = (KT1 > KS2 ? KT1 : KS2) * 1024;
  uint4* xf = reinterpret_cast<uint4*>(smem);
  float* ssw = reinterpret_cast<float*>(smem + XF);
  f32x4* red = reinterpret_cast<f32x4*>(smem + XF + W * 64);

  // Every global load below is issued unconditionally (straight-line code, fixed counts): a load in
  // a runtime branch makes the compiler's vmcnt bookkeeping fall back to vmcnt(0) at the join, which
  // drains the whole weight stream at every group. Slots past a range are buffer loads at an offset
  // beyond the resource (OOB_OFF): they return zeros and touch no memory.
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(a.x), rA = rsrc_of(a.wgu), rB = rsrc_of(a.wd);

  // ---- x rows -> LDS fragments (loads issued first: vmcnt retires in issue order) ----
  const int mrow = r16 < a.M ? r16 : a.M - 1;  // padded rows duplicate a real row (never stored)
  const uint32_t xoff = (uint32_t)(((size_t)mrow * a.ldx + 8 * g4) * 2);
  uint4 xv[XPW];
  if (w == 0) MLP_STAMP(1);
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int kk = w + i * W;
    xv[i] = bld<0>(rx, kk < KT1 ? xoff + (uint32_t)kk * 64u : OOB_OFF);
  }
  if (w == 0) MLP_STAMP(2);

  // ---- phase A weight stream: this wave's contiguous (tile, k-step) range, NGA groups of UA ----
  const int p0 = (PA * w) / W, p1 = (PA * (w + 1)) / W;
  const int bndA = (p0 / KT1 + 1) * KT1;  // pairs >= bndA belong to the wave's second tile
  const uint32_t abase = (uint32_t)(((size_t)t0 * KT1 * 64 + lane) * 16);
  auto loadA = [&](uint4 (&v)[UA], int q0) {
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int q = q0 + u;
      v[u] = bld<AUX_NT>(rA, q < p1 ? abase + (uint32_t)q * 1024u : OOB_OFF);
    }
  };
  // down weights of this wave's range (issued once the last gate_up group is in flight)
  const int LB = pb1 - pb0;
  const int r0 = pb0 + (LB * w) / W, r1 = pb0 + (LB * (w + 1)) / W;
  const int bndB = (r0 / KS2 + 1) * KS2;
  uint4 bw[NB];
  auto loadB = [&]() {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = r0 + i;
      const uint32_t off = (uint32_t)((((size_t)(q / KS2) * KT2 + s * KS2 + q % KS2) * 64 + lane) * 16);
      bw[i] = bld<AUX_NT>(rB, q < r1 ? off : OOB_OFF);
    }
  };

  // residual words of the n-tile this wave would finalise (read only by an n-tile's last arriver;
  // loaded now so the combine at the end waits for nothing but the slabs)
  const int LB0 = pb1 - pb0;
  const int uA0 = pb0 / KS2, nfin = LB0 > 0 ? (pb1 - 1) / KS2 - uA0 + 1 : 0;
  uint2 resw;
  {  // (unconditional buffer load: zeros past the range, no branch around a load)
    const __amdgpu_buffer_rsrc_t rr = rsrc_of(a.res != nullptr ? a.res : a.x);
    const uint32_t off = (uint32_t)(((size_t)mrow * a.ldr + (uA0 + w) * 16 + 4 * g4) * 2);
    const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rr, (a.res != nullptr && w < nfin) ? off : OOB_OFF, 0, 0);
    const uint32_t v2 = __builtin_amdgcn_raw_buffer_load_b32(rr, (a.res != nullptr && w < nfin) ? off + 4 : OOB_OFF, 0, 0);
    resw = make_uint2(v, v2);
  }
  // XWAIT: the x rows land before any weight load is issued — a CU's loads return at the rate of
  // its whole burst, in any issue order (MI355X_MICROARCH.md, prologue HBM burst): x issued ahead of
  // 192 KB of weight groups still arrived ~5.5 us late and held back the first MFMA and every refill
  if constexpr (XWAIT) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (w == 0) MLP_STAMP(3);
  }
  uint4 b0[UA], b1[UA];
  loadA(b0, p0);
  if constexpr (NGA > 1) loadA(b1, p0 + UA);
  if constexpr (BEARLY) loadB();  // down weights right behind the first gate_up groups

  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int kk = w + i * W;
    float f[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += f[e] * f[e];  // zeros past KT1
    if (kk < KT1) xf[kk * 64 + lane] = xv[i];
  }
  ss += xor16(ss);
  ss += xor32(ss);
  if (lane < 16) ssw[w * 16 + lane] = ss;
  lds_barrier();
  if (w == 0) MLP_STAMP(4);

  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  auto mmaA = [&](const uint4 (&v)[UA], int q0) {
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int q = q0 + u;
      if (q < p1) {  // scalar branch (q is wave-uniform); no load inside
        const uint4 xq = xf[(q % KT1) * 64 + lane];
        if (q < bndA) acc0 = mfma16(as_bf16x8(v[u]), as_bf16x8(xq), acc0);
        else acc1 = mfma16(as_bf16x8(v[u]), as_bf16x8(xq), acc1);
      }
    }
  };
  // ping-pong: consume group g, refill its registers with group g + 2; the down weights go out at
  // the first refill slot with no gate_up group left to issue (the last group is then in flight)
#pragma unroll
  for (int g = 0; g < NGA; ++g) {
    uint4 (&buf)[UA] = (g & 1) ? b1 : b0;
    mmaA(buf, p0 + g * UA);
    if (g + 2 < NGA) loadA(buf, p0 + (g + 2) * UA);
    else if (!BEARLY && g == (NGA >= 2 ? NGA - 2 : 0)) loadB();
  }

  // ---- phase A epilogue: partial tiles meet in LDS (wave order), row scale, SiLU, h granules ----
  red[(w * 2) * 64 + lane] = acc0;
  red[(w * 2 + 1) * 64 + lane] = acc1;
  lds_barrier();
  if (w == 0) MLP_STAMP(5);  // (every wave's gate_up range done)
  if (w < tl1 - tl0) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int ww = 0; ww < W; ++ww) {
      const int q0 = (PA * ww) / W, q1 = (PA * (ww + 1)) / W;
      if (q1 <= q0) continue;
      if (q0 / KT1 == w) v += red[(ww * 2) * 64 + lane];
      else if ((q1 - 1) / KT1 == w) v += red[(ww * 2 + 1) * 64 + lane];
    }
    float sr = 0.f;
    for (int ww = 0; ww < W; ++ww) sr += ssw[ww * 16 + r16];
    v *= rsqrtf(sr / (float)a.H + a.eps);
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = silu(v[i]) * xor32(v[i]);  // gate lanes: silu(gate) * up
    if (lane < 32 && r16 < a.M) {
      // h columns 8 t + 4 g4 + i of row r16: granules (c, c + 1) = one 16-B sc1 store
      const uint4 gv = make_uint4(pack_bf2(o[0], o[1]), tag, pack_bf2(o[2], o[3]), tag);
      const uint32_t off = (uint32_t)(((size_t)r16 * (a.I >> 2) + 2 * (t0 + w) + g4) * 16);
      st_sc1_x4(a.hbuf, off, as_f4(gv));
    }
  }
  if (w == 0) MLP_STAMP(6);

  // ---- phase B: stage the slice's h (poll the granules) -> LDS fragments ----
  uint4* hf = xf;  // x fragments are dead (every wave passed the barrier above)
  {
    f32x4 hv[HPW][2];
    const size_t rowq = (size_t)mrow * (a.I >> 2);
    auto poll = [&]() {
#pragma unroll
      for (int i = 0; i < HPW; ++i) {
        const int kk = w + i * W;
        if (kk < KS2) {
          const uint32_t off = (uint32_t)((rowq + (size_t)(s * KS2 + kk) * 8 + 2 * g4) * 16);
          hv[i][0] = ld_sc1_x4(a.hbuf, off);
          hv[i][1] = ld_sc1_x4(a.hbuf, off + 16);
        }
      }
    };
    poll();
    for (int spin = 0;; ++spin) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < HPW; ++i) {
        const int kk = w + i * W;
        if (kk < KS2 && r16 < a.M) {
          const uint4 c0 = as_u4(hv[i][0]), c1 = as_u4(hv[i][1]);
          ok = ok && c0.y == tag && c0.w == tag && c1.y == tag && c1.w == tag;
        }
      }
      if (__all(ok)) break;
      if (spin >= MLP_SPIN) {
        if (lane == 0) atomicOr(a.err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      poll();
    }
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int kk = w + i * W;
      if (kk < KS2) {
        const uint4 c0 = as_u4(hv[i][0]), c1 = as_u4(hv[i][1]);
        hf[kk * 64 + lane] = r16 < a.M ? make_uint4(c0.x, c0.z, c1.x, c1.z) : make_uint4(0, 0, 0, 0);
      }
    }
  }
  lds_barrier();
  if (w == 0) MLP_STAMP(7);

  // ---- phase B MFMAs: weights in registers, h from LDS ----
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = r0 + i;
    if (q < r1) {
      const uint4 hq = hf[(q % KS2) * 64 + lane];
      if (q < bndB) c0 = mfma16(as_bf16x8(bw[i]), as_bf16x8(hq), c0);
      else c1 = mfma16(as_bf16x8(bw[i]), as_bf16x8(hq), c1);
    }
  }
  red[(w * 2) * 64 + lane] = c0;
  red[(w * 2 + 1) * 64 + lane] = c1;
  lds_barrier();
  if (w == 0) MLP_STAMP(8);
  if (LB <= 0) return;
  const int uA = pb0 / KS2, uZ = (pb1 - 1) / KS2;
  if (w > uZ - uA) return;
  const int u = uA + w;  // the n-tile this wave finalises (its piece of it)
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  for (int ww = 0; ww < W; ++ww) {
    const int q0 = pb0 + (LB * ww) / W, q1 = pb0 + (LB * (ww + 1)) / W;
    if (q1 <= q0) continue;
    if (q0 / KS2 == u) v += red[(ww * 2) * 64 + lane];
    else if ((q1 - 1) / KS2 == u) v += red[(ww * 2 + 1) * 64 + lane];
  }
  const int jf = sp.owner(u * KS2), jl = sp.owner((u + 1) * KS2 - 1);
  const int npc = jl - jf + 1, k = j - jf;
  const uint32_t slot = (uint32_t)(((size_t)u * S + s) * MLP_KMAX + k) * 1024u;
  st_sc1_x4(a.slabs, slot + lane * 16u, v);
  drain_stores();
  uint32_t old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(a.tickets + u, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  const uint32_t total = (uint32_t)(S * npc);
  if (w == 0) MLP_STAMP(9);
  if (old != total - 1) return;
  if (lane == 0) __hip_atomic_store(a.tickets + u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // last arriver: every (slice, piece) slab in fixed order; all loads issued before the adds
  f32x4 y = {0.f, 0.f, 0.f, 0.f};
  for (int z0 = 0; z0 < S; z0 += 4) {
    f32x4 r[4][MLP_KMAX];
#pragma unroll
    for (int zz = 0; zz < 4; ++zz)
#pragma unroll
      for (int kk = 0; kk < MLP_KMAX; ++kk) {
        const int z = min(z0 + zz, S - 1), kc = min(kk, npc - 1);
        r[zz][kk] = ld_sc1_x4(a.slabs, (uint32_t)(((size_t)u * S + z) * MLP_KMAX + kc) * 1024u + lane * 16u);
      }
#pragma unroll
    for (int zz = 0; zz < 4; ++zz)
#pragma unroll
      for (int kk = 0; kk < MLP_KMAX; ++kk)
        if (z0 + zz < S && kk < npc) y += r[zz][kk];
  }
  if (r16 < a.M) {
    const int n = u * 16 + 4 * g4;
    float o[4] = {y[0], y[1], y[2], y[3]};
    if (a.res != nullptr) {
      const uint2 rw = resw;  // (prefetched at the start: this wave's n-tile u = uA0 + w)
      const float rr[4] = {__uint_as_float(rw.x << 16), __uint_as_float(rw.x & 0xffff0000u),
                           __uint_as_float(rw.y << 16), __uint_as_float(rw.y & 0xffff0000u)};
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = bf2f(f2bf(o[i])) + rr[i];  // torch: (h @ Wd^T).bf16() + res
    }
    uint2 pk;
    pk.x = pack_bf2(o[0], o[1]);
    pk.y = pack_bf2(o[2], o[3]);
    *reinterpret_cast<uint2*>(a.out + (size_t)r16 * a.ldo + n) = pk;
  }
  MLP_STAMP(10);
#undef MLP_STAMP
}

int cu_count_mlp() {
  static const int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
  }();
  return n;
}

}  // namespace

// Host-side check of the work split (the same formulas as Split): every workgroup's tiles fit the
// wave ranges (<= 2 tiles / units per wave, <= W of each per workgroup), the down shares are
// non-negative, and no down n-tile is shared by more than MLP_KMAX workgroups of a slice.
static bool mlp_split_ok(int G, int S, int H, int I, int W, int NB, int XPW, int HPW) {
  if (S < 1 || S > MLP_SMAX || G % S) return false;
  if (H % 32 || I % (32 * S)) return false;
  const int KT1 = H / 32, TPS = (I / 8) / S, KS2 = (I / 32) / S, NT2 = H / 16, BPS = G / S;
  if ((KT1 + W - 1) / W > XPW || (KS2 + W - 1) / W > HPW) return false;
  const long long QT = (long long)TPS * KT1 + (long long)NT2 * KS2;
  if ((long long)BPS * QT >= (1LL << 31) || (long long)BPS * TPS >= (1LL << 31)) return false;
  auto tA = [&](int j) { return (int)(((long long)j * TPS) / BPS); };
  auto pB = [&](int j) { return (int)(((long long)j * QT) / BPS) - tA(j) * KT1; };
  int prev_owner_start = 0;
  for (int jj = 0; jj < BPS; ++jj) {
    const int T = tA(jj + 1) - tA(jj);
    if (T > W) return false;
    const int lb = pB(jj + 1) - pB(jj);
    if (lb < 0) return false;
    if (lb > 0) {
      if ((lb + W - 1) / W > NB) return false;
      if ((pB(jj + 1) - 1) / KS2 - pB(jj) / KS2 + 1 > W) return false;
    }
    (void)prev_owner_start;
  }
  // pieces per n-tile
  for (int u = 0; u < NT2; ++u) {
    int first = -1, last = -1;
    for (int jj = 0; jj < BPS; ++jj) {
      const int a0 = pB(jj), a1 = pB(jj + 1);
      if (a1 <= a0) continue;
      if (a0 < (u + 1) * KS2 && a1 > u * KS2) {
        if (first < 0) first = jj;
        last = jj;
      }
    }
    if (first < 0 || last - first + 1 > MLP_KMAX) return false;
    // the kernel's owner() scan must agree: first = block holding pair u*KS2, contiguous pieces
    for (int jj = first; jj <= last; ++jj)
      if (pB(jj + 1) <= pB(jj)) return false;  // an empty share inside a unit's span
  }
  return true;
}

bool launch_mlp_decode(const MlpDecodeArgs& g, hipStream_t st) {
  if (g.M < 1 || g.M > 16) return false;
  const int G = g.grid > 0 ? g.grid : cu_count_mlp();
  const int S = g.slices > 0 ? g.slices : 8;
  constexpr int W = 8, UA = 8, NB = 16, XPW = 8, HPW = 8;
  if (!mlp_split_ok(G, S, g.H, g.I, W, NB, XPW, HPW)) return false;
  // gate_up groups per wave: the longest wave range of the grid
  const int KT1w = g.H / 32, TPS = (g.I / 8) / S, BPS = G / S;
  int maxA = 0;
  for (int jj = 0; jj < BPS; ++jj) {
    const int T = (int)(((long long)(jj + 1) * TPS) / BPS) - (int)(((long long)jj * TPS) / BPS);
    maxA = std::max(maxA, (T * KT1w + W - 1) / W);
  }
  const int nga = (maxA + UA - 1) / UA;
  if (nga > 8) return false;
  const int NT2 = g.H / 16;
  if ((size_t)NT2 * S * MLP_KMAX * 1024 > g.slab_bytes || NT2 > g.max_tickets) return false;
  const int KT1 = g.H / 32, KS2 = (g.I / 32) / S;
  const size_t lds_need = (size_t)(KT1 > KS2 ? KT1 : KS2) * 1024 + W * 64 + W * 2 * 1024;
  if (lds_need > 160 * 1024) return false;
  const size_t lds = lds_need > 81 * 1024 ? lds_need : 81 * 1024;  // > 80 KiB: one workgroup per CU
  MlpParams p{};
  p.x = reinterpret_cast<const bf16_t*>(g.x); p.ldx = g.ldx; p.M = g.M;
  p.wgu = reinterpret_cast<const uint4*>(g.wgu); p.wd = reinterpret_cast<const uint4*>(g.wd);
  p.H = g.H; p.I = g.I;
  p.out = reinterpret_cast<bf16_t*>(g.out); p.ldo = g.ldo;
  p.res = reinterpret_cast<const bf16_t*>(g.res); p.ldr = g.ldr;
  p.eps = g.eps;
  p.hbuf = reinterpret_cast<float*>(g.hbuf);
  p.slabs = g.slabs; p.tickets = g.tickets; p.err = g.err;
  p.epoch = g.epoch; p.layer = g.layer; p.S = S;
  p.tl = tl_take("mlp_fused", G);
  p.dbg = g.dbg;
#define VG_MLP(NG, BE, XW) hipLaunchKernelGGL((mlp_decode_kernel<W, UA, NG, NB, XPW, HPW, BE, XW>), dim3(G), dim3(64 * W), lds, st, p)
#define VG_MLP_NG(BE, XW) do { if (nga <= 2) VG_MLP(2, BE, XW); else if (nga <= 4) VG_MLP(4, BE, XW); else VG_MLP(8, BE, XW); } while (0)
  // b_early bit 0: down weights right behind the first gate_up groups; bit 1: do NOT wait for x first
  const bool be = (g.b_early & 1) != 0, xw = (g.b_early & 2) == 0;
  if (be) { if (xw) VG_MLP_NG(true, true); else VG_MLP_NG(true, false); }
  else { if (xw) VG_MLP_NG(false, true); else VG_MLP_NG(false, false); }
#undef VG_MLP_NG
#undef VG_MLP
  return true;
}

}  // namespace vgate
