// Decode-attention building blocks shared by the attention launches (attention.hip) and the
// fused QKV-projection + decode-attention launch (qkv_attn.hip): the K / V chunk loads, the
// online-softmax step, the V^T . P^T update and the per-(sequence, KV head, partition) decode block.
// Layout and MFMA orientation: attention.hip (file comment).
#pragma once
#include <type_traits>

#include "gemm_epilogue.h"

namespace vgate {

constexpr int D_ = 128;
constexpr int BS_ = 16;
constexpr int CHUNK = 32;
constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ int v_lds_off(int r, int c) {  // element offset, c % 4 == 0
  return r * D_ + ((((c >> 2) ^ ((r & 7) << 2))) << 2);
}

// Stage a 32-token V chunk into the swizzled LDS image. `valid` = tokens < valid are real.
// Instruction i: lane reads 16 B at element (4i + l>>4, 8(l&15)) -> 1 KiB coalesced.
// rb >= 0 (fused QKV + attention launch): cache row rb of block vb0 (s0) / vb1 (s1) is still being
// written by this launch; its lanes read the neighbouring row (rb ^ 1) instead — ONE extra per-lane
// offset, selected per load by a wave-uniform test — and the caller patches them after the wait.
__device__ __forceinline__ void load_v_regs(uint4 (&vr)[8], const bf16_t* vb0, const bf16_t* vb1,
                                            int lane, int rb = -1, bool s0 = false, bool s1 = false) {
  const int dv = rb >= 0 && (lane >> 4) == (rb & 3) ? ((rb & 1) ? -D_ : D_) : 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = 4 * i + (lane >> 4);
    const int c = 8 * (lane & 15) + (((i < 4 ? s0 : s1) && (i & 3) == (rb >> 2)) ? dv : 0);
    const bf16_t* src = (r < 16 ? vb0 + r * D_ : vb1 + (r - 16) * D_) + c;
    vr[i] = *reinterpret_cast<const uint4*>(src);
  }
}

__device__ __forceinline__ void store_v_lds(bf16_t* lds, const uint4 (&vr)[8], int lane, int valid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = 4 * i + (lane >> 4);
    const int c = 8 * (lane & 15);
    const uint4 v = r < valid ? vr[i] : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(lds + v_lds_off(r, c)) = v;
  }
}

// O^T[16mt + ..][col] += V^T(chunk) . P^T ; pb = P^T fragment (bf16x8)
__device__ __forceinline__ void pv_update(f32x4 (&o)[8], const bf16_t* lds, const bf16x8& pb,
                                          int lane) {
  const int g = lane >> 4;
  const int q = (lane >> 2) & 3;
  const int p = lane & 3;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int c = 16 * mt + 4 * p;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (lds_bf16x4*)(lds + v_lds_off(4 * g + q, c)));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (lds_bf16x4*)(lds + v_lds_off(16 + 4 * g + q, c)));
    bf16x8 a;
    a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
    a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
    o[mt] = mfma16(a, pb, o[mt]);
  }
}

__device__ __forceinline__ bf16x8 pack_p(const f32x4& s0, const f32x4& s1) {
  bf16x8 b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    b[i] = (__bf16)s0[i];
    b[4 + i] = (__bf16)s1[i];
  }
  return b;
}

// S^T tile for 16 tokens starting at kbase (row-major [16][D] in cache)
__device__ __forceinline__ f32x4 qk_tile(const bf16_t* kbase, const uint4 (&qf)[4], int lane) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bf16_t* kp = kbase + (lane & 15) * D_ + 8 * (lane >> 4);
  uint4 kf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) kf[kk] = *reinterpret_cast<const uint4*>(kp + 32 * kk);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) acc = mfma16(as_bf16x8(kf[kk]), as_bf16x8(qf[kk]), acc);
  return acc;
}

// Online-softmax step over one 32-token chunk for the lane's query column.
// tok_lo: absolute token index of chunk row 0; lim: tokens >= lim are masked for this column.
__device__ __forceinline__ bf16x8 softmax_step(f32x4& s0, f32x4& s1, float& m, float& l,
                                               f32x4 (&o)[8], int tok_lo, int lim, float cscale,
                                               int lane) {
  const int g = lane >> 4;
  float cmax = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t0 = tok_lo + 4 * g + i, t1 = tok_lo + 16 + 4 * g + i;
    s0[i] = t0 < lim ? s0[i] * cscale : -INFINITY;
    s1[i] = t1 < lim ? s1[i] * cscale : -INFINITY;
    cmax = fmaxf(cmax, fmaxf(s0[i], s1[i]));
  }
  cmax = fmaxf(cmax, xor16(cmax));
  cmax = fmaxf(cmax, xor32(cmax));
  const float mn = fmaxf(m, cmax);
  // a fully masked column keeps m = -inf: exponentiate against 0 instead, so masked
  // scores give exp2(-inf) = 0 and alpha only multiplies zeros (no per-element selects).
  // Raw v_exp_f32: the arguments are <= 0 and underflow to 0 is the wanted result.
  const float mref = mn == -INFINITY ? 0.f : mn;
  const float alpha = __builtin_amdgcn_exp2f(m - mref);
  float ps = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s0[i] = __builtin_amdgcn_exp2f(s0[i] - mref);
    s1[i] = __builtin_amdgcn_exp2f(s1[i] - mref);
    ps += s0[i] + s1[i];
  }
  l = l * alpha + ps;
  m = mn;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) o[mt] *= alpha;
  return pack_p(s0, s1);
}

// LDS: max(decode: one V image (then o partial) per wave + (m, l) + flag, prefill double buffer)
__host__ __device__ constexpr int attn_lds_bytes(int nw) {
  return nw * CHUNK * D_ * 2 + nw * 32 * 4 + 16 > 2 * CHUNK * D_ * 2 ? nw * CHUNK * D_ * 2 + nw * 32 * 4 + 16
                                                                     : 2 * CHUNK * D_ * 2;
}

// ---------------------------------------------------------------- decode ----
// ONE WORKGROUP per (sequence, KV head, partition); its nw waves take the partition's
// 32-token chunks round-robin (chunk c -> wave c % nw), so a short context has every chunk's
// K/V loads in flight at once (one HBM round trip instead of one per chunk: a single wave is
// latency-bound at ~16 KB per round trip, MI355X_MICROARCH.md handoff-payload). Each wave
// keeps its own online-softmax state; the waves' (m, l, o) are merged through LDS (the o
// partials reuse each wave's V image). Query columns = the G = Hq/Hkv heads sharing the KV
// head. Partitions of one (sequence, head) — contexts longer than part_size — are merged
// by the last-arriving block (sc1 hand-off + ticket, no second launch).
// Only sequences with a single new query token are decode work.
#define ATTN_STAMP(i)                                                                          \
  do {                                                                                         \
    if (a.dbg_ts != nullptr && threadIdx.x == 0 && s == 0 && h == 0 && part == 0)              \
      a.dbg_ts[i] = __builtin_amdgcn_s_memrealtime();                                          \
  } while (0)

__device__ __forceinline__ void load_k_regs(uint4 (&kf)[8], const bf16_t* kb0, const bf16_t* kb1, int lane,
                                            int rb = -1, bool s0 = false, bool s1 = false) {  // (rb: load_v_regs)
  const int dk = rb >= 0 && (lane & 15) == rb ? ((rb & 1) ? -D_ : D_) : 0;
  const bf16_t* k0 = kb0 + (lane & 15) * D_ + 8 * (lane >> 4) + (s0 ? dk : 0);
  const bf16_t* k1 = kb1 + (lane & 15) * D_ + 8 * (lane >> 4) + (s1 ? dk : 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) kf[kk] = *reinterpret_cast<const uint4*>(k0 + 32 * kk);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) kf[4 + kk] = *reinterpret_cast<const uint4*>(k1 + 32 * kk);
}

// LDS of a decode block: [nw][CHUNK * D_] bf16 V images (then the waves' fp32 o partials,
// 16 cols x 128 d = the same 8 KiB) | [nw][16][2] (m, l) | flag
__host__ __device__ constexpr int dec_ml_off(int nw) { return nw * CHUNK * D_ * 2; }

// Output stores. SC1: write-through (device-coherent) stores, for a consumer that reads the
// result inside the same launch (a consumer in the same launch loads it with sc1 loads)
template <bool SC1>
__device__ __forceinline__ void out_store16(bf16_t* base, size_t elem, uint4 v) {
  if constexpr (SC1) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v), rsrc_of(base), (uint32_t)(elem * 2), 0, 16);
  } else {
    *reinterpret_cast<uint4*>(base + elem) = v;
  }
}
template <bool SC1>
__device__ __forceinline__ void out_store8(bf16_t* base, size_t elem, uint2 v) {
  if constexpr (SC1) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, rsrc_of(base), (uint32_t)(elem * 2), 0, 16);
  } else {
    *reinterpret_cast<uint2*>(base + elem) = v;
  }
}

// Fused QKV projection + decode attention (qkv_attn.hip): the handed-off values travel as data-tagged
// granules, 8 B = {a bf16 pair, tag} with tag = position + 1 of the row, written by the GEMM epilogue
// (16-B write-through stores of two granules) and polled by the consumer with 16-B sc1 loads until
// every tag matches (MI355X_MICROARCH.md handoff-1to1 / R2: no flag, no drain, no fence). The consumer
// clears what it read, so a later launch never meets a stale tag. qa_get8: the 8 bf16 at granule
// (pair) index `pair` (even) -> v; true when all four tags match.
__device__ __forceinline__ bool qa_get8(const QaSync& q, uint32_t pair, uint32_t tag, uint4& v) {
  const float* gb = reinterpret_cast<const float*>(q.gran);
  const uint4 x = __builtin_bit_cast(uint4, ld_sc1_x4(gb, pair * 8u));
  const uint4 y = __builtin_bit_cast(uint4, ld_sc1_x4(gb, pair * 8u + 16u));
  v = make_uint4(x.x, x.z, y.x, y.z);
  return x.y == tag && x.w == tag && y.y == tag && y.w == tag;
}

// FUSED: the block runs in the fused QKV + attention launch. Everything that does not depend on this
// step's projection — context length, block table, every wave's first K / V chunk — is requested at
// once; the query fragments and the new token's K / V row (position ctx - 1) come from the producer
// blocks' granules (qa_get8), never through a plain load of the cache row the producer is writing
// (the prefetched chunk reads the neighbouring row in its place and is patched).
template <bool SC1 = false, bool FUSED = false>
__device__ __forceinline__ void decode_block(const AttnArgs& a, int s, int h, int part, char* smem,
                                             const QaSync* qs = nullptr) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  ATTN_STAMP(0);
  const int pstart = part * a.part_size;
  const int* bt = a.block_tables + (size_t)s * a.max_blocks;
  // every independent load of the dependency chain up front: context length, query
  // bounds, the partition's block-table window (one entry per lane: chunk addresses come
  // from v_readlane, never from a per-chunk global load) and the query fragments
  const int ctx = a.context_lens[s];
  const int qbeg = a.query_start ? a.query_start[s] : s;
  const int qend = a.query_start ? a.query_start[s + 1] : s + 1;
  const int btv = bt[min(pstart / BS_ + lane, a.max_blocks - 1)];
  const int G = a.Hq / a.Hkv;
  const int col = lane & 15;
  const bool cok = col < G;
  uint4 qf[4];  // (FUSED: from the producer's granules, after the wait)
  if constexpr (!FUSED) {
    const bf16_t* qp = a.q + (size_t)qbeg * a.q_stride + (size_t)(h * G + (cok ? col : 0)) * D_ + 8 * (lane >> 4);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) qf[kk] = cok ? *reinterpret_cast<const uint4*>(qp + 32 * kk) : make_uint4(0, 0, 0, 0);
  }
  if (ctx <= 0 || pstart >= ctx || qend - qbeg != 1) return;  // block-uniform
  ATTN_STAMP(1);
  const int pend = min(ctx, pstart + a.part_size);
  const int nparts = (ctx + a.part_size - 1) / a.part_size;
  const int nch = (pend - pstart + CHUNK - 1) / CHUNK;
  const int myn = nch > wid ? (nch - wid + nw - 1) / nw : 0;  // chunks wid, wid + nw, ...
  const size_t head_off = (size_t)h * BS_ * D_;
  const size_t blk_stride = (size_t)a.Hkv * BS_ * D_;
  const float cscale = a.scale * LOG2E;
  bf16_t* vl = reinterpret_cast<bf16_t*>(smem) + wid * (CHUNK * D_);
  float m = -INFINITY, l = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // j-th chunk of this wave covers tokens [tb, tb + 32) = cache blocks (b0, b1). Two
  // register sets ping-pong: chunk j+1's K/V loads are issued before chunk j is consumed.
  // FUSED: the new token (chunk cnew of this partition, row rnew in it; cache block nb, row rb)
  const int tnew = ctx - 1 - pstart;
  const int cnew = FUSED && tnew < pend - pstart ? tnew / CHUNK : -1;
  const int rnew = tnew % CHUNK, rb = tnew % BS_;
  const int nb = cnew >= 0 ? __builtin_amdgcn_readlane(btv, tnew / BS_) : 0;
  auto issue = [&](uint4 (&kf)[8], uint4 (&vr)[8], int j) {
    const int c = wid + j * nw;
    const int tb = pstart + c * CHUNK;
    const int n0 = __builtin_amdgcn_readlane(btv, 2 * c);
    const int n1 = (tb + BS_ < pend) ? __builtin_amdgcn_readlane(btv, 2 * c + 1) : n0;
    const bool sk0 = cnew >= 0 && n0 == nb, sk1 = cnew >= 0 && n1 == nb;
    load_k_regs(kf, a.k_cache + (size_t)n0 * blk_stride + head_off, a.k_cache + (size_t)n1 * blk_stride + head_off,
                lane, FUSED ? rb : -1, sk0, sk1);
    load_v_regs(vr, a.v_cache + (size_t)n0 * blk_stride + head_off, a.v_cache + (size_t)n1 * blk_stride + head_off,
                lane, FUSED ? rb : -1, sk0, sk1);
  };
  // FUSED: poll the granules of this sequence's row — the query fragments (with_q) and / or the new
  // token's K row (lanes of row rb, half rnew / 16) and V row (lanes rnew % 4 of slot rnew / 4) into
  // the prefetched chunk (with_new) — until every tag is this step's; bounded (fault bit 32)
  const uint32_t tag = (uint32_t)ctx;  // position + 1 of the new token
  const uint32_t row0 = FUSED ? (uint32_t)qbeg * (uint32_t)qs->n2 : 0u;
  auto poll = [&](bool with_q, bool with_new, uint4 (&kf)[8], uint4 (&vr)[8]) {
    const uint32_t qp = row0 + (uint32_t)(((h * G + (cok ? col : 0)) * D_ + 8 * (lane >> 4)) >> 1);
    const uint32_t kp = row0 + (uint32_t)(((a.Hq + h) * D_ + 8 * (lane >> 4)) >> 1);
    const uint32_t vp = row0 + (uint32_t)(((a.Hq + a.Hkv + h) * D_ + 8 * (lane & 15)) >> 1);
    int spins = 0;
    while (true) {
      uint4 qv[4], kn[4], vn;
      bool ok = true;
      if (with_q) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) ok = qa_get8(*qs, qp + 16 * kk, tag, qv[kk]) && ok;
      }
      if (with_new) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) ok = qa_get8(*qs, kp + 16 * kk, tag, kn[kk]) && ok;
        ok = qa_get8(*qs, vp, tag, vn) && ok;
      }
      const bool all = __all(ok);
      if (all && with_q) ATTN_STAMP(6);  // profiling: the query granules are this step's
      if (all || ++spins > (1 << 20)) {  // bounded: the step fails loudly (fault word), never hangs
        if (!all && lane == 0 && qs->fault != nullptr) atomicOr(qs->fault, 32u);
        if (with_q) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) qf[kk] = cok ? qv[kk] : make_uint4(0, 0, 0, 0);
        }
        if (with_new) {
          if ((lane & 15) == rb) {
            if (rnew < 16) {
#pragma unroll
              for (int kk = 0; kk < 4; ++kk) kf[kk] = kn[kk];
            } else {
#pragma unroll
              for (int kk = 0; kk < 4; ++kk) kf[4 + kk] = kn[kk];
            }
          }
          if ((lane >> 4) == (rnew & 3)) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if (i == (rnew >> 2)) vr[i] = vn;
          }
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  auto consume = [&](uint4 (&kf)[8], uint4 (&vr)[8], int j) {
    const int tb = pstart + (wid + j * nw) * CHUNK;
    if (j == 0 && a.dbg_ts != nullptr) {  // profiling: the first chunk's K / V have landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ATTN_STAMP(4);
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) s0 = mfma16(as_bf16x8(kf[kk]), as_bf16x8(qf[kk]), s0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) s1 = mfma16(as_bf16x8(kf[4 + kk]), as_bf16x8(qf[kk]), s1);
    const bf16x8 pb = softmax_step(s0, s1, m, l, o, tb, pend, cscale, lane);
    // rows past the context hold finite cache contents (the pool is zero-initialised)
    // and meet p = 0: stored unmasked
    store_v_lds(vl, vr, lane, CHUNK);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pv_update(o, vl, pb, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  if constexpr (FUSED) {
    // every wave's first chunk in flight, then the granule poll (the first issue is repeated in each
    // branch: hoisted above them it costs the ping-pong loop a spill)
    if (myn == 1) {
      uint4 ka[8], va[8];
      issue(ka, va, 0);
      poll(true, wid == cnew, ka, va);
      consume(ka, va, 0);
    } else if (myn == 2) {
      // both chunks in flight before the poll (contexts up to 64 * nw tokens)
      uint4 ka[8], va[8], kb[8], vb[8];
      issue(ka, va, 0);
      issue(kb, vb, 1);
      if (wid + nw == cnew) poll(true, true, kb, vb);
      else poll(true, wid == cnew, ka, va);
      consume(ka, va, 0);
      consume(kb, vb, 1);
    } else if (myn > 2) {
      // the new token sits in the context's last chunk: a wave that owns it runs its other chunks
      // through the ping-pong loop and that one after it (the patch's registers stay out of the loop)
      const bool last_new = wid + (myn - 1) * nw == cnew;
      const int ml = last_new ? myn - 1 : myn;
      uint4 ka[8], va[8], kb[8], vb[8];
      issue(ka, va, 0);
      poll(true, false, ka, va);
      for (int j = 0; j < ml; j += 2) {
        issue(kb, vb, min(j + 1, ml - 1));
        consume(ka, va, j);
        issue(ka, va, min(j + 2, ml - 1));
        if (j + 1 < ml) consume(kb, vb, j + 1);
      }
      if (last_new) {
        issue(ka, va, myn - 1);
        poll(false, true, ka, va);
        consume(ka, va, myn - 1);
      }
    }
  } else if (myn == 1) {
    // one chunk (every wave of a context <= 32 * nw): a single load round, no look-ahead. The
    // ping-pong below would re-read the chunk twice more (clamped look-ahead issues), tripling
    // the KV bytes the block's CU moves (first K/V landed 2.5 -> 1.9 us at ctx 128 with the
    // re-reads cut, benchmarks/attn_phases.py)
    uint4 ka[8], va[8];
    issue(ka, va, 0);
    consume(ka, va, 0);
  } else if (myn > 1) {
    // Loads are issued UNCONDITIONALLY (an index past the end re-reads the last chunk):
    // straight-line issue lets the compiler keep partial vmcnt waits across the back-edge.
    uint4 ka[8], va[8], kb[8], vb[8];
    issue(ka, va, 0);
    for (int j = 0; j < myn; j += 2) {
      issue(kb, vb, min(j + 1, myn - 1));
      consume(ka, va, j);
      issue(ka, va, min(j + 2, myn - 1));
      if (j + 1 < myn) consume(kb, vb, j + 1);
    }
  }
  if (myn > 0) {
    l += xor16(l);
    l += xor32(l);
  }
  ATTN_STAMP(2);
  // ---- merge the waves through LDS: o partial [w][col][d] fp32 over the wave's V image
  float* opart = reinterpret_cast<float*>(smem);
  float* mlp = reinterpret_cast<float*>(smem + dec_ml_off(nw));
  int* flag = reinterpret_cast<int*>(mlp + nw * 32);
  {
    float* ow = opart + wid * (16 * D_);
    const int g = lane >> 4;
    // 16-B chunk k of query column c lives at chunk k ^ c of its row: the 16 columns of one
    // store (same k) land in 16 different bank groups (unswizzled, every column's row starts
    // on the same bank: a 16-way conflict, profiles/r1_pmc_sq.txt)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) *reinterpret_cast<f32x4*>(ow + col * D_ + 4 * ((4 * mt + g) ^ col)) = o[mt];
    if (lane < 16) {
      mlp[(wid * 16 + lane) * 2] = m;
      mlp[(wid * 16 + lane) * 2 + 1] = l;
    }
  }
  __syncthreads();
  ATTN_STAMP(5);
  if constexpr (FUSED) {
    // every wave has consumed its granules: clear them (zeros) for the next launch — the new K / V
    // rows here (the block of the last partition), the query here when there is one partition, else
    // by the partitions' last arriver below
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    float* gb = reinterpret_cast<float*>(qs->gran);
    if (cnew >= 0 && threadIdx.x < 64) {
      const uint32_t t = threadIdx.x;
      const uint32_t pr = t < 32 ? row0 + (uint32_t)((a.Hq + h) * D_ / 2) + 2 * t
                                 : row0 + (uint32_t)((a.Hq + a.Hkv + h) * D_ / 2) + 2 * (t - 32);
      st_sc1_x4(gb, pr * 8u, z);
    }
    if (nparts == 1) {
      for (int i = threadIdx.x; i < G * 32; i += blockDim.x)
        st_sc1_x4(gb, (row0 + (uint32_t)(h * G * D_ / 2) + 2u * (uint32_t)i) * 8u, z);
    }
  }
  // one thread per (query column, 8 d): rescale and sum the waves' partials. Unrolled over the
  // (<= 8) waves with every LDS read issued before the arithmetic: the loop with a per-wave
  // `continue` serialised ~12 dependent LDS round trips (merge + store 1.1 us of a 4.6 us block
  // at ctx 64, benchmarks/attn_phases.py). Fixed wave order: bit-reproducible.
  const int items = G * 16;
  float M = -INFINITY, L = 0.f;
  float acc[8];
  const int it = threadIdx.x;
  const int icol = it >> 4, d0 = (it & 15) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  // only the waves that had chunks carry partials (the others: l = 0, weight 0): a context of <= 4
  // chunks merges 4 slots, not the block's 8 — the same sum, half the LDS reads and exponentials
  const int nwa = min(nw, nch);
  auto merge = [&](auto wc) {
    constexpr int WP = decltype(wc)::value;  // slots per pass (<= 8), mw slots = 16 / (8 / WP)
    constexpr int MWN = WP == 8 ? 16 : WP;
    float mw[MWN];
#pragma unroll
    for (int w = 0; w < MWN; ++w) mw[w] = mlp[((w < nwa ? w : 0) * 16 + icol) * 2];
#pragma unroll
    for (int w = 0; w < MWN; ++w)
      if (w < nwa) M = fmaxf(M, mw[w]);
    const float Mref = M == -INFINITY ? 0.f : M;
    for (int base = 0; base < nwa; base += WP) {  // <= 2 passes (G <= 16)
      float lw[WP];
      f32x4 v0[WP], v1[WP];
#pragma unroll
      for (int i = 0; i < WP; ++i) {
        const int ww = base + i < nwa ? base + i : base;  // clamped: surplus slots weighted 0 below
        lw[i] = mlp[(ww * 16 + icol) * 2 + 1];
        const float* row = opart + ww * (16 * D_) + icol * D_;
        v0[i] = *reinterpret_cast<const f32x4*>(row + 4 * ((d0 >> 2) ^ icol));
        v1[i] = *reinterpret_cast<const f32x4*>(row + 4 * (((d0 >> 2) + 1) ^ icol));
      }
#pragma unroll
      for (int i = 0; i < WP; ++i) {
        const int w = base + i;
        // a wave without tokens has l = 0 and m = -inf: weight exactly 0 (no 0 * inf)
        float mv = mw[0];
#pragma unroll
        for (int k = 1; k < MWN; ++k)
          if (k == w) mv = mw[k];
        const float e = (w < nwa && lw[i] > 0.f) ? __builtin_amdgcn_exp2f(mv - Mref) : 0.f;
        L += lw[i] * e;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] += e * v0[i][j];
          acc[4 + j] += e * v1[i][j];
        }
      }
    }
  };
  if (it < items) {
    if (nwa <= 4) merge(std::integral_constant<int, 4>{});
    else merge(std::integral_constant<int, 8>{});
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int hq = h * G + icol;
  if (nparts == 1) {
    if (it < items) {
      uint4 pk;
      pk.x = pack_bf2(acc[0] * inv, acc[1] * inv);
      pk.y = pack_bf2(acc[2] * inv, acc[3] * inv);
      pk.z = pack_bf2(acc[4] * inv, acc[5] * inv);
      pk.w = pack_bf2(acc[6] * inv, acc[7] * inv);
      out_store16<SC1>(a.out, (size_t)qbeg * a.out_stride + (size_t)hq * D_ + d0, pk);
    }
    ATTN_STAMP(3);
    return;
  }
  // partial (normalised o, running max M, sum L) by device-coherent stores
  if (it < items) {
    float* po = a.part_o + (((size_t)s * a.Hq + hq) * a.num_parts + part) * D_ + d0;
    st_sc1_f4(po, acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
    st_sc1_f4(po + 4, acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
    if ((it & 15) == 0) {
      float* pm = a.part_ml + (((size_t)s * a.Hq + hq) * a.num_parts + part) * 2;
      st_sc1(pm, M);
      st_sc1(pm + 1, L);
    }
  }
  if (a.tickets == nullptr) return;  // separate reduce launch
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* t = a.tickets + (size_t)s * a.Hkv + h;
    const uint32_t old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (uint32_t)(nparts - 1);
    if (last) __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  if constexpr (FUSED) {  // every partition has read the query granules
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < G * 32; i += blockDim.x)
      st_sc1_x4(reinterpret_cast<float*>(qs->gran), (row0 + (uint32_t)(h * G * D_ / 2) + 2u * (uint32_t)i) * 8u, z);
  }
  // last arriver: merge the nparts partials of the G heads (one thread per (head, 4 d))
  for (int idx = threadIdx.x; idx < G * (D_ / 4); idx += blockDim.x) {
    const int hh = h * G + idx / (D_ / 4);
    const int dd = (idx % (D_ / 4)) * 4;
    const float* pm = a.part_ml + ((size_t)s * a.Hq + hh) * a.num_parts * 2;
    const float* po = a.part_o + ((size_t)s * a.Hq + hh) * a.num_parts * D_ + dd;
    float MM = -INFINITY;
    for (int p = 0; p < nparts; ++p) MM = fmaxf(MM, ld_sc1(pm + 2 * p));
    float LL = 0.f, r[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < nparts; ++p) {
      const float w = ld_sc1(pm + 2 * p + 1) * exp2f(ld_sc1(pm + 2 * p) - MM);
      const f32x4 v = ld_sc1_f4(po + (size_t)p * D_);
      LL += w;
      r[0] += w * v[0]; r[1] += w * v[1]; r[2] += w * v[2]; r[3] += w * v[3];
    }
    const float iv = LL > 0.f ? 1.f / LL : 0.f;
    uint2 pk;
    pk.x = pack_bf2(r[0] * iv, r[1] * iv);
    pk.y = pack_bf2(r[2] * iv, r[3] * iv);
    out_store8<SC1>(a.out, (size_t)qbeg * a.out_stride + (size_t)hh * D_ + dd, pk);
  }
}

// Host side of the fused QKV projection + decode attention launch (qkv_attn.hip, gemm_kx.h): the
// attention blocks' arguments and the launch's LDS for gx x slices GEMM blocks of `waves` waves;
// false when the step or shape is not one it takes (the caller launches the two kernels).
static inline bool qa_setup(GemmParams& p, const GemmArgs& g, int gx, int slices, int waves, size_t lds_gemm,
                            AttnArgs& a, QaSync& q, size_t& lds) {
  if (g.fa == nullptr || g.fa_gran == nullptr || g.fa_done == nullptr) return false;
  if ((size_t)g.M * (size_t)(g.N / 2) * 8 > g.fa_gran_bytes) return false;
  a = *g.fa;
  const int G = a.Hq / a.Hkv;
  // the decode block's merge: G query columns x 16 threads; partitions merged in-launch (tickets)
  if (waves < 1 || waves > 8 || G * 16 > 64 * waves || a.tickets == nullptr || a.num_tiles > 0) return false;
  if (a.S * a.num_parts * a.Hkv <= 0) return false;
  lds = std::max(lds_gemm, (size_t)attn_lds_bytes(waves));
  if (lds > 160 * 1024) return false;
  q = QaSync{g.fa_gran, g.N / 2, gx * slices, g.fault};
  p.qa_gran = reinterpret_cast<uint4*>(g.fa_gran);
  p.vgx = gx;
  a.tl = nullptr;
  return true;
}

template <typename K>
static void qa_launch(K kern, const GemmParams& p, const AttnArgs& a, const QaSync& q, int waves, size_t lds,
                      hipStream_t st) {
  if (lds > 64 * 1024) {
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    (void)attr;
  }
  hipLaunchKernelGGL(kern, dim3(q.nprod + a.S * a.num_parts * a.Hkv), dim3(64 * waves), lds, st, p, a, q);
}

}  // namespace vgate
