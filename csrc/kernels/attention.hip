// Paged attention for gfx950: decode (split-K / flash-decoding) and varlen
// causal prefill (chunked-prefill capable: queries attend to the paged cache).
//
// KV cache layout (per layer): [num_blocks][Hkv][BS=16][D=128] bf16.
//
// Both kernels use the "swapped" product S^T = K . Q^T on v_mfma_f32_16x16x32_bf16:
//   A = K tile (lane: K[tok l&15][d 8(l>>4)+j]  -> a plain 16-B row load),
//   B = Q^T   (lane: Q[col l&15][d 8(l>>4)+j]   -> a plain 16-B row load),
//   C = S^T   (lane: S[col l&15][tok 4(l>>4)+i]) -> every softmax statistic of a
//               query column lives in ONE lane group: the row max/sum need only
//               two xor-shuffles (16, 32) and the O rescale is lane-local.
// Then O^T = V^T . P^T:
//   B = P^T: built in-register from two S^T tiles with the k-order permuted to
//            {4g..4g+3, 16+4g..16+4g+3} (g = l>>4),
//   A = V^T: read from an LDS image of the V chunk with ds_read_b64_tr_b16, whose
//            4-row x 16-col transposed gather delivers exactly that k-order.
// The LDS image of V is XOR-swizzled on 8-B chunks (chunk ^= 4*(row&7)), which
// makes the transposed reads conflict-free (cdna_hip_programming.md T10).
#include "attn_decode.h"

namespace vgate {

// Combine split-K partitions: grid (S, Hq), block 128 (one thread per d).
__global__ __launch_bounds__(128) void attn_decode_reduce_kernel(AttnArgs a) {
  TLScope tl_scope(a.tl);
  const int s = blockIdx.x, hq = blockIdx.y, d = threadIdx.x;
  const int ctx = a.context_lens[s];
  if (ctx <= 0) return;
  if (a.query_start && a.query_start[s + 1] - a.query_start[s] != 1) return;
  const int nparts = (ctx + a.part_size - 1) / a.part_size;
  if (nparts <= 1) return;
  const float* pm = a.part_ml + ((size_t)s * a.Hq + hq) * a.num_parts * 2;
  const float* po = a.part_o + ((size_t)s * a.Hq + hq) * a.num_parts * D_;
  float M = -INFINITY;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, pm[2 * p]);
  float L = 0.f, acc = 0.f;
  for (int p = 0; p < nparts; ++p) {
    const float w = pm[2 * p + 1] * exp2f(pm[2 * p] - M);
    L += w;
    acc += w * po[p * D_ + d];
  }
  const int qtok = a.query_start ? a.query_start[s + 1] - 1 : s;
  a.out[(size_t)qtok * a.out_stride + (size_t)hq * D_ + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

// --------------------------------------------------------------- prefill ----
// One block per (16-query tile, KV head); wave w < G owns query head h*G + w and
// its 16 query columns; every wave walks the same KV chunks, V is staged once per
// block into a double-buffered LDS image (one barrier per chunk).
template <bool SC1 = false>
__device__ __forceinline__ void prefill_body(const AttnArgs& a, int tile, int h, char* smem) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nthr = blockDim.x;
  const int s = a.tile_seq[tile];
  if (s < 0) return;  // padding tile of a graph bucket (uniform over the block)
  const int q0 = a.tile_q0[tile];
  const int qs = a.query_start[s];
  const int qlen = a.query_start[s + 1] - qs;
  const int ctx = a.context_lens[s];
  const int G = a.Hq / a.Hkv;
  const bool wave_ok = wid < G;
  const int hq = h * G + (wave_ok ? wid : 0);
  const int col = lane & 15;
  const int qi = q0 + col;
  const bool qok = wave_ok && qi < qlen;
  const int qpos = ctx - qlen + qi;
  const int lim = qok ? qpos + 1 : 0;
  const int kv_end = min(ctx, ctx - qlen + min(q0 + 16, qlen));

  uint4 qf[4];
  {
    const bf16_t* qp = a.q + (size_t)(qs + (qok ? qi : 0)) * a.q_stride + (size_t)hq * D_ + 8 * (lane >> 4);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      qf[kk] = qok ? *reinterpret_cast<const uint4*>(qp + 32 * kk) : make_uint4(0, 0, 0, 0);
  }
  const float cscale = a.scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) o[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16_t* vls = reinterpret_cast<bf16_t*>(smem);
  const int* bt = a.block_tables + (size_t)s * a.max_blocks;
  const size_t head_off = (size_t)h * BS_ * D_;
  const size_t blk_stride = (size_t)a.Hkv * BS_ * D_;
  const int nch = (kv_end + CHUNK - 1) / CHUNK;
  const int lane64 = threadIdx.x & 63;
  int btv = 0;  // a 64-entry window of the block table, one entry per lane (see decode_wave)
  for (int c = 0; c < nch; ++c) {
    const int tb = c * CHUNK;
    if ((c & 31) == 0) btv = bt[min(2 * c + lane64, a.max_blocks - 1)];
    const int b0 = __builtin_amdgcn_readlane(btv, (2 * c) & 63);
    const int b1 = (tb + BS_ < kv_end) ? __builtin_amdgcn_readlane(btv, (2 * c + 1) & 63) : b0;
    const bf16_t* vb0 = a.v_cache + (size_t)b0 * blk_stride + head_off;
    const bf16_t* vb1 = a.v_cache + (size_t)b1 * blk_stride + head_off;
    bf16_t* vl = vls + (c & 1) * (CHUNK * D_);
    for (int e = threadIdx.x; e < CHUNK * D_ / 8; e += nthr) {
      const int r = e >> 4, cc = (e & 15) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (tb + r < kv_end) v = *reinterpret_cast<const uint4*>((r < 16 ? vb0 + r * D_ : vb1 + (r - 16) * D_) + cc);
      *reinterpret_cast<uint4*>(vl + v_lds_off(r, cc)) = v;
    }
    const bf16_t* kb0 = a.k_cache + (size_t)b0 * blk_stride + head_off;
    const bf16_t* kb1 = a.k_cache + (size_t)b1 * blk_stride + head_off;
    f32x4 s0 = qk_tile(kb0, qf, lane);
    f32x4 s1 = qk_tile(kb1, qf, lane);
    const bf16x8 pb = softmax_step(s0, s1, m, l, o, tb, min(lim, kv_end), cscale, lane);
    __syncthreads();
    pv_update(o, vl, pb, lane);
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (!qok) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  const size_t orow = (size_t)(qs + qi) * a.out_stride + (size_t)hq * D_;
  const int g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    uint2 pk;
    pk.x = pack_bf2(o[mt][0] * inv, o[mt][1] * inv);
    pk.y = pack_bf2(o[mt][2] * inv, o[mt][3] * inv);
    out_store8<SC1>(a.out, orow + 16 * mt + 4 * g, pk);
  }
}

// ------------------------------------------------------- flash prefill ----
// Causal (chunked-prefill capable) attention of a block of QPB = 16 CT QG query tokens x the G
// query heads of one KV head. NW = QG G waves: wave w owns head h G + w % G for the CT 16-query
// MFMA column tiles of query group w / G; Q lives in registers. K / V stream through LDS in
// 64-token chunks, SHARED by the block's waves (GQA: one K/V byte serves G heads x QPB queries),
// moved by LDS-DMA (global_load_lds_dwordx4: no VGPRs; every wave issues P = ceil(32 / NW) of
// the chunk's 32 1-KiB pieces, padded with repeats of its own last piece so every wave's vmcnt
// bookkeeping is the same constant). NST-stage ring: chunk c + NST - 1 is issued at the top of
// iteration c, so a chunk's DMA has NST - 1 chunks of compute to land — with two stages (one
// chunk ahead) the kernel ran at the DMA's issue-to-land latency per chunk (~3.4 us, 109 us for
// Llama-3-8B causal 2048, profiles/r3_flash_prefill.log). One barrier per chunk.
//   S^T = K Q^T (swapped: softmax statistics lane-local, row reductions by two xor-swaps); K image
//   16-B chunks XOR-swizzled by row & 15 (conflict-free ds_read_b128 of the A operand);
//   O^T += V^T P^T with V^T read by ds_read_b64_tr_b16 from the 8-B-chunk-swizzled V image and P^T
//   built in registers (pack_p), as in the decode kernel.
// Softmax per chunk: the causal mask only on chunks that cross a query's bound (the others are
// below every query of the block), the scale folded into the exp2 argument (one fma), and the
// O / l rescale only when some column's running max moved (wave-uniform test; exact: alpha = 1
// otherwise).
// The host's 16-query tile list is reused: a block whose tile starts a QPB-aligned group leads it
// (others exit at once). The host lists the group leaders first, longest causal range first
// (ops.tile_order), so the working blocks are the grid's first ones, spread over all 8 XCDs and
// the longest start first. Chunks past the causal bound are not read (the ring's look-ahead past
// the last chunk re-reads the last one into a free stage).
extern int g_flash_prefill;
constexpr int FL_KV = 64;
constexpr int FL_STAGE = 2 * FL_KV * D_ * 2;  // K + V of one chunk (32 KiB)
constexpr int FL_NST_MAX = 4;                 // ring stages (<= 128 KiB: one block per CU)

// f32 max of values known not to be NaN: one v_max / v_max3 each (fmaxf's IEEE-mode lowering
// canonicalises every MFMA-produced input first: an extra v_max x, x per value)
__device__ __forceinline__ float fmax3_(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float fmax_(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ constexpr int vm_imm(int n) {  // s_waitcnt vmcnt(n), other counters untouched
  return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8);
}

// dec_seqs > 0: the step's decode rows ride in the same launch — grid rows y >= num_tiles are
// (sequence, partition) decode blocks (part z == 0 of each KV head), so a prefill or mixed step has
// ONE attention launch (in a prefill-only step those blocks see no single-token sequence and exit)
template <int CT, int NW, int FL_NST, bool SWP>
__global__ __launch_bounds__(64 * NW) void attn_flash_kernel(AttnArgs a, int lazy, int dec_seqs) {
  constexpr int P = (32 + NW - 1) / NW;  // DMA pieces per wave per chunk
  constexpr int FL_LDS = FL_NST * FL_STAGE;
  static_assert((FL_NST - 2) * P < 64, "vmcnt immediate");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(a.tl);
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = a.Hq / a.Hkv;
  const int QG = NW / G;
  const int QPB = 16 * CT * QG;
  // grid (Hkv x halves, tiles): the KV heads (and a split range's two halves) of one tile are
  // adjacent in dispatch order, so the tile list's longest-first order holds across every head
  const int zs = gridDim.x / a.Hkv;
  const int h = blockIdx.x / zs;
  const int tile = blockIdx.y;
  if (tile >= a.num_tiles) {  // block-uniform: a decode block
    const int r = tile - a.num_tiles;
    if (blockIdx.x % zs == 0 && dec_seqs > 0) decode_block(a, r % dec_seqs, h, r / dec_seqs, smem);
    return;
  }
  const int s = a.tile_seq[tile];
  if (s < 0) return;
  const int q0 = a.tile_q0[tile];
  if (q0 % QPB) return;  // block-uniform: not a group leader
  const int qs = a.query_start[s];
  const int qlen = a.query_start[s + 1] - qs;
  // a single-query sequence is a decode row, computed by this launch's decode blocks: a tile of it
  // (a tile list that names every sequence) must not write the same output row concurrently
  if (qlen == 1 && dec_seqs > 0) return;  // block-uniform
  const int ctx = a.context_lens[s];
  const int hq = h * G + wid % G;
  const int qw0 = q0 + 16 * CT * (wid / G);  // this wave's first query
  const int qhi = min(q0 + QPB, qlen);       // the block's queries: [q0, qhi)
  const int kv_end = ctx - qlen + qhi;       // the block's causal bound (exclusive)
  const int nch = (kv_end + FL_KV - 1) / FL_KV;
  const int nfull = max(0, ctx - qlen + q0 + 1) / FL_KV;  // chunks below every query's bound
  // K split (zs parts per KV head, launch_attention): a range of nch chunks runs as nsp =
  // min(zs, nch / 2) parts of whole chunks (>= 2 each), part z on [nch z / nsp, nch (z+1) / nsp),
  // met in the epilogue; the causal triangle's long tail then costs 1 / nsp of a range per block.
  // Parts past nsp exit at once. Block-uniform, before any barrier.
  const int z = blockIdx.x % zs;
  const int nsp = SWP ? 1 : min(zs, nch / 2);
  const bool split = nsp > 1;
  if (z >= max(nsp, 1)) return;
  const int c0 = split ? nch * z / nsp : 0;
  const int c1 = split ? nch * (z + 1) / nsp : nch;
  const int col = lane & 15, g4 = lane >> 4;
  // Q fragments (B operand of S^T = K Q^T): CT column tiles x 4 k-slices
  uint4 qf[CT][4];
  int lim[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int qi = qw0 + 16 * ct + col;
    const bool ok = qi < qhi;
    lim[ct] = ok ? ctx - qlen + qi + 1 : 0;
    const bf16_t* qp = a.q + (size_t)(qs + (ok ? qi : 0)) * a.q_stride + (size_t)hq * D_ + 8 * g4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) qf[ct][kk] = ok ? *reinterpret_cast<const uint4*>(qp + 32 * kk) : make_uint4(0, 0, 0, 0);
  }
  const size_t blk_stride = (size_t)a.Hkv * BS_ * D_;
  const size_t head_off = (size_t)h * BS_ * D_;
  // the sequence's block-table entries of the causal range, staged in LDS once: a DMA's source page
  // is then an LDS broadcast read, not a global load whose wait would serialise behind the DMAs
  // already in flight (vmcnt counts both)
  int* s_bt = reinterpret_cast<int*>(smem + FL_LDS);
  const int npg = (kv_end + BS_ - 1) / BS_;
  {
    const int* bt = a.block_tables + (size_t)s * a.max_blocks;
    for (int i = threadIdx.x; i < npg; i += blockDim.x) s_bt[i] = bt[i];
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // Q fragments and the block table
  __builtin_amdgcn_s_barrier();
  // chunk c's 32 DMA pieces (16 K, 16 V) over the block's waves, into stage c % NST; past the last
  // chunk the last one is re-read (the ring keeps NST - 1 chunks in flight, a constant vmcnt).
  // Piece i of a chunk: K rows 4 i .. 4 i + 3 (i < 16; lane -> physical 16-B chunk l & 15 holds
  // logical chunk ^ (row & 15)) or V half (i - 16) / 8, rows 4 ((i - 16) % 8) .. + 3 of that half
  // (v_lds_off's 8-B chunk swizzle). Everything but the 4 pages of the chunk is chunk-invariant:
  // the lane's element offset inside its page and the piece's page slot / LDS offset are set once.
  uint32_t loff[P];  // lane's element offset inside the page
  int pslot[P], pisv[P], pdst[P];  // wave-uniform: page slot 0..3, V?, LDS byte offset in the stage
#pragma unroll
  for (int k = 0; k < P; ++k) {
    int i = wid + k * NW;
    if (i >= 32) i = wid + (k - 1) * NW;  // pad: this wave's previous piece again (same bytes, same place)
    const int isv = i >> 4, pi = i & 15;
    int r, d0;
    if (!isv) {
      r = 4 * pi + g4;
      d0 = 8 * (col ^ (r & 15));
    } else {
      const int rh = 4 * (pi & 7) + g4;
      r = 32 * (pi >> 3) + rh;
      d0 = (8 * col) ^ (16 * (rh & 7));
    }
    loff[k] = (uint32_t)((r & 15) * D_ + d0);
    pslot[k] = isv ? 2 * (pi >> 3) + ((pi & 7) >> 2) : pi >> 2;  // rows of a piece share one page
    pisv[k] = isv;
    pdst[k] = (isv ? FL_KV * D_ * 2 : 0) + pi * 1024;
  }
  auto issue = [&](int c) {
    const uint32_t stage = lds_addr_of(smem) + (uint32_t)((c % FL_NST) * FL_STAGE);
    const int cc = min(c, c1 - 1);
    int pg[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pg[j] = __builtin_amdgcn_readfirstlane(s_bt[min(4 * cc + j, npg - 1)]);  // past the bound: the last page
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int page = pslot[k] == 0 ? pg[0] : pslot[k] == 1 ? pg[1] : pslot[k] == 2 ? pg[2] : pg[3];
      const bf16_t* base = (pisv[k] ? a.v_cache : a.k_cache) + (size_t)page * blk_stride + head_off;
      glds16(base + loff[k], stage + (uint32_t)pdst[k]);
    }
  };
  const float cscale = a.scale * LOG2E;
  float m[CT], l[CT];  // running max (scaled, log2 domain) and sum per column
  f32x4 o[CT][8];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    m[ct] = -INFINITY;
    l[ct] = 0.f;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) o[ct][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int q = (lane >> 2) & 3, p4 = lane & 3;
  // S^T tiles of chunk c: 4 token tiles x CT column tiles (K from stage c % NST)
  auto qk = [&](int c, f32x4 (&st)[4][CT]) {
    const char* kb = smem + (c % FL_NST) * FL_STAGE;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) st[tt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* krow = kb + (16 * tt + col) * 256;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const uint4 kf = *reinterpret_cast<const uint4*>(krow + (((4 * kk + g4) ^ col) << 4));
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) st[tt][ct] = mfma16(as_bf16x8(kf), as_bf16x8(qf[ct][kk]), st[tt][ct]);
      }
    }
  };
  // online softmax of chunk c per column tile over its 64 tokens (lane: column col, tokens
  // 16 tt + 4 g4 + i) -> P^T fragments. SWP: branch-free (mask by select, rescale every chunk),
  // so the next chunk's QK MFMAs issued before it interleave with this VALU in one basic block
  auto softmax = [&](int c, f32x4 (&st)[4][CT], bf16x8 (&pb)[CT][2]) {
    const bool masked = c >= nfull;  // block-uniform
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      if (SWP || masked) {
        // token t = c 64 + 16 tt + 4 g4 + i is masked when t >= lim: i.e. 16 tt + i >= lim - c 64 - 4 g4
        const int rel = (SWP && !masked ? 0x3fffffff : lim[ct]) - c * FL_KV - 4 * g4;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (16 * tt + i >= rel) st[tt][ct][i] = -INFINITY;
      }
      // max without NaN canonicalisation (the scores are finite or -inf): v_max3 chains
      float cmax = -INFINITY;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
        cmax = fmax3_(cmax, fmax3_(st[tt][ct][0], st[tt][ct][1], st[tt][ct][2]), st[tt][ct][3]);
      cmax = fmax_(cmax, xor16(cmax));
      cmax = fmax_(cmax, xor32(cmax));
      const float mn = fmaxf(m[ct], cmax * cscale);
      if (SWP || !lazy || __any(mn > m[ct])) {  // wave-uniform: rescale only when a running max moved
        const float alpha = __builtin_amdgcn_exp2f(m[ct] - (mn == -INFINITY ? 0.f : mn));
        l[ct] *= alpha;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) o[ct][mt] *= alpha;
        m[ct] = mn;
      }
      const float mref = m[ct] == -INFINITY ? 0.f : m[ct];  // fully masked column: exp2(-inf) = 0, no NaN
      float ps = 0.f;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          st[tt][ct][i] = __builtin_amdgcn_exp2f(fmaf(st[tt][ct][i], cscale, -mref));
          ps += st[tt][ct][i];
        }
      l[ct] += ps;
      pb[ct][0] = pack_p(st[0][ct], st[1][ct]);
      pb[ct][1] = pack_p(st[2][ct], st[3][ct]);
    }
  };
  // O^T += V^T P^T of chunk c: each V^T fragment (ds_read_b64_tr_b16) feeds every column tile
  auto pv = [&](int c, const bf16x8 (&pb)[CT][2]) {
    const bf16_t* vb = reinterpret_cast<const bf16_t*>(smem + (c % FL_NST) * FL_STAGE + FL_KV * D_ * 2);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const bf16_t* vh = vb + half * (32 * D_);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int cc = 16 * mt + 4 * p4;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vh + v_lds_off(4 * g4 + q, cc)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vh + v_lds_off(16 + 4 * g4 + q, cc)));
        bf16x8 av;
        av[0] = lo[0]; av[1] = lo[1]; av[2] = lo[2]; av[3] = lo[3];
        av[4] = hi[0]; av[5] = hi[1]; av[6] = hi[2]; av[7] = hi[3];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) o[ct][mt] = mfma16(av, pb[ct][half], o[ct][mt]);
      }
    }
  };
  if constexpr (!SWP) {
    if (c1 > c0) {
#pragma unroll
      for (int c = 0; c < FL_NST - 1; ++c) issue(c0 + c);
    }
    __builtin_amdgcn_s_waitcnt(vm_imm((FL_NST - 2) * P));  // chunk c0 landed (this wave's pieces)
    __builtin_amdgcn_s_barrier();                          // everyone's
    for (int c = c0; c < c1; ++c) {
      issue(c + FL_NST - 1);  // into the stage every wave finished reading last iteration
      f32x4 st[4][CT];
      bf16x8 pb[CT][2];
      qk(c, st);
      softmax(c, st, pb);
      pv(c, pb);
      __builtin_amdgcn_s_waitcnt(vm_imm((FL_NST - 2) * P));  // this wave's pieces of chunk c + 1 landed
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // everyone's; stage c % NST free
    }
  } else {
    // software-pipelined: iteration c computes S of chunk c + 1 (MFMA) beside the softmax of chunk c
    // (VALU), then P V of chunk c. Live stages: c (V), c + 1 (K), c + 2 (landing), c + 3 (issued)
    static_assert(FL_NST >= 4, "the pipelined loop keeps four chunks resident");
    if (nch > 0) {
#pragma unroll
      for (int c = 0; c < FL_NST - 1; ++c) issue(c);
    }
    __builtin_amdgcn_s_waitcnt(vm_imm((FL_NST - 3) * P));  // chunks 0 and 1 landed (this wave's pieces)
    __builtin_amdgcn_s_barrier();                          // everyone's
    f32x4 sc[4][CT];
    if (nch > 0) qk(0, sc);
    for (int c = 0; c < nch; ++c) {
      issue(c + FL_NST - 1);  // into stage (c - 1) % NST: every wave finished its P V in iteration c - 1
      f32x4 sn[4][CT];
      bf16x8 pb[CT][2];
      qk(c + 1, sn);  // past the last chunk: the re-read last chunk, discarded
      softmax(c, sc, pb);
      pv(c, pb);
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) sc[tt][ct] = sn[tt][ct];
      __builtin_amdgcn_s_waitcnt(vm_imm((FL_NST - 3) * P));  // this wave's pieces of chunk c + 2 landed
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // everyone's; stage c % NST free
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the look-ahead DMAs drained before the block exits
  if (split) {
    // The parts meet per wave. Each rounds its partial to bf16 normalised by its own sum (o / l),
    // (m, l) in fp32, and takes the wave's ticket first: the nsp - 1 early arrivers publish
    // (16-B sc1 stores, drain, +1 on the ready word) and exit; the last waits for ready = nsp - 1
    // (the others never wait, so they always get there), re-arms both words and merges every
    // part's ROUNDED partial in fixed part order: the result does not depend on arrival order.
    // Slot: the leader's rank over the step (every earlier sequence holds ceil(qlen / QPB)
    // leaders), KV head, wave; the host sized fl_ws for (tiles 16 / QPB + S + 1) Hkv NW <= 32768
    // slots of zs parts.
    int before = 0;
    for (int i = lane; i < s; i += 64) {
      const int ql = a.query_start[i + 1] - a.query_start[i];
      before += (ql + QPB - 1) / QPB;
    }
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) before += __shfl_xor(before, sh);
    const uint32_t wslot = (uint32_t)(((before + q0 / QPB) * a.Hkv + h) * NW + wid);
    uint32_t* ticket = a.fl_tickets + wslot;
    uint32_t* ready = a.fl_tickets + 32768 + wslot;
    float ll[CT];
    uint4 pw[CT][4];  // this part's o / l, bf16, mt pairs
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      ll[ct] = l[ct];
      ll[ct] += xor16(ll[ct]);
      ll[ct] += xor32(ll[ct]);
      const float inv = ll[ct] > 0.f ? 1.f / ll[ct] : 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const f32x4 x0 = o[ct][2 * w], x1 = o[ct][2 * w + 1];
        pw[ct][w] = make_uint4(pack_bf2(x0[0] * inv, x0[1] * inv), pack_bf2(x0[2] * inv, x0[3] * inv),
                               pack_bf2(x1[0] * inv, x1[1] * inv), pack_bf2(x1[2] * inv, x1[3] * inv));
      }
    }
    constexpr uint32_t PW = CT * 4 + 1;  // 16-B words per lane and part: the bf16 partial, then (m, l) pairs
    const uint32_t lane_off = lane * 16u;
    auto part_off = [&](int p) { return (wslot * (uint32_t)zs + (uint32_t)p) * PW * 1024u + lane_off; };
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0);
    if (old + 1 < (uint32_t)nsp) {
      const uint32_t off = part_off(z);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int w = 0; w < 4; ++w)
          st_sc1_x4(a.fl_ws, off + (uint32_t)(ct * 4 + w) * 1024u, __builtin_bit_cast(f32x4, pw[ct][w]));
      st_sc1_x4(a.fl_ws, off + CT * 4 * 1024u, f32x4{m[0], ll[0], m[CT - 1], ll[CT - 1]});
      drain_stores();
      if (lane == 0) __hip_atomic_fetch_add(ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (lane == 0) {
      uint32_t spins = 0;
      bool late = false;
      while (__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 < (uint32_t)nsp) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { late = true; break; }  // bounded: never hang the GPU
      }
      if (late) {
        // the result is wrong and a late part may still add to `ready`: leave the words as they are and
        // raise the sticky fault word, which the step's last node hands to the host (engine fails)
        if (a.fault != nullptr) atomicOr(a.fault, 2u);
      } else {
        __hip_atomic_store(ready, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("" ::: "memory");  // the partials' loads stay behind the flag
    // every part's (m, l) -> weights, then the partials in part order
    f32x4 ml[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
      ml[p] = (p < nsp && p != z) ? ld_sc1_x4(a.fl_ws, part_off(p) + CT * 4 * 1024u)
                                  : f32x4{m[0], ll[0], m[CT - 1], ll[CT - 1]};
    auto lo_f = [](uint32_t u) { return __uint_as_float(u << 16); };
    auto hi_f = [](uint32_t u) { return __uint_as_float(u & 0xffff0000u); };
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      float mm = -INFINITY;
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (p < nsp) mm = fmaxf(mm, ml[p][2 * ct]);
      const float mref = mm == -INFINITY ? 0.f : mm;
      float wt[4], lt = 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        wt[p] = p < nsp ? __builtin_amdgcn_exp2f(ml[p][2 * ct] - mref) * ml[p][2 * ct + 1] : 0.f;
        lt += wt[p];
      }
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      float acc[32];
#pragma unroll
      for (int e = 0; e < 32; ++e) acc[e] = 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (p >= nsp) continue;
        uint4 q4[4];
#pragma unroll
        for (int w = 0; w < 4; ++w)
          q4[w] = p == z ? pw[ct][w] : __builtin_bit_cast(uint4, ld_sc1_x4(a.fl_ws, part_off(p) + (uint32_t)(ct * 4 + w) * 1024u));
        const float wp = wt[p] * inv;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const uint32_t u[4] = {q4[w].x, q4[w].y, q4[w].z, q4[w].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[8 * w + 2 * k] += lo_f(u[k]) * wp;
            acc[8 * w + 2 * k + 1] += hi_f(u[k]) * wp;
          }
        }
      }
      const int qi = qw0 + 16 * ct + col;
      if (qi >= qhi) continue;
      const size_t orow = (size_t)(qs + qi) * a.out_stride + (size_t)hq * D_;
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        uint2 pk;
        pk.x = pack_bf2(acc[4 * mt], acc[4 * mt + 1]);
        pk.y = pack_bf2(acc[4 * mt + 2], acc[4 * mt + 3]);
        *reinterpret_cast<uint2*>(a.out + orow + 16 * mt + 4 * g4) = pk;
      }
    }
    return;
  }
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    float ll = l[ct];
    ll += xor16(ll);
    ll += xor32(ll);
    const int qi = qw0 + 16 * ct + col;
    if (qi >= qhi) continue;
    const float inv = ll > 0.f ? 1.f / ll : 0.f;
    const size_t orow = (size_t)(qs + qi) * a.out_stride + (size_t)hq * D_;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      uint2 pk;
      pk.x = pack_bf2(o[ct][mt][0] * inv, o[ct][mt][1] * inv);
      pk.y = pack_bf2(o[ct][mt][2] * inv, o[ct][mt][3] * inv);
      *reinterpret_cast<uint2*>(a.out + orow + 16 * mt + 4 * g4) = pk;
    }
  }
}

// flash configuration for a head group of G (ct = 0: not supported): waves NW = 8 when G | 8
// (G query groups of 8 / G), 6 for G = 3, 6; two 16-query column tiles per wave for G <= 4
// (Llama: 64-query blocks), one above (16-query blocks keep >= one block per CU at 2k tokens for
// the 1-2 KV-head layouts; two there were slower at every length, profiles/r3_flash_split.log)
struct FlashCfg { int ct, nw; };
static FlashCfg flash_cfg(const AttnArgs& a) {
  if (a.D != D_ || a.BS != BS_ || a.Hkv <= 0 || a.Hq % a.Hkv) return {0, 0};
  const int G = a.Hq / a.Hkv;
  const int nw = 8 % G == 0 ? 8 : (6 % G == 0 ? 6 : 0);
  if (nw == 0) return {0, 0};
  const int ct = G <= 4 ? 2 : 1;
  return {ct, nw};
}

static bool flash_enabled() {
  static const int v = [] { const char* e = getenv("VGATE_FLASH_PREFILL"); return e ? atoi(e) : 1; }();
  return g_flash_prefill >= 0 ? g_flash_prefill != 0 : v != 0;
}

// ------------------------------------------------------------- unified launch ----
// grid.x = [decode blocks: one per (sequence, partition), partition-major: bx = p*S + s]
//          ++ [prefill tiles], grid.y = KV heads. One launch serves a decode-only,
// prefill-only or mixed (chunked-prefill) step; waves / blocks without work exit.
// MAXT: 512 threads (G <= 8 query heads per KV head) leaves 256 VGPRs per wave for the
// prefetched K + in-flight V + O accumulators; 1024 only for G > 8.
template <int MAXT>
__global__ __launch_bounds__(MAXT) void attn_kernel(AttnArgs a, int dec_seqs, int dec_blocks) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TLScope tl_scope(a.tl);
  const int bx = blockIdx.x;
  if (bx < dec_blocks) {
    decode_block(a, bx % dec_seqs, blockIdx.y, bx / dec_seqs, smem);  // block = (sequence, partition)
  } else {
    // (a tile of a single-query sequence: that row is a decode block's, see attn_flash_kernel)
    const int s = a.tile_seq[bx - dec_blocks];
    if (dec_seqs > 0 && s >= 0 && a.query_start[s + 1] - a.query_start[s] == 1) return;
    prefill_body(a, bx - dec_blocks, blockIdx.y, smem);
  }
}

static int attn_waves(const AttnArgs& a) {
  const int G = a.Hq / a.Hkv;
  return G > 4 ? G : 4;
}

int g_flash_prefill = -1;  // -1: VGATE_FLASH_PREFILL (default on); 0 / 1: set_flash_prefill (tests)
void set_flash_prefill(int on) { g_flash_prefill = on; }

static int cu_count();

void launch_attention(const AttnArgs& a, int dec_seqs, hipStream_t st) {
  int tiles = a.num_tiles > 0 ? a.num_tiles : 0;
  // prefill tiles on the flash kernel (its own launch; a decode-only graph bucket carries no tile
  // list, StepMeta.view), the unified kernel keeps the decode rows
  const FlashCfg fc = tiles > 0 && flash_enabled() ? flash_cfg(a) : FlashCfg{0, 0};
  if (fc.ct > 0) {
    AttnArgs f = a;
    f.num_tiles = tiles;
    // the decode rows join this launch (grid rows past the tiles): no second attention launch
    const int dec_rows = dec_seqs > 0 ? dec_seqs * a.num_parts : 0;
    // a 2-stage K/V ring with the lazy rescale (4 stages and eager rescale measured no faster:
    // profiles/r3_flash_split.log)
    constexpr int lazy = 1;
    const size_t lds = (size_t)2 * FL_STAGE + (size_t)a.max_blocks * 4;
    // K split of the long causal ranges (zs parts per KV head, adjacent in grid.x) when the
    // workspace holds every wave's partials: 2 parts while the step's working blocks fill less
    // than two waves of the chip's block slots (CT = 2 blocks hold a CU alone, CT = 1 two), 4
    // while 4 parts per block still fit in one wave (profiles/r3_flash_split.log: 4 parts won
    // only there: Llama-3-70B TP=8 2048 39.8 -> 31.9 us, lost at Qwen 2048 46 -> 50, Llama-8B
    // 1024 35 -> 45); none once the blocks alone fill two waves (they balance the triangle)
    int zs = 1;
    if (f.fl_ws != nullptr && f.fl_tickets != nullptr) {
      const int qpb = 16 * fc.ct * (fc.nw / (a.Hq / a.Hkv));
      const size_t leaders = (size_t)tiles * 16 / qpb + (size_t)a.S + 1;
      const size_t slots = leaders * a.Hkv * fc.nw;
      const size_t blocks = (size_t)tiles * 16 / qpb * a.Hkv;
      const size_t cap = (size_t)cu_count() * (fc.ct == 2 ? 1 : 2);
      if (blocks < 2 * cap) zs = 2;
      if (blocks * 4 <= cap) zs = 4;
      if (slots > 32768 || slots * zs * (fc.ct * 4 + 1) * 1024 > f.fl_ws_bytes) zs = 1;
    }
    const dim3 grid(a.Hkv * zs, tiles + dec_rows, 1), block(64 * fc.nw);
    f.tl = tl_take("attn_flash", (tiles + dec_rows) * a.Hkv * zs);
    const size_t lds_all = std::max(lds, (size_t)attn_lds_bytes(fc.nw));
#define VG_FL(CT_, NW_) hipLaunchKernelGGL((attn_flash_kernel<CT_, NW_, 2, false>), grid, block, lds_all, st, f, lazy, dec_seqs)
    if (fc.nw == 8) {
      if (fc.ct == 2) VG_FL(2, 8); else VG_FL(1, 8);
    } else {
      if (fc.ct == 2) VG_FL(2, 6); else VG_FL(1, 6);
    }
#undef VG_FL
    if (dec_seqs > 0 && a.num_parts > 1 && a.tickets == nullptr) {
      AttnArgs b = a;
      b.tl = tl_take("attn_reduce", dec_seqs * a.Hq);
      hipLaunchKernelGGL(attn_decode_reduce_kernel, dim3(dec_seqs, a.Hq), dim3(128), 0, st, b);
    }
    return;
  }
  const int nw = attn_waves(a);
  const int dec_blocks = dec_seqs > 0 ? dec_seqs * a.num_parts : 0;
  const int nx = dec_blocks + tiles;
  if (nx <= 0) return;
  AttnArgs b = a;
  b.num_tiles = tiles;
  b.tl = tl_take("attention", nx * a.Hkv);
  if (nw <= 8)
    hipLaunchKernelGGL(attn_kernel<512>, dim3(nx, a.Hkv, 1), dim3(64 * nw), attn_lds_bytes(nw), st, b, dec_seqs, dec_blocks);
  else
    hipLaunchKernelGGL(attn_kernel<1024>, dim3(nx, a.Hkv, 1), dim3(64 * nw), attn_lds_bytes(nw), st, b, dec_seqs, dec_blocks);
  if (dec_seqs > 0 && a.num_parts > 1 && a.tickets == nullptr) {
    b.tl = tl_take("attn_reduce", dec_seqs * a.Hq);
    hipLaunchKernelGGL(attn_decode_reduce_kernel, dim3(dec_seqs, a.Hq), dim3(128), 0, st, b);
  }
}

static int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 1;
  }();
  return n;
}

void launch_attn_decode(const AttnArgs& a, hipStream_t st) {
  AttnArgs b = a;
  b.num_tiles = 0;
  launch_attention(b, a.S, st);
}

void launch_attn_prefill(const AttnArgs& a, hipStream_t st) {
  launch_attention(a, 0, st);
}

}  // namespace vgate
