// Weight-streaming MFMA GEMMs for the decode / small-M regime on gfx950, with the
// transformer's neighbouring ops fused in so a decoder layer is 4 GEMM launches.
//
//   out[m][n] = epilogue( sum_k prologue(x)[m][k] * W[n][k] )
//
// Weights are pre-packed ONCE at load time into "fragment-major" order so that
// one wave-instruction of 16 B/lane reads 1 KiB of contiguous HBM that is
// exactly the A operand of v_mfma_f32_16x16x32_bf16:
//
//   Wp[nt][kt][lane][j] = W[16*nt + (lane & 15)][32*kt + 8*(lane >> 4) + j]
//
// No LDS staging of weights: in the M <= 64 regime each weight byte is used by one
// wave only, so the bytes go straight to VGPRs with non-temporal loads
// (cdna_hip_programming.md §5 'GEMV / M <= 16 decode weights').
//
// Decomposition: grid = (n-tile groups, m-chunks of 16*MB rows, SPLITK k-slices).
// Inside a block, W waves split the block's k-slice into contiguous ranges and
// their accumulators are reduced through LDS. With SPLITK > 1 every block writes
// an fp32 partial slab and the LAST-ARRIVING block of the tile (sc1 slab stores ->
// drain -> ticket atomic; sc1 slab loads: no L2-wide release/acquire fences, see
// common.h) sums the slabs and runs the epilogue — no second launch, and the
// small-N projections (o_proj / down_proj: 96 tiles) still fill all 256 CUs.
//
// Fusions:
//   NORM          : RMSNorm folded into the GEMM with a DEFERRED row scale:
//                   out = rsqrt(mean(x^2) + eps) * (bf16(x * w) @ W^T). The sum of squares
//                   is accumulated from the same x fragments the MFMA loop already loads
//                   (no prologue pass, no serial latency before the weight stream) and
//                   applied per row in the epilogue (RMSNorm never runs as a kernel);
//   row_idx       : rows gathered by index (LM head reads only sampled rows);
//   epilogues     : +bias, +residual (in place), SiLU(gate)*up,
//                   f32 logits, and QKV: bias + NeoX RoPE + paged KV-cache write
//                   (one 16-column tile holds 8 rotation pairs / 8 gate-up pairs; the
//                   partners sit on lanes l, l ^ 32, see gemm_epilogue.h).
//
// Orientation: D = Wfrag(A) x xfrag(B) -> lane holds D[n = 4(l>>4)+i][m = l&15]:
// 4 consecutive output columns of one row -> 8-byte stores.
//
// AWQ W4A16 variant: int4 weights in the same fragment order, 4 k-tiles per 16-B
// lane load ([nt][kt/4][lane][4] uint32, nibble j = element j), group-wise
// (scale, scale*zero) applied in registers before the bf16 MFMA.
// The kernel templates and their launch logic live in gemm_decode.h; each epilogue's
// instantiations are compiled in gemm_epi_{bf16,f32,silu,qkv}.hip.
#include "gemm_decode.h"

namespace vgate {

int g_dec_u = -100;  // -100: the launcher's rule; else the forced decode register group size (tests)
void set_dec_u(int u) { g_dec_u = u; }

VG_EXTERN_EPI(EPI_BF16)
VG_EXTERN_EPI(EPI_F32)
VG_EXTERN_EPI(EPI_SILU)
VG_EXTERN_EPI(EPI_QKV)
VG_EXTERN_EPI(EPI_BF16_AR)

// ---- AWQ prefill operand: int4 fragments -> bf16 fragments (same fragment order) ----
// Long AWQ steps run the LDS-tiled bf16 prefill kernel (gemm_prefill.hip) on a per-call scratch
// copy of ONE matrix, dequantised here in the packed layout the kernel reads: lane l's k-step
// fragment of tile nt is element-wise (v - z) * s [* gamma_k] of the int4 fragment that the decode
// kernels feed to the MFMA as raw8. Folding the RMSNorm gamma in here turns the gamma-in-registers
// prologue (which the prefill kernel does not take) into the row-scale-only mode. No bf16 copy of
// the model is kept: the scratch is the largest single matrix (gate_up: 55 MB for Qwen2.5-1.5B).
// One thread per (tile, k-quad, lane): 16 B int4 in, 4 x 16 B bf16 out.
__global__ __launch_bounds__(256) void awq_dequant_packed_kernel(const uint4* __restrict__ wq,
                                                                 const bf16_t* __restrict__ scales,
                                                                 const bf16_t* __restrict__ sz,
                                                                 const bf16_t* __restrict__ gamma, uint4* __restrict__ out,
                                                                 int N, int K, int group) {
  const int KQ = K >> 7;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // ((nt * KQ) + kq) * 64 + lane
  if (idx >= (size_t)(N >> 4) * KQ * 64) return;
  const int lane = (int)(idx & 63);
  const size_t tq = idx >> 6;
  const int kq = (int)(tq % KQ), nt = (int)(tq / KQ);
  const int n = nt * 16 + (lane & 15);
  const uint4 q = wq[idx];
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k0 = (kq * 4 + u) * 32 + 8 * (lane >> 4);
    const int g = k0 / group;
    const float s = bf2f(scales[(size_t)g * N + n]), zs = bf2f(sz[(size_t)g * N + n]);
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)((qw[u] >> ((j & 1) * 16 + 4 * (j >> 1))) & 0xF) * s - zs;
    if (gamma != nullptr) {
      float g8[8];
      unpack8(*reinterpret_cast<const uint4*>(gamma + k0), g8);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= g8[j];
    }
    out[(((size_t)nt * (K >> 5)) + kq * 4 + u) * 64 + lane] = pack8(f);
  }
}

void launch_awq_dequant(const void* wq, const uint16_t* scales, const uint16_t* sz, const uint16_t* gamma,
                        void* out, int N, int K, int group, hipStream_t st) {
  const size_t n = (size_t)(N / 16) * (K / 128) * 64;
  hipLaunchKernelGGL(awq_dequant_packed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint4*>(wq), reinterpret_cast<const bf16_t*>(scales),
                     reinterpret_cast<const bf16_t*>(sz), reinterpret_cast<const bf16_t*>(gamma),
                     reinterpret_cast<uint4*>(out), N, K, group);
}

template <bool AWQ>
static void launch_dispatch(GemmParams p, const GemmArgs& g, hipStream_t st) {
  switch (g.epi) {
    case EPI_SILU: dispatch_epi<EPI_SILU, AWQ>(p, g, st); break;
    case EPI_QKV: dispatch_epi<EPI_QKV, AWQ>(p, g, st); break;
    case EPI_F32: dispatch_epi<EPI_F32, AWQ>(p, g, st); break;
    default: dispatch_epi<EPI_BF16, AWQ>(p, g, st);
  }
}

static GemmParams to_params(const GemmArgs& g) {
  GemmParams p{};
  p.x = g.x; p.lda = g.lda; p.M = g.M; p.row_idx = g.row_idx;
  p.wp = reinterpret_cast<const uint4*>(g.wp); p.N = g.N; p.K = g.K;
  p.norm_w = g.norm_w; p.eps = g.eps;
  p.bias = g.bias; p.res = g.res; p.ldr = g.ldr;
  p.out = g.out; p.ldo = g.ldo;
  p.slabs = g.slabs; p.counters = g.counters;
  p.gran = nullptr; p.fault = g.fault;  // (granule split-K: set by the decode launchers when it fits)
  p.positions = g.positions; p.slots = g.slots; p.cos_sin = g.cos_sin;
  p.k_cache = g.k_cache; p.v_cache = g.v_cache; p.hq = g.hq; p.hkv = g.hkv; p.bs = g.bs;
  p.scales = g.scales; p.zeros = g.zeros; p.group = g.group; p.szp = g.awq_szp;
  p.dbg_ts = g.dbg_ts;
  p.hg = g.hg; p.hg_gamma = g.hg_gamma; p.ssp_out = g.ssp_out; p.ssp_in = g.ssp_in; p.ssn = g.ssn;
  p.ar = ArFused{};
  if (g.ar_world > 0) {
    for (int r = 0; r < 8; ++r) p.ar.base[r] = g.ar_fused[r];
    p.ar.err = g.ar_err; p.ar.rank = g.ar_rank; p.ar.world = g.ar_world; p.ar.spin = ar_spin();
  }
  return p;
}

void launch_gemm(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return;
  // TP row-parallel decode GEMM with the all-reduce in the epilogue: the tile-per-block decode kernels
  // (one wave finishes a whole 16-row tile: epilogue_ar's lane layout); the binding checked the shape
  if (g.ar_world > 0) {
    dispatch_epi<EPI_BF16_AR, false>(to_params(g), g, st);
    return;
  }
  // long steps (prefill chunks): the LDS-tiled MFMA kernel (gemm_prefill.hip) on the same packed
  // weights; it declines shapes / modes it does not take
  // mixed prefill + decode steps (16 < M <= 64): the medium-M kernel when the start-up tuner
  // measured it faster (path 2, gemm_mid.hip); it declines shapes / modes it does not take
  if (g.path == 2 && launch_gemm_mid(g, st)) return;
  // decode rows on the register-stationary kernel (path 4: a decode plan / forced; gemm_kx_bf16.hip)
  if (g.path == 4) {
    GemmArgs h = g;
    if (h.ntb > -12 || h.ntb < -14) h.ntb = 0;
    if (launch_dense_kx(h, st)) return;
    h.path = 0; h.waves = 0; h.splitk = 0; h.ntb = 0;
    launch_dispatch<false>(to_params(h), h, st);
    return;
  }
  // decode rows on the stream-K kernel (path 3: a decode plan / forced), else the tile-per-block kernels
  if (g.path == 3) {
    if (launch_gemm_sk(g, st)) return;
    // declined (shape / mode / occupancy): a stream-K plan's (waves, blocks per CU, k-group) fields
    // mean nothing to the tile kernels — fall back on the launcher's own heuristic
    GemmArgs h = g;
    h.path = 0; h.waves = 0; h.splitk = 0; h.ntb = 0;
    launch_dispatch<false>(to_params(h), h, st);
    return;
  }
  if (g.path == 1 || (g.path == 0 && g.M >= 128 && g.waves == 0 && g.splitk == 0)) {
    GemmArgs h = g;
    if (g.path == 0) h.ntb = 0;
    if (launch_gemm_prefill(h, st)) return;
  }
  launch_dispatch<false>(to_params(g), g, st);
}

void launch_awq_gemm(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return;
  if (g.ar_world > 0) {  // fused all-reduce: the K-split int4 kernel (gemm_finish -> epilogue_ar)
    GemmArgs h = g;
    h.ntb = -2;
    dispatch_epi<EPI_BF16_AR, true>(to_params(h), h, st);
    return;
  }
  // decode (M <= 16) on the register-stationary int4 kernel: the launcher's choice (no forced waves /
  // tiles per block), or g.ntb = -12 / -13 / -14 (1 / 2 / 4 tiles per block) with the forced waves / slices
  if (g.path == 0 && ((g.ntb == 0 && g.waves == 0) || (g.ntb <= -12 && g.ntb >= -14)) && launch_awq_kx(g, st)) return;
  // mixed prefill + decode steps (16 < M <= 64) on the int4 medium kernel (path 2)
  if (g.path == 2 && launch_awq_mid(g, st)) return;
  launch_dispatch<true>(to_params(g), g, st);
}

}  // namespace vgate