// Weight-streaming MFMA GEMMs for the decode / small-M regime on gfx950.
//
//   out[m][n] = epilogue( sum_k x[m][k] * W[n][k] )
//
// Weights are pre-packed ONCE at load time into "fragment-major" order so that
// one wave-instruction of 16 B/lane reads 1 KiB of contiguous HBM that is
// exactly the A operand of v_mfma_f32_16x16x32_bf16:
//
//   Wp[nt][kt][lane][j] = W[16*nt + (lane & 15)][32*kt + 8*(lane >> 4) + j]
//
// (nt = 16-row n-tile, kt = 32-wide k-tile). No LDS staging of weights: in the
// M <= 64 regime each weight byte is used by one wave only, so the bytes go
// straight to VGPRs with non-temporal loads (cdna_hip_programming.md §5 'GEMV /
// M <= 16 decode weights' row). Activation (x) fragments are L2-resident.
//
// Decomposition: one workgroup owns NTB n-tiles for a 16*MB row chunk of x and
// ALL of K; its W waves split K into contiguous ranges (each wave streams one
// contiguous weight region) and the partial accumulators are reduced through
// LDS. The epilogue (bias, residual add, SiLU*mul, f32 logits) is fused, so no
// split-K workspace or second launch exists.
//
// Orientation: D = Wfrag(A) x xfrag(B) -> lane holds D[n = 4(l>>4)+i][m = l&15],
// i.e. 4 consecutive output columns of one row -> 8-byte stores.
//
// AWQ W4A16 variant: int4 weights packed in the same fragment order, 4 k-tiles
// per 16-B lane load ([nt][kt/4][lane][4] uint32, nibble j = element j), with
// group-wise (scale, scale*zero) applied in registers before the bf16 MFMA.
#include "common.h"
#include "launchers.h"

namespace vgate {

enum GemmEpi : int { EPI_BF16 = 0, EPI_F32 = 1, EPI_SILU = 2 };

// Cross-wave LDS reduction of acc[MB][NTB] + fused epilogue + store.
template <int MB, int NTB, int EPI>
__device__ __forceinline__ void gemm_finish(f32x4 (&acc)[MB][NTB], float* red, int M, int m_base,
                                            int nt0, const bf16_t* __restrict__ bias,
                                            const bf16_t* res, int ldr, void* out, int ldo) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  constexpr int SLOTS = MB * NTB * 64;  // f32x4 slots per wave
  f32x4* red4 = reinterpret_cast<f32x4*>(red);
  if (nw > 1) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int j = 0; j < NTB; ++j) red4[wid * SLOTS + (mb * NTB + j) * 64 + lane] = acc[mb][j];
    __syncthreads();
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
      // single-wave block (thread == lane): select this m-block's registers statically
#pragma unroll
      for (int mm = 0; mm < MB; ++mm)
        if (mm == mb)
#pragma unroll
          for (int j = 0; j < NTB; ++j) v[j] = acc[mm][j];
    }
    if (m >= M) continue;
    const int nsub = 4 * (l >> 4);
    if constexpr (EPI == EPI_SILU) {
      static_assert(NTB == 2, "silu epilogue pairs a gate tile with an up tile");
      const int n = (nt0 >> 1) * 16 + nsub;  // output column (N/2 wide)
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = silu(v[0][i]) * v[1][i];
      bf16_t* op = reinterpret_cast<bf16_t*>(out) + (size_t)m * ldo + n;
      uint2 pk;
      pk.x = pack_bf2(o[0], o[1]);
      pk.y = pack_bf2(o[2], o[3]);
      *reinterpret_cast<uint2*>(op) = pk;
    } else {
#pragma unroll
      for (int j = 0; j < NTB; ++j) {
        const int n = (nt0 + j) * 16 + nsub;
        float o[4] = {v[j][0], v[j][1], v[j][2], v[j][3]};
        if (bias) {
          const uint2 b = *reinterpret_cast<const uint2*>(bias + n);
          o[0] += __uint_as_float(b.x << 16); o[1] += __uint_as_float(b.x & 0xffff0000u);
          o[2] += __uint_as_float(b.y << 16); o[3] += __uint_as_float(b.y & 0xffff0000u);
        }
        if constexpr (EPI == EPI_F32) {
          float* op = reinterpret_cast<float*>(out) + (size_t)m * ldo + n;
          *reinterpret_cast<float4*>(op) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
          if (res) {
            // round the GEMM result to bf16 first (matches torch: (x@W).bf16() + res)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = bf2f(f2bf(o[i]));
            const uint2 r = *reinterpret_cast<const uint2*>(res + (size_t)m * ldr + n);
            o[0] += __uint_as_float(r.x << 16); o[1] += __uint_as_float(r.x & 0xffff0000u);
            o[2] += __uint_as_float(r.y << 16); o[3] += __uint_as_float(r.y & 0xffff0000u);
          }
          bf16_t* op = reinterpret_cast<bf16_t*>(out) + (size_t)m * ldo + n;
          uint2 pk;
          pk.x = pack_bf2(o[0], o[1]);
          pk.y = pack_bf2(o[2], o[3]);
          *reinterpret_cast<uint2*>(op) = pk;
        }
      }
    }
  }
}

template <int MB>
__device__ __forceinline__ void x_rows(const bf16_t* (&xrow)[MB], const bf16_t* x, int lda, int M,
                                       int m_base, int lane) {
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    int m = m_base + mb * 16 + (lane & 15);
    m = m < M ? m : M - 1;  // clamp: duplicated rows are computed but never stored
    xrow[mb] = x + (size_t)m * lda + 8 * (lane >> 4);
  }
}

template <int MB, int NTB, int U, int EPI>
__global__ __launch_bounds__(1024) void gemm_skinny_kernel(
    const bf16_t* __restrict__ x, int lda, int M, const uint4* __restrict__ Wp, int N, int K,
    const bf16_t* __restrict__ bias, const bf16_t* res, int ldr, void* out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const int KT = K >> 5;
  const int nt0 = blockIdx.x * NTB;
  const int m_base = blockIdx.y * 16 * MB;
  const int kbeg = (KT * wid) / nw;
  const int kend = (KT * (wid + 1)) / nw;

  f32x4 acc[MB][NTB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NTB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint4* wbase[NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) wbase[j] = Wp + ((size_t)(nt0 + j) * KT) * 64 + lane;
  const bf16_t* xrow[MB];
  x_rows<MB>(xrow, x, lda, M, m_base, lane);

  int kt = kbeg;
  for (; kt + U <= kend; kt += U) {
    uint4 b[U][NTB];
    uint4 a[U][MB];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NTB; ++j) b[u][j] = ld_nt16(wbase[j] + (size_t)(kt + u) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        a[u][mb] = *reinterpret_cast<const uint4*>(xrow[mb] + (kt + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NTB; ++j)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb][j] = mfma16(as_bf16x8(b[u][j]), as_bf16x8(a[u][mb]), acc[mb][j]);
  }
  for (; kt < kend; ++kt) {
    uint4 b[NTB], a[MB];
#pragma unroll
    for (int j = 0; j < NTB; ++j) b[j] = ld_nt16(wbase[j] + (size_t)kt * 64);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) a[mb] = *reinterpret_cast<const uint4*>(xrow[mb] + kt * 32);
#pragma unroll
    for (int j = 0; j < NTB; ++j)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(as_bf16x8(b[j]), as_bf16x8(a[mb]), acc[mb][j]);
  }
  gemm_finish<MB, NTB, EPI>(acc, red, M, m_base, nt0, bias, res, ldr, out, ldo);
}

// ---- AWQ W4A16 ----
// dequant 8 nibbles of one 32-bit word: w = q * s - sz  (sz = s * zero)
__device__ __forceinline__ bf16x8 dq8(uint32_t q, float s, float sz) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)((float)((q >> (4 * j)) & 0xF) * s - sz);
  return r;
}

template <int MB, int NTB, int EPI>
__global__ __launch_bounds__(1024) void awq_gemm_kernel(
    const bf16_t* __restrict__ x, int lda, int M, const uint4* __restrict__ qw,
    const bf16_t* __restrict__ scales, const bf16_t* __restrict__ zeros, int group, int N, int K,
    const bf16_t* __restrict__ bias, const bf16_t* res, int ldr, void* out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const int KQ = K >> 7;  // 128-wide k quads (4 k-tiles per 16-B lane load)
  const int nt0 = blockIdx.x * NTB;
  const int m_base = blockIdx.y * 16 * MB;
  const int qbeg = (KQ * wid) / nw;
  const int qend = (KQ * (wid + 1)) / nw;
  f32x4 acc[MB][NTB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NTB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16_t* xrow[MB];
  x_rows<MB>(xrow, x, lda, M, m_base, lane);
  for (int kq = qbeg; kq < qend; ++kq) {
    uint4 w[NTB];
#pragma unroll
    for (int j = 0; j < NTB; ++j) w[j] = ld_nt16(qw + ((size_t)(nt0 + j) * KQ + kq) * 64 + lane);
    uint4 a[4][MB];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        a[u][mb] = *reinterpret_cast<const uint4*>(xrow[mb] + (kq * 4 + u) * 32);
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      const int n = (nt0 + j) * 16 + (lane & 15);
      const uint32_t wq[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = (kq * 4 + u) * 32 + 8 * (lane >> 4);
        const int gi = k / group;
        const float s = bf2f(scales[(size_t)gi * N + n]);
        const float sz = bf2f(zeros[(size_t)gi * N + n]);
        const bf16x8 wf = dq8(wq[u], s, sz);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][j] = mfma16(wf, as_bf16x8(a[u][mb]), acc[mb][j]);
      }
    }
  }
  gemm_finish<MB, NTB, EPI>(acc, red, M, m_base, nt0, bias, res, ldr, out, ldo);
}

static int pick_waves(int total_blocks, int ksteps, int mb, int ntb, int forced) {
  if (forced > 0) return forced;
  int w = 1;
  while (w < 16 && total_blocks * w < 4096) w <<= 1;
  while (w > 1 && ksteps / w < 4) w >>= 1;
  while (w > 1 && w * mb * ntb > 64) w >>= 1;
  return w;
}

template <int MB, int NTB, int EPI>
static void launch_mb(const GemmArgs& g, hipStream_t st) {
  const int KT = g.K / 32;
  const int nblk = g.N / 16 / NTB;
  const int mchunks = (g.M + 16 * MB - 1) / (16 * MB);
  const int w = pick_waves(nblk * mchunks, KT, MB, NTB, g.waves);
  const size_t lds = (w > 1) ? (size_t)w * MB * NTB * 64 * 16 : 0;
  hipLaunchKernelGGL((gemm_skinny_kernel<MB, NTB, 4, EPI>), dim3(nblk, mchunks), dim3(64 * w), lds, st,
                     g.x, g.lda, g.M, reinterpret_cast<const uint4*>(g.wp), g.N, g.K, g.bias, g.res,
                     g.ldr, g.out, g.ldo);
}

template <int NTB, int EPI>
static void launch_ntb(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 16) launch_mb<1, NTB, EPI>(g, st);
  else if (g.M <= 32) launch_mb<2, NTB, EPI>(g, st);
  else launch_mb<4, NTB, EPI>(g, st);
}

void launch_gemm(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return;
  const int ntiles = g.N / 16;
  if (g.epi == EPI_SILU) {
    launch_ntb<2, EPI_SILU>(g, st);
  } else if (g.epi == EPI_F32) {
    if (ntiles % 2 == 0 && ntiles >= 1024) launch_ntb<2, EPI_F32>(g, st);
    else launch_ntb<1, EPI_F32>(g, st);
  } else {
    if (ntiles % 2 == 0 && ntiles >= 1024) launch_ntb<2, EPI_BF16>(g, st);
    else launch_ntb<1, EPI_BF16>(g, st);
  }
}

template <int MB, int NTB, int EPI>
static void awq_launch_mb(const AwqGemmArgs& g, hipStream_t st) {
  const int KQ = g.K / 128;
  const int nblk = g.N / 16 / NTB;
  const int mchunks = (g.M + 16 * MB - 1) / (16 * MB);
  const int w = pick_waves(nblk * mchunks, KQ * 2, MB, NTB, 0);
  const size_t lds = (w > 1) ? (size_t)w * MB * NTB * 64 * 16 : 0;
  hipLaunchKernelGGL((awq_gemm_kernel<MB, NTB, EPI>), dim3(nblk, mchunks), dim3(64 * w), lds, st, g.x,
                     g.lda, g.M, reinterpret_cast<const uint4*>(g.qw), g.scales, g.zeros, g.group,
                     g.N, g.K, g.bias, g.res, g.ldr, g.out, g.ldo);
}

template <int NTB, int EPI>
static void awq_launch_ntb(const AwqGemmArgs& g, hipStream_t st) {
  if (g.M <= 16) awq_launch_mb<1, NTB, EPI>(g, st);
  else if (g.M <= 32) awq_launch_mb<2, NTB, EPI>(g, st);
  else awq_launch_mb<4, NTB, EPI>(g, st);
}

void launch_awq_gemm(const AwqGemmArgs& g, hipStream_t st) {
  if (g.M <= 0) return;
  if (g.epi == EPI_SILU) awq_launch_ntb<2, EPI_SILU>(g, st);
  else if (g.epi == EPI_F32) awq_launch_ntb<1, EPI_F32>(g, st);
  else awq_launch_ntb<1, EPI_BF16>(g, st);
}

}  // namespace vgate
