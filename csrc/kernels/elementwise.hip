// Memory-bound kernels: RMSNorm (+fused residual add), embedding gather,
// NeoX RoPE + paged KV-cache write. All bf16 traffic is 16-B vectorised
// (cdna_hip_programming.md Guideline 13); trig comes from a host-built table.
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace vgate {

// One workgroup per row; each thread owns up to VPT 8-element vectors kept in
// registers between the sum-of-squares pass and the scale pass (one HBM read).
template <int VPT>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_t* __restrict__ x, int ldx,
                                                       bf16_t* res, int ldres,
                                                       const bf16_t* __restrict__ w,
                                                       bf16_t* __restrict__ y, int ldy, int H,
                                                       float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = H >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * ldx);
  uint4* rr = res ? reinterpret_cast<uint4*>(res + (size_t)row * ldres) : nullptr;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      unpack8(xr[c], v[i]);
      if (rr) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        // residual stream is stored in bf16: normalise the rounded value
        const uint4 pk = pack8(v[i]);
        rr[c] = pk;
        unpack8(pk, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_reduce_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * ldy);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(wr[c], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // match torch: (x * inv).to(bf16) * w
        o[j] = bf2f(f2bf(v[i][j] * inv)) * wf[j];
      }
      yr[c] = pack8(o);
    }
  }
}

void launch_rmsnorm(const uint16_t* x, int ldx, uint16_t* res, int ldres, const uint16_t* w,
                    uint16_t* y, int ldy, int M, int H, float eps, hipStream_t st) {
  if (M <= 0) return;
  const int nvec = H / 8;
  int threads = nvec < 256 ? ((nvec + 63) / 64) * 64 : 256;
  const int vpt = (nvec + threads - 1) / threads;
  dim3 grid(M), block(threads);
  if (vpt <= 1)
    hipLaunchKernelGGL(rmsnorm_kernel<1>, grid, block, 0, st, x, ldx, res, ldres, w, y, ldy, H, eps);
  else if (vpt <= 2)
    hipLaunchKernelGGL(rmsnorm_kernel<2>, grid, block, 0, st, x, ldx, res, ldres, w, y, ldy, H, eps);
  else if (vpt <= 4)
    hipLaunchKernelGGL(rmsnorm_kernel<4>, grid, block, 0, st, x, ldx, res, ldres, w, y, ldy, H, eps);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<8>, grid, block, 0, st, x, ldx, res, ldres, w, y, ldy, H, eps);
}

// ids[t] < 0 refers to a token sampled by the PREVIOUS step that the host has not seen
// yet (asynchronous scheduling): id = prev[-ids[t] - 1], read on the device.
__global__ __launch_bounds__(256) void embedding_kernel(const int32_t* __restrict__ ids,
                                                         const int32_t* __restrict__ prev,
                                                         const bf16_t* __restrict__ table,
                                                         bf16_t* __restrict__ out, int H,
                                                         int vstart, int vrows, unsigned long long* tl) {
  TLScope tl_scope(tl);
  const int t = blockIdx.x;
  int tok = ids[t];
  if (tok < 0 && prev != nullptr) tok = prev[-tok - 1];
  const int id = tok - vstart;
  const bool ok = id >= 0 && id < vrows;
  const uint4* src = reinterpret_cast<const uint4*>(table + (size_t)(ok ? id : 0) * H);
  uint4* dst = reinterpret_cast<uint4*>(out + (size_t)t * H);
  for (int c = threadIdx.x; c < (H >> 3); c += blockDim.x) dst[c] = ok ? src[c] : make_uint4(0, 0, 0, 0);
}

void launch_embedding(const int32_t* ids, const uint16_t* table, uint16_t* out, int T, int H,
                      int vstart, int vrows, hipStream_t st, const int32_t* prev) {
  if (T <= 0) return;
  hipLaunchKernelGGL(embedding_kernel, dim3(T), dim3(256), 0, st, ids, prev, table, out, H, vstart, vrows,
                     tl_take("embedding", T));
}

// One workgroup per token. Work items:
//   rotate:  (Hq + Hkv) heads x (D/2)/4 quads  -> each rotates 4 (x1, x2) pairs
//   v copy:  Hkv heads x D/8 vectors
__global__ __launch_bounds__(256) void rope_kv_kernel(bf16_t* __restrict__ qkv,
                                                       const int32_t* __restrict__ positions,
                                                       const int32_t* __restrict__ slots,
                                                       const float* __restrict__ cos_sin,
                                                       bf16_t* __restrict__ k_cache,
                                                       bf16_t* __restrict__ v_cache, int Hq,
                                                       int Hkv, int D, int BS, bf16_t* __restrict__ q_out,
                                                       int ldq) {
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int slot = slots ? slots[t] : -1;
  const int half = D >> 1;
  const int qpr = half >> 2;  // quads per head
  const int row_elems = (Hq + 2 * Hkv) * D;
  bf16_t* row = qkv + (size_t)t * row_elems;
  const float* cs = cos_sin + (size_t)pos * D;
  const int blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  const int nrot = (Hq + Hkv) * qpr;
  for (int it = threadIdx.x; it < nrot; it += blockDim.x) {
    const int h = it / qpr;
    const int i0 = (it % qpr) * 4;
    bf16_t* base = row + h * D;
    const uint2 a = *reinterpret_cast<const uint2*>(base + i0);
    const uint2 b = *reinterpret_cast<const uint2*>(base + half + i0);
    const float4 c = *reinterpret_cast<const float4*>(cs + i0);
    const float4 s = *reinterpret_cast<const float4*>(cs + half + i0);
    float x1[4] = {__uint_as_float(a.x << 16), __uint_as_float(a.x & 0xffff0000u),
                   __uint_as_float(a.y << 16), __uint_as_float(a.y & 0xffff0000u)};
    float x2[4] = {__uint_as_float(b.x << 16), __uint_as_float(b.x & 0xffff0000u),
                   __uint_as_float(b.y << 16), __uint_as_float(b.y & 0xffff0000u)};
    const float cc[4] = {c.x, c.y, c.z, c.w}, ssn[4] = {s.x, s.y, s.z, s.w};
    float o1[4], o2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o1[j] = x1[j] * cc[j] - x2[j] * ssn[j];
      o2[j] = x2[j] * cc[j] + x1[j] * ssn[j];
    }
    uint2 p1, p2;
    p1.x = pack_bf2(o1[0], o1[1]); p1.y = pack_bf2(o1[2], o1[3]);
    p2.x = pack_bf2(o2[0], o2[1]); p2.y = pack_bf2(o2[2], o2[3]);
    if (q_out == nullptr) {  // in place
      *reinterpret_cast<uint2*>(base + i0) = p1;
      *reinterpret_cast<uint2*>(base + half + i0) = p2;
    } else if (h < Hq) {  // rotated q straight into the attention input (k only goes to the cache)
      bf16_t* qd = q_out + (size_t)t * ldq + h * D;
      *reinterpret_cast<uint2*>(qd + i0) = p1;
      *reinterpret_cast<uint2*>(qd + half + i0) = p2;
    }
    if (h >= Hq && slot >= 0) {
      const int kh = h - Hq;
      bf16_t* dst = k_cache + (((size_t)blk * Hkv + kh) * BS + off) * D;
      *reinterpret_cast<uint2*>(dst + i0) = p1;
      *reinterpret_cast<uint2*>(dst + half + i0) = p2;
    }
  }
  if (slot >= 0) {
    const int vpr = D >> 3;
    for (int it = threadIdx.x; it < Hkv * vpr; it += blockDim.x) {
      const int h = it / vpr;
      const int c = it % vpr;
      const uint4 v = *reinterpret_cast<const uint4*>(row + (Hq + Hkv + h) * D + c * 8);
      bf16_t* dst = v_cache + (((size_t)blk * Hkv + h) * BS + off) * D;
      *reinterpret_cast<uint4*>(dst + c * 8) = v;
    }
  }
}

void launch_rope_kv(uint16_t* qkv, const int32_t* positions, const int32_t* slots,
                    const float* cos_sin, uint16_t* k_cache, uint16_t* v_cache, int T, int Hq,
                    int Hkv, int D, int BS, hipStream_t st, uint16_t* q_out, int ldq) {
  if (T <= 0) return;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(256), 0, st, qkv, positions, slots, cos_sin,
                     k_cache, v_cache, Hq, Hkv, D, BS, q_out, ldq);
}

// out[m, i] = silu(y[m, i]) * y[m, I + i] (fp32 math, bf16 out): the SiLU*mul epilogue of the
// library (hipBLASLt) gate_up GEMM. 8 columns per thread, 16-B accesses; I % 8 == 0.
__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16_t* __restrict__ y, int ldy, bf16_t* __restrict__ out,
                                                       int ldo, int I, int M) {
  const int per_row = I >> 3;
  const size_t n = (size_t)M * per_row;
  for (size_t it = (size_t)blockIdx.x * blockDim.x + threadIdx.x; it < n; it += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(it / per_row), c = (int)(it % per_row) * 8;
    const bf16_t* r = y + (size_t)m * ldy;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(r + c), g);
    unpack8(*reinterpret_cast<const uint4*>(r + I + c), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    *reinterpret_cast<uint4*>(out + (size_t)m * ldo + c) = pack8(o);
  }
}

void launch_silu_mul(const uint16_t* y, int ldy, uint16_t* out, int ldo, int I, int M, hipStream_t st) {
  if (M <= 0 || I <= 0) return;
  const size_t n = (size_t)M * (I >> 3);
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(silu_mul_kernel, dim3(blocks), dim3(256), 0, st, y, ldy, out, ldo, I, M);
}

// Read-only sweep of a byte range with the DEFAULT cache policy (not nt): the lines land in
// the memory-side Infinity Cache (MALL, 256 MB) so a later non-temporal weight stream of the
// same bytes hits there instead of HBM. Used on latency-bound phases (attention, small GEMMs)
// whose HBM is otherwise idle. Nothing is written (the sink test is never true).
__global__ __launch_bounds__(256) void prefetch_kernel(const uint4* __restrict__ p, size_t n16, uint32_t* sink,
                                                        unsigned long long* tl) {
  TLScope tl_scope(tl);
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x9E3779B9u && sink != nullptr) *sink = acc;
}

void launch_prefetch(const void* p, size_t bytes, int blocks, hipStream_t st) {
  const size_t n16 = bytes / 16;
  if (n16 == 0) return;
  if (blocks <= 0) blocks = 256;
  hipLaunchKernelGGL(prefetch_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const uint4*>(p), n16,
                     nullptr, tl_take("prefetch", blocks));
}

// Host <-> device copies of the step loop as a kernel on the compute queue. Per decode step the
// engine moves ~40 KB of step metadata to the device and the sampled ids back; as hipMemcpyAsync
// the metadata went through an SDMA engine, and the compute queue <-> SDMA hand-offs left the GPU
// idle for ~25-40 us between two steps (benchmarks/trace_gaps.py: sampler end -> 9 us -> D2H blit
// -> 11 us -> SDMA H2D -> 10 us -> next step). Here every 16-B piece is one load + one store by its
// own thread (all in flight at once: one PCIe round trip); pinned host memory is device-mapped.
// Stores to host memory are made system-visible before the kernel ends.
__global__ __launch_bounds__(256) void copy16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16,
                                                     int to_host) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) dst[i] = src[i];
  if (to_host) __threadfence_system();
}

// The step graph's last node: the sampled ids of the step -> slot `*slot` of a pinned host ring
// (device-mapped), so the host reads them once the graph has completed, with no copy launched
// after the graph (the graph-end -> next-dispatch boundary was ~9 us of the gap between steps).
__global__ __launch_bounds__(64) void ids_to_host_kernel(const int32_t* __restrict__ ids, int32_t* __restrict__ ring,
                                                         const int32_t* __restrict__ slot, int stride, int n,
                                                         const uint32_t* __restrict__ ar,
                                                         const uint32_t* __restrict__ fault) {
  const int s = *slot;
  for (int i = threadIdx.x; i < n; i += 64) ring[(size_t)s * stride + i] = ids[i];
  if (ar != nullptr && threadIdx.x < 3)  // custom all-reduce {error, ticks, calls}: sticky / running words
    ring[(size_t)s * stride + stride - 4 + threadIdx.x] =
        (int32_t)__hip_atomic_load(ar + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (fault != nullptr && threadIdx.x == 3)  // in-launch hand-off give-ups (flash K split, fused MLP): sticky
    ring[(size_t)s * stride + stride - 1] = (int32_t)__hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
}

void launch_ids_to_host(const int32_t* ids, int32_t* ring, const int32_t* slot, int stride, int n, hipStream_t st,
                        const uint32_t* ar, const uint32_t* fault) {
  if (n <= 0 && ar == nullptr && fault == nullptr) return;
  hipLaunchKernelGGL(ids_to_host_kernel, dim3(1), dim3(64), 0, st, ids, ring, slot, stride, n, ar, fault);
}

void launch_copy16(const void* src, void* dst, size_t bytes, bool to_host, hipStream_t st) {
  const int n16 = (int)(bytes / 16);
  if (n16 <= 0) return;
  hipLaunchKernelGGL(copy16_kernel, dim3((n16 + 255) / 256), dim3(256), 0, st, reinterpret_cast<const uint4*>(src),
                     reinterpret_cast<uint4*>(dst), n16, to_host ? 1 : 0);
}

}  // namespace vgate
