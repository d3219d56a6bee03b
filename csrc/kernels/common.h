// Shared device helpers for the vgate gfx950 (CDNA4 / MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * bf16 is moved as raw 16-bit words (uint16_t / uint4 of 8 elements) and
//     converted with bit operations; MFMA operands are `bf16x8` ext-vectors.
//   * MFMA shape is v_mfma_f32_16x16x32_bf16. Operand lane maps (gfx950):
//       A: lane l holds A[row l&15][k 8(l>>4)+j], j=0..7
//       B: lane l holds B[k 8(l>>4)+j][col l&15]
//       C: lane l holds C[row 4(l>>4)+i][col l&15], i=0..3
//   * Every launcher takes an explicit hipStream_t so the whole forward pass is
//     hipGraph-capturable (no allocation / sync inside launchers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vgate {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;  // storage type

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN stays NaN via the compiler's cvt path)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack_bf2(f[0], f[1]); r.y = pack_bf2(f[2], f[3]);
  r.z = pack_bf2(f[4], f[5]); r.w = pack_bf2(f[6], f[7]);
  return r;
}

__device__ __forceinline__ bf16x8 as_bf16x8(const uint4& v) {
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ T wave_reduce_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` needs >= 16 floats of LDS.
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_reduce_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}

__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_reduce_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
  return r;
}

// Non-temporal 16-B load for once-read weight streams (decode GEMV regime).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// plain 16-B load as a value (a uint4 struct assignment from global memory can lower to a
// memcpy through scratch that SROA does not undo)
__device__ __forceinline__ uint4 ld16(const void* p) {
  const u32x4 v = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// ---- cross-row lane exchange on the VALU (gfx950 v_permlane16/32_swap), no LDS pipe ----
// xor32(v): lane l gets lane l^32's value; xor16(v): lane l gets lane l^16's value.
// (__shfl_xor lowers to ds_bpermute: an LDS round trip on the critical path of a
// softmax reduction.)
__device__ __forceinline__ float xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}

// ---- in-launch cross-workgroup hand-off (cross-XCD safe, no cache-wide fences) ----
// The per-XCD L2s are not coherent, and an agent-scope release/acquire fence compiles to
// buffer_wbl2 / buffer_inv of the WHOLE L2 (write back every dirty line, drop every clean
// one: the weights and activations the next kernels want). Instead, hand-off data travels
// with device-coherent (sc1) stores and loads only: producer sc1 stores -> s_waitcnt
// vmcnt(0) -> relaxed agent-scope atomic (ticket / counter); consumer observes the atomic
// -> sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1_f4(float* p, float a, float b, float c, float d) {
  st_sc1(p, a); st_sc1(p + 1, b); st_sc1(p + 2, c); st_sc1(p + 3, d);
}
__device__ __forceinline__ f32x4 ld_sc1_f4(const float* p) {
  return f32x4{ld_sc1(p), ld_sc1(p + 1), ld_sc1(p + 2), ld_sc1(p + 3)};
}
// Bulk hand-off payloads: ONE 16-B write-through (sc1) vector store / sc1 load per lane through a
// buffer descriptor (four dword sc1 stores of the same bytes are 3-20x slower to publish:
// cdna_hip_programming.md Guideline 16, Pitfall 7). `base` must be wave-uniform (a kernel
// argument or a blockIdx-derived pointer), the per-lane part goes in the byte offset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_sc1_x4(float* base, uint32_t off_bytes, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc_of(base), off_bytes, 0, 16 /* sc1 */);
}
__device__ __forceinline__ f32x4 ld_sc1_x4(const float* base, uint32_t off_bytes) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base), off_bytes, 0, 16 /* sc1 */);
}
// all of this thread's stores have reached the device-coherent level
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS-DMA of one 16-B piece per lane (global_load_lds_dwordx4; the wave's 64 pieces land at
// lds_addr + 16 * lane). Written as inline asm so hipcc's alias analysis does not treat the
// in-flight DMA as an LDS write that every later ds_read must wait for (it emits vmcnt(0) in
// front of the first ds_read of the OTHER ring buffer otherwise, which serialises the stage
// pipeline). The caller owns the vmcnt bookkeeping (cdna_hip_programming.md §5.7 item 1).
// lds_addr must be wave-uniform; M0 is saved / restored inside the statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_addr) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  // generic -> LDS address-space cast (addrspacecast: the aperture offset), then its 32 bits
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// Workgroup barrier for LDS hand-offs that leaves global loads in flight: __syncthreads()
// is a release/acquire fence, which on gfx9 waits vmcnt(0) and so drains every outstanding
// weight prefetch; this waits only for this wave's LDS traffic (lgkmcnt) and then barriers.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

}  // namespace vgate

// ---- launch timeline (profiling, benchmarks/timeline.py) ----
// A kernel that receives a non-null `tl` stamps its block's [start, end] with the 100 MHz
// s_memrealtime clock at tl[2 * bid] / tl[2 * bid + 1]: start by thread 0 on entry, end as
// the max over the block's waves on every exit path (destructor). The host carves `tl` out
// of one device buffer per launch (tl_take), so a captured hipGraph keeps its slots and
// every replay rewrites them: inter-kernel gaps = next kernel's first start - last end.
struct TLScope {
  unsigned long long* p;
  __device__ __forceinline__ explicit TLScope(unsigned long long* tl) {
    p = nullptr;
    if (tl != nullptr) {
      const size_t bid = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
      p = tl + 2 * bid;
      if (threadIdx.x == 0) p[0] = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ ~TLScope() {
    if (p != nullptr && (threadIdx.x & 63) == 0)
      __hip_atomic_fetch_max(p + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
};
