// Can a latency-bound producer and a weight-streaming consumer share ONE launch? (MI355X, gfx950)
//
// Decode layer boundaries cost ~1.6 us each in a replayed graph (profiles/r2_grid_barrier_probe.log,
// 143 per Qwen2.5-1.5B step), and the consumer GEMM cannot request a single weight byte before the
// producer's launch has fully drained. Round 3 tried overlap across two queues (graph branches,
// profiles/r3_chain_overlap_negative.log: the spinning consumer starved the other queue's producer).
// Here producer and consumer are blocks of the SAME launch: block ids [0, NA) are producers, [NA,
// NA + NB) consumers. Workgroups are dispatched in id order on each XCD, so every producer is placed
// before any consumer of its XCD and a consumer only ever waits on blocks that are running or done.
//   producer ("attention"-like): a two-round-trip dependent load chain, a little ALU, the output
//     rows stored write-through (sc1), drained, then one device-scope arrival increment;
//   consumer ("o_proj"-like, one 16-column tile per block, W waves splitting K): EVERY weight
//     fragment requested at launch, then the wave spins (bounded, s_sleep) on the arrival counter,
//     then loads x (sc1), MFMAs, stores.
// Modes: 0 = two launches (producer kernel, consumer kernel without waiting), 1 = one fused launch.
// Arrival targets grow by NA per iteration (iteration index passed per launch), so no reset is needed.
// A consumer that gives up sets an error word (counted below), nothing hangs.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/fused_pair_probe benchmarks/probes/fused_pair_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ u32x4 ld_nt(const u32x4* p) { return __builtin_nontemporal_load(p); }

struct Args {
  const u32x4* kv;      // producer input (L2-cold ring copy), 64 KiB per producer block
  const int* idx;       // producer indirection (the "block table")
  u32x4* out;           // producer output rows = consumer x: K bf16 per row, 8 rows
  const u32x4* w;       // consumer weights: [ntiles][KT][64] fragment-packed
  float* y;             // consumer output
  unsigned* arrivals;   // producer arrival counter
  unsigned* err;        // consumer give-up count
  int NA, KT, iter;
};

__device__ void producer(const Args& a, int b) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // round trip 1: the indirection; round trip 2: the data it points at (as attention's block table -> K/V)
  const int j = a.idx[b * 64 + lane];
  const u32x4* src = a.kv + (size_t)b * 4096 + (size_t)(j & 63) * 64;
  u32x4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = src[(size_t)u * 1024 + wid * 64 + lane - (wid * 64 + lane) % 64 + lane];
  unsigned acc = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) acc ^= v[u].x + v[u].y * 3u + v[u].z * 5u + v[u].w * 7u;
  // this block's slice of the 8 output rows (write-through stores: the consumer reads them in-launch)
  const int per = (a.KT * 32) / a.NA;  // u32x4 (8 bf16) pieces of the 8 x K image per producer block
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    u32x4 val = {acc & 0x3f003f00u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, val),
                                           __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7fffffff, 0x00020000),
                                           (uint32_t)((b * per + i) * 16), 0, 16);
  }
  // write-through stores drained, then a relaxed arrival (no cache-wide release fence: the data never
  // sat dirty in an L2)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(a.arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool WAIT>
__device__ void consumer(const Args& a, int t) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int k0 = (a.KT * wid) / nw, k1 = (a.KT * (wid + 1)) / nw;  // <= 8 k-steps per wave (host)
  u32x4 w[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) w[u] = ld_nt(a.w + ((size_t)t * a.KT + min(k0 + u, k1 - 1)) * 64 + lane);
  if (WAIT) {
    const unsigned target = (unsigned)(a.iter + 1) * (unsigned)a.NA;
    int spins = 0;
    while (true) {
      const unsigned v = __hip_atomic_load(a.arrivals, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(v - target) >= 0) break;
      if (++spins > (1 << 16)) {
        if (lane == 0) atomicAdd(a.err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");  // the x loads (device-coherent) stay behind the poll
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (k0 + u < k1) {
      // x fragment of k-step k0+u: 16 rows x 32 k -> this lane's 8 bf16 (rows >= 8 re-read row 7)
      const int row = (lane & 15) < 8 ? (lane & 15) : 7;
      const uint32_t off = (uint32_t)(((size_t)row * a.KT * 4 + (size_t)(k0 + u) * 4 + (lane >> 4)) * 16);
      const f32x4 xv = __builtin_amdgcn_raw_buffer_load_b128(
          __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7fffffff, 0x00020000), off, 0, 16);
      acc = mfma16(w[u], __builtin_bit_cast(u32x4, xv), acc);
    }
  }
  __shared__ f32x4 red[16][64];
  red[wid][lane] = acc;
  __syncthreads();
  if (wid == 0) {
    f32x4 s = red[0][lane];
    for (int i = 1; i < nw; ++i) s += red[i][lane];
    *reinterpret_cast<f32x4*>(a.y + ((size_t)t * 64 + lane) * 4) = s;
  }
}

__global__ __launch_bounds__(1024) void k_producer(Args a) { producer(a, blockIdx.x); }
__global__ __launch_bounds__(1024) void k_consumer(Args a) { consumer<false>(a, blockIdx.x); }
__global__ __launch_bounds__(1024) void k_fused(Args a) {
  if ((int)blockIdx.x < a.NA) producer(a, blockIdx.x);
  else consumer<true>(a, blockIdx.x - a.NA);
}

int main() {
  const int NA = 16, ntiles = 96, K = 1536, KT = K / 32, W = 12;  // o_proj: 96 tiles x 48 k-steps
  const int R = 20;
  const size_t kv_bytes = (size_t)NA * 4096 * 16;
  const size_t w_bytes = (size_t)ntiles * KT * 64 * 16;
  const int ncopy = 64;  // cold weights / producer input: a ring of copies
  char *kv, *wb;
  CK(hipMalloc(&kv, kv_bytes * ncopy));
  CK(hipMalloc(&wb, w_bytes * ncopy));
  CK(hipMemset(kv, 1, kv_bytes * ncopy));
  CK(hipMemset(wb, 0, w_bytes * ncopy));
  int* idx;
  CK(hipMalloc(&idx, NA * 64 * 4));
  CK(hipMemset(idx, 0, NA * 64 * 4));
  u32x4* out;
  CK(hipMalloc(&out, (size_t)8 * K * 2 + 4096));
  CK(hipMemset(out, 0, (size_t)8 * K * 2 + 4096));
  float* y;
  CK(hipMalloc(&y, (size_t)ntiles * 64 * 16));
  unsigned *arr, *err;
  CK(hipMalloc(&arr, 4));
  CK(hipMalloc(&err, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(arr, 0, 4));
      CK(hipMemset(err, 0, 4));
      CK(hipDeviceSynchronize());
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int r = 0; r < R; ++r) {
        Args a{reinterpret_cast<const u32x4*>(kv + (size_t)(r % ncopy) * kv_bytes), idx, out,
               reinterpret_cast<const u32x4*>(wb + (size_t)(r % ncopy) * w_bytes), y, arr, err, NA, KT, r};
        if (mode == 0) {
          hipLaunchKernelGGL(k_producer, dim3(NA), dim3(64 * W), 0, st, a);
          hipLaunchKernelGGL(k_consumer, dim3(ntiles), dim3(64 * W), 0, st, a);
        } else {
          hipLaunchKernelGGL(k_fused, dim3(NA + ntiles), dim3(64 * W), 0, st, a);
        }
      }
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned h_err = 0, h_arr = 0;
      CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&h_arr, arr, 4, hipMemcpyDeviceToHost));
      printf("{\"mode\": %d, \"rep\": %d, \"us_per_pair\": %.2f, \"arrivals\": %u, \"consumer_giveups\": %u}\n", mode, rep,
             1e3 * ms / R, h_arr, h_err);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
