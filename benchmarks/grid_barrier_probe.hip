// Grid-barrier cost on gfx950 (MI355X): how long does a device-wide arrive + release take for
// a persistent grid, compared with the ~2-6 us kernel-boundary gaps the decode step pays
// (gpurun_out r2_timeline2: 548 us of gaps in a 1708 us step)? Decides whether a persistent
// decode-layer kernel (phases joined by in-kernel barriers, next-phase weights prefetched while
// waiting) can beat one launch per op.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/grid_barrier_probe benchmarks/grid_barrier_probe.hip
//   /tmp/grid_barrier_probe   -> one JSON line per configuration
//
// Every spin is bounded (a block that cannot see the others exits with an error count), so a
// non-co-resident grid ends instead of hanging. Cross-XCD visibility: counters are touched only
// with agent-scope atomics (sc1: past the per-XCD L2), never with plain loads.
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

constexpr unsigned kSpin = 1u << 22;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_agent(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// mode 0: one flat counter, every block arrives and polls it
// mode 1: per-XCD counters (blockIdx % 8), the last arriver of an XCD bumps the global counter;
//         everyone polls the global counter
// mode 2: flat arrive, but only one wave per block polls and the others wait at s_barrier
//         (same as 0 here: thread 0 polls) + a 16 KiB per-block HBM read between barriers
__global__ __launch_bounds__(256) void barrier_kernel(unsigned* ctr, int rounds, int mode, unsigned* err,
                                                      const uint4* src, uint4* sink) {
  const int nb = gridDim.x;
  unsigned* glob = ctr;
  unsigned* xcd = ctr + 64;  // 8 counters, 64 B apart
  uint4 accv = make_uint4(0, 0, 0, 0);
  __shared__ int bail;
  if (threadIdx.x == 0) bail = 0;
  for (int r = 1; r <= rounds; ++r) {
    if (mode == 2) {
      const u32x4* s = reinterpret_cast<const u32x4*>(src) + ((size_t)(r % 64) * nb + blockIdx.x) * 1024;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u32x4 v = __builtin_nontemporal_load(s + i * 256 + threadIdx.x);
        accv.x ^= v.x; accv.y ^= v.y; accv.z ^= v.z; accv.w ^= v.w;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (mode == 1) {
        const int x = blockIdx.x & 7;
        const unsigned per = (unsigned)((nb - x + 7) / 8);  // blocks of this XCD
        const unsigned old = add_agent(xcd + 16 * x, 1);
        if (old + 1 == per * (unsigned)r) add_agent(glob, 1);
        const unsigned target = 8u * (unsigned)r;
        unsigned n = 0;
        while (ld_agent(glob) < target && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
        if (n >= kSpin) {
          atomicAdd(err, 1u);
          bail = 1;
        }
      } else {
        add_agent(glob, 1);
        const unsigned target = (unsigned)nb * (unsigned)r;
        unsigned n = 0;
        while (ld_agent(glob) < target && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
        if (n >= kSpin) {
          atomicAdd(err, 1u);
          bail = 1;
        }
      }
    }
    __syncthreads();
    if (bail) break;  // a block that could not see the others leaves: the grid always drains
  }
  if (accv.x == 0x12345678u) sink[threadIdx.x] = accv;
}

__global__ void empty_kernel(int* p) {
  if (p != nullptr && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *p = 0;
}

int main() {
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  unsigned *ctr, *err;
  CK(hipMalloc(&ctr, 4096));
  CK(hipMalloc(&err, 4));
  uint4 *src, *sink;
  const size_t src_bytes = (size_t)64 * 1024 * 16 * 1024;  // 64 rounds x 1024 blocks x 16 KiB = 1 GiB
  CK(hipMalloc(&src, src_bytes));
  CK(hipMemset(src, 1, src_bytes));
  CK(hipMalloc(&sink, 4096 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, barrier_kernel, 256, 0));
  printf("{\"cus\": %d, \"occupancy_blocks_per_cu\": %d}\n", prop.multiProcessorCount, occ);
  // kernel-boundary reference: back-to-back empty launches, and back-to-back 256-block launches
  for (int blocks : {1, 256, 1024}) {
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, 0, nullptr);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, 0, nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"test\": \"empty_launch\", \"blocks\": %d, \"us_per_launch\": %.3f}\n", blocks, ms * 1e3f / 2000);
  }
  // same in a graph (the engine's decode step is one hipGraph)
  {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, nullptr);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"test\": \"graph_empty_launch\", \"blocks\": 256, \"us_per_node\": %.3f}\n", ms * 1e3f / 2000);
  }
  const int max_blocks = prop.multiProcessorCount * (occ < 4 ? occ : 4);
  for (int mode : {0, 1, 2}) {
    for (int blocks : {prop.multiProcessorCount, 2 * prop.multiProcessorCount, 4 * prop.multiProcessorCount}) {
      if (blocks > max_blocks || blocks > 1024) continue;
      const int rounds = 2000;
      float best = 1e30f;
      unsigned herr = 0;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(ctr, 0, 4096));
        CK(hipMemset(err, 0, 4));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(barrier_kernel, dim3(blocks), dim3(256), 0, 0, ctr, rounds, mode, err, src, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned e;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        herr += e;
        if (ms < best) best = ms;
      }
      printf("{\"test\": \"grid_barrier\", \"mode\": %d, \"blocks\": %d, \"us_per_barrier\": %.3f, \"errors\": %u}\n",
             mode, blocks, best * 1e3f / rounds, herr);
      fflush(stdout);
    }
  }
  return 0;
}
