// Where does a decode GEMM's weight stream come from, and how fast? (MI355X, gfx950)
//
// Streams S bytes with a grid-stride 16-B-per-lane read sweep (4 loads in flight per thread per
// iteration) in three cache states, timed as a hipGraph of R launches (time per launch):
//   cold  : launch i reads copy i of a ring of copies > 1 GiB in all (every launch misses L2 and the
//           256 MiB Infinity Cache / MALL);
//   mall  : every launch reads the SAME copy, block b starting at the chunk block b+1 read last time
//           (another XCD: its L2 misses, the die-level MALL holds the bytes);
//   l2    : the same copy with the same block -> chunk mapping every launch (XCD L2 hits where the
//           copy fits in 8 x 4 MiB).
// Loads: default policy or nontemporal (nt). The answer decides whether warming the MALL for the
// next bandwidth-bound kernel (on the CUs a latency-bound kernel leaves idle) can pay.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/mall_stream_probe benchmarks/probes/mall_stream_probe.hip
//   build/mall_stream_probe   -> one JSON line per (bytes, blocks, policy, state)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// chunk-contiguous sweep: block b streams chunk (b + rot) % nblk of the buffer
template <bool NT>
__global__ __launch_bounds__(256) void sweep(const u32x4* __restrict__ p, size_t n16, int rot, unsigned* sink) {
  const int nb = gridDim.x;
  const int b = (blockIdx.x + rot) % nb;
  const size_t per = (n16 + nb - 1) / nb;
  const size_t lo = (size_t)b * per, hi = lo + per < n16 ? lo + per : n16;
  unsigned acc = 0;
  size_t i = lo + threadIdx.x;
  for (; i + 3 * 256 < hi; i += 4 * 256) {
    const u32x4 a = ld<NT>(p + i), c = ld<NT>(p + i + 256), d = ld<NT>(p + i + 512), e = ld<NT>(p + i + 768);
    acc ^= a[0] ^ c[1] ^ d[2] ^ e[3];
  }
  for (; i < hi; i += 256) acc ^= ld<NT>(p + i)[0];
  if (acc == 0x9E3779B9u && sink != nullptr) *sink = acc;
}

int main() {
  const size_t sizes[] = {55050240, 27525120, 6291456};  // Qwen2.5-1.5B gate_up / down / qkv weights (bf16)
  const int blocks_list[] = {256, 512, 1024, 2048};
  const int R = 20;
  const size_t ring_bytes = (size_t)1400 << 20;
  char* base = nullptr;
  CK(hipMalloc(&base, ring_bytes));
  CK(hipMemset(base, 1, ring_bytes));
  unsigned* sink = nullptr;
  CK(hipMalloc(&sink, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t S : sizes) {
    const size_t n16 = S / 16;
    const size_t stride = (S + 4095) / 4096 * 4096;
    const int ncopy = (int)(ring_bytes / stride);
    for (int nb : blocks_list) {
      for (int nt = 0; nt < 2; ++nt) {
        for (int state = 0; state < 3; ++state) {  // 0 cold, 1 mall, 2 l2
          hipGraph_t g;
          hipGraphExec_t ge;
          CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
          for (int r = 0; r < R; ++r) {
            const int copy = state == 0 ? (r % ncopy) : 0;
            const int rot = state == 1 ? r : 0;
            const u32x4* p = reinterpret_cast<const u32x4*>(base + (size_t)copy * stride);
            if (nt) hipLaunchKernelGGL(sweep<true>, dim3(nb), dim3(256), 0, st, p, n16, rot, sink);
            else hipLaunchKernelGGL(sweep<false>, dim3(nb), dim3(256), 0, st, p, n16, rot, sink);
          }
          CK(hipStreamEndCapture(st, &g));
          CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
          float best = 1e30f;
          for (int rep = 0; rep < 5; ++rep) {
            if (state != 0) {  // warm the shared copy first
              hipLaunchKernelGGL(sweep<false>, dim3(nb), dim3(256), 0, st,
                                 reinterpret_cast<const u32x4*>(base), n16, 0, sink);
            }
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
          }
          const double us = 1e3 * best / R;
          printf("{\"bytes\": %zu, \"blocks\": %d, \"nt\": %d, \"state\": \"%s\", \"us_per_launch\": %.2f, \"tb_s\": %.2f}\n",
                 S, nb, nt, state == 0 ? "cold" : state == 1 ? "mall" : "l2", us, S / us / 1e6);
          fflush(stdout);
          CK(hipGraphExecDestroy(ge));
          CK(hipGraphDestroy(g));
        }
      }
    }
  }
  CK(hipFree(base));
  return 0;
}
