// Do independent branches of a hipGraph run concurrently on gfx950 / ROCm 7.2?
// Kernels stamp [start, end] (s_memrealtime, 100 MHz) of block 0; printed relative to kernel 0.
//   A: eager, two streams, two 30 us kernels
//   B: hipGraph, fork / join (two branches, one kernel each)
//   C: hipGraph chain of 8 kernels alternating two streams, K_n depends only on K_{n-2}
//      (the pattern a "next kernel prefetches while the previous one drains" decode step needs)
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ovl benchmarks/overlap_probe.hip && /tmp/ovl
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

__global__ void spin_kernel(unsigned long long* st, int id, int ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) st[2 * id] = t0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(2);
  if (blockIdx.x == 0 && threadIdx.x == 0) st[2 * id + 1] = __builtin_amdgcn_s_memrealtime();
}

static void report(const char* name, unsigned long long* d, int n) {
  unsigned long long h[64];
  CK(hipMemcpy(h, d, 2 * n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  printf("{\"test\": \"%s\", \"kernels\": [", name);
  for (int i = 0; i < n; ++i)
    printf("%s[%.2f, %.2f]", i ? ", " : "", (h[2 * i] - h[0]) / 100.0, (h[2 * i + 1] - h[0]) / 100.0);
  int overl = 0;
  for (int i = 1; i < n; ++i) overl += h[2 * i] < h[2 * (i - 1) + 1];
  printf("], \"overlapping_pairs\": %d}\n", overl);
  fflush(stdout);
}

int main() {
  CK(hipSetDevice(0));
  unsigned long long* st;
  CK(hipMalloc(&st, 4096));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int T = 3000;  // 30 us
  const int blocks = 64;
  // A: eager
  CK(hipMemset(st, 0, 4096));
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s1, st, 0, T);
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s2, st, 1, T);
  CK(hipDeviceSynchronize());
  report("eager_two_streams", st, 2);
  // B: graph fork / join
  hipEvent_t ef, ej;
  CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(ef, s1));
    CK(hipStreamWaitEvent(s2, ef, 0));
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s1, st, 0, T);
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s2, st, 1, T);
    CK(hipEventRecord(ej, s2));
    CK(hipStreamWaitEvent(s1, ej, 0));
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemsetAsync(st, 0, 4096, s1));
      CK(hipGraphLaunch(ge, s1));
      CK(hipStreamSynchronize(s1));
      report("graph_fork_join", st, 2);
    }
  }
  // C: alternating chain, K_n depends on K_{n-2} only
  {
    const int N = 8;
    hipEvent_t ev[N];
    for (int i = 0; i < N; ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(ef, s1));
    CK(hipStreamWaitEvent(s2, ef, 0));
    for (int n = 0; n < N; ++n) {
      hipStream_t s = (n & 1) ? s2 : s1;
      hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s, st, n, T);
    }
    CK(hipEventRecord(ej, s2));
    CK(hipStreamWaitEvent(s1, ej, 0));
    CK(hipStreamEndCapture(s1, &g));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    printf("{\"chain_graph_nodes\": %zu}\n", nn);
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemsetAsync(st, 0, 4096, s1));
      CK(hipGraphLaunch(ge, s1));
      CK(hipStreamSynchronize(s1));
      report("graph_alternating_chain", st, N);
    }
  }
  return 0;
}
