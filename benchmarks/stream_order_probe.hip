// Does the ORDER in which the decode GEMM's waves walk the weight matrix limit HBM bandwidth?
//
// The decode GEMMs give every wave a contiguous fragment range (tile-major packing: a tile's K is
// contiguous), so at any instant ~2000 waves each read 1 KiB at ~24 KiB-strided positions all over
// the matrix. A float4 copy kernel (6.3 TB/s) reads a contiguous window instead. This probe streams
// the same bytes through register groups + one MFMA per fragment (as gemm_kernel does) in two orders:
//   order 0: wave w reads fragments [w F / NW, (w + 1) F / NW)       (today's layout)
//   order 1: wave w reads fragments w, w + NW, w + 2 NW, ...          (step-major: a contiguous
//            NW KiB window per step across the chip)
// for the Qwen2.5-1.5B gate_up (55 MB) and down (27.5 MB) sizes and the LM head (466 MB), 28
// launches per graph on 28 different copies (1.5 GB: no MALL reuse), per grid shape.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sorder benchmarks/stream_order_probe.hip && /tmp/sorder
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

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void stream_kernel(const char* base, unsigned frags, int order, float* sink) {
  const int lane = threadIdx.x & 63;
  const unsigned nw = gridDim.x * (blockDim.x >> 6);
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  unsigned f0, f1, stride;
  if (order == 0) {
    f0 = (unsigned)(((unsigned long long)frags * w) / nw);
    f1 = (unsigned)(((unsigned long long)frags * (w + 1)) / nw);
    stride = 1;
  } else {
    f0 = w;
    f1 = frags;
    stride = nw;
  }
  const unsigned n = f1 > f0 ? (f1 - f0 + stride - 1) / stride : 0;
  const bf16x8 bx = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                     (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const u32x4* p = reinterpret_cast<const u32x4*>(base) + lane;
  auto ld = [&](u32x4 (&r)[U], unsigned j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned j = min(j0 + u, n - 1);
      r[u] = __builtin_nontemporal_load(p + (size_t)(f0 + j * stride) * 64);
    }
  };
  auto use = [&](const u32x4 (&r)[U], unsigned j0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (j0 + u < n) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r[u]), bx, acc, 0, 0, 0);
  };
  if (n > 0) {
    u32x4 a[U], b[U];
    ld(a, 0);
    for (unsigned j = 0; j < n; j += 2 * U) {
      ld(b, j + U);
      use(a, j);
      if (j + 2 * U < n) ld(a, j + 2 * U);
      use(b, j + U);
    }
  }
  if (acc[0] == 1234.5f) sink[threadIdx.x] = acc[1];
}

int main() {
  CK(hipSetDevice(0));
  const size_t sizes[3] = {55050240, 27525120, 466747392};
  const char* names[3] = {"gate_up", "down", "lm_head"};
  const int L = 28;
  char* buf;
  const size_t cap = (size_t)1600 << 20;
  CK(hipMalloc(&buf, cap));
  CK(hipMemset(buf, 0x3c, cap));
  float* sink;
  CK(hipMalloc(&sink, 4096));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int k = 0; k < 3; ++k) {
    const size_t sz = sizes[k];
    const int copies = (int)((cap / sz) < (size_t)L ? cap / sz : L);
    const unsigned frags = (unsigned)(sz / 1024);
    for (int cfg = 0; cfg < 4; ++cfg) {
      const int blocks = cfg == 0 ? 512 : cfg == 1 ? 1024 : cfg == 2 ? 2048 : 4096;
      const int thr = 256;
      for (int order = 0; order < 2; ++order) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int l = 0; l < L; ++l)
          hipLaunchKernelGGL(stream_kernel<8>, dim3(blocks), dim3(thr), 0, s, buf + (size_t)(l % copies) * sz, frags,
                             order, sink);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        float best = 1e30f;
        for (int rep = 0; rep < 6; ++rep) {
          CK(hipEventRecord(e0, s));
          CK(hipGraphLaunch(ge, s));
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (rep > 0 && ms < best) best = ms;
        }
        printf("{\"op\": \"%s\", \"mb\": %.1f, \"copies\": %d, \"blocks\": %d, \"threads\": %d, \"order\": %d, "
               "\"us_per_launch\": %.2f, \"tb_s\": %.2f}\n",
               names[k], sz / 1e6, copies, blocks, thr, order, best * 1e3f / L, sz * L / (best * 1e-3) / 1e12);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
    }
  }
  return 0;
}
