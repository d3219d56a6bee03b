// Which part of the decode GEMM's weight stream costs time? (MI355X, gfx950)
//
// The bf16 decode GEMM of a Qwen2.5-1.5B gate_up projection (M = 8, N = 17920, K = 1536: 1120 column
// tiles x 48 k-steps of 1 KiB fragment-packed weights, 55 MB) runs at ~4.5 TB/s over its span while a
// plain read sweep of the same bytes reaches ~6.4 TB/s (mall_stream_probe). This probe streams the
// same 55 MB in the GEMM's own shapes — cold (a ring of copies > 1 GiB), no MFMA — to price each
// structural choice separately:
//   layout  contig : wave w of a tile block streams k-steps [w*KW, (w+1)*KW) (the GEMM today)
//           inter  : wave w streams k-steps w, w+nw, w+2nw, ... (the block's waves advance side by side)
//   waves   per tile block (1 tile per block: 1120 blocks)
//   act     one extra L2-resident 16-B "activation" load per 2 weight loads (the GEMM's XP = 2 B operand)
//   U       k-steps per register group (two groups in flight, ping-pong, as the GEMM)
// Time = graph of R launches / R (includes the ~1.5 us launch boundary).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/decode_stream_probe benchmarks/probes/decode_stream_probe.hip
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

__device__ __forceinline__ u32x4 ldnt(const u32x4* p) { return __builtin_nontemporal_load(p); }

// one tile per block: KT k-steps of 64 lanes x 16 B; NW waves; U-deep groups, two in flight
template <int U, bool INTER, bool ACT>
__global__ __launch_bounds__(512) void tile_stream(const u32x4* __restrict__ w, const u32x4* __restrict__ x, int KT,
                                                   unsigned* sink) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const u32x4* base = w + (size_t)blockIdx.x * KT * 64 + lane;
  // this wave's k-steps: contig = [k0, k1); inter = wid, wid + nw, ...
  const int per = (KT + nw - 1) / nw;
  const int k0 = INTER ? 0 : wid * per;
  const int n = INTER ? (KT - wid + nw - 1) / nw : (min(KT, k0 + per) - k0);
  auto kstep = [&](int i) { return INTER ? wid + i * nw : k0 + i; };
  unsigned acc = 0;
  u32x4 a[U], b[U], xa[U], xb[U];
  auto load = [&](u32x4 (&r)[U], u32x4 (&xr)[U], int g) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(g * U + u, n - 1);
      r[u] = ldnt(base + (size_t)kstep(i) * 64);
      if (ACT && (u & 1) == 0) xr[u] = x[(kstep(i) * 64 + lane) & 1023];
    }
  };
  auto use = [&](const u32x4 (&r)[U], const u32x4 (&xr)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc ^= r[u][0] ^ r[u][3];
      if (ACT && (u & 1) == 0) acc += xr[u][1];
    }
  };
  const int ng = (n + U - 1) / U;
  if (ng > 0) {
    load(a, xa, 0);
    int g = 0;
    for (; g + 2 <= ng; g += 2) {
      load(b, xb, g + 1);
      use(a, xa);
      if (g + 2 < ng) load(a, xa, g + 2);
      use(b, xb);
    }
    if (g < ng) use(a, xa);
  }
  if (acc == 0x9E3779B9u && sink != nullptr) *sink = acc;
}

template <int U, bool INTER, bool ACT>
void run(const char* name, char* base, size_t stride, int ncopy, const u32x4* x, unsigned* sink, int ntiles, int KT,
         int nw, hipStream_t st) {
  const int R = 20;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < R; ++r)
    hipLaunchKernelGGL((tile_stream<U, INTER, ACT>), dim3(ntiles), dim3(64 * nw), 0, st,
                       reinterpret_cast<const u32x4*>(base + (size_t)(r % ncopy) * stride), x, KT, sink);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double us = 1e3 * best / R;
  const double bytes = (double)ntiles * KT * 1024;
  printf("{\"probe\": \"%s\", \"tiles\": %d, \"KT\": %d, \"waves\": %d, \"U\": %d, \"inter\": %d, \"act\": %d, "
         "\"us_per_launch\": %.2f, \"tb_s\": %.2f}\n",
         name, ntiles, KT, nw, U, (int)INTER, (int)ACT, us, bytes / us / 1e6);
  fflush(stdout);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
}

int main() {
  const size_t ring = (size_t)1400 << 20;
  char* base = nullptr;
  CK(hipMalloc(&base, ring));
  CK(hipMemset(base, 1, ring));
  u32x4* x = nullptr;
  CK(hipMalloc(&x, 1024 * 16));
  CK(hipMemset(x, 2, 1024 * 16));
  unsigned* sink = nullptr;
  CK(hipMalloc(&sink, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Shape { const char* name; int ntiles, KT; };
  const Shape shapes[] = {{"gate_up", 1120, 48}, {"down_as_tiles", 96 * 2, 140}};
  for (const Shape& s : shapes) {
    const size_t bytes = (size_t)s.ntiles * s.KT * 1024;
    const size_t stride = (bytes + 65535) / 65536 * 65536;
    const int ncopy = (int)(ring / stride);
    for (int nw : {2, 4, 8}) {
      run<8, false, true>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);   // the GEMM today (nw 2)
      run<8, false, false>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);
      run<8, true, true>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);
      run<8, true, false>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);
      run<4, false, true>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);
      run<4, true, true>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);
      run<2, true, true>(s.name, base, stride, ncopy, x, sink, s.ntiles, s.KT, nw, st);
    }
  }
  CK(hipFree(base));
  return 0;
}
