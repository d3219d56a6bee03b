// Would a decode step run faster if each kernel started streaming its weights while the
// previous kernel drains? Models one Qwen2.5-1.5B decode layer x 28 as weight-streaming kernels
// with the engine's grid shapes (qkv 6.3 MB 128x512, attention 80x384 latency-only, o 4.7 MB
// 96x512, gate_up 55 MB 1120x128, down 27.5 MB 192x512):
//   mode 0: one stream, every kernel a graph node after the previous one (today's decode step)
//   mode 1: two streams alternating, K_n's graph edge is K_{n-2}; K_n issues its first two register
//           groups of weights, then waits (bounded sc1 poll) until every block of K_{n-1} has
//           published (sc1 stores -> vmcnt(0) -> agent atomic), then reads one 16-B word of K_{n-1}'s
//           output (the activation round trip) and consumes its weights
// Every spin is bounded (error count printed): a dependency that never arrives cannot hang.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/chain benchmarks/chain_overlap_probe.hip && /tmp/chain
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

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct KArgs {
  const char* w;          // weights of this kernel (nullptr: latency kernel)
  unsigned frags;         // 1 KiB fragments
  unsigned* done_prev;    // previous kernel's arrival counter (nullptr: no wait)
  unsigned prev_blocks;
  unsigned* done_me;
  float* out_prev;        // previous kernel's output (one 16-B word per block)
  float* out_me;
  unsigned* err;
};

constexpr unsigned kSpin = 1u << 22;

__device__ __forceinline__ unsigned ld_sc1_u32(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// poll through a returning atomic (executes at the memory side: never an L2-cached stale copy;
// a plain sc1 load poll kept reading a stale line of the poller's XCD L2 in this probe)
__device__ __forceinline__ unsigned poll_u32(unsigned* p) {
  return __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int U>
__global__ __launch_bounds__(512) void chain_kernel(KArgs a) {
  const int lane = threadIdx.x & 63;
  const unsigned nw = gridDim.x * (blockDim.x >> 6);
  const unsigned wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const unsigned f0 = a.w ? (unsigned)(((unsigned long long)a.frags * wv) / nw) : 0;
  const unsigned f1 = a.w ? (unsigned)(((unsigned long long)a.frags * (wv + 1)) / nw) : 0;
  const unsigned n = f1 - f0;
  const bf16x8 bx = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                     (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const u32x4* p = reinterpret_cast<const u32x4*>(a.w) + lane;
  u32x4 ra[U], rb[U];
  auto ld = [&](u32x4 (&r)[U], unsigned j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(p + (size_t)(f0 + min(j0 + u, n - 1)) * 64);
  };
  auto use = [&](const u32x4 (&r)[U], unsigned j0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (j0 + u < n) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r[u]), bx, acc, 0, 0, 0);
  };
  if (n > 0) {
    ld(ra, 0);
    ld(rb, U);
  }
  // dependency: every block of the previous kernel published
  float xin = 0.f;
  if (a.done_prev != nullptr) {
    unsigned spins = 0, v = 0;
    if (lane == 0) {
      while ((v = poll_u32(a.done_prev)) < a.prev_blocks && ++spins < kSpin) __builtin_amdgcn_s_sleep(2);
      if (spins >= kSpin) atomicAdd(a.err, 1u);
    }
    v = __builtin_amdgcn_readfirstlane(v);
    // the activation round trip: one word of the previous kernel's output
    xin = __uint_as_float(ld_sc1_u32(reinterpret_cast<const unsigned*>(a.out_prev) + (blockIdx.x * 4 + lane) % 256));
  }
  if (n > 0) {
    for (unsigned j = 0; j < n; j += 2 * U) {
      use(ra, j);
      if (j + 2 * U < n) ld(ra, j + 2 * U);
      use(rb, j + U);
      if (j + 3 * U < n) ld(rb, j + 3 * U);
    }
  } else {
    // latency kernel (attention stand-in): one more dependent round trip
    xin += __uint_as_float(ld_sc1_u32(reinterpret_cast<const unsigned*>(a.out_prev ? a.out_prev : a.out_me) + lane));
  }
  // publish: sc1 store of this block's word, drain, one arrival per block
  if (threadIdx.x < 4)
    __hip_atomic_store(reinterpret_cast<unsigned*>(a.out_me) + blockIdx.x * 4 + threadIdx.x,
                       __float_as_uint(acc[0] + xin), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && a.done_me != nullptr)
    __hip_atomic_fetch_add(a.done_me, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  CK(hipSetDevice(0));
  const int L = 28;
  struct K { size_t bytes; int blocks, threads; };
  const K layer[5] = {{6291456, 128, 512}, {0, 80, 384}, {4718592, 96, 512}, {55050240, 1120, 128}, {27525120, 192, 512}};
  size_t total = 0;
  for (int i = 0; i < 5; ++i) total += layer[i].bytes;
  char* w;
  CK(hipMalloc(&w, total * L + 4096));
  CK(hipMemset(w, 0x3c, total * L + 4096));
  const int NK = 5 * L;
  unsigned* ctr;
  float* outs;
  unsigned* err;
  CK(hipMalloc(&ctr, NK * 64 * sizeof(unsigned)));
  CK(hipMalloc(&outs, (size_t)NK * 8192 * sizeof(float)));
  CK(hipMalloc(&err, 64));
  CK(hipMemset(outs, 0, (size_t)NK * 8192 * sizeof(float)));
  std::vector<KArgs> ka(NK);
  size_t off = 0;
  for (int l = 0; l < L; ++l)
    for (int i = 0; i < 5; ++i) {
      const int k = 5 * l + i;
      ka[k].w = layer[i].bytes ? w + off : nullptr;
      ka[k].frags = (unsigned)(layer[i].bytes / 1024);
      off += layer[i].bytes;
      ka[k].done_me = ctr + 64 * k;
      ka[k].out_me = outs + (size_t)8192 * k;
      ka[k].err = err;
      ka[k].done_prev = nullptr;
      ka[k].out_prev = k > 0 ? outs + (size_t)8192 * (k - 1) : nullptr;
      ka[k].prev_blocks = k > 0 ? (unsigned)layer[(i + 4) % 5].blocks : 0;
    }
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ef, ej, e0, e1;
  CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int nk_env = getenv("CHAIN_NK") ? atoi(getenv("CHAIN_NK")) : NK;
  for (int mode = 0; mode < 4; ++mode) {
    // mode 2: alternating streams, no waits (concurrency only); mode 3: waits + a graph edge on
    // K_{n-1} too (the flags are always set already: protocol check, no overlap)
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    CK(hipMemsetAsync(ctr, 0, NK * 64 * sizeof(unsigned), s1));
    const bool two = mode == 1 || mode == 2;
    if (two) {
      CK(hipEventRecord(ef, s1));
      CK(hipStreamWaitEvent(s2, ef, 0));
    }
    for (int k = 0; k < nk_env; ++k) {
      KArgs a = ka[k];
      if ((mode == 1 || mode == 3) && k > 0) a.done_prev = ka[k - 1].done_me;
      hipStream_t s = (two && (k & 1)) ? s2 : s1;
      const K& kk = layer[k % 5];
      hipLaunchKernelGGL(chain_kernel<8>, dim3(kk.blocks), dim3(kk.threads), 0, s, a);
    }
    if (two) {
      CK(hipEventRecord(ej, s2));
      CK(hipStreamWaitEvent(s1, ej, 0));
    }
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float best = 1e30f;
    unsigned herr = 0;
    for (int rep = 0; rep < 8; ++rep) {
      CK(hipMemsetAsync(err, 0, 64, s1));
      CK(hipEventRecord(e0, s1));
      CK(hipGraphLaunch(ge, s1));
      CK(hipEventRecord(e1, s1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned e;
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      herr += e;
      if (rep > 1 && ms < best) best = ms;
      if (e) {
        std::vector<unsigned> hc(NK * 64);
        CK(hipMemcpy(hc.data(), ctr, NK * 64 * sizeof(unsigned), hipMemcpyDeviceToHost));
        printf("{\"mode\": %d, \"arrivals\": [", mode);
        for (int k = 0; k < nk_env && k < 20; ++k) printf("%s%u/%d", k ? ", " : "", hc[64 * k], layer[k % 5].blocks);
        printf("]}\n");
        break;
      }
    }
    printf("{\"mode\": %d, \"kernels\": %d, \"ms\": %.4f, \"us_per_layer\": %.2f, \"errors\": %u}\n", mode, nk_env, best,
           best * 1e3f * 5 / nk_env, herr);
    fflush(stdout);
  }
  return 0;
}
