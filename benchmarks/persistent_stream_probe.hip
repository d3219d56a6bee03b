// Decode-step skeleton on gfx950: does ONE persistent kernel that streams every layer's weights
// through an LDS-DMA ring (glds16), joins phases with a hierarchical grid barrier and keeps the
// NEXT phase's weight chunks in flight across that barrier beat one graph node per op?
//
// Phases per layer = the Qwen2.5-1.5B decode ops: qkv 6.3 MB, attention (no weights: one
// dependent round trip), o_proj 4.7 MB, gate_up 55.1 MB, down 27.5 MB; 28 layers (2.6 GB).
// Every 1 KiB weight fragment is read from LDS once and fed to one 16x16x32 MFMA, as the decode
// GEMM does for M <= 16.
//
//   mode 0: one kernel per phase, captured in a hipGraph (the engine's structure today)
//   mode 1: persistent, ring drained at every phase end (barrier cost, no overlap)
//   mode 2: persistent, chunks of the next phase issued before the barrier (overlap)
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/pstream benchmarks/persistent_stream_probe.hip && /tmp/pstream
//
// Every spin is bounded and a block that times out leaves (error count printed): the grid drains.
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

constexpr int NT = 512;       // 8 waves
constexpr int NW = NT / 64;
constexpr int CH = 16;        // fragments (1 KiB) per chunk: 2 per wave
constexpr int R = 8;          // ring slots (128 KiB)
constexpr unsigned kSpin = 1u << 22;

struct Phase {
  const char* base;
  unsigned frags;  // 0: a latency phase (attention stand-in)
};

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_addr) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_agent(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// this block's fragment range of a phase
__device__ __forceinline__ void frag_range(const Phase& ph, unsigned& f0, unsigned& f1) {
  const unsigned nb = gridDim.x, b = blockIdx.x;
  f0 = (unsigned)(((unsigned long long)ph.frags * b) / nb);
  f1 = (unsigned)(((unsigned long long)ph.frags * (b + 1)) / nb);
}

// hierarchical grid barrier (per-XCD counter, last arriver bumps the global one); returns false
// on timeout. `gen` = number of barriers passed so far + 1.
__device__ bool grid_barrier(unsigned* ctr, unsigned gen, unsigned* err) {
  __shared__ int ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nb = gridDim.x, x = blockIdx.x & 7;
    const unsigned per = (unsigned)((nb - x + 7) / 8);
    unsigned* xc = ctr + 64 + 16 * x;
    const unsigned old = add_agent(xc, 1);
    if (old + 1 == per * gen) add_agent(ctr, 1);
    unsigned n = 0;
    while (ld_agent(ctr) < 8u * gen && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
    ok = n < kSpin;
    if (!ok) atomicAdd(err, 1u);
  }
  __syncthreads();
  return ok;
}

// stream phases [p0, p1) of `ph` through the ring; mode 2 lets chunk issue run ahead across
// phase boundaries, mode 0/1 drain at each phase end. Returns false if a barrier timed out.
__device__ bool run_phases(const Phase* ph, int p0, int p1, int mode, unsigned* ctr, unsigned* err,
                           unsigned& gen, f32x4& acc, char* ring) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bf16x8 bx = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                     (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  // issue cursor (phase, next fragment) and consume cursor
  int ip = p0;
  unsigned if0 = 0, if1 = 0;
  if (ip < p1) frag_range(ph[ip], if0, if1);
  int issued = 0, consumed = 0;
  // chunk descriptors of the in-flight ring: phase index and fragment count per slot
  __shared__ int slot_phase[R];
  __shared__ unsigned slot_n[R];
  auto issue_one = [&](int limit_phase) -> bool {
    // advance past empty / latency phases
    while (ip < p1 && (ph[ip].frags == 0 || if0 >= if1)) {
      if (ip >= limit_phase) return false;
      ++ip;
      if (ip < p1) frag_range(ph[ip], if0, if1);
    }
    if (ip >= p1 || ip > limit_phase) return false;
    const unsigned n = min((unsigned)CH, if1 - if0);
    const int s = issued % R;
    char* dst = ring + (size_t)s * CH * 1024;
#pragma unroll
    for (int j = 0; j < CH / NW; ++j) {
      const unsigned idx = wid * (CH / NW) + j;
      const unsigned f = if0 + min(idx, n - 1);  // clamped duplicate: uniform vmcnt per chunk
      glds16(ph[ip].base + (size_t)f * 1024 + lane * 16,
             __builtin_amdgcn_readfirstlane(lds_addr_of(dst + idx * 1024)));
    }
    if (threadIdx.x == 0) {
      slot_phase[s] = ip;
      slot_n[s] = n;
    }
    if0 += n;
    ++issued;
    return true;
  };
  // the phase the issue cursor may run ahead to
  int cur = p0;
  auto limit = [&]() { return mode == 2 ? p1 - 1 : cur; };
  while (issued < R && issue_one(limit())) {}
  for (cur = p0; cur < p1; ++cur) {
    if (ph[cur].frags == 0) {
      // attention stand-in: one dependent global round trip per block
      const unsigned* q = reinterpret_cast<const unsigned*>(ph[cur - 1].base) + blockIdx.x * 64 + lane;
      unsigned v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      acc[0] += (float)(v & 1);
    } else {
      unsigned f0, f1;
      frag_range(ph[cur], f0, f1);
      const int nch = (int)((f1 - f0 + CH - 1) / CH);
      for (int c = 0; c < nch; ++c) {
        // chunks in flight after `consumed`: issued - consumed; wait for the oldest
        const int ahead = issued - consumed - 1;
        if (ahead >= 7) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        else if (ahead == 6) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else if (ahead == 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else if (ahead == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (ahead == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if (ahead == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // + slot_n written by thread 0
        const int s = consumed % R;
        const unsigned n = slot_n[s];
        const char* src = ring + (size_t)s * CH * 1024;
#pragma unroll
        for (int j = 0; j < CH / NW; ++j) {
          const unsigned idx = wid * (CH / NW) + j;
          if (idx < n) {
            const u32x4 w = *reinterpret_cast<const u32x4*>(src + idx * 1024 + lane * 16);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w), bx, acc, 0, 0, 0);
          }
        }
        ++consumed;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // slot free for reuse
        issue_one(limit());
      }
    }
    if (cur + 1 < p1 && mode != 0) {
      if (!grid_barrier(ctr, ++gen, err)) return false;
      if (mode == 1)
        while (issued < consumed + R && issue_one(cur + 1)) {}
    }
  }
  return true;
}

__global__ __launch_bounds__(NT, 1) void stream_kernel(const Phase* ph, int p0, int p1, int mode, unsigned* ctr,
                                                       unsigned* err, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char ring[];
  unsigned gen = 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  run_phases(ph, p0, p1, mode, ctr, err, gen, acc, ring);
  if (acc[0] == 1234.5f) sink[threadIdx.x] = acc[1];
}


// ---- register-pipelined variant: every wave streams ITS OWN fragment range (a decode GEMM's
// weight fragment feeds exactly one MFMA of one wave, so no LDS sharing is needed) with a
// ping-pong pair of U-fragment register groups. Groups never span phases; in mode 2 the group
// after a phase's last one (the next phase's first) is issued before the grid barrier.
struct WCur {
  int p;
  unsigned f, f1;
};

__device__ __forceinline__ void wave_range(const Phase& ph, unsigned& f0, unsigned& f1) {
  unsigned b0, b1;
  frag_range(ph, b0, b1);
  const unsigned w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  f0 = b0 + ((b1 - b0) * w) / nw;
  f1 = b0 + ((b1 - b0) * (w + 1)) / nw;
}

template <int U>
__device__ __forceinline__ int load_group(const Phase* ph, int p1, int limit, WCur& c, u32x4 (&r)[U], unsigned& nv) {
  const int lane = threadIdx.x & 63;
  while (c.f >= c.f1 && c.p < limit) {  // next phase with weights (latency phases have none)
    ++c.p;
    if (c.p < p1) wave_range(ph[c.p], c.f, c.f1);
    else c.f = c.f1 = 0;
  }
  if (c.f >= c.f1) {
    nv = 0;
    return -1;
  }
  nv = min((unsigned)U, c.f1 - c.f);
  const char* base = ph[c.p].base;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const unsigned f = c.f + min((unsigned)u, nv - 1);
    r[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)f * 1024) + lane);
  }
  c.f += nv;
  return c.p;
}

template <int U>
__global__ __launch_bounds__(NT) void reg_stream_kernel(const Phase* ph, int p0, int p1, int mode, unsigned* ctr,
                                                           unsigned* err, float* sink) {
  const bf16x8 bx = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                     (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  unsigned gen = 0;
  WCur c{p0, 0, 0};
  wave_range(ph[p0], c.f, c.f1);
  int cur = p0;  // phase being computed
  u32x4 ra[U], rb[U];
  unsigned na = 0, nb2 = 0;
  bool fail = false;
  auto consume = [&](const u32x4 (&r)[U], unsigned n) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if ((unsigned)u < n) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r[u]), bx, acc, 0, 0, 0);
  };
  // advance `cur` to phase `to`, running the barriers (and latency phases) in between
  auto goto_phase = [&](int to) {
    while (cur < to && !fail) {
      if (mode != 0) fail = !grid_barrier(ctr, ++gen, err);
      ++cur;
      if (ph[cur].frags == 0) {
        const unsigned* q = reinterpret_cast<const unsigned*>(ph[cur - 1].base) + blockIdx.x * 64 + (threadIdx.x & 63);
        acc[1] += (float)(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1);
      }
    }
  };
  auto stream = [&](int limit) {
    int pa = load_group<U>(ph, p1, limit, c, ra, na);
    while (pa >= 0 && !fail) {
      const int pb = load_group<U>(ph, p1, limit, c, rb, nb2);
      goto_phase(pa);
      consume(ra, na);
      if (pb < 0) break;
      pa = load_group<U>(ph, p1, limit, c, ra, na);
      goto_phase(pb);
      consume(rb, nb2);
    }
  };
  if (mode == 1) {  // no overlap: a phase's loads are issued only after its barrier
    for (int p = p0; p < p1 && !fail; ++p) {
      goto_phase(p);
      if (ph[p].frags == 0) continue;
      c.p = p;
      wave_range(ph[p], c.f, c.f1);
      stream(p);
    }
  } else {
    stream(p1 - 1);
  }
  if (!fail) goto_phase(p1 - 1);
  if (acc[0] == 1234.5f) sink[threadIdx.x] = acc[1];
}

// mode 3: persistent, 8 streaming waves + 1 dedicated sync wave. The streaming waves join a
// phase barrier with a bare s_barrier (no fence: their next-phase loads stay in flight); only
// the sync wave, which has no loads outstanding, runs the device-scope arrive / poll.
template <int U>
__global__ __launch_bounds__(NT + 64) void reg_stream_sync_kernel(const Phase* ph, int p0, int p1, unsigned* ctr,
                                                                  unsigned* err, float* sink) {
  __shared__ int fail_s;
  const int wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) fail_s = 0;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const int nbar = p1 - 1 - p0;
  if (wid == NW) {  // sync wave
    for (int g = 1; g <= nbar; ++g) {
      asm volatile("s_barrier" ::: "memory");  // streaming waves finished phase g-1
      if ((threadIdx.x & 63) == 0) {
        const int nb = gridDim.x, x = blockIdx.x & 7;
        const unsigned per = (unsigned)((nb - x + 7) / 8);
        unsigned* xc = ctr + 64 + 16 * x;
        const unsigned old = add_agent(xc, 1);
        if (old + 1 == per * (unsigned)g) add_agent(ctr, 1);
        unsigned n = 0;
        while (ld_agent(ctr) < 8u * (unsigned)g && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
        if (n >= kSpin) {
          atomicAdd(err, 1u);
          fail_s = 1;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // release
      if (fail_s) break;  // the streaming waves leave too: nobody waits on a dead barrier
    }
    return;
  }
  const bf16x8 bx = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                     (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // wave ranges computed over the 8 streaming waves only
  auto wrange = [&](const Phase& ph_, unsigned& f0, unsigned& f1) {
    unsigned b0, b1;
    frag_range(ph_, b0, b1);
    f0 = b0 + ((b1 - b0) * wid) / NW;
    f1 = b0 + ((b1 - b0) * (wid + 1)) / NW;
  };
  const int lane = threadIdx.x & 63;
  int cp = p0;
  unsigned cf = 0, cf1 = 0;
  wrange(ph[p0], cf, cf1);
  auto load = [&](u32x4 (&r)[U], unsigned& nv) -> int {
    while (cf >= cf1 && cp < p1 - 1) {
      ++cp;
      wrange(ph[cp], cf, cf1);
    }
    if (cf >= cf1) {
      nv = 0;
      return -1;
    }
    nv = min((unsigned)U, cf1 - cf);
    const char* base = ph[cp].base;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned f = cf + min((unsigned)u, nv - 1);
      r[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)f * 1024) + lane);
    }
    cf += nv;
    return cp;
  };
  int cur = p0;
  bool fail = false;
  auto goto_phase = [&](int to) {
    while (cur < to && !fail) {
      asm volatile("s_barrier" ::: "memory");                          // arrive (loads stay in flight)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // released by the sync wave
      fail = fail_s != 0;
      ++cur;
      if (ph[cur].frags == 0) {
        const unsigned* q = reinterpret_cast<const unsigned*>(ph[cur - 1].base) + blockIdx.x * 64 + lane;
        acc[1] += (float)(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1);
      }
    }
  };
  auto consume = [&](const u32x4 (&r)[U], unsigned n) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if ((unsigned)u < n) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r[u]), bx, acc, 0, 0, 0);
  };
  u32x4 ra[U], rb[U];
  unsigned na = 0, nb2 = 0;
  int pa = load(ra, na);
  while (pa >= 0 && !fail) {
    const int pb = load(rb, nb2);
    goto_phase(pa);
    consume(ra, na);
    if (pb < 0) break;
    pa = load(ra, na);
    goto_phase(pb);
    consume(rb, nb2);
  }
  goto_phase(p1 - 1);  // every streaming wave takes part in all nbar barriers
  if (acc[0] == 1234.5f) sink[threadIdx.x] = acc[1];
}

int main() {
  CK(hipSetDevice(0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int L = 28;
  const size_t sz[5] = {6291456, 0, 4718592, 55050240, 27525120};
  const char* names[5] = {"qkv", "attn", "o", "gate_up", "down"};
  size_t total = 0;
  for (int i = 0; i < 5; ++i) total += sz[i];
  total *= L;
  char* w;
  CK(hipMalloc(&w, total + 4096));
  CK(hipMemset(w, 0x3c, total + 4096));
  std::vector<Phase> hp;
  size_t off = 0;
  for (int l = 0; l < L; ++l)
    for (int i = 0; i < 5; ++i) {
      hp.push_back(Phase{w + off, (unsigned)(sz[i] / 1024)});
      off += sz[i];
    }
  Phase* dph;
  CK(hipMalloc(&dph, hp.size() * sizeof(Phase)));
  CK(hipMemcpy(dph, hp.data(), hp.size() * sizeof(Phase), hipMemcpyHostToDevice));
  unsigned *ctr, *err;
  float* sink;
  CK(hipMalloc(&ctr, 4096));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&sink, 4096));
  const size_t lds = (size_t)R * CH * 1024;
  CK(hipFuncSetAttribute((const void*)stream_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, stream_kernel, NT, lds));
  const int nb = prop.multiProcessorCount;
  printf("{\"cus\": %d, \"occupancy\": %d, \"weights_gb\": %.3f}\n", nb, occ, total / 1e9);
  if (occ < 1) return 1;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int P = (int)hp.size();
  for (int mode : {0, 1, 2}) {
    hipGraphExec_t ge = nullptr;
    if (mode == 0) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int p = 0; p < P; ++p) {
        if (hp[p].frags == 0) continue;  // the attention stand-in needs a kernel of its own: add below
        hipLaunchKernelGGL(stream_kernel, dim3(nb), dim3(NT), lds, s, dph, p, p + 1, 0, ctr, err, sink);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    float best = 1e30f;
    unsigned herr = 0;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipMemsetAsync(ctr, 0, 4096, s));
      CK(hipMemsetAsync(err, 0, 4, s));
      CK(hipEventRecord(e0, s));
      if (mode == 0) CK(hipGraphLaunch(ge, s));
      else hipLaunchKernelGGL(stream_kernel, dim3(nb), dim3(NT), lds, s, dph, 0, P, mode, ctr, err, sink);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned e;
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      herr += e;
      if (rep > 0 && ms < best) best = ms;
      if (e) break;
    }
    printf("{\"mode\": %d, \"ms_28_layers\": %.4f, \"us_per_layer\": %.2f, \"tb_s\": %.2f, \"errors\": %u}\n", mode, best,
           best * 1e3f / L, total / (best * 1e-3) / 1e12, herr);
    fflush(stdout);
    if (herr) return 2;
  }
  for (int v = 0; v < 2; ++v)
    for (int mode : {0, 1, 2}) {
      auto kern = v == 0 ? reg_stream_kernel<8> : reg_stream_kernel<16>;
      hipGraphExec_t ge = nullptr;
      if (mode == 0) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int p = 0; p < P; ++p) {
          if (hp[p].frags == 0) continue;
          hipLaunchKernelGGL(kern, dim3(nb), dim3(NT), 0, s, dph, p, p + 1, 0, ctr, err, sink);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      }
      float best = 1e30f;
      unsigned herr = 0;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipMemsetAsync(ctr, 0, 4096, s));
        CK(hipMemsetAsync(err, 0, 4, s));
        CK(hipEventRecord(e0, s));
        if (mode == 0) CK(hipGraphLaunch(ge, s));
        else hipLaunchKernelGGL(kern, dim3(nb), dim3(NT), 0, s, dph, 0, P, mode, ctr, err, sink);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned e;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        herr += e;
        if (rep > 0 && ms < best) best = ms;
        if (e) break;
      }
      printf("{\"variant\": \"regs_U%d\", \"mode\": %d, \"ms_28_layers\": %.4f, \"us_per_layer\": %.2f, \"tb_s\": %.2f, "
             "\"errors\": %u}\n", v == 0 ? 8 : 16, mode, best, best * 1e3f / L, total / (best * 1e-3) / 1e12, herr);
      fflush(stdout);
      if (herr) return 2;
    }
  for (int v = 0; v < 2; ++v) {
    auto kern = v == 0 ? reg_stream_sync_kernel<8> : reg_stream_sync_kernel<16>;
    float best = 1e30f;
    unsigned herr = 0;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipMemsetAsync(ctr, 0, 4096, s));
      CK(hipMemsetAsync(err, 0, 4, s));
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(kern, dim3(nb), dim3(NT + 64), 0, s, dph, 0, P, ctr, err, sink);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned e;
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      herr += e;
      if (rep > 0 && ms < best) best = ms;
      if (e) break;
    }
    printf("{\"variant\": \"regs_syncwave_U%d\", \"mode\": 3, \"ms_28_layers\": %.4f, \"us_per_layer\": %.2f, "
           "\"tb_s\": %.2f, \"errors\": %u}\n", v == 0 ? 8 : 16, best, best * 1e3f / L, total / (best * 1e-3) / 1e12, herr);
    fflush(stdout);
    if (herr) return 2;
  }
  // standalone streaming cost per op size: 28 launches of one kind in a graph, per grid shape
  for (int k : {0, 2, 3, 4}) {
    for (int cfg = 0; cfg < 4; ++cfg) {
      const int blocks = cfg == 0 ? nb : cfg == 1 ? 2 * nb : cfg == 2 ? 4 * nb : 8 * nb;
      const int thr = cfg == 0 ? 512 : 256;
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int l = 0; l < L; ++l)
        hipLaunchKernelGGL(reg_stream_kernel<8>, dim3(blocks), dim3(thr), 0, s, dph, 5 * l + k, 5 * l + k + 1, 0, ctr,
                           err, sink);
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
      printf("{\"op\": \"%s\", \"mb\": %.1f, \"blocks\": %d, \"threads\": %d, \"us_per_launch\": %.2f, \"tb_s\": %.2f}\n",
             names[k], sz[k] / 1e6, blocks, thr, best * 1e3f / L, sz[k] * L / (best * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
