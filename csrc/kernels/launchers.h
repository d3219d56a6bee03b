// Host-side launcher declarations for the vgate HIP kernels.
// The kernels (*.hip) are compiled by hipcc without any torch headers; the
// torch binding layer (csrc/runtime/bindings.cpp) only sees these plain structs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vgate {

struct AttnArgs;

struct GemmArgs {
  const uint16_t* x;  // [M, K] bf16, row stride lda (rows gathered through row_idx if set)
  int lda;
  int M;
  const int32_t* row_idx;  // optional [M] row gather (LM head over sampled rows)
  const void* wp;     // fragment-packed weight (bf16 [N/16][K/32][64][8] or AWQ int4 [N/16][K/128][64][4])
  int N;
  int K;
  const uint16_t* norm_w;  // optional fused RMSNorm weight [K] (null + rownorm: gamma pre-folded into W)
  float eps;
  int rownorm;             // 1: apply the RMSNorm row scale (gamma folded into the packed weight)
  const uint16_t* bias;  // [N] bf16 or null
  const uint16_t* res;   // residual [M, N] bf16 (stride ldr) or null; may alias out
  int ldr;
  void* out;          // bf16 [M, N] (silu: [M, N/2]; f32 for EPI_F32; qkv: q [M, hq*128])
  int ldo;
  int epi;            // 0 bf16, 1 f32, 2 silu*mul (gate/up tiles interleaved), 3 qkv+rope+kv-write
  int waves;          // 0 = heuristic
  int splitk;         // 0 = heuristic
  int ntb;            // 16-column tiles per block for plain / f32 epilogues (0 = heuristic; 1, 2, 4)
  int path;           // M > 16 dense: 0 auto (prefill kernel at M >= 128), 1 force prefill kernel,
                      // 2 medium-M kernel (16 < M <= 64), -1 never (tile / decode kernels)
  float* slabs;       // split-K fp32 partial slabs (workspace) or null
  size_t slab_bytes;
  uint32_t* counters; // split-K arrival tickets, zero-initialised, self-resetting
  int max_counters;
  // EPI_QKV
  const int32_t* positions;
  const int32_t* slots;
  const float* cos_sin;  // [max_pos, 128] f32
  uint16_t* k_cache;
  uint16_t* v_cache;
  int hq;
  int hkv;
  int bs;
  // AWQ
  const uint16_t* awq_szp = nullptr;  // AWQ decode: fragment-packed (s, s*z) [N/16][K/128][4][8]
  const uint16_t* scales;  // [K/group][N] bf16
  const uint16_t* zeros;   // [K/group][N] bf16 (= scale * zero)
  int group;
  // profiling only: per-block [start, end] s_memrealtime stamps (2 x blocks u64), or null
  unsigned long long* dbg_ts;
  // RMSNorm hand-off to the int4 consumers (decode, M <= 16; gemm_epilogue.h GemmParams::hg):
  // producer (epi 0): hg [M, N] bf16 = out * hg_gamma, ssp_out [M][N/16] f32 per-tile sums of out^2;
  // consumer (AWQ): x is hg, ssp_in [M][ssn] the producer's sums (gamma not re-applied)
  uint16_t* hg = nullptr;
  const uint16_t* hg_gamma = nullptr;
  float* ssp_out = nullptr;
  const float* ssp_in = nullptr;
  int ssn = 0;
  // stream-K decode kernel (path 3, gemm_streamk.hip): zeroed publisher-slot workspace and the
  // sticky fault word (bit 2: a partial poll gave up)
  void* sk_pub = nullptr;
  size_t sk_bytes = 0;
  uint32_t* fault = nullptr;
  // TP row-parallel decode GEMM with the all-reduce in its epilogue (ar_world >= 1; gemm_epilogue.h
  // epilogue_ar): every rank's fused region (IPC-mapped, AR_FUSED_BYTES) and the own sticky error word
  char* ar_fused[8] = {};
  uint32_t* ar_err = nullptr;
  int ar_rank = 0;
  int ar_world = 0;
  // decode-only step, EPI_QKV: the step's decode attention rides in the same launch when the decode
  // tile kernel takes the shape (qkv_attn.hip; fa_done set), else the caller launches it after
  const AttnArgs* fa = nullptr;
  void* fa_gran = nullptr;      // zeroed granule buffer (QaSync::gran), fa_gran_bytes long
  size_t fa_gran_bytes = 0;
  bool* fa_done = nullptr;
};
void launch_gemm(const GemmArgs& g, hipStream_t st);
// stream-K decode GEMM (gemm_streamk.hip): M <= 16 dense rows, one equal share of the packed weight
// stream per CU; returns false (nothing launched) for a shape / mode it does not take
bool launch_gemm_sk(const GemmArgs& g, hipStream_t st);
// LDS-tiled prefill GEMM (gemm_prefill.hip) for long steps; returns false for a shape / mode it
// does not take (caller falls back). g.ntb: forced tile width (0 heuristic, 64, 128).
bool launch_gemm_prefill(const GemmArgs& g, hipStream_t st);
// medium-M GEMM (gemm_mid.hip, 16 < M <= 64): W = g.waves tiles per block, g.splitk K slices
// (0 = heuristic); returns false for a shape / mode it does not take (caller falls back)
bool launch_gemm_mid(const GemmArgs& g, hipStream_t st);
// Decode GEMMs with register-stationary activations (gemm_kx.h; M <= 16; WIDE one block per CU / GROUP
// 1-4 tiles per block + K slices): AWQ W4A16 (group 128, packed scales) and bf16. False: shape / mode
// not taken (the caller falls back on the other decode kernels).
bool launch_awq_kx(const GemmArgs& g, hipStream_t st);
bool launch_dense_kx(const GemmArgs& g, hipStream_t st);
// AWQ W4A16 medium-M kernel (gemm_awq_mid.hip, 16 < M <= 64): g.waves tiles per block (8: one block
// per CU owning whole tiles), g.splitk K slices; false for a shape / mode it does not take
bool launch_awq_mid(const GemmArgs& g, hipStream_t st);
// AWQ int4 fragments -> bf16 fragment-packed copy (optionally gamma-folded) for the prefill kernel
void launch_awq_dequant(const void* wq, const uint16_t* scales, const uint16_t* sz, const uint16_t* gamma,
                        void* out, int N, int K, int group, hipStream_t st);

// ---- custom one-shot all-reduce over xGMI peer memory (allreduce.hip) ----
// bases[p]: rank p's IPC-mapped allocation = [AR_SIGNAL_BYTES signal area][2 x max_bytes data];
// bf16 in/out (may alias), nbytes % 16 == 0, nbytes <= max_bytes
constexpr int64_t AR_SIGNAL_BYTES = 65536;
// fused row-parallel GEMM + all-reduce (gemm_epilogue.h epilogue_ar): a region after the two data
// buffers = arrival words [AR_FUSED_TILES][8] u32, then two parity buffers of one fp32 16 x 16 tile
// (1 KiB) per 16-column output tile
constexpr int AR_FUSED_TILES = 1024;
constexpr int64_t AR_FUSED_FLAG_BYTES = (int64_t)AR_FUSED_TILES * 8 * 4;
constexpr int64_t AR_FUSED_DATA = (int64_t)AR_FUSED_TILES * 1024;
constexpr int64_t AR_FUSED_BYTES = AR_FUSED_FLAG_BYTES + 2 * AR_FUSED_DATA;
uint32_t ar_spin();  // the wait bound of every all-reduce kind (VGATE_AR_SPIN_LIMIT)
void launch_custom_allreduce(const void* in, void* out, int64_t nbytes, char* const* bases, int rank, int world,
                             int64_t max_bytes, hipStream_t st, int two_shot = 0);
// all-gather over the same buffers: out = [rank 0's in | rank 1's in | ...] (nbytes each)
void launch_custom_allgather(const void* in, void* out, int64_t nbytes, char* const* bases, int rank, int world,
                             int64_t max_bytes, hipStream_t st);
// byte offsets in the signal area: the sticky wait-timeout word, then {ticks, calls} (ArSignal)
int64_t ar_error_offset();
int64_t ar_blocks_used();

// ---- launch timeline (profiling; csrc/runtime/timeline.cpp, benchmarks/timeline.py) ----
// While a timeline is active every launcher takes 2 x blocks u64 stamps for its kernel
// (TLScope in common.h) and records (name, offset, blocks); null when inactive or full.
unsigned long long* tl_take(const char* name, int nblocks);
void tl_start(unsigned long long* base, int64_t capacity);
int64_t tl_stop();
int tl_count();
const char* tl_name(int i);
int64_t tl_offset(int i);
int tl_blocks(int i);
void launch_awq_gemm(const GemmArgs& g, hipStream_t st);

// y = rmsnorm(x) * w ; if res != null: res = x + res (in place) and the norm is of the sum.
void launch_rmsnorm(const uint16_t* x, int ldx, uint16_t* res, int ldres, const uint16_t* w,
                    uint16_t* y, int ldy, int M, int H, float eps, hipStream_t st);

// Embedding gather with vocab-shard masking (TP): rows outside [vstart, vstart+vrows) -> 0.
void launch_embedding(const int32_t* ids, const uint16_t* table, uint16_t* out, int T, int H,
                      int vstart, int vrows, hipStream_t st, const int32_t* prev = nullptr);

// Default-policy read sweep of [p, p + bytes) over `blocks` workgroups (MALL warm-up).
void launch_prefetch(const void* p, size_t bytes, int blocks, hipStream_t st);
// bytes % 16 == 0; src / dst device pointers (pinned host memory: its device-mapped address)
void set_dec_u(int u);  // decode GEMM register group: -100 the launcher's rule, 6 / 8 / 10 / 12 forced (tests)
void set_flash_prefill(int on);  // prefill tiles on the flash kernel: 1 on, 0 off (16-query tiles), -1 env
void launch_copy16(const void* src, void* dst, size_t bytes, bool to_host, hipStream_t st);
// ids[0, n) -> ring[*slot * stride + i] (ring: device-mapped pinned host memory); with `ar` (the
// own custom all-reduce signal area's error word, or null) also its {error, ticks, calls} words ->
// ring[*slot * stride + stride - 4 + {0, 1, 2}] (the TP collective health / time, no host sync); with
// `fault` (ops.fault_word: the sticky give-up word of the in-launch hand-offs) also -> stride - 1
void launch_ids_to_host(const int32_t* ids, int32_t* ring, const int32_t* slot, int stride, int n, hipStream_t st,
                        const uint32_t* ar = nullptr, const uint32_t* fault = nullptr);

// NeoX RoPE on q,k inside the fused qkv buffer + paged KV-cache write.
// qkv: [T, (Hq + 2*Hkv) * D]; cos_sin: [max_pos, D] f32 (cos | sin halves)
// k_cache/v_cache: [num_blocks, Hkv, BS, D]; slot < 0 => skip write.
void launch_rope_kv(uint16_t* qkv, const int32_t* positions, const int32_t* slots,
                    const float* cos_sin, uint16_t* k_cache, uint16_t* v_cache, int T, int Hq,
                    int Hkv, int D, int BS, hipStream_t st,
                    uint16_t* q_out = nullptr, int ldq = 0);
void launch_silu_mul(const uint16_t* y, int ldy, uint16_t* out, int ldo, int I, int M, hipStream_t st);

struct AttnArgs {
  const uint16_t* q;  // [T, Hq, D] with row stride q_stride (elements, per token)
  int q_stride;
  const uint16_t* k_cache;  // [num_blocks, Hkv, BS, D]
  const uint16_t* v_cache;
  const int32_t* block_tables;  // [S, max_blocks]
  int max_blocks;
  const int32_t* context_lens;  // [S] total kv length (incl. new tokens)
  const int32_t* query_start;   // [S+1] cumulative query offsets (prefill); null => decode
  uint16_t* out;                // [T, Hq, D]
  int out_stride;
  float* part_o;    // decode split-K workspace [S, Hq, P, D]
  float* part_ml;   // [S, Hq, P, 2]
  int S;
  int Hq;
  int Hkv;
  int D;
  int BS;
  int num_parts;    // decode: partitions per sequence (grid z)
  int part_size;    // tokens per partition (multiple of 32)
  float scale;
  // prefill tiling (host computed): tile -> (seq, q offset)
  const int32_t* tile_seq;
  const int32_t* tile_q0;
  int num_tiles;
  // decode partitions merged in-launch by the last-arriving partition block of each
  // (sequence, KV head): zero-initialised, self-resetting [S * Hkv] tickets (null ->
  // separate reduce launch)
  uint32_t* tickets;
  // profiling only: phase timestamps (s_memtime) of block (0,0,0) wave 0, or null
  unsigned long long* dbg_ts;
  unsigned long long* tl;  // launch timeline slot (set by the launcher), or null
  // flash prefill K split (attention.hip attn_flash_kernel, two blocks per KV head): the two halves of a long
  // causal range meet through bf16 partials + fp32 (m, l) in fl_ws and a zeroed, self-resetting
  // ticket + ready word per (leader, KV head, wave) (fl_tickets: 65536 words); null -> no split
  float* fl_ws = nullptr;
  size_t fl_ws_bytes = 0;
  uint32_t* fl_tickets = nullptr;
  // sticky kernel-fault word (bit 1: a flash K-split waiter gave up), copied to the host each step by
  // launch_ids_to_host; null = none
  uint32_t* fault = nullptr;
};
// In-launch hand-off of the fused QKV projection + decode attention (qkv_attn.hip): the nprod GEMM
// blocks write q and the new K / V rows also as data-tagged granules {bf16 pair, position + 1} into
// `gran` ([M][n2 = N / 2] x 8 B, zeroed once: ops.qa_granules); the attention blocks poll them and
// clear what they read. fault: the sticky fault word (bit 32: a poll gave up).
struct QaSync {
  void* gran;
  int n2;
  int nprod;
  uint32_t* fault;
};
void launch_attn_decode(const AttnArgs& a, hipStream_t st);
void launch_attn_prefill(const AttnArgs& a, hipStream_t st);
// One launch for a mixed step: decode blocks for sequences [0, dec_seqs) (only those
// with a single query token do work) + prefill tiles (tile_seq < 0 = padding).
void launch_attention(const AttnArgs& a, int dec_seqs, hipStream_t st);


struct SampleArgs {
  const float* logits;  // [B, V] f32, row stride ldl
  int ldl;
  int B;
  int V;
  const float* temperature;  // [B]
  const float* top_p;        // [B]
  const int32_t* top_k;      // [B]
  const uint64_t* seeds;     // [B]
  const int64_t* offsets;    // [B] per-row philox offset (e.g. generated-token count)
  int32_t* out;              // [B]
  float* out_logprob;        // [B] or null
  unsigned long long* tl;    // launch timeline slot (set by the launcher), or null
  // segmented mode (sampling.hip sample_gran_kernel, B <= SAMPLE_GRAN_ROWS): tagged partial granules,
  // a fixed region of SAMPLE_GRAN_ROW uint4 per row, and per-row epochs [B] (zero-initialised,
  // self-advancing); null -> one block per row. fault: sticky word (bit 16: a row's wait gave up)
  void* gran = nullptr;
  uint32_t* epoch = nullptr;
  uint32_t* fault = nullptr;
};
// sampler workspace (int32 words): [0, SAMPLE_WS_GRAN) per-row epochs, then the granule regions
constexpr int SAMPLE_GRAN_SEGS = 64;                        // max segments per row
constexpr int SAMPLE_GRAN_ROWS = 128;                       // rows of the segmented mode (nseg >= 2)
constexpr int SAMPLE_GRAN_ROW = 2 * SAMPLE_GRAN_SEGS * 2;   // uint4 per row: [parity][segment][2]
constexpr int SAMPLE_WS_GRAN = 256;                         // int32 offset of the granules (16-B aligned)
constexpr int SAMPLE_WS_WORDS = SAMPLE_WS_GRAN + SAMPLE_GRAN_ROWS * SAMPLE_GRAN_ROW * 4;
void launch_sample(const SampleArgs& s, hipStream_t st);
int sample_segments(int B, int V);
void set_sample_nseg(int n);  // cap on segments per row, 1..SAMPLE_GRAN_SEGS (1 = one block per row)

// Custom one-shot all-reduce over IPC-mapped peer buffers (xGMI).
struct AllReduceArgs {
  void* const* peers;     // device array of world_size peer buffer pointers
  uint32_t* const* flags; // device array of world_size peer flag pointers
  int rank;
  int world;
  uint16_t* out;
  int64_t numel;
  uint32_t epoch;
};
void launch_allreduce_oneshot(const AllReduceArgs& a, hipStream_t st);

}  // namespace vgate
