// Fused QKV projection + decode attention: ONE launch per layer for a decode-only step.
//
// A decode layer is qkv GEMM -> attention -> o_proj -> gate_up -> down_proj, and the attention launch
// is a dependency chain the kernel boundary serialises: context length + block table (one round trip),
// then the K / V chunks (a second), then q . K^T, softmax, V, the wave merge. Only the query and the
// NEW token's K / V row depend on the projection; everything else (the whole cached history) was
// written by earlier launches. So the attention blocks ride behind the GEMM blocks of the projection
// launch (block ids [nprod, nprod + ncons)): each requests its context metadata and the first K / V
// chunk of every wave at launch, while the GEMM streams its weights on other CUs, then waits for the
// GEMM blocks' arrivals and loads only q and the new row (attn_decode.h decode_block<.., FUSED>).
//
// Hand-off (MI355X_MICROARCH.md handoff-1to1, R2 granules): the producer epilogue writes q and the new
// K / V rows a second time as data-tagged granules {bf16 pair, position + 1} (16-B write-through
// stores, gemm_epilogue.h epilogue, p.qa_gran); each consumer wave polls the granules it needs with
// 16-B sc1 loads until every tag is this step's, and the consumer block clears them after use. No
// flag, drain or fence sits between the GEMM's last MFMA and the attention's first: a first attempt
// with drained write-through stores + an arrival counter + a barrier took 12.6 us for the pair
// against 11.0 us for two launches (store drain, atomic, poll and payload load are four serial memory
// latencies). Workgroups are dispatched in id order, so every producer is resident or done before
// any consumer can wait on it. A poll that gives up sets fault bit 32 (the step fails loudly).
//
// The reference serves decode through vLLM's separate attention + GEMM kernels
// (/root/reference/vgate/backends/vllm_backend.py); this launch is MI355X-specific structure.
#include "attn_decode.h"
#include "gemm_decode.h"

namespace vgate {

template <int U, int XP, int NORM>
__global__ __launch_bounds__(512) void qkv_attn_kernel(GemmParams p, AttnArgs a, QaSync q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < q.nprod) {
    gemm_block<1, 1, U, EPI_QKV, NORM, true, XP>(p);
    return;
  }
  TLScope tl_scope(p.dbg_ts);
  // consumer r = (KV head, partition, sequence), sequence fastest (as attn_kernel's decode blocks)
  const int r = (int)blockIdx.x - q.nprod;
  const int S = a.S, P = a.num_parts;
  decode_block<false, true>(a, r % S, r / (S * P), (r / S) % P, smem, &q);
}

template <int NORM>
static bool qa_dispatch(int u, int xp, const GemmParams& p, const AttnArgs& a, const QaSync& q, int waves,
                        size_t lds, hipStream_t st) {
  if (xp == 4 && u == 8) { qa_launch(qkv_attn_kernel<8, 4, NORM>, p, a, q, waves, lds, st); return true; }
  if (xp == 2 && u == 6) { qa_launch(qkv_attn_kernel<6, 2, NORM>, p, a, q, waves, lds, st); return true; }
  if (xp == 2 && u == 8) { qa_launch(qkv_attn_kernel<8, 2, NORM>, p, a, q, waves, lds, st); return true; }
  if (xp == 1 && u == 6) { qa_launch(qkv_attn_kernel<6, 1, NORM>, p, a, q, waves, lds, st); return true; }
  if (xp == 1 && u == 8) { qa_launch(qkv_attn_kernel<8, 1, NORM>, p, a, q, waves, lds, st); return true; }
  return false;
}

// gx x slices GEMM blocks (K slices combined in-launch as in the two-launch form: granules / slabs),
// carried z-major in the 1-D grid (GemmParams::vgx), then the attention blocks
bool launch_qkv_attn(int u, int xp, int norm, GemmParams p, int gx, int slices, int waves, size_t lds_gemm,
                     const GemmArgs& g, hipStream_t st) {
  if (norm != 2 && norm != 3) return false;  // the decode QKV projections: gamma folded / hand-off
  const bool inst = (xp == 4 && u == 8) || ((xp == 2 || xp == 1) && (u == 6 || u == 8));
  if (!inst) return false;
  AttnArgs a;
  QaSync q;
  size_t lds;
  if (!qa_setup(p, g, gx, slices, waves, lds_gemm, a, q, lds)) return false;
  if (p.dbg_ts == nullptr) p.dbg_ts = tl_take("qkv_attn", q.nprod + a.S * a.num_parts * a.Hkv);
  if (norm == 2) return qa_dispatch<2>(u, xp, p, a, q, waves, lds, st);
  return qa_dispatch<3>(u, xp, p, a, q, waves, lds, st);
}

}  // namespace vgate
