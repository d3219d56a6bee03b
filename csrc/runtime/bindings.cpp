// Torch / pybind11 binding layer for the vgate gfx950 kernels.
//
// This is the only translation unit that sees torch headers; kernels are plain
// HIP objects (csrc/kernels/*.hip) reached through csrc/kernels/launchers.h.
// Every op launches on torch's current HIP stream, so ops are hipGraph
// capturable via torch.cuda.graph / vgate.runtime.graphs.
#include <cstring>

#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include "../kernels/launchers.h"
#include "allocator.h"
#include "lru_cache.h"

namespace {

using torch::Tensor;

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_DT(t, d) do { TORCH_CHECK((t).scalar_type() == (d), #t " has wrong dtype ", (t).scalar_type()); } while (0)
#define CHECK_LASTDIM(t) TORCH_CHECK((t).stride(-1) == 1, #t " must be contiguous in its last dim")

// torch-ROCm exposes HIP devices as DeviceType::CUDA ("masquerading")
hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

const uint16_t* bf16p(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bf16p_mut(Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

const uint16_t* opt_bf16(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t);
  CHECK_DT(*t, torch::kBFloat16);
  return reinterpret_cast<const uint16_t*>(t->data_ptr());
}

template <typename T>
T* opt_ptr(const c10::optional<Tensor>& t, c10::ScalarType dt, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t->scalar_type() == dt, name, " has wrong dtype ", t->scalar_type());
  return reinterpret_cast<T*>(t->data_ptr());
}

vgate::AttnArgs attn_common(const Tensor& q, int64_t q_stride, const Tensor& k_cache,
                            const Tensor& v_cache, const Tensor& block_tables,
                            const Tensor& context_lens, Tensor& out, int64_t Hq, int64_t Hkv,
                            double scale);

// out = epilogue(prologue(x) @ W^T); W fragment-packed [N/16, K/32, 64, 8] bf16, or AWQ
// int4 [N/16, K/128, 64, 4] int32 with scales/zeros. ws = int32 workspace: [0, 65536)
// split-K tickets (zeroed once, self-resetting), the rest fp32 slabs.
void gemm(const Tensor& x, const Tensor& wp, int64_t N, int64_t K, Tensor& out, int64_t epi,
          const c10::optional<Tensor>& bias, const c10::optional<Tensor>& res,
          const c10::optional<Tensor>& norm_w, double eps, const c10::optional<Tensor>& row_idx,
          const c10::optional<Tensor>& ws, int64_t waves, int64_t splitk,
          const c10::optional<Tensor>& positions, const c10::optional<Tensor>& slots,
          const c10::optional<Tensor>& cos_sin, const c10::optional<Tensor>& k_cache,
          const c10::optional<Tensor>& v_cache, int64_t hq, int64_t hkv,
          const c10::optional<Tensor>& awq_scales, const c10::optional<Tensor>& awq_zeros, int64_t group,
          bool rownorm, const c10::optional<Tensor>& dbg_ts, int64_t ntb, int64_t path,
          const c10::optional<Tensor>& awq_szp, const c10::optional<Tensor>& hg_out,
          const c10::optional<Tensor>& hg_gamma, const c10::optional<Tensor>& ssp_out,
          const c10::optional<Tensor>& ssp_in, const c10::optional<Tensor>& sk_ws,
          const c10::optional<Tensor>& fault, const std::vector<int64_t>& ar_bases, int64_t ar_rank,
          int64_t ar_fused_off, const c10::optional<Tensor>& fa_block_tables,
          const c10::optional<Tensor>& fa_context_lens, const c10::optional<Tensor>& fa_query_start,
          const c10::optional<Tensor>& fa_out, const c10::optional<Tensor>& fa_part_o,
          const c10::optional<Tensor>& fa_part_ml, const c10::optional<Tensor>& fa_tickets,
          const c10::optional<Tensor>& fa_sync, int64_t fa_part_size, double fa_scale,
          const c10::optional<Tensor>& fa_dbg_ts) {
  CHECK_DEV(x); CHECK_DEV(wp); CHECK_DEV(out);
  CHECK_DT(x, torch::kBFloat16);
  CHECK_LASTDIM(x); CHECK_LASTDIM(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "gemm: x/out must be 2-D");
  TORCH_CHECK(K % 32 == 0 && N % 16 == 0, "gemm: K%32 / N%16");
  TORCH_CHECK(x.size(1) >= K, "gemm: x has ", x.size(1), " cols < K=", K);
  const bool awq = awq_scales.has_value() && awq_scales->defined();
  if (awq) {
    CHECK_DT(wp, torch::kInt32);
    TORCH_CHECK(K % 128 == 0 && K % group == 0 && group % 32 == 0, "awq: K/group");
    TORCH_CHECK(wp.numel() == N * K / 8, "awq: packed qweight numel");
    TORCH_CHECK(awq_scales->size(0) == K / group && awq_scales->size(1) == N, "awq: scales shape");
  } else {
    CHECK_DT(wp, torch::kBFloat16);
    TORCH_CHECK(wp.numel() == N * K, "gemm: packed weight numel mismatch");
  }
  int64_t M = x.size(0);
  const int32_t* ridx = opt_ptr<const int32_t>(row_idx, torch::kInt32, "row_idx");
  if (ridx) M = row_idx->numel();
  const int64_t ncols = (epi == 2) ? N / 2 : N;
  if (epi == 1) CHECK_DT(out, torch::kFloat32); else CHECK_DT(out, torch::kBFloat16);
  if (epi == 3) TORCH_CHECK((N / 16) % 2 == 0, "qkv epilogue needs an even tile count");
  if (epi == 3) {
    TORCH_CHECK(N == (hq + 2 * hkv) * 128, "qkv epilogue: N must be (hq + 2 hkv) * 128");
    TORCH_CHECK(out.size(1) >= hq * 128, "qkv epilogue: q out cols");
    TORCH_CHECK(positions.has_value() && slots.has_value() && cos_sin.has_value() && k_cache.has_value() &&
                v_cache.has_value(), "qkv epilogue needs positions/slots/cos_sin/k_cache/v_cache");
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == hkv && k_cache->size(3) == 128, "qkv: cache shape");
    TORCH_CHECK(cos_sin->size(1) == 128, "qkv: cos_sin must be [max_pos, 128]");
  } else {
    TORCH_CHECK(out.size(1) >= ncols, "gemm: out cols");
  }
  TORCH_CHECK(out.size(0) >= M, "gemm: out rows");
  vgate::GemmArgs g{};
  g.x = bf16p(x); g.lda = (int)x.stride(0); g.M = (int)M; g.row_idx = ridx;
  g.wp = wp.data_ptr(); g.N = (int)N; g.K = (int)K;
  g.norm_w = opt_bf16(norm_w); g.eps = (float)eps; g.rownorm = rownorm ? 1 : 0;
  g.dbg_ts = reinterpret_cast<unsigned long long*>(opt_ptr<int64_t>(dbg_ts, torch::kInt64, "dbg_ts"));
  if (g.norm_w) TORCH_CHECK(norm_w->numel() == K, "norm_w must have K elements");
  g.bias = opt_bf16(bias);
  g.res = opt_bf16(res);
  g.ldr = g.res ? (int)res->stride(0) : 0;
  if (g.res) TORCH_CHECK(res->size(0) >= M && res->size(1) >= N, "gemm: residual shape");
  g.out = out.data_ptr(); g.ldo = (int)out.stride(0);
  g.epi = (int)epi; g.waves = (int)waves; g.splitk = (int)splitk; g.ntb = (int)ntb; g.path = (int)path;
  if (ws.has_value() && ws->defined()) {
    CHECK_DEV(*ws); CHECK_DT(*ws, torch::kInt32);
    TORCH_CHECK(ws->numel() > 65536 * 2, "gemm: workspace too small");
    g.counters = reinterpret_cast<uint32_t*>(ws->data_ptr());
    g.max_counters = 65536;
    g.slabs = reinterpret_cast<float*>(reinterpret_cast<int32_t*>(ws->data_ptr()) + 65536);
    g.slab_bytes = (size_t)(ws->numel() - 65536) * 4;
  }
  g.positions = opt_ptr<const int32_t>(positions, torch::kInt32, "positions");
  g.slots = opt_ptr<const int32_t>(slots, torch::kInt32, "slots");
  g.cos_sin = opt_ptr<const float>(cos_sin, torch::kFloat32, "cos_sin");
  g.k_cache = opt_ptr<uint16_t>(k_cache, torch::kBFloat16, "k_cache");
  g.v_cache = opt_ptr<uint16_t>(v_cache, torch::kBFloat16, "v_cache");
  g.hq = (int)hq; g.hkv = (int)hkv; g.bs = k_cache.has_value() && k_cache->defined() ? (int)k_cache->size(2) : 16;
  g.scales = opt_bf16(awq_scales); g.zeros = opt_bf16(awq_zeros); g.group = (int)group;
  if (awq_szp.has_value() && awq_szp->defined()) {
    CHECK_DEV(*awq_szp); CHECK_DT(*awq_szp, torch::kBFloat16);
    TORCH_CHECK(group == 128 && awq_szp->numel() == N / 16 * (K / 128) * 32, "awq_szp: [N/16][K/128][4][8], group 128");
    g.awq_szp = reinterpret_cast<const uint16_t*>(awq_szp->data_ptr());
  }
  if (ssp_out.has_value() && ssp_out->defined()) {
    // producer of the next RMSNorm's hand-off: decode rows, bf16 residual epilogue. It stores the
    // per-(row, 16-column tile) sums of squares of its output; for int4 consumers also hg = out * gamma
    TORCH_CHECK(epi == 0 && M <= 16, "ssp_out: epi 0, M <= 16");
    CHECK_DEV(*ssp_out); CHECK_DT(*ssp_out, torch::kFloat32);
    TORCH_CHECK(ssp_out->numel() >= M * (N / 16), "ssp_out: [M][N/16]");
    g.ssp_out = reinterpret_cast<float*>(ssp_out->data_ptr());
    if (hg_out.has_value() && hg_out->defined()) {
      CHECK_DEV(*hg_out); CHECK_DT(*hg_out, torch::kBFloat16); CHECK_LASTDIM(*hg_out);
      TORCH_CHECK(hg_out->stride(0) == out.stride(0) && hg_out->size(0) >= M && hg_out->size(1) >= N, "hg_out: like out");
      TORCH_CHECK(hg_gamma.has_value() && hg_gamma->numel() == N, "hg_gamma: N elements");
      g.hg = reinterpret_cast<uint16_t*>(hg_out->data_ptr());
      g.hg_gamma = opt_bf16(hg_gamma);
    }
  } else {
    TORCH_CHECK(!(hg_out.has_value() && hg_out->defined()), "hg_out needs ssp_out");
  }
  if (ssp_in.has_value() && ssp_in->defined()) {
    // consumer: int4 (x = h * gamma) or bf16 with gamma folded into the packed weights (x = h)
    TORCH_CHECK(M <= 16 && !g.norm_w && !rownorm, "ssp_in: decode consumers without another norm mode");
    CHECK_DEV(*ssp_in); CHECK_DT(*ssp_in, torch::kFloat32);
    TORCH_CHECK(ssp_in->numel() >= M * (K / 16) && (reinterpret_cast<uintptr_t>(ssp_in->data_ptr()) % 16) == 0,
                "ssp_in: [M][K/16], 16-B aligned");
    g.ssp_in = reinterpret_cast<const float*>(ssp_in->data_ptr());
    g.ssn = (int)(K / 16);
  }
  if (sk_ws.has_value() && sk_ws->defined()) {
    CHECK_DEV(*sk_ws); CHECK_DT(*sk_ws, torch::kInt32);
    TORCH_CHECK(sk_ws->is_contiguous(), "sk_ws: contiguous");
    g.sk_pub = sk_ws->data_ptr();
    g.sk_bytes = (size_t)sk_ws->numel() * 4;
  }
  g.fault = reinterpret_cast<uint32_t*>(opt_ptr<int32_t>(fault, torch::kInt32, "fault"));
  if (!ar_bases.empty()) {
    // TP row-parallel decode GEMM + all-reduce in the epilogue (vgate/parallel/custom_allreduce.py)
    const int world = (int)ar_bases.size();
    TORCH_CHECK(world <= 8 && ar_rank >= 0 && ar_rank < world, "gemm ar: world 1..8, rank in range");
    TORCH_CHECK(epi == 0 && M <= 16 && !g.ssp_out && N / 16 <= vgate::AR_FUSED_TILES,
                "gemm ar: bf16 epilogue, M <= 16, no norm hand-off, N <= 16 * AR_FUSED_TILES");
    TORCH_CHECK(ar_fused_off >= vgate::AR_SIGNAL_BYTES, "gemm ar: fused region offset");
    for (int r = 0; r < world; ++r) g.ar_fused[r] = reinterpret_cast<char*>(ar_bases[r]) + ar_fused_off;
    g.ar_err = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ar_bases[ar_rank]) + vgate::ar_error_offset());
    g.ar_rank = (int)ar_rank;
    g.ar_world = world;
  }
  // decode-only step: the step's decode attention (q = this projection's output) in the same launch
  // when the decode tile kernel takes it (qkv_attn.hip), else launched right after the projection
  vgate::AttnArgs fa{};
  bool fa_done = false;
  const bool fused_attn = fa_out.has_value() && fa_out->defined();
  if (fused_attn) {
    TORCH_CHECK(epi == 3 && M <= 16, "fused attention: the decode QKV projection (epi 3, M <= 16)");
    TORCH_CHECK(fa_block_tables.has_value() && fa_context_lens.has_value() && fa_query_start.has_value() &&
                    fa_part_o.has_value() && fa_part_ml.has_value() && fa_tickets.has_value() && fa_sync.has_value(),
                "fused attention: block_tables, context_lens, query_start, part_o, part_ml, tickets, sync");
    Tensor fo = *fa_out;
    fa = attn_common(out, out.stride(0), *k_cache, *v_cache, *fa_block_tables, *fa_context_lens, fo, hq, hkv,
                     fa_scale);
    TORCH_CHECK(fa_part_size % 32 == 0 && fa_part_size <= 1024, "fused attention: part_size");
    CHECK_DT(*fa_part_o, torch::kFloat32); CHECK_DT(*fa_part_ml, torch::kFloat32);
    CHECK_DT(*fa_query_start, torch::kInt32);
    TORCH_CHECK(fa_query_start->numel() >= fa.S + 1, "fused attention: query_start needs S+1 entries");
    fa.query_start = reinterpret_cast<const int32_t*>(fa_query_start->data_ptr());
    fa.num_parts = (int)fa_part_o->size(2);
    fa.part_size = (int)fa_part_size;
    TORCH_CHECK((int64_t)fa.num_parts * fa_part_size >= fa_block_tables->size(1) * 16,
                "fused attention: partitions do not cover max context");
    TORCH_CHECK(fa_part_o->size(0) >= fa.S && fa_part_o->size(1) == hq, "fused attention: part_o shape");
    fa.part_o = reinterpret_cast<float*>(fa_part_o->data_ptr());
    fa.part_ml = reinterpret_cast<float*>(fa_part_ml->data_ptr());
    CHECK_DEV(*fa_tickets); CHECK_DT(*fa_tickets, torch::kInt32);
    TORCH_CHECK(fa_tickets->numel() >= (int64_t)fa.S * hkv, "fused attention: tickets need S*Hkv zeroed int32");
    fa.tickets = reinterpret_cast<uint32_t*>(fa_tickets->data_ptr());
    CHECK_DEV(*fa_sync); CHECK_DT(*fa_sync, torch::kInt32);
    TORCH_CHECK(fa_sync->is_contiguous(), "fused attention: granule buffer contiguous");
    fa.fault = g.fault;
    if (fa_dbg_ts.has_value() && fa_dbg_ts->defined()) {  // profiling: attention phase stamps (qa_phases.py)
      CHECK_DEV(*fa_dbg_ts); CHECK_DT(*fa_dbg_ts, torch::kInt64);
      TORCH_CHECK(fa_dbg_ts->numel() >= 16, "fused attention: dbg_ts needs 16 int64");
      fa.dbg_ts = reinterpret_cast<unsigned long long*>(fa_dbg_ts->data_ptr());
    }
    g.fa = &fa;
    g.fa_gran = fa_sync->data_ptr();
    g.fa_gran_bytes = (size_t)fa_sync->numel() * 4;
    g.fa_done = &fa_done;
  }
  c10::DeviceGuard guard(x.device());
  if (awq) vgate::launch_awq_gemm(g, cur_stream());
  else vgate::launch_gemm(g, cur_stream());
  if (fused_attn && !fa_done) vgate::launch_attention(fa, fa.S, cur_stream());
}

// AWQ int4 packed weight -> bf16 packed weight (same fragment order / row permutation)
void awq_dequant(const Tensor& wq, const Tensor& scales, const Tensor& sz, int64_t N, int64_t K, int64_t group,
                 Tensor& out, const c10::optional<Tensor>& gamma) {
  CHECK_DEV(wq); CHECK_DEV(scales); CHECK_DEV(sz); CHECK_DEV(out);
  CHECK_DT(wq, torch::kInt32); CHECK_DT(scales, torch::kBFloat16); CHECK_DT(sz, torch::kBFloat16);
  CHECK_DT(out, torch::kBFloat16);
  TORCH_CHECK(N % 16 == 0 && K % 128 == 0 && K % group == 0 && group % 32 == 0, "awq_dequant: N/K/group");
  TORCH_CHECK(wq.numel() == N * K / 8 && out.numel() >= N * K, "awq_dequant: sizes");
  TORCH_CHECK(scales.size(0) == K / group && scales.size(1) == N && sz.sizes() == scales.sizes(), "awq_dequant: scales");
  const uint16_t* g = opt_bf16(gamma);
  if (g) TORCH_CHECK(gamma->numel() == K, "awq_dequant: gamma has K elements");
  c10::DeviceGuard guard(wq.device());
  vgate::launch_awq_dequant(wq.data_ptr(), bf16p(scales), bf16p(sz), g, out.data_ptr(), (int)N, (int)K, (int)group,
                            cur_stream());
}

// y = rmsnorm(x [+ res]) * w ; res (if given) is updated in place to x + res
void rmsnorm(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& w, Tensor& y,
             double eps) {
  CHECK_DEV(x); CHECK_DEV(w); CHECK_DEV(y);
  CHECK_DT(x, torch::kBFloat16); CHECK_DT(w, torch::kBFloat16); CHECK_DT(y, torch::kBFloat16);
  CHECK_LASTDIM(x); CHECK_LASTDIM(y);
  const int64_t M = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "rmsnorm: H");
  uint16_t* rp = nullptr;
  int ldr = 0;
  if (res.has_value() && res->defined()) {
    CHECK_DT(*res, torch::kBFloat16);
    rp = reinterpret_cast<uint16_t*>(res->data_ptr());
    ldr = (int)res->stride(0);
  }
  c10::DeviceGuard guard(x.device());
  vgate::launch_rmsnorm(bf16p(x), (int)x.stride(0), rp, ldr, bf16p(w), bf16p_mut(y),
                        (int)y.stride(0), (int)M, (int)H, (float)eps, cur_stream());
}

void embedding(const Tensor& ids, const Tensor& table, Tensor& out, int64_t vstart,
               const c10::optional<Tensor>& prev) {
  CHECK_DEV(ids); CHECK_DEV(table); CHECK_DEV(out);
  CHECK_DT(ids, torch::kInt32); CHECK_DT(table, torch::kBFloat16); CHECK_DT(out, torch::kBFloat16);
  TORCH_CHECK(table.is_contiguous() && out.is_contiguous(), "embedding: contiguous");
  const int64_t T = ids.numel(), H = table.size(1);
  TORCH_CHECK(H % 8 == 0 && out.numel() >= T * H, "embedding: shapes");
  c10::DeviceGuard guard(ids.device());
  vgate::launch_embedding(reinterpret_cast<const int32_t*>(ids.data_ptr()), bf16p(table),
                          bf16p_mut(out), (int)T, (int)H, (int)vstart, (int)table.size(0),
                          cur_stream(), opt_ptr<const int32_t>(prev, torch::kInt32, "prev"));
}

void rope_kv(Tensor& qkv, const Tensor& positions, const c10::optional<Tensor>& slots,
             const Tensor& cos_sin, Tensor& k_cache, Tensor& v_cache, int64_t Hq, int64_t Hkv,
             int64_t D, const c10::optional<Tensor>& q_out) {
  CHECK_DEV(qkv); CHECK_DEV(positions); CHECK_DEV(cos_sin);
  CHECK_DT(qkv, torch::kBFloat16); CHECK_DT(positions, torch::kInt32);
  CHECK_DT(cos_sin, torch::kFloat32);
  TORCH_CHECK(qkv.is_contiguous() && qkv.size(1) == (Hq + 2 * Hkv) * D, "rope_kv: qkv shape");
  TORCH_CHECK(D % 8 == 0 && cos_sin.size(1) == D, "rope_kv: D / cos_sin");
  const int32_t* sp = nullptr;
  if (slots.has_value() && slots->defined()) {
    CHECK_DT(*slots, torch::kInt32);
    sp = reinterpret_cast<const int32_t*>(slots->data_ptr());
  }
  const int BS = (int)k_cache.size(2);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D, "rope_kv: cache shape");
  uint16_t* qo = nullptr;
  int ldq = 0;
  if (q_out.has_value() && q_out->defined()) {
    CHECK_DEV(*q_out); CHECK_DT(*q_out, torch::kBFloat16); CHECK_LASTDIM(*q_out);
    TORCH_CHECK(q_out->dim() == 2 && q_out->size(0) >= qkv.size(0) && q_out->size(1) >= Hq * D, "rope_kv: q_out shape");
    qo = reinterpret_cast<uint16_t*>(q_out->data_ptr());
    ldq = (int)q_out->stride(0);
  }
  c10::DeviceGuard guard(qkv.device());
  vgate::launch_rope_kv(bf16p_mut(qkv), reinterpret_cast<const int32_t*>(positions.data_ptr()), sp,
                        reinterpret_cast<const float*>(cos_sin.data_ptr()), bf16p_mut(k_cache),
                        bf16p_mut(v_cache), (int)qkv.size(0), (int)Hq, (int)Hkv, (int)D, BS,
                        cur_stream(), qo, ldq);
}

// out [M, I] = silu(y[:, :I]) * y[:, I:2I]
void silu_mul(const Tensor& y, Tensor& out) {
  CHECK_DEV(y); CHECK_DEV(out);
  CHECK_DT(y, torch::kBFloat16); CHECK_DT(out, torch::kBFloat16);
  CHECK_LASTDIM(y); CHECK_LASTDIM(out);
  const int64_t I = out.size(1);
  TORCH_CHECK(y.dim() == 2 && out.dim() == 2 && y.size(1) == 2 * I && out.size(0) == y.size(0) && I % 8 == 0,
              "silu_mul: y [M, 2I], out [M, I], I % 8 == 0");
  c10::DeviceGuard guard(y.device());
  vgate::launch_silu_mul(bf16p(y), (int)y.stride(0), bf16p_mut(out), (int)out.stride(0), (int)I, (int)y.size(0),
                         cur_stream());
}

vgate::AttnArgs attn_common(const Tensor& q, int64_t q_stride, const Tensor& k_cache,
                            const Tensor& v_cache, const Tensor& block_tables,
                            const Tensor& context_lens, Tensor& out, int64_t Hq, int64_t Hkv,
                            double scale) {
  CHECK_DEV(q); CHECK_DEV(k_cache); CHECK_DEV(v_cache); CHECK_DEV(block_tables);
  CHECK_DEV(context_lens); CHECK_DEV(out);
  CHECK_DT(q, torch::kBFloat16); CHECK_DT(out, torch::kBFloat16);
  CHECK_DT(block_tables, torch::kInt32); CHECK_DT(context_lens, torch::kInt32);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 16 && k_cache.size(3) == 128,
              "attention: cache must be [nblk, Hkv, 16, 128]");
  TORCH_CHECK(Hq % Hkv == 0 && Hq / Hkv <= 16, "attention: GQA group must be <= 16");
  TORCH_CHECK(block_tables.is_contiguous(), "attention: block_tables contiguous");
  vgate::AttnArgs a{};
  a.q = bf16p(q); a.q_stride = (int)q_stride;
  a.k_cache = bf16p(k_cache); a.v_cache = bf16p(v_cache);
  a.block_tables = reinterpret_cast<const int32_t*>(block_tables.data_ptr());
  a.max_blocks = (int)block_tables.size(1);
  a.context_lens = reinterpret_cast<const int32_t*>(context_lens.data_ptr());
  a.out = bf16p_mut(out); a.out_stride = (int)(Hq * 128);
  TORCH_CHECK(out.is_contiguous(), "attention: out contiguous");
  a.S = (int)context_lens.numel();
  a.Hq = (int)Hq; a.Hkv = (int)Hkv; a.D = 128; a.BS = 16;
  a.scale = (float)scale;
  return a;
}

void attn_decode(const Tensor& q, int64_t q_stride, const Tensor& k_cache, const Tensor& v_cache,
                 const Tensor& block_tables, const Tensor& context_lens,
                 const c10::optional<Tensor>& query_start, Tensor& out, Tensor& part_o,
                 Tensor& part_ml, int64_t Hq, int64_t Hkv, int64_t part_size, double scale) {
  auto a = attn_common(q, q_stride, k_cache, v_cache, block_tables, context_lens, out, Hq, Hkv, scale);
  CHECK_DT(part_o, torch::kFloat32); CHECK_DT(part_ml, torch::kFloat32);
  TORCH_CHECK(part_size % 32 == 0 && part_size <= 1024, "attention: part_size must be a multiple of 32, <= 1024");
  TORCH_CHECK(part_o.dim() == 4 && part_o.size(0) >= a.S && part_o.size(1) == Hq && part_o.size(3) == 128,
              "attention: part_o must be [S, Hq, P, 128]");
  a.num_parts = (int)part_o.size(2);
  TORCH_CHECK((int64_t)a.num_parts * part_size >= block_tables.size(1) * 16,
              "attention: partitions do not cover max context");
  a.part_size = (int)part_size;
  a.part_o = reinterpret_cast<float*>(part_o.data_ptr());
  a.part_ml = reinterpret_cast<float*>(part_ml.data_ptr());
  a.query_start = nullptr;
  if (query_start.has_value() && query_start->defined()) {
    CHECK_DT(*query_start, torch::kInt32);
    a.query_start = reinterpret_cast<const int32_t*>(query_start->data_ptr());
  }
  c10::DeviceGuard guard(q.device());
  vgate::launch_attn_decode(a, cur_stream());
}

// the flash prefill K split's workspace: the GEMM workspace (ops.workspace), 65536 zeroed
// self-resetting tickets, then fp32 slabs; a flash launch never overlaps a GEMM on the stream
static void set_flash_ws(vgate::AttnArgs& a, const c10::optional<Tensor>& flash_ws,
                         const c10::optional<Tensor>& fault = c10::nullopt) {
  a.fault = reinterpret_cast<uint32_t*>(opt_ptr<int32_t>(fault, torch::kInt32, "fault"));
  if (!flash_ws.has_value() || !flash_ws->defined()) return;
  CHECK_DEV(*flash_ws); CHECK_DT(*flash_ws, torch::kInt32);
  TORCH_CHECK(flash_ws->numel() > 65536, "attention: flash_ws is the GEMM workspace");
  a.fl_tickets = reinterpret_cast<uint32_t*>(flash_ws->data_ptr());
  a.fl_ws = reinterpret_cast<float*>(flash_ws->data_ptr()) + 65536;
  a.fl_ws_bytes = (size_t)(flash_ws->numel() - 65536) * 4;
}

void attn_prefill(const Tensor& q, int64_t q_stride, const Tensor& k_cache, const Tensor& v_cache,
                  const Tensor& block_tables, const Tensor& context_lens,
                  const Tensor& query_start, const Tensor& tile_seq, const Tensor& tile_q0,
                  Tensor& out, int64_t Hq, int64_t Hkv, double scale, const c10::optional<Tensor>& flash_ws,
                  const c10::optional<Tensor>& fault) {
  auto a = attn_common(q, q_stride, k_cache, v_cache, block_tables, context_lens, out, Hq, Hkv, scale);
  set_flash_ws(a, flash_ws, fault);
  CHECK_DT(query_start, torch::kInt32); CHECK_DT(tile_seq, torch::kInt32); CHECK_DT(tile_q0, torch::kInt32);
  a.query_start = reinterpret_cast<const int32_t*>(query_start.data_ptr());
  a.tile_seq = reinterpret_cast<const int32_t*>(tile_seq.data_ptr());
  a.tile_q0 = reinterpret_cast<const int32_t*>(tile_q0.data_ptr());
  a.num_tiles = (int)tile_seq.numel();
  c10::DeviceGuard guard(q.device());
  vgate::launch_attn_prefill(a, cur_stream());
}

void attention(const Tensor& q, int64_t q_stride, const Tensor& k_cache, const Tensor& v_cache,
               const Tensor& block_tables, const Tensor& context_lens, const Tensor& query_start,
               const Tensor& tile_seq, const Tensor& tile_q0, Tensor& out, Tensor& part_o, Tensor& part_ml,
               int64_t Hq, int64_t Hkv, int64_t part_size, double scale, int64_t out_stride,
               const c10::optional<Tensor>& tickets, const c10::optional<Tensor>& dbg_ts,
               const c10::optional<Tensor>& flash_ws, const c10::optional<Tensor>& fault) {
  auto a = attn_common(q, q_stride, k_cache, v_cache, block_tables, context_lens, out, Hq, Hkv, scale);
  set_flash_ws(a, flash_ws, fault);
  if (out_stride > 0) a.out_stride = (int)out_stride;
  CHECK_DT(query_start, torch::kInt32); CHECK_DT(tile_seq, torch::kInt32); CHECK_DT(tile_q0, torch::kInt32);
  CHECK_DT(part_o, torch::kFloat32); CHECK_DT(part_ml, torch::kFloat32);
  TORCH_CHECK(part_size % 32 == 0 && part_size <= 1024, "attention: part_size must be a multiple of 32, <= 1024");
  TORCH_CHECK(query_start.numel() >= a.S + 1, "attention: query_start needs S+1 entries");
  a.query_start = reinterpret_cast<const int32_t*>(query_start.data_ptr());
  a.tile_seq = reinterpret_cast<const int32_t*>(tile_seq.data_ptr());
  a.tile_q0 = reinterpret_cast<const int32_t*>(tile_q0.data_ptr());
  a.num_tiles = (int)tile_seq.numel();
  a.num_parts = (int)part_o.size(2);
  a.part_size = (int)part_size;
  TORCH_CHECK((int64_t)a.num_parts * part_size >= block_tables.size(1) * 16,
              "attention: partitions do not cover max context");
  TORCH_CHECK(part_o.size(0) >= a.S && part_o.size(1) == Hq, "attention: part_o shape");
  a.part_o = reinterpret_cast<float*>(part_o.data_ptr());
  a.part_ml = reinterpret_cast<float*>(part_ml.data_ptr());
  if (tickets.has_value() && tickets->defined()) {
    CHECK_DEV(*tickets); CHECK_DT(*tickets, torch::kInt32);
    TORCH_CHECK(tickets->numel() >= (int64_t)a.S * Hkv, "attention: tickets need S*Hkv zeroed int32");
    a.tickets = reinterpret_cast<uint32_t*>(tickets->data_ptr());
  }
  if (dbg_ts.has_value() && dbg_ts->defined()) {
    CHECK_DEV(*dbg_ts); CHECK_DT(*dbg_ts, torch::kInt64);
    TORCH_CHECK(dbg_ts->numel() >= 16, "attention: dbg_ts needs 16 int64");
    a.dbg_ts = reinterpret_cast<unsigned long long*>(dbg_ts->data_ptr());
  }
  c10::DeviceGuard guard(q.device());
  vgate::launch_attention(a, a.S, cur_stream());
}

void sample(const Tensor& logits, const c10::optional<Tensor>& temperature,
            const c10::optional<Tensor>& top_p, const c10::optional<Tensor>& top_k,
            const c10::optional<Tensor>& seeds, const c10::optional<Tensor>& offsets, Tensor& out,
            const c10::optional<Tensor>& out_logprob, const c10::optional<Tensor>& ws,
            const c10::optional<Tensor>& fault) {
  CHECK_DEV(logits); CHECK_DEV(out);
  CHECK_DT(logits, torch::kFloat32); CHECK_DT(out, torch::kInt32);
  CHECK_LASTDIM(logits);
  vgate::SampleArgs s{};
  s.logits = reinterpret_cast<const float*>(logits.data_ptr());
  s.ldl = (int)logits.stride(0);
  s.B = (int)logits.size(0);
  s.V = (int)logits.size(1);
  TORCH_CHECK(s.V % 4 == 0 && s.ldl % 4 == 0 && (reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16) == 0,
              "sample: vocab and row stride must be multiples of 4 floats (16-B aligned rows)");
  auto fp = [](const c10::optional<Tensor>& t, c10::ScalarType dt) -> const void* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == dt, "sample: dtype mismatch");
    TORCH_CHECK(t->is_cuda(), "sample: GPU tensor expected");
    return t->data_ptr();
  };
  s.temperature = static_cast<const float*>(fp(temperature, torch::kFloat32));
  s.top_p = static_cast<const float*>(fp(top_p, torch::kFloat32));
  s.top_k = static_cast<const int32_t*>(fp(top_k, torch::kInt32));
  s.seeds = static_cast<const uint64_t*>(fp(seeds, torch::kInt64));
  s.offsets = static_cast<const int64_t*>(fp(offsets, torch::kInt64));
  s.out = reinterpret_cast<int32_t*>(out.data_ptr());
  s.out_logprob = const_cast<float*>(static_cast<const float*>(fp(out_logprob, torch::kFloat32)));
  if (ws.has_value() && ws->defined()) {
    // per-row epochs, then one fixed granule region per row (launchers.h SAMPLE_WS_*)
    TORCH_CHECK(ws->scalar_type() == torch::kInt32 && ws->is_cuda() && ws->numel() >= vgate::SAMPLE_WS_WORDS,
                "sample: ws must be int32[>=", vgate::SAMPLE_WS_WORDS, "]");
    if (s.B <= vgate::SAMPLE_GRAN_ROWS) {
      s.epoch = reinterpret_cast<uint32_t*>(ws->data_ptr());
      s.gran = reinterpret_cast<int32_t*>(ws->data_ptr()) + vgate::SAMPLE_WS_GRAN;
    }
  }
  s.fault = reinterpret_cast<uint32_t*>(opt_ptr<int32_t>(fault, torch::kInt32, "fault"));
  c10::DeviceGuard guard(logits.device());
  vgate::launch_sample(s, cur_stream());
}

// Warm the memory-side cache with a tensor's bytes (default-policy read sweep, nothing written).
// Copy the first `nbytes` (rounded up to 16, within both tensors) between a pinned host tensor and
// a device tensor with a kernel on the current stream (no SDMA engine hand-off, see elementwise.hip).
static void* device_view(const Tensor& t) {
  if (t.is_cuda()) return t.data_ptr();
  TORCH_CHECK(t.is_pinned(), "kernel_copy: host tensor must be pinned");
  void* d = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&d, t.data_ptr(), 0) == hipSuccess && d != nullptr,
              "kernel_copy: pinned host memory is not device-mapped");
  return d;
}

void kernel_copy(Tensor& dst, const Tensor& src, int64_t nbytes) {
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous(), "kernel_copy: contiguous tensors");
  TORCH_CHECK(dst.is_cuda() != src.is_cuda(), "kernel_copy: one host (pinned) and one device tensor");
  const int64_t n = (nbytes + 15) / 16 * 16;
  TORCH_CHECK(n <= (int64_t)(dst.numel() * dst.element_size()) && n <= (int64_t)(src.numel() * src.element_size()),
              "kernel_copy: 16-B rounded size exceeds a tensor");
  const Tensor& dev = dst.is_cuda() ? dst : src;
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "kernel_copy: 16-B aligned tensors");
  c10::DeviceGuard guard(dev.device());
  vgate::launch_copy16(device_view(src), device_view(dst), (size_t)n, !dst.is_cuda(), cur_stream());
}

void ids_to_host(const Tensor& ids, Tensor& ring, const Tensor& slot, int64_t n, int64_t ar_base,
                 const c10::optional<Tensor>& fault) {
  CHECK_DEV(ids); CHECK_DEV(slot);
  CHECK_DT(ids, torch::kInt32); CHECK_DT(ring, torch::kInt32); CHECK_DT(slot, torch::kInt32);
  TORCH_CHECK(ring.dim() == 2 && ring.is_contiguous() && !ring.is_cuda(), "ids_to_host: ring = pinned int32 [slots, stride]");
  TORCH_CHECK(n >= 0 && n <= ids.numel() && n <= ring.size(1), "ids_to_host: n exceeds ids or a ring slot");
  const uint32_t* fw = reinterpret_cast<const uint32_t*>(opt_ptr<int32_t>(fault, torch::kInt32, "fault"));
  TORCH_CHECK((ar_base == 0 && fw == nullptr) || n <= ring.size(1) - 4,
              "ids_to_host: the all-reduce / fault words need the slot's last 4 ints");
  const uint32_t* ar = ar_base ? reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(ar_base) + vgate::ar_error_offset())
                               : nullptr;
  c10::DeviceGuard guard(ids.device());
  vgate::launch_ids_to_host(reinterpret_cast<const int32_t*>(ids.data_ptr()), reinterpret_cast<int32_t*>(device_view(ring)),
                            reinterpret_cast<const int32_t*>(slot.data_ptr()), (int)ring.size(1), (int)n, cur_stream(), ar,
                            fw);
}

void prefetch(const Tensor& t, int64_t blocks) {
  CHECK_DEV(t);
  TORCH_CHECK(t.is_contiguous(), "prefetch: contiguous tensor");
  c10::DeviceGuard guard(t.device());
  vgate::launch_prefetch(t.data_ptr(), (size_t)t.numel() * t.element_size(), (int)blocks, cur_stream());
}

// Launch timeline (profiling): every launch while active takes 2 x blocks u64 stamps of buf.
void timeline_start(Tensor& buf) {
  CHECK_DEV(buf); CHECK_DT(buf, torch::kInt64);
  TORCH_CHECK(buf.is_contiguous(), "timeline buffer must be contiguous");
  vgate::tl_start(reinterpret_cast<unsigned long long*>(buf.data_ptr()), buf.numel());
}

std::vector<std::tuple<std::string, int64_t, int64_t>> timeline_entries() {
  std::vector<std::tuple<std::string, int64_t, int64_t>> r;
  for (int i = 0; i < vgate::tl_count(); ++i) r.emplace_back(vgate::tl_name(i), vgate::tl_offset(i), vgate::tl_blocks(i));
  return r;
}

// ---- custom all-reduce: IPC-shared uncached buffers (vgate/parallel/custom_allreduce.py) ----
#define HIP_OK(x) do { hipError_t e_ = (x); TORCH_CHECK(e_ == hipSuccess, #x ": ", hipGetErrorString(e_)); } while (0)

int64_t ar_alloc(int64_t bytes) {
  void* p = nullptr;
  HIP_OK(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached));
  HIP_OK(hipMemset(p, 0, (size_t)bytes));
  HIP_OK(hipDeviceSynchronize());
  return reinterpret_cast<int64_t>(p);
}

void ar_free(int64_t ptr) { HIP_OK(hipFree(reinterpret_cast<void*>(ptr))); }

Tensor ar_ipc_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  Tensor t = torch::empty({(int64_t)sizeof(h)}, torch::kUInt8);
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

int64_t ar_open(const Tensor& handle) {
  TORCH_CHECK(handle.numel() == (int64_t)sizeof(hipIpcMemHandle_t) && !handle.is_cuda(), "ar_open: 64-byte CPU handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  void* p = nullptr;
  HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<int64_t>(p);
}

void ar_close(int64_t ptr) { HIP_OK(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr))); }

// error word of the own signal area (a wait timed out); clears it
int64_t ar_error(int64_t own_base) {
  uint32_t v = 0, z = 0;
  const size_t off = (size_t)vgate::ar_error_offset();
  HIP_OK(hipMemcpy(&v, reinterpret_cast<char*>(own_base) + off, 4, hipMemcpyDeviceToHost));
  if (v) HIP_OK(hipMemcpy(reinterpret_cast<char*>(own_base) + off, &z, 4, hipMemcpyHostToDevice));
  return v;
}

void custom_allreduce(const Tensor& inp, Tensor& out, const std::vector<int64_t>& bases, int64_t rank,
                      int64_t max_bytes, int64_t two_shot) {
  CHECK_DEV(inp); CHECK_DEV(out);
  CHECK_DT(inp, torch::kBFloat16); CHECK_DT(out, torch::kBFloat16);
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.numel() == out.numel(), "custom_allreduce: contiguous, same size");
  const int64_t nbytes = inp.numel() * 2;
  TORCH_CHECK(nbytes % 16 == 0 && nbytes <= max_bytes, "custom_allreduce: bytes ", nbytes, " (need %16, <= ", max_bytes, ")");
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "custom_allreduce: world 1..8");
  std::vector<char*> b(world);
  for (int i = 0; i < world; ++i) b[i] = reinterpret_cast<char*>(bases[i]);
  c10::DeviceGuard guard(inp.device());
  vgate::launch_custom_allreduce(inp.data_ptr(), out.data_ptr(), nbytes, b.data(), (int)rank, world, max_bytes,
                                 cur_stream(), (int)two_shot);
}

void custom_allgather(const Tensor& inp, Tensor& out, const std::vector<int64_t>& bases, int64_t rank,
                      int64_t max_bytes) {
  CHECK_DEV(inp); CHECK_DEV(out);
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.scalar_type() == out.scalar_type(),
              "custom_allgather: contiguous, same dtype");
  const int world = (int)bases.size();
  const int64_t nbytes = inp.numel() * inp.element_size();
  TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "custom_allgather: world 1..8");
  TORCH_CHECK(nbytes % 16 == 0 && nbytes <= max_bytes, "custom_allgather: bytes ", nbytes, " (need %16, <= ", max_bytes, ")");
  TORCH_CHECK(out.numel() == inp.numel() * world, "custom_allgather: out must hold world x input");
  std::vector<char*> b(world);
  for (int i = 0; i < world; ++i) b[i] = reinterpret_cast<char*>(bases[i]);
  c10::DeviceGuard guard(inp.device());
  vgate::launch_custom_allgather(inp.data_ptr(), out.data_ptr(), nbytes, b.data(), (int)rank, world, max_bytes,
                                 cur_stream());
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "vgate gfx950 (MI355X) HIP kernels and native runtime";
  namespace py = pybind11;
  m.def("gemm", &gemm, "fragment-packed MFMA GEMM (+RMSNorm prologue, split-K, fused epilogues; bf16 or AWQ int4)",
        py::arg("x"), py::arg("wp"), py::arg("N"), py::arg("K"), py::arg("out"), py::arg("epi") = 0,
        py::arg("bias") = py::none(), py::arg("res") = py::none(), py::arg("norm_w") = py::none(),
        py::arg("eps") = 1e-6, py::arg("row_idx") = py::none(), py::arg("ws") = py::none(),
        py::arg("waves") = 0, py::arg("splitk") = 0, py::arg("positions") = py::none(),
        py::arg("slots") = py::none(), py::arg("cos_sin") = py::none(), py::arg("k_cache") = py::none(),
        py::arg("v_cache") = py::none(), py::arg("hq") = 0, py::arg("hkv") = 0,
        py::arg("awq_scales") = py::none(), py::arg("awq_zeros") = py::none(), py::arg("group") = 128,
        py::arg("rownorm") = false, py::arg("dbg_ts") = py::none(), py::arg("ntb") = 0, py::arg("path") = 0,
        py::arg("awq_szp") = py::none(), py::arg("hg_out") = py::none(), py::arg("hg_gamma") = py::none(),
        py::arg("ssp_out") = py::none(), py::arg("ssp_in") = py::none(), py::arg("sk_ws") = py::none(),
        py::arg("fault") = py::none(), py::arg("ar_bases") = std::vector<int64_t>{}, py::arg("ar_rank") = 0,
        py::arg("ar_fused_off") = 0, py::arg("fa_block_tables") = py::none(), py::arg("fa_context_lens") = py::none(),
        py::arg("fa_query_start") = py::none(), py::arg("fa_out") = py::none(), py::arg("fa_part_o") = py::none(),
        py::arg("fa_part_ml") = py::none(), py::arg("fa_tickets") = py::none(), py::arg("fa_sync") = py::none(),
        py::arg("fa_part_size") = 512, py::arg("fa_scale") = 1.0, py::arg("fa_dbg_ts") = py::none());
  m.def("attention", &attention, "unified paged attention: decode (partitions merged in-launch) + varlen prefill tiles",
        py::arg("q"), py::arg("q_stride"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"),
        py::arg("context_lens"), py::arg("query_start"), py::arg("tile_seq"), py::arg("tile_q0"), py::arg("out"),
        py::arg("part_o"), py::arg("part_ml"), py::arg("Hq"), py::arg("Hkv"), py::arg("part_size"), py::arg("scale"),
        py::arg("out_stride") = 0, py::arg("tickets") = py::none(), py::arg("dbg_ts") = py::none(),
        py::arg("flash_ws") = py::none(), py::arg("fault") = py::none());
  m.def("embedding", &embedding, "vocab-sharded embedding gather (negative ids: previous step's samples)",
        py::arg("ids"), py::arg("table"), py::arg("out"), py::arg("vstart") = 0, py::arg("prev") = py::none());
  m.def("rmsnorm", &rmsnorm, "RMSNorm with optional fused residual add");
  m.def("rope_kv", &rope_kv, "NeoX RoPE + paged KV-cache write (rotated q in place or into q_out)",
        py::arg("qkv"), py::arg("positions"), py::arg("slots"), py::arg("cos_sin"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"), py::arg("q_out") = py::none());
  m.def("awq_dequant", &awq_dequant, "AWQ int4 packed -> bf16 fragment-packed (prefill operand; optional gamma fold)",
        py::arg("wq"), py::arg("scales"), py::arg("sz"), py::arg("N"), py::arg("K"), py::arg("group"), py::arg("out"),
        py::arg("gamma") = py::none());
  m.def("silu_mul", &silu_mul, "out = silu(y[:, :I]) * y[:, I:] (library gate_up epilogue)");
  m.def("attn_decode", &attn_decode, "paged split-K decode attention");
  m.def("attn_prefill", &attn_prefill, "paged varlen causal prefill attention",
        py::arg("q"), py::arg("q_stride"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"),
        py::arg("context_lens"), py::arg("query_start"), py::arg("tile_seq"), py::arg("tile_q0"), py::arg("out"),
        py::arg("Hq"), py::arg("Hkv"), py::arg("scale"), py::arg("flash_ws") = py::none(),
        py::arg("fault") = py::none());
  m.def("sample", &sample, "temperature/top-k/top-p sampling (segmented Gumbel-max + exact rejection)",
        py::arg("logits"), py::arg("temperature"), py::arg("top_p"), py::arg("top_k"), py::arg("seeds"),
        py::arg("offsets"), py::arg("out"), py::arg("out_logprob") = py::none(), py::arg("ws") = py::none(),
        py::arg("fault") = py::none());
  m.def("sample_segments", &vgate::sample_segments, "blocks per row the sampler uses for (B, V)");
  m.def("set_sample_nseg", &vgate::set_sample_nseg, "cap the sampler's segments per row (1 = one block per row)");
  m.attr("SAMPLE_WS_WORDS") = vgate::SAMPLE_WS_WORDS;
  m.def("kernel_copy", &kernel_copy, "pinned host <-> device copy by a kernel on the current stream (no SDMA)",
        py::arg("dst"), py::arg("src"), py::arg("nbytes"));
  m.def("set_flash_prefill", &vgate::set_flash_prefill, "flash prefill attention: 1 on, 0 off, -1 environment");
  m.def("set_dec_u", &vgate::set_dec_u, "decode GEMM register group: 0 auto, -1 round-2 rule, 6/8/10/12 forced, -100 environment");
  m.def("ids_to_host", &ids_to_host, "sampled ids -> slot *slot of a pinned host ring (graph-capturable, device-read slot)",
        py::arg("ids"), py::arg("ring"), py::arg("slot"), py::arg("n"), py::arg("ar_base") = 0,
        py::arg("fault") = py::none());
  m.def("prefetch", &prefetch, "read a tensor once with the default cache policy (MALL warm-up)",
        py::arg("t"), py::arg("blocks") = 256);
  m.def("ar_alloc", &ar_alloc, "uncached device allocation for the custom all-reduce (zeroed)");
  m.def("ar_free", &ar_free);
  m.def("ar_ipc_handle", &ar_ipc_handle, "hipIpcMemHandle of an ar_alloc pointer (64 bytes, CPU uint8)");
  m.def("ar_open", &ar_open, "map a peer's ar_alloc buffer (hipIpcOpenMemHandle)");
  m.def("ar_close", &ar_close);
  m.def("ar_error", &ar_error, "read-and-clear the wait-timeout word of the own signal area");
  m.def("ar_fused_bytes", [] { return vgate::AR_FUSED_BYTES; },
        "bytes of the fused row-parallel GEMM + all-reduce region (after the two data buffers)");
  m.def("ar_blocks", &vgate::ar_blocks_used, "workgroups per custom all-reduce call (VGATE_AR_BLOCKS)");
  m.def("custom_allreduce", &custom_allreduce, "one-shot bf16 all-reduce over IPC-mapped peer buffers",
        py::arg("inp"), py::arg("out"), py::arg("bases"), py::arg("rank"), py::arg("max_bytes"),
        py::arg("two_shot") = 0);
  m.def("custom_allgather", &custom_allgather, "all-gather over IPC-mapped peer buffers (rank-major output)",
        py::arg("inp"), py::arg("out"), py::arg("bases"), py::arg("rank"), py::arg("max_bytes"));
  m.def("timeline_start", &timeline_start, "start a launch timeline in an int64 device buffer (zero it first)");
  m.def("timeline_stop", &vgate::tl_stop, "stop handing out timeline slots; returns the slots used");
  m.def("timeline_entries", &timeline_entries, "(kernel, offset, blocks) per launch since timeline_start");
  vgate::bind_runtime(m);
  vgate::bind_step_ring(m);
  py::class_<vgate::ShardedLRU>(m, "ShardedLRU", "sharded LRU of bytes values (result cache backend 'native')")
      .def(py::init<int64_t, int64_t>(), py::arg("capacity"), py::arg("shards") = 16)
      .def("get", [](vgate::ShardedLRU& c, const std::string& k) -> py::object {
             std::optional<std::string> v;
             {
               py::gil_scoped_release nogil;
               v = c.get(k);
             }
             if (!v) return py::none();
             return py::bytes(*v);
           })
      .def("put", [](vgate::ShardedLRU& c, const std::string& k, py::bytes v) {
             std::string val = v;  // copied under the GIL
             py::gil_scoped_release nogil;
             return c.put(k, std::move(val));
           })
      .def("erase", &vgate::ShardedLRU::erase, py::call_guard<py::gil_scoped_release>())
      .def("clear", &vgate::ShardedLRU::clear, py::call_guard<py::gil_scoped_release>())
      .def("__len__", &vgate::ShardedLRU::size)
      .def_property_readonly("capacity", &vgate::ShardedLRU::capacity)
      .def_property_readonly("num_shards", &vgate::ShardedLRU::num_shards)
      .def_property_readonly("hits", &vgate::ShardedLRU::hits)
      .def_property_readonly("misses", &vgate::ShardedLRU::misses)
      .def_property_readonly("evictions", &vgate::ShardedLRU::evictions);
}
