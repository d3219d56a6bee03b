// int4 (AWQ W4A16) instantiations of the register-stationary decode GEMM (gemm_kx.h).
#include "gemm_kx.h"

namespace vgate {

bool launch_awq_kx(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.M > 16 || g.awq_szp == nullptr || g.group != 128 || g.N % 16 != 0 || g.K % 128 != 0 ||
      g.rownorm || g.ar_world > 0 || (g.ssp_in != nullptr && g.norm_w != nullptr) || g.epi == EPI_F32)
    return false;
  const GemmParams p = kx_params(g);
  const int norm = g.norm_w != nullptr ? 1 : g.ssp_in != nullptr ? 3 : 0;
#define VG_KX(E)                                              \
  return norm == 1 ? kx_launch<true, E, 1>(p, g, st)          \
       : norm == 3 ? kx_launch<true, E, 3>(p, g, st)          \
                   : kx_launch<true, E, 0>(p, g, st)
  switch (g.epi) {
    case EPI_SILU: VG_KX(EPI_SILU);
    case EPI_QKV: VG_KX(EPI_QKV);
    default: VG_KX(EPI_BF16);
  }
#undef VG_KX
}

}  // namespace vgate
