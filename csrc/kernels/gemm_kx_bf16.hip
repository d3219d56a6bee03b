// bf16 instantiations of the register-stationary decode GEMM (gemm_kx.h): the dense decode
// projections with the same grid forms as the int4 kernel (WIDE one block per CU owning whole tiles,
// GROUP 1-4 tiles per block + K slices), every weight fragment of a wave requested at once.
#include "gemm_kx.h"

namespace vgate {

bool launch_dense_kx(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.M > 16 || g.N % 16 != 0 || g.K % 128 != 0 || g.norm_w != nullptr || g.ar_world > 0 ||
      g.row_idx != nullptr || g.epi == EPI_F32 || (g.ssp_in != nullptr && g.rownorm))
    return false;
  const GemmParams p = kx_params(g);
  const int norm = g.rownorm ? 2 : g.ssp_in != nullptr ? 3 : 0;
#define VG_KX(E)                                               \
  return norm == 2 ? kx_launch<false, E, 2>(p, g, st)          \
       : norm == 3 ? kx_launch<false, E, 3>(p, g, st)          \
                   : kx_launch<false, E, 0>(p, g, st)
  switch (g.epi) {
    case EPI_SILU: VG_KX(EPI_SILU);
    case EPI_QKV: VG_KX(EPI_QKV);
    default: VG_KX(EPI_BF16);
  }
#undef VG_KX
}

}  // namespace vgate
