// EPI_BF16_AR instantiations (TP row-parallel decode GEMMs with the all-reduce in the epilogue,
// gemm_epilogue.h epilogue_ar): only the one-wave-per-tile decode kernels, no norm modes.
#include "gemm_decode.h"

namespace vgate {
template void dispatch_epi<EPI_BF16_AR, false>(GemmParams, const GemmArgs&, hipStream_t);
template void dispatch_epi<EPI_BF16_AR, true>(GemmParams, const GemmArgs&, hipStream_t);
}  // namespace vgate
