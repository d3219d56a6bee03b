// EPI_BF16 instantiations of the decode / small-M GEMM family (gemm_decode.h), one translation unit
// per epilogue so the kernel variants compile in parallel (csrc/build.py).
#include "gemm_decode.h"

namespace vgate {
template void dispatch_epi<EPI_BF16, false>(GemmParams, const GemmArgs&, hipStream_t);
template void dispatch_epi<EPI_BF16, true>(GemmParams, const GemmArgs&, hipStream_t);
}  // namespace vgate
