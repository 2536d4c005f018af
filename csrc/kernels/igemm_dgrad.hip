// Implicit-GEMM instantiations: conv data gradient (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
void igemm_dgrad_pointwise(IgemmArgs& a, hipStream_t s) { launch_epi<KM_DENSE, MN_DENSE, EPI_BNB>(a, s, FAM_DGRAD_PW); }
void igemm_dgrad_general(IgemmArgs& a, hipStream_t s) { launch_epi<KM_DGRAD_DY, MN_DGRAD_W, EPI_BNB>(a, s, FAM_DGRAD_X); }
}  // namespace tfx
