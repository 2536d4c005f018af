// Implicit-GEMM instantiations: conv forward (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
void igemm_fwd_pointwise(IgemmArgs& a, hipStream_t s) { launch_epi<KM_DENSE, KM_DENSE, EPI_STATS>(a, s, FAM_FWD_PW); }
void igemm_fwd_im2col(IgemmArgs& a, hipStream_t s) {
  if (a.tapmask) launch_epi<KM_FWD_XT, KM_DENSE, EPI_STATS>(a, s, FAM_FWD_X);  // C % 64 == 0: one tap per k-tile
  else launch_epi<KM_FWD_X, KM_DENSE, EPI_STATS>(a, s, FAM_FWD_X);
}
}  // namespace tfx
