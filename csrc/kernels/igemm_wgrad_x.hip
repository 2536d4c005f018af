// Implicit-GEMM instantiations: gathered weight gradient (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
// a 64-pixel k-tile covers whole output rows of one image, or whole images (MN_WGRAD_XT)
static bool xt_ok(const IgemmArgs& a) {
  const int PQ = a.P * a.Q;
  return igemm_xt_enabled() && ((PQ % 64 == 0 && 64 % a.Q == 0) || (64 % PQ == 0));
}
void igemm_wgrad_x(IgemmArgs& a, hipStream_t s) {
  if (xt_ok(a)) launch_shape<MN_DENSE, MN_WGRAD_XT, false>(a, s, FAM_WGRAD_X);
  else launch_shape<MN_DENSE, MN_WGRAD_X, false>(a, s, FAM_WGRAD_X);
}
void igemm_wgrad_t_x(IgemmArgs& a, hipStream_t s) {
  if (xt_ok(a)) launch_shape<MN_WGRAD_XT, MN_DENSE, false>(a, s, FAM_WGRAD_T_X);
  else launch_shape<MN_WGRAD_X, MN_DENSE, false>(a, s, FAM_WGRAD_T_X);
}
}  // namespace tfx
