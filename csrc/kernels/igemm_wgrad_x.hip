// Implicit-GEMM instantiations: gathered weight gradient (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
void igemm_wgrad_x(IgemmArgs& a, hipStream_t s) { launch_shape<MN_DENSE, MN_WGRAD_X, false>(a, s, FAM_WGRAD_X); }
void igemm_wgrad_t_x(IgemmArgs& a, hipStream_t s) { launch_shape<MN_WGRAD_X, MN_DENSE, false>(a, s, FAM_WGRAD_T_X); }
}  // namespace tfx
