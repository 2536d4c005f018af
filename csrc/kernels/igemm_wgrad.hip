// Implicit-GEMM instantiations: 1x1 weight gradient (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
void igemm_wgrad_dense(IgemmArgs& a, hipStream_t s) { launch_shape<MN_DENSE, MN_DENSE, false>(a, s, FAM_WGRAD_DENSE); }
}  // namespace tfx
