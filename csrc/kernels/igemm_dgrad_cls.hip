// Implicit-GEMM instantiations: stride-2 data gradient parity classes (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
void igemm_dgrad_cls_dense(IgemmArgs& a, hipStream_t s) { launch_shape<KM_DENSE, MN_DENSE>(a, s, FAM_DGRAD_CLS_DENSE); }
void igemm_dgrad_cls(IgemmArgs& a, hipStream_t s) { launch_shape<KM_DGRAD_DY, MN_DGRAD_W2>(a, s, FAM_DGRAD_CLS); }
}  // namespace tfx
