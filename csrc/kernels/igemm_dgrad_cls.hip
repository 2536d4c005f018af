// Implicit-GEMM instantiations: stride-2 data gradient parity classes (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
// (+ the fused BN-backward partials: the four class launches add into the same slots, each output pixel
// belongs to exactly one class -- conv_dgrad_bn at stride 2)
void igemm_dgrad_cls_dense(IgemmArgs& a, hipStream_t s) {
  launch_epi<KM_DENSE, MN_DENSE, EPI_BNB>(a, s, FAM_DGRAD_CLS_DENSE);
}
void igemm_dgrad_cls(IgemmArgs& a, hipStream_t s) { launch_epi<KM_DGRAD_DY, MN_DGRAD_W2, EPI_BNB>(a, s, FAM_DGRAD_CLS); }
}  // namespace tfx
