// Implicit-GEMM instantiations: stride-2 data gradient parity classes (kernel template: igemm_impl.h).
// Plain bf16 epilogue (+ addend): the BN-backward reduction of a stride-2 conv's input runs in the
// tail blocks of the same conv's weight-gradient launch instead (ops/nn.py _SR_FUSE2).
#include "igemm_impl.h"

namespace tfx {
void igemm_dgrad_cls_dense(IgemmArgs& a, hipStream_t s) {
  launch_shape<KM_DENSE, MN_DENSE, true, EPI_PLAIN>(a, s, FAM_DGRAD_CLS_DENSE);
}
void igemm_dgrad_cls(IgemmArgs& a, hipStream_t s) {
  launch_shape<KM_DGRAD_DY, MN_DGRAD_W2, true, EPI_PLAIN>(a, s, FAM_DGRAD_CLS);
}
}  // namespace tfx
