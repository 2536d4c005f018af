// Implicit-GEMM instantiation: stride-1 3x3 (pad 1) data gradient run as the FORWARD conv of dY with
// the flipped, channel-transposed filter Wf[c][r][s][ko] = W[ko][2-r][2-s][c]: dX = conv(dY, Wf).
// The A operand is then the forward's K-major im2col gather of dY and B a dense K-major weight
// image (ds_read_b128), instead of the data-gradient's MN-major W staging (ds_read_b64_tr) -- the
// same GEMM dims as the forward of that conv, with the data gradient's fused BN-backward epilogue.
#include "igemm_impl.h"

namespace tfx {
void igemm_dgrad_flip(IgemmArgs& a, hipStream_t s) {
  if (a.tapmask) launch_epi<KM_FWD_XT, KM_DENSE, EPI_BNB>(a, s, FAM_DGRAD_FLIP);  // Ko % 64 == 0
  else launch_epi<KM_FWD_X, KM_DENSE, EPI_BNB>(a, s, FAM_DGRAD_FLIP);
}
}  // namespace tfx
