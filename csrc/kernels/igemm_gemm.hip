// Implicit-GEMM instantiations: plain GEMM (kernel template: igemm_impl.h).
#include "igemm_impl.h"

namespace tfx {
void igemm_gemm(IgemmArgs& a, hipStream_t s) {
  // skinny f32-accumulated GEMMs (the recurrent h @ W_hh^T / dgates @ W_hh of an LSTM step:
  // M = batch <= 128, a few thousand columns): latency-bound, so cut them into many short
  // blocks -- 128x64 tiles, split-K down to min_kps k-tiles per block
  if (a.out_mode == OUT_F32_ATOMIC && a.M <= 128 && kSkinnyMinKps > 0) {
    const int mk = kSkinnyMinKps;
    if (a.a_kmajor && a.b_kmajor) launch_t<KM_DENSE, KM_DENSE, 128, 64>(a, s, 1, mk);
    else if (a.a_kmajor) launch_t<KM_DENSE, MN_DENSE, 128, 64>(a, s, 1, mk);
    else if (a.b_kmajor) launch_t<MN_DENSE, KM_DENSE, 128, 64>(a, s, 1, mk);
    else launch_t<MN_DENSE, MN_DENSE, 128, 64>(a, s, 1, mk);
    return;
  }
  if (a.a_kmajor && a.b_kmajor) launch_t<KM_DENSE, KM_DENSE, 128, 128>(a, s);
  else if (a.a_kmajor) launch_t<KM_DENSE, MN_DENSE, 128, 128>(a, s);
  else if (a.b_kmajor) launch_t<MN_DENSE, KM_DENSE, 128, 128>(a, s);
  else launch_t<MN_DENSE, MN_DENSE, 128, 128>(a, s);
}
}  // namespace tfx
