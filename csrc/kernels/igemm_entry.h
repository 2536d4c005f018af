// Entry points of the implicit-GEMM kernel families, one translation unit per group (igemm_*.hip)
// so the heavy template instantiations compile in parallel.  igemm.hip's igemm_launch validates the
// arguments and dispatches here.
#pragma once
#include "tfx_kernels.h"

namespace tfx {
void igemm_fwd_pointwise(IgemmArgs& a, hipStream_t s);   // X[M][C] . W[Ko][C]^T (+ fused BN stats)
void igemm_fwd_im2col(IgemmArgs& a, hipStream_t s);      // im2col(X) . W^T (+ fused BN stats)
void igemm_dgrad_pointwise(IgemmArgs& a, hipStream_t s); // dY[M][Ko] . W[Ko][C] (+ fused BN backward)
void igemm_dgrad_general(IgemmArgs& a, hipStream_t s);   // gathered dY . W (+ fused BN backward)
void igemm_dgrad_cls_dense(IgemmArgs& a, hipStream_t s); // single-tap stride-2 parity class
void igemm_dgrad_cls(IgemmArgs& a, hipStream_t s);       // stride-2 parity class, gathered
void igemm_wgrad_dense(IgemmArgs& a, hipStream_t s);     // dY^T . X (1x1) -- f32 atomics, split-K
void igemm_wgrad_x(IgemmArgs& a, hipStream_t s);         // dY^T . im2col(X)
void igemm_wgrad_t_x(IgemmArgs& a, hipStream_t s);       // im2col(X)^T . dY (transposed store)
void igemm_gemm(IgemmArgs& a, hipStream_t s);            // plain GEMMs (FC layers, LSTM)
}  // namespace tfx
