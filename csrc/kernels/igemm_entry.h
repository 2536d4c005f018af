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
void igemm_dgrad_flip(IgemmArgs& a, hipStream_t s);      // 3x3 s1: im2col(dY) . Wf^T (+ fused BN backward)
void igemm_dgrad_cls_dense(IgemmArgs& a, hipStream_t s); // single-tap stride-2 parity class
void igemm_dgrad_cls(IgemmArgs& a, hipStream_t s);       // stride-2 parity class, gathered
void igemm_wgrad_dense(IgemmArgs& a, hipStream_t s);     // dY^T . X (1x1) -- f32 atomics, split-K
void igemm_wgrad_x(IgemmArgs& a, hipStream_t s);         // dY^T . im2col(X)
void igemm_wgrad_t_x(IgemmArgs& a, hipStream_t s);       // im2col(X)^T . dY (transposed store)
void igemm_gemm(IgemmArgs& a, hipStream_t s);            // plain GEMMs (FC layers, LSTM)
// persistent 1x1 forward (igemm_persist.hip): one continuous LDS-DMA ring over all of a block's tiles
bool igemm_fwd_persist_ok(const IgemmArgs& a);
void igemm_fwd_persist(IgemmArgs& a, hipStream_t s);

// ---- measured launch configurations (igemm.hip; table from scripts/tune_convs.py)
// family = which entry above launched; a config overrides the built-in heuristics of launch_shape /
// launch_t: tile 1 = 128x128, 2 = 128x64, 3 = 256x64 (bf16-output families only); ks 1 / 2 =
// in-block split-K groups (f32-atomic families); gls = LDS-DMA ring depth (0 = register pipeline);
// want = split-K block target.  0 / -1 = keep the heuristic's choice.
enum {
  FAM_FWD_PW = 0, FAM_FWD_X, FAM_DGRAD_PW, FAM_DGRAD_X, FAM_DGRAD_CLS_DENSE, FAM_DGRAD_CLS, FAM_WGRAD_DENSE,
  FAM_WGRAD_X, FAM_WGRAD_T_X, FAM_DGRAD_FLIP, FAM_COUNT
};
struct TuneCfg {
  int tile = 0, ks = 0, gls = -1, want = 0;
};
bool igemm_tune_lookup(int fam, int M, int N, int K, TuneCfg* out);  // also records the launch when tracing
void igemm_tune_set(int fam, int M, int N, int K, TuneCfg c);
void igemm_tune_clear();
void igemm_tune_force(int fam, TuneCfg c);  // every launch of `fam` (fam < 0: clear every force)
void igemm_tune_trace(bool on);             // start (clearing) / stop recording launches
int igemm_tune_traced(int* out, int cap);   // recorded launches as (fam, M, N, K) quadruples
}  // namespace tfx
