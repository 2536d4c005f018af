// Implicit-GEMM dispatcher: argument validation and routing to the per-mode kernel families
// (igemm_impl.h: the kernel template; igemm_fwd / _dgrad / _dgrad_cls / _wgrad / _wgrad_x / _gemm.hip:
// their instantiations).  Reference: the matmuls of R/distributed/distributed.py:96-98 and their TF1
// gradients; conv/FC layers of the north-star models (BASELINE.json configs 2-5).
#include "tfx_common.h"
#include "tfx_kernels.h"
#include "igemm_entry.h"

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace tfx {
// TFX_IGEMM_XT=0 routes the 3x3 convs to the round-3 per-element-decode operands (KM_FWD_X /
// MN_WGRAD_X) instead of the tap-uniform ones (A/B and numerics bisection hook; read once)
bool igemm_xt_enabled() {
  static const int on = [] {
    const char* e = getenv("TFX_IGEMM_XT");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}


constexpr int BKT_HOST = 64;  // k-tile depth of igemm_impl.h (BKT)

// ------------------------------------------------------------------ measured launch configurations
// Written at import (tensorflow_examples_amd/ops/tuning.py loads the committed table) or by the
// tuner; read on every launch.  A mutex keeps the rare writes and the reads apart (autograd's device
// thread launches the backward kernels).
namespace {
struct TuneEntry {
  int fam, M, N, K;
  TuneCfg c;
};
std::mutex g_tune_mu;
std::vector<TuneEntry> g_tune;
TuneCfg g_force[FAM_COUNT];
bool g_forced[FAM_COUNT] = {};
bool g_tracing = false;
std::vector<int> g_trace;
}  // namespace

bool igemm_tune_lookup(int fam, int M, int N, int K, TuneCfg* out) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  if (g_tracing) g_trace.insert(g_trace.end(), {fam, M, N, K});
  if (fam < 0 || fam >= FAM_COUNT) return false;
  if (g_forced[fam]) {
    *out = g_force[fam];
    return true;
  }
  for (const auto& e : g_tune)
    if (e.fam == fam && e.M == M && e.N == N && e.K == K) {
      *out = e.c;
      return true;
    }
  return false;
}

void igemm_tune_set(int fam, int M, int N, int K, TuneCfg c) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  for (auto& e : g_tune)
    if (e.fam == fam && e.M == M && e.N == N && e.K == K) {
      e.c = c;
      return;
    }
  g_tune.push_back({fam, M, N, K, c});
}

void igemm_tune_clear() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tune.clear();
}

void igemm_tune_force(int fam, TuneCfg c) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  if (fam < 0) {
    for (int i = 0; i < FAM_COUNT; ++i) g_forced[i] = false;
    return;
  }
  if (fam < FAM_COUNT) {
    g_force[fam] = c;
    g_forced[fam] = true;
  }
}

void igemm_tune_trace(bool on) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  if (on) g_trace.clear();
  g_tracing = on;
}

int igemm_tune_traced(int* out, int cap) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  const int n = (int)g_trace.size() / 4;
  for (int i = 0; i < n && 4 * i + 3 < cap; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = g_trace[4 * i + j];
  return n;
}

void igemm_launch(IgemmArgs a, int mode, hipStream_t s) {
  if (a.out_mode == OUT_F32_ATOMIC && a.zero_out) {
    const size_t rows = a.trans_out ? a.N : a.M;
    TFX_HIP_CHECK(hipMemsetAsync(a.Cp, 0, sizeof(float) * rows * a.ldc, s));
  }
  // a masked addend is applied only by the bf16 16-byte-store epilogue path
  if (a.addend_mask && !(a.addend && a.out_mode == OUT_BF16 && !a.trans_out && (a.ldc & 7) == 0 && (a.N & 7) == 0)) {
    fprintf(stderr, "igemm_launch: masked addend needs a bf16 output with 8-aligned columns\n");
    abort();
  }
  // a stride-2 compact addend likewise (and never with mask bits or a parity-class output)
  if (a.addend_s2 && !(a.addend && !a.addend_mask && !a.cls && a.out_mode == OUT_BF16 && !a.trans_out &&
                       (a.ldc & 7) == 0 && (a.N & 7) == 0)) {
    fprintf(stderr, "igemm_launch: stride-2 compact addend needs a bf16 16-byte-store output\n");
    abort();
  }
  // fused-BN epilogues live in the bf16 16-byte-store path of the forward / data-gradient kernels
  if (a.stats || a.bnb_x) {
    if (!(a.out_mode == OUT_BF16 && !a.trans_out && (a.ldc & 7) == 0 && (a.N & 7) == 0 &&
          (mode == MODE_FWD ||
           (a.bnb_x && (mode == MODE_DGRAD || mode == MODE_DGRAD_FLIP))) &&
          (a.stats == nullptr || a.bnb_x == nullptr))) {
      fprintf(stderr, "igemm_launch: unsupported fused-BN epilogue configuration\n");
      abort();
    }
  }
  // the A-operand BN transform: pointwise forward with the fused statistics epilogue, single k-tile only
  // (the register path's single-tile kernel is the one that applies it)
  if (a.a_scale && !(a.stats && mode == MODE_FWD && a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 &&
                     a.pw == 0 && a.a_shift && a.K % 8 == 0 && a.K <= BKT_HOST)) {
    fprintf(stderr, "igemm_launch: A-operand transform needs a 1x1 stride-1 forward with BN stats and K <= 64\n");
    abort();
  }
  // 1x1 stride-1 unpadded convs (two thirds of ResNet-50's) are plain GEMMs over the NHWC rows:
  // dense loaders instead of the im2col / parity gathers -- no per-row address decode at all.
  const bool pointwise = mode != MODE_GEMM && a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 &&
                         a.pw == 0;
  if (pointwise) {
    switch (mode) {
      case MODE_FWD:  // X[M][C] . W[Ko][C]^T
        a.lda = a.C; a.ldb = a.C;
        if (igemm_fwd_persist_ok(a)) igemm_fwd_persist(a, s);  // one ring over all of a block's tiles
        else igemm_fwd_pointwise(a, s);
        return;
      case MODE_DGRAD:  // dY[M][Ko] . W[Ko][C]
        a.lda = a.Ko; a.ldb = a.C;
        igemm_dgrad_pointwise(a, s);
        return;
      case MODE_WGRAD:  // dY^T[Ko][pix] . X[pix][C]
        a.lda = a.Ko; a.ldb = a.C;
        igemm_wgrad_dense(a, s);
        return;
      case MODE_WGRAD_T:  // X^T[C][pix] . dY[pix][Ko]
        a.lda = a.C; a.ldb = a.Ko;
        igemm_wgrad_dense(a, s);
        return;
      case MODE_DGRAD_CLS:
        // single-tap class aligned with dY (1x1 stride-2 even pixels, 3x3 stride-2 (even, even)):
        // dY[M][Ko] . W[:, tap, :] -- dense operands, the tap folded into B's base; rows remapped
        if (a.H == a.P && a.W == a.Q) {
          const int64_t tap_off = (int64_t)(a.cr0 * a.wS + a.cs0) * a.C;
          a.B += tap_off;
          a.b_bytes -= tap_off * 2;
          a.lda = a.Ko; a.ldb = a.wR * a.wS * a.C;
          igemm_dgrad_cls_dense(a, s);
          return;
        }
        break;
    }
  }
  // im2col operand (forward, flipped-filter data gradient) whose k-tiles each lie in one filter tap
  if ((mode == MODE_FWD || mode == MODE_DGRAD_FLIP) && a.C % BKT_HOST == 0 && a.R * a.S <= 32 && !a.a_scale &&
      igemm_xt_enabled())
    a.tapmask = 1;
  switch (mode) {
    case MODE_FWD: igemm_fwd_im2col(a, s); break;
    case MODE_DGRAD: igemm_dgrad_general(a, s); break;
    case MODE_DGRAD_FLIP: igemm_dgrad_flip(a, s); break;
    case MODE_DGRAD_CLS: igemm_dgrad_cls(a, s); break;
    case MODE_WGRAD: igemm_wgrad_x(a, s); break;
    case MODE_WGRAD_T: igemm_wgrad_t_x(a, s); break;
    default: igemm_gemm(a, s);
  }
}

}  // namespace tfx
