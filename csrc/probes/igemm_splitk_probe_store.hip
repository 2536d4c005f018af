// Cost probe of the split-K 1x1 weight gradient's epilogue (scripts/dev/splitk_atomic_probe.py): the
// production kernel igemm_kernel<MN_DENSE, MN_DENSE, 128, 64, .., KS 2, ring 3> launched with the
// production launch configuration, built twice -- with the f32 atomic epilogue and with plain stores
// in its place (wrong sums; timing only).  Not part of libtfx_ops.so (build: scripts/dev/build_probes.sh).
#define TFX_PROBE_SPLITK_STORE 1
#include "../kernels/igemm_impl.h"

extern "C" int tfx_probe_wgrad_store(const void* dy, const void* x, float* dw, int npix, int Ko, int C, int want,
                                  void* stream) {
  using namespace tfx;
  IgemmArgs a;
  a.A = static_cast<const uint16_t*>(dy);
  a.B = static_cast<const uint16_t*>(x);
  a.a_bytes = (int64_t)npix * Ko * 2;
  a.b_bytes = (int64_t)npix * C * 2;
  a.M = Ko; a.N = C; a.K = npix;
  a.lda = Ko; a.ldb = C; a.ldc = C;
  a.out_mode = OUT_F32_ATOMIC;
  a.zero_out = 0;
  a.Cp = dw;
  if (Ko % 128 || C % 64 || npix % 64) return -1;  // the shapes the probe's grid assumes
  g_tc = TuneCfg{2, 2, 3, want};
  launch_t<MN_DENSE, MN_DENSE, 128, 64, EPI_PLAIN, 2>(a, static_cast<hipStream_t>(stream));
  return (int)hipGetLastError();
}
