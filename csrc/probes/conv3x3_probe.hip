// Cost probes of the stage-1 fused 3x3 conv kernels (scripts/dev/conv3x3_probe.py): the production kernels
// of conv3x3_fused.hip instantiated with their PROBE bits (phases skipped; outputs wrong, timing only).
// Not part of libtfx_ops.so (build: scripts/dev/build_probes.sh).
#include "../kernels/conv3x3_fused.hip"

namespace tfx {
namespace {
template <int P>
void fwd_p(const Conv3Args& a, hipStream_t s) {
  conv3x3_fwd_fused_kernel<P><<<std::min(256, a.N * (a.H / C3_TR)), PW_NT, 0, s>>>(a);
}
template <int P>
void bwd_p(const Conv3BwdArgs& a, hipStream_t s) {
  conv3x3_bwd_fused_kernel<P><<<std::min(256, a.N * (a.H / C3_TR)), PW_NT, 0, s>>>(a);
}
}  // namespace
}  // namespace tfx

// x / y1 / y2 / g2 / dx: [N][H][32][64] bf16; save*: [4][64]; red2 [2][64]; w [64][3][3][64]; slots [64][2][64];
// slab [256][64 * 576] f32
extern "C" int tfx_probe_conv3_fwd(int probe, const void* x, const float* save_in, const void* w, void* y, float* slots,
                                   int N, int H, void* stream) {
  using namespace tfx;
  if (!conv3x3_fused_ok(N, H, 32, 64, 64)) return -1;
  Conv3Args a;
  a.x = (const uint16_t*)x; a.save_in = save_in; a.w = (const uint16_t*)w; a.y = (uint16_t*)y; a.slots = slots;
  a.N = N; a.H = H;
  hipStream_t s = (hipStream_t)stream;
  switch (probe) {
    case 0: fwd_p<0>(a, s); break;
    case 1: fwd_p<1>(a, s); break;
    case 2: fwd_p<2>(a, s); break;
    case 3: fwd_p<3>(a, s); break;
    case 4: fwd_p<4>(a, s); break;
    case 7: fwd_p<7>(a, s); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int tfx_probe_conv3_bwd(int probe, const void* g2, const void* y2, const float* save2, const float* red2,
                                   const void* y1, const float* save1, const void* w, void* dx, float* slots1,
                                   float* slab, int N, int H, void* stream) {
  using namespace tfx;
  if (!conv3x3_fused_ok(N, H, 32, 64, 64)) return -1;
  Conv3BwdArgs a;
  a.g2 = (const uint16_t*)g2; a.y2 = (const uint16_t*)y2; a.save2 = save2; a.red2 = red2;
  a.y1 = (const uint16_t*)y1; a.save1 = save1; a.w = (const uint16_t*)w; a.dx = (uint16_t*)dx;
  a.slots1 = slots1; a.slab = slab; a.N = N; a.H = H;
  hipStream_t s = (hipStream_t)stream;
  switch (probe) {
#define P(v) case v: bwd_p<v>(a, s); break;
    P(0) P(1) P(2) P(3) P(4) P(8) P(16) P(24) P(27) P(31) P(28) P(7)
#undef P
    default: return -2;
  }
  return (int)hipGetLastError();
}
