// Input-pipeline kernel: uint8 NHWC images -> the bf16 NHWC compute tensor of the CNN stems.
//
// y[p][c] = (x[p][c] / 255 - mean[c]) / std[c] for c < cin, 0 for cin <= c < cout (the stem's padded
// channels, which must stay exactly zero).  One thread per pixel: cin byte loads, one 16-byte store
// for cout = 8.  Replaces the ~8 elementwise launches (cast, scale, subtract, divide, zero-fill,
// slice copy) of the PyTorch formulation at the head of every training step.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

struct Norm4 {
  float scale[4], shift[4];  // y = x * scale + shift  (scale = 1 / (255 std), shift = -mean / std)
};

template <int COUT>
__global__ void __launch_bounds__(256) image_norm_kernel(const uint8_t* __restrict__ x, int64_t npix, int cin,
                                                         Norm4 nm, uint16_t* __restrict__ y) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < npix; p += (int64_t)gridDim.x * 256) {
    float f[COUT];
#pragma unroll
    for (int c = 0; c < COUT; ++c) f[c] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < cin) f[c] = fmaf((float)x[p * cin + c], nm.scale[c], nm.shift[c]);
    if constexpr (COUT == 8) {
      reinterpret_cast<U4*>(y)[p] = pack8(f);
    } else {
#pragma unroll
      for (int c = 0; c < COUT; ++c) y[p * COUT + c] = f32_to_bf16(f[c]);
    }
  }
}

}  // namespace

void image_normalize(const uint8_t* x, int64_t npix, int cin, int cout, const float* mean, const float* stdv,
                     uint16_t* y, hipStream_t s) {
  Norm4 nm{};
  for (int c = 0; c < 4; ++c) {
    const float m = c < cin ? mean[c] : 0.f, sd = c < cin ? stdv[c] : 1.f;
    nm.scale[c] = 1.f / (255.f * sd);
    nm.shift[c] = -m / sd;
  }
  int64_t g = (npix + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (cout == 8) image_norm_kernel<8><<<(int)g, 256, 0, s>>>(x, npix, cin, nm, y);
  else image_norm_kernel<4><<<(int)g, 256, 0, s>>>(x, npix, cin, nm, y);
}

}  // namespace tfx
