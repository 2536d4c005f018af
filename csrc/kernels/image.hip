// Input-pipeline kernel: uint8 NHWC images -> the bf16 NHWC compute tensor of the CNN stems.
//
// y[p][c] = (x[p][c] / 255 - mean[c]) / std[c] for c < cin, 0 for cin <= c < cout (the stem's padded
// channels, which must stay exactly zero).  One thread per pixel: cin byte loads, one 16-byte store
// for cout = 8.  Replaces the ~8 elementwise launches (cast, scale, subtract, divide, zero-fill,
// slice copy) of the PyTorch formulation at the head of every training step.  Optionally the batch's
// int64 labels ride along (lab -> lab_out), so a captured step's static label buffer is filled by the
// same launch instead of a separate copy.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

struct Norm4 {
  float scale[4], shift[4];  // y = x * scale + shift  (scale = 1 / (255 std), shift = -mean / std)
};

template <int COUT>
__global__ void __launch_bounds__(256) image_norm_kernel(const uint8_t* __restrict__ x, int64_t npix, int cin,
                                                         Norm4 nm, uint16_t* __restrict__ y,
                                                         const int64_t* __restrict__ lab, int64_t* __restrict__ lab_out,
                                                         int nlab) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nlab; i += gridDim.x * 256) lab_out[i] = lab[i];
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

// Training augmentation fused with the normalisation: pad-P random crop + horizontal flip of an HxW
// uint8 NHWC batch, written as the normalised bf16 NHWC compute tensor in one pass.
// off[n] = {ox, oy, f}: the crop origin in the padded image (0 .. 2P) and flip = f & 1.  Padding
// pixels are uint8 zeros before the normalisation (as torch.nn.functional.pad of the uint8 batch).
template <int COUT>
__global__ void __launch_bounds__(256) augment_norm_kernel(const uint8_t* __restrict__ x, int N, int H, int W, int cin,
                                                           int pad, const int32_t* __restrict__ off, Norm4 nm,
                                                           uint16_t* __restrict__ y) {
  const int64_t npix = (int64_t)N * H * W;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < npix; p += (int64_t)gridDim.x * 256) {
    const int n = (int)(p / (H * W)), yx = (int)(p - (int64_t)n * H * W), yy = yx / W, xx = yx - yy * W;
    const int ox = off[3 * n], oy = off[3 * n + 1], fl = off[3 * n + 2] & 1;
    const int sy = yy + oy - pad, sx = (fl ? W - 1 - xx : xx) + ox - pad;
    const bool in = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
    const uint8_t* src = x + (((int64_t)n * H + (in ? sy : 0)) * W + (in ? sx : 0)) * cin;
    float f[COUT];
#pragma unroll
    for (int c = 0; c < COUT; ++c) f[c] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < cin) f[c] = fmaf(in ? (float)src[c] : 0.f, nm.scale[c], nm.shift[c]);
    if constexpr (COUT == 8) {
      reinterpret_cast<U4*>(y)[p] = pack8(f);
    } else {
#pragma unroll
      for (int c = 0; c < COUT; ++c) y[p * COUT + c] = f32_to_bf16(f[c]);
    }
  }
}

}  // namespace

void augment_normalize(const uint8_t* x, int N, int H, int W, int cin, int cout, int pad, const int32_t* off,
                       const float* mean, const float* stdv, uint16_t* y, hipStream_t s) {
  Norm4 nm{};
  for (int c = 0; c < 4; ++c) {
    const float m = c < cin ? mean[c] : 0.f, sd = c < cin ? stdv[c] : 1.f;
    nm.scale[c] = 1.f / (255.f * sd);
    nm.shift[c] = -m / sd;
  }
  int64_t g = ((int64_t)N * H * W + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (cout == 8) augment_norm_kernel<8><<<(int)g, 256, 0, s>>>(x, N, H, W, cin, pad, off, nm, y);
  else augment_norm_kernel<4><<<(int)g, 256, 0, s>>>(x, N, H, W, cin, pad, off, nm, y);
}

void image_normalize(const uint8_t* x, int64_t npix, int cin, int cout, const float* mean, const float* stdv,
                     uint16_t* y, hipStream_t s, const int64_t* lab, int64_t* lab_out, int nlab) {
  Norm4 nm{};
  for (int c = 0; c < 4; ++c) {
    const float m = c < cin ? mean[c] : 0.f, sd = c < cin ? stdv[c] : 1.f;
    nm.scale[c] = 1.f / (255.f * sd);
    nm.shift[c] = -m / sd;
  }
  int64_t g = (npix + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (cout == 8) image_norm_kernel<8><<<(int)g, 256, 0, s>>>(x, npix, cin, nm, y, lab, lab_out, nlab);
  else image_norm_kernel<4><<<(int)g, 256, 0, s>>>(x, npix, cin, nm, y, lab, lab_out, nlab);
}

}  // namespace tfx
