// The CIFAR ResNet stem (3x3, stride 1, pad 1, 8 padded input channels, 32x32 images, 64 outputs) for
// gfx950: its weight gradient, and (below) its forward with the BN statistics.
//
// As an implicit GEMM this is dW[Ko][72] = dY^T[Ko][P] . im2col(X)[P][72] over P = N*32*32 pixels: the
// generic kernels tile its 72 columns into a 128-wide tile (44 % padding), gather im2col pieces of
// 16 B per (pixel, tap) and split P over blocks with f32 atomics (31 us per step,
// profiles/r03_s2sq/step_trace.txt).  Here one block per image: the whole image's dY (128 KB, 32 16-B
// loads per thread) and the image itself (16 KB, to LDS with a zero border, 34 x 34 pixels) are put in
// flight at once and staged in LDS as they are -- no im2col, no transposes.  Both MFMA operands are
// then read with the transposed LDS read (ds_read_b64_tr_b16, cdna_hip_programming.md T10), whose
// lanes each supply their own row address: the A fragment (dY^T, k = 8 pixels of a row) straight from
// the dY rows, and the B fragment (im2col, column n = (tap, c)) from the image at the tap's shifted
// pixel -- a 16-column block spans two taps, columns 8..15 addressed at the second tap's pixel.
// Per wave: one 16-row ko tile, 5 column tiles (taps 0..8 in pairs, the 10th "tap" reads the zero
// border), 32 image rows x 5 MFMAs (16x16x32).  Every block adds its dW into one of ST_COPIES copies of
// a workspace (256 blocks into ONE 18 KB dW would serialise on the atomic units: MI355X_MICROARCH.md
// "Global float atomics", contention rows), and a small second launch sums the copies into dW and
// re-zeroes them (the workspace is zero between uses).
// Reference: the first conv layer of the north-star ResNet-50 (BASELINE.json config 3); SURVEY §2.7.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {
namespace {

constexpr int ST_W = 32, ST_HW = 34, ST_NT = 256;  // 32x32 images (+ a 1-pixel border), 4 waves
constexpr int ST_COPIES = 32;                      // dW workspace copies (4-8 blocks per address)

typedef short st_s4 __attribute__((ext_vector_type(4)));
typedef short st_s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) st_s4 st_lds_s4;
typedef __attribute__((address_space(3))) char st_lds_char;

template <int KO>
__global__ void __launch_bounds__(ST_NT) stem_wgrad_kernel(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ dy, int N,
                                                           float* __restrict__ wsall) {
  static_assert(KO == 64, "one 16-row ko tile per wave, one 16-B dY piece per thread and row");
  constexpr int H = ST_W, XB = ST_HW * ST_HW * 16, DB = H * ST_W * KO * 2;
  __shared__ __attribute__((aligned(16))) char smem[XB + 16 + DB];  // image (+ trash slot), dY
  char* ximg = smem;
  char* dimg = smem + XB + 16;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = blockIdx.x;
  float* ws = wsall + (size_t)(n % ST_COPIES) * (KO * 72);
  const int64_t img_px = (int64_t)H * ST_W;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(x), 0,
                                                                      (int)(N * img_px * 8 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(dy), 0,
                                                                      (int)(N * img_px * KO * 2), 0x00020000);
  constexpr uint32_t BADO = 0x80000000u;

  // ---- everything in flight: the image (zero border via out-of-range loads), then dY, row-major
  U4 xv[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int p = t + ST_NT * i, py = p / ST_HW, px = p % ST_HW;
    const bool in = (p < ST_HW * ST_HW) & (py >= 1) & (py <= H) & (px >= 1) & (px <= ST_W);
    const uint32_t o = in ? (uint32_t)((n * img_px + (py - 1) * ST_W + (px - 1)) * 16) : BADO;
    xv[i] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0));
  }
  U4 dv[H];
#pragma unroll
  for (int y = 0; y < H; ++y)
    dv[y] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(
                                       rd, (uint32_t)((n * img_px * KO + y * ST_W * KO + t * 8) * 2), 0, 0));
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int p = t + ST_NT * i;
    *reinterpret_cast<U4*>(ximg + (p < ST_HW * ST_HW ? p * 16 : XB)) = xv[i];  // past the image: trash slot
  }
#pragma unroll
  for (int y = 0; y < H; ++y) *reinterpret_cast<U4*>(dimg + y * (ST_W * KO * 2) + t * 16) = dv[y];
  __syncthreads();

  // ---- fragments by transposed reads: 16-lane group g, lane 4q+p supplies row q of a 4-row block,
  // columns 4p..4p+3; the lane receives column (lane & 15) of the block, rows in its elements
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto tr2 = [](const char* base0, const char* base1) -> bf16x8_t {
    const st_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((st_lds_s4*)(st_lds_char*)base0);
    const st_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((st_lds_s4*)(st_lds_char*)base1);
    st_s8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, r);
  };
  f32x4_t acc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int y = 0; y < H; ++y) {
    // A = dY^T: rows ko 16 wv .. +15, k = pixels 8g .. 8g+7 of row y
    const char* drow = dimg + y * (ST_W * KO * 2) + (16 * wv + 4 * p) * 2;
    const bf16x8_t fa = tr2(drow + (8 * g + q) * (KO * 2), drow + (8 * g + 4 + q) * (KO * 2));
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      // B = im2col: columns 16j .. 16j+15 = taps 2j (p < 2) and 2j+1 (p >= 2), channels 4 (p & 1) .. +3
      const int tap = 2 * j + (p >> 1), r = tap / 3, s = tap - 3 * r;
      const int c4 = 8 * (p & 1);  // byte offset of the channel quartet in the 16-B pixel
      const char* b0 = tap < 9 ? ximg + ((y + r) * ST_HW + 8 * g + q + s) * 16 + c4 : ximg + c4;  // pixel (0,0): zero
      const char* b1 = tap < 9 ? b0 + 4 * 16 : ximg + c4;
      const bf16x8_t fb = tr2(b0, b1);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[j], 0, 0, 0);
    }
  }
  // ---- acc[j] lane element r = dW[ko = 16 wv + 4 (lane >> 4) + r][n = 16 j + (lane & 15)]
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int col = 16 * j + (lane & 15);
    if (col < 72) {
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(ws + (16 * wv + 4 * (lane >> 4) + r) * 72 + col, acc[j][r]);
    }
  }
}

// ---- forward: y[n][y][x][ko] = sum over (r, s, c) of X[n][y+r-1][x+s-1][c] W[ko][r][s][c], and the
// BN statistics of the bf16 y (igemm.hip EPI_STATS math) into the BN layer's slots.  One block per
// image: the bordered image and W go to LDS once; per output row each wave (one 16-wide ko tile, its 3
// B fragments held in registers for the whole image) reads 6 A fragments -- a pixel's 8 channels of one
// tap are 16 contiguous bytes of the image, so no im2col -- and runs 6 MFMAs into y^T tiles (lanes hold
// 4 consecutive ko: 8-byte bf16 stores).  No barrier after the staging: the block is store-bound.
template <int KO>
__global__ void __launch_bounds__(ST_NT) stem_fwd_kernel(const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ w, int N,
                                                         uint16_t* __restrict__ y, float* __restrict__ slots) {
  static_assert(KO == 64, "one 16-wide ko tile per wave");
  constexpr int H = ST_W, XB = ST_HW * ST_HW * 16;
  __shared__ __attribute__((aligned(16))) char ximg[XB + 16];  // + a zero pixel for the padded taps
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = blockIdx.x;
  const int64_t img_px = (int64_t)H * ST_W;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(x), 0,
                                                                      (int)(N * img_px * 8 * 2), 0x00020000);
  constexpr uint32_t BADO = 0x80000000u;
  U4 xv[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int p = t + ST_NT * i, py = p / ST_HW, px = p % ST_HW;
    const bool in = (p < ST_HW * ST_HW) & (py >= 1) & (py <= H) & (px >= 1) & (px <= ST_W);
    const uint32_t o = in ? (uint32_t)((n * img_px + (py - 1) * ST_W + (px - 1)) * 16) : BADO;
    xv[i] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0));
  }
  // B fragments: lane holds W[ko = 16 wv + (lane & 15)][tap = 4 ks + (lane >> 4)][c 0..7]; taps 9..11 zero
  bf16x8_t fb[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int tap = 4 * ks + (lane >> 4), ko = 16 * wv + (lane & 15);
    U4 v = U4{0u, 0u, 0u, 0u};
    if (tap < 9) v = *reinterpret_cast<const U4*>(w + (ko * 9 + tap) * 8);
    fb[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int p = t + ST_NT * i;
    *reinterpret_cast<U4*>(ximg + (p < ST_HW * ST_HW ? p * 16 : XB)) = xv[i];  // past the image: the zero pixel
  }
  if (t == 0) *reinterpret_cast<U4*>(ximg + XB) = U4{0u, 0u, 0u, 0u};
  __syncthreads();

  float bs[4] = {0.f, 0.f, 0.f, 0.f}, bq[4] = {0.f, 0.f, 0.f, 0.f};
  const int ko0 = 16 * wv + 4 * (lane >> 4);
  uint16_t* yimg = y + (int64_t)n * img_px * KO;
#pragma unroll 2
  for (int yy = 0; yy < H; ++yy) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int px = 16 * mt + (lane & 15);
      f32x4_t acc = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int tap = 4 * ks + (lane >> 4), r = tap / 3, s = tap - 3 * r;
        const int off = tap < 9 ? ((yy + r) * ST_HW + px + s) * 16 : XB;
        const bf16x8_t fa = *(const __attribute__((address_space(3))) bf16x8_t*)(
            (__attribute__((address_space(3))) char*)ximg + off);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks], fa, acc, 0, 0, 0);  // y^T: rows ko, cols px
      }
      const uint32_t lo = pack_bf16x2(acc[0], acc[1]), hi = pack_bf16x2(acc[2], acc[3]);
      *reinterpret_cast<uint2*>(yimg + (yy * ST_W + px) * KO + ko0) = make_uint2(lo, hi);
      const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u), __uint_as_float(hi << 16),
                          __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bs[r] += v[r];
        bq[r] = fmaf(v[r], v[r], bq[r]);
      }
    }
  }
  // the 16 lanes of a DPP row hold the same 4 ko (different pixels): reduce, one atomic pair per ko
  float* slot = slots + (size_t)(n % NSLOT) * 2 * KO;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float sv = row16_sum(bs[r]), qv = row16_sum(bq[r]);
    if ((lane & 15) == 0) {
      atomicAdd(slot + ko0 + r, sv);
      atomicAdd(slot + KO + ko0 + r, qv);
    }
  }
}

// dw[e] += sum of the ST_COPIES workspace copies of element e, which are re-zeroed
__global__ void __launch_bounds__(256) stem_reduce_kernel(float* __restrict__ ws, int E, float* __restrict__ dw) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float v[ST_COPIES];
#pragma unroll
  for (int c = 0; c < ST_COPIES; ++c) v[c] = ws[(size_t)c * E + e];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < ST_COPIES; ++c) {
    sum += v[c];
    ws[(size_t)c * E + e] = 0.f;
  }
  dw[e] += sum;
}

}  // namespace

bool stem_wgrad_ok(int N, int H, int W, int C, int Ko) {
  return C == 8 && W == ST_W && H == ST_W && Ko == 64 && N >= 1 && (int64_t)N * H * W * Ko * 2 < (1ll << 31);
}

int stem_wgrad_ws_floats(int Ko) { return ST_COPIES * Ko * 72; }

void stem_fwd(const uint16_t* x, const uint16_t* w, int N, int Ko, uint16_t* y, float* slots, hipStream_t s) {
  (void)Ko;
  stem_fwd_kernel<64><<<N, ST_NT, 0, s>>>(x, w, N, y, slots);
}

void stem_wgrad(const uint16_t* x, const uint16_t* dy, int N, int Ko, float* ws, float* dw, hipStream_t s) {
  stem_wgrad_kernel<64><<<N, ST_NT, 0, s>>>(x, dy, N, ws);
  const int E = Ko * 72;
  stem_reduce_kernel<<<(E + 255) / 256, 256, 0, s>>>(ws, E, dw);
}

}  // namespace tfx
