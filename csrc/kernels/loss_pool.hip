// Softmax cross-entropy (fused fwd + bwd), accuracy, and global average pooling.
//
// softmax_xent: one wave per row (C <= a few thousand: classes of MNIST/CIFAR/char vocab).
//   mode 0 (stable): loss_r = logsumexp(z) - z[label]; dz = (p - onehot) * gscale
//   mode 1 (naive, reference parity R/distributed/distributed.py:99,102):
//       p = softmax(z), loss_r = -sum y*log(p)  (log of the softmax OUTPUT, may be -inf/NaN like TF1)
//       dz = (g - sum(g*p)) * p  with g = -y/p * gscale  (TF1's Log-grad -> SoftmaxGrad chain)
// Targets are either class indices (int64) or dense rows (f32, one-hot or soft).
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

template <typename TIN>
__device__ __forceinline__ float ld(const TIN* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }

template <typename T>
__device__ __forceinline__ void st_dz(T* p, int64_t i, float v);
template <>
__device__ __forceinline__ void st_dz<float>(float* p, int64_t i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st_dz<uint16_t>(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }

// One row on one wave; returns the row's loss (every lane holds it).
template <typename TIN, typename TDZ>
__device__ __forceinline__ float xent_row(const TIN* __restrict__ z, int row, int C, int lane,
                                          const int64_t* __restrict__ lab_idx, const float* __restrict__ lab_dense,
                                          int naive, float gscale, TDZ* __restrict__ dz, float* __restrict__ probs) {
  const TIN* zr = z + (int64_t)row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, ld(zr, c));
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(ld(zr, c) - m);
  s = wave_sum(s);
  const float inv_s = 1.f / s;
  const float lse = m + __logf(s);
  const int64_t lab = lab_idx ? lab_idx[row] : -1;
  float loss = 0.f, gp = 0.f;
  // pass 1: loss (+ for naive mode sum(g*p))
  for (int c = lane; c < C; c += 64) {
    const float zc = ld(zr, c);
    const float y = lab_dense ? lab_dense[(int64_t)row * C + c] : (c == lab ? 1.f : 0.f);
    if (naive) {
      const float p = __expf(zc - m) * inv_s;
      if (y != 0.f) loss -= y * logf(p);
      const float g = -y / p * gscale;  // NaN when y=0,p=0 is avoided below
      gp += (y != 0.f ? g : 0.f) * p;
    } else {
      if (y != 0.f) loss += y * (lse - zc);
    }
  }
  loss = wave_sum(loss);
  if (naive) gp = wave_sum(gp);
  if (!dz && !probs) return loss;
  for (int c = lane; c < C; c += 64) {
    const float zc = ld(zr, c);
    const float p = __expf(zc - m) * inv_s;
    const float y = lab_dense ? lab_dense[(int64_t)row * C + c] : (c == lab ? 1.f : 0.f);
    if (probs) probs[(int64_t)row * C + c] = p;
    if (dz) {
      float d;
      if (naive) {
        const float g = y != 0.f ? -y / p * gscale : 0.f;
        d = (g - gp) * p;
      } else {
        d = (p - y) * gscale;
      }
      st_dz(dz, (int64_t)row * C + c, d);
    }
  }
  return loss;
}

template <typename TIN>
__global__ void __launch_bounds__(256) softmax_xent_kernel(const TIN* __restrict__ z, int B, int C,
                                                           const int64_t* __restrict__ lab_idx,
                                                           const float* __restrict__ lab_dense, int naive,
                                                           float gscale, float* __restrict__ loss_rows,
                                                           float* __restrict__ dz, float* __restrict__ probs) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float loss = xent_row(z, row, C, lane, lab_idx, lab_dense, naive, gscale, dz, probs);
  if (lane == 0 && loss_rows) loss_rows[row] = loss;
}

// Small batches (the training step's loss): one block of 16 waves walks every row and also writes
// the batch-mean loss (fixed-order LDS sum: deterministic), with dz stored in the logits' dtype --
// the separate mean-reduction and scale/cast launches of the training step's loss are gone.
template <typename TIN, typename TDZ>
__global__ void __launch_bounds__(1024) softmax_xent_mean_kernel(const TIN* __restrict__ z, int B, int C,
                                                                 const int64_t* __restrict__ lab_idx,
                                                                 const float* __restrict__ lab_dense, int naive,
                                                                 float gscale, float* __restrict__ loss_mean,
                                                                 TDZ* __restrict__ dz) {
  __shared__ float part[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  if (C <= 32) {
    // thread = row: the whole row lives in one thread's registers (no cross-lane reductions, whose
    // serial shuffle latency -- ~3 per row -- dominates a one-block launch)
    for (int row = threadIdx.x; row < B; row += 1024) {
      float zv[32];
      const int64_t lab = lab_idx ? lab_idx[row] : -1;
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < 32; ++c)
        if (c < C) {
          zv[c] = ld(z, (int64_t)row * C + c);
          m = fmaxf(m, zv[c]);
        }
      float sum = 0.f;
#pragma unroll
      for (int c = 0; c < 32; ++c)
        if (c < C) sum += __expf(zv[c] - m);
      const float inv_s = 1.f / sum, lse = m + __logf(sum);
      float l = 0.f, gp = 0.f;
#pragma unroll
      for (int c = 0; c < 32; ++c)
        if (c < C) {
          const float y = lab_dense ? lab_dense[(int64_t)row * C + c] : (c == lab ? 1.f : 0.f);
          if (naive) {
            const float p = __expf(zv[c] - m) * inv_s;
            if (y != 0.f) {
              l -= y * logf(p);
              gp += -y / p * gscale * p;
            }
          } else if (y != 0.f) {
            l += y * (lse - zv[c]);
          }
        }
      if (dz) {
#pragma unroll
        for (int c = 0; c < 32; ++c)
          if (c < C) {
            const float y = lab_dense ? lab_dense[(int64_t)row * C + c] : (c == lab ? 1.f : 0.f);
            const float p = __expf(zv[c] - m) * inv_s;
            float d;
            if (naive) {
              const float g = y != 0.f ? -y / p * gscale : 0.f;
              d = (g - gp) * p;
            } else {
              d = (p - y) * gscale;
            }
            st_dz(dz, (int64_t)row * C + c, d);
          }
      }
      acc += l;
    }
    acc = wave_sum(acc);
  } else if (C <= 64) {
    // lane = class: every load of a chunk of RPW rows is issued before any math (one memory round
    // trip per chunk instead of ~5 dependent ones per row), then the rows reduce from registers
    constexpr int RPW = 16;
    for (int base = w; base < B; base += 16 * RPW) {
      float zc[RPW], yv[RPW];
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int row = base + 16 * k;
        const bool v = row < B && lane < C;
        zc[k] = v ? ld(z, (int64_t)row * C + lane) : -INFINITY;
        if (lab_dense) yv[k] = v ? lab_dense[(int64_t)row * C + lane] : 0.f;
        else yv[k] = (v && lab_idx[row] == lane) ? 1.f : 0.f;
      }
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int row = base + 16 * k;
        if (row >= B) break;  // wave-uniform
        const bool v = lane < C;
        const float m = wave_max(zc[k]);
        const float e = v ? __expf(zc[k] - m) : 0.f;
        const float sum = wave_sum(e);
        const float p = e / sum, y = yv[k];
        float l, d;
        if (naive) {
          l = wave_sum(y != 0.f ? -y * logf(p) : 0.f);
          const float g = y != 0.f ? -y / p * gscale : 0.f;
          const float gp = wave_sum(g * p);
          d = (g - gp) * p;
        } else {
          l = wave_sum(y != 0.f ? y * (m + __logf(sum) - zc[k]) : 0.f);
          d = (p - y) * gscale;
        }
        if (dz && v) st_dz(dz, (int64_t)row * C + lane, d);
        acc += l;
      }
    }
  } else {
    for (int row = w; row < B; row += 16) acc += xent_row(z, row, C, lane, lab_idx, lab_dense, naive, gscale, dz,
                                                          (float*)nullptr);
  }
  if (lane == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 16; ++i) t += part[i];
    loss_mean[0] = t / (float)B;
  }
}

// correct[row] = argmax(z[row]) == argmax(target[row]) (first max wins, as tf.argmax)
template <typename TIN>
__global__ void __launch_bounds__(256) accuracy_kernel(const TIN* __restrict__ z, int B, int C,
                                                       const int64_t* __restrict__ lab_idx,
                                                       const float* __restrict__ lab_dense,
                                                       float* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  float hit = 0.f;
  if (row < B) {
    float bv = -INFINITY, tv = -INFINITY;
    int bi = C, ti = C;
    for (int c = lane; c < C; c += 64) {
      const float v = ld(z + (int64_t)row * C, c);
      if (v > bv) { bv = v; bi = c; }
      if (lab_dense) {
        const float t = lab_dense[(int64_t)row * C + c];
        if (t > tv) { tv = t; ti = c; }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      const float otv = __shfl_xor(tv, o, 64);
      const int oti = __shfl_xor(ti, o, 64);
      if (otv > tv || (otv == tv && oti < ti)) { tv = otv; ti = oti; }
    }
    const int target = lab_idx ? (int)lab_idx[row] : ti;
    hit = (lane == 0 && bi == target) ? 1.f : 0.f;
  }
  if (lane == 0 && row < B && hit != 0.f) atomicAdd(count, 1.f);
}

// Global average pool NHWC: x [N][HW][C] bf16 -> y [N][C] (bf16 or f32)
// 8 channels per thread: 16-byte loads over the HW pixels, one 16-byte (bf16) / 2x16-byte (f32) store
__global__ void __launch_bounds__(256) gap_fwd_vec_kernel(const uint16_t* __restrict__ x, int N, int HW, int C,
                                                          uint16_t* __restrict__ y16, float* __restrict__ y32) {
  const int C8 = C >> 3;
  const int v = blockIdx.x * 256 + threadIdx.x;  // (n, c8)
  if (v >= N * C8) return;
  const int n = v / C8, c = (v - n * C8) * 8;
  const U4* xp = reinterpret_cast<const U4*>(x + (int64_t)n * HW * C + c);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < HW; ++i) {
    float f[8];
    unpack8(xp[(int64_t)i * C8], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += f[k];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] *= inv;
  if (y16) reinterpret_cast<U4*>(y16)[v] = pack8(s);
  if (y32) {
    float4* o = reinterpret_cast<float4*>(y32 + (int64_t)n * C + c);
    o[0] = make_float4(s[0], s[1], s[2], s[3]);
    o[1] = make_float4(s[4], s[5], s[6], s[7]);
  }
}

// dx[n][p][c] = dy[n][c] / HW, 8 channels per thread (16-byte stores), 32-bit index math
template <typename TG>
__global__ void __launch_bounds__(256) gap_bwd_vec_kernel(const TG* __restrict__ dy, int nvec, int HWC8, int C8,
                                                          float inv, uint16_t* __restrict__ dx) {
  for (int v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    const int n = v / HWC8, c8 = (v - n * HWC8) % C8;
    const TG* g = dy + ((int64_t)n * C8 + c8) * 8;
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = ld(g, k) * inv;
    reinterpret_cast<U4*>(dx)[v] = pack8(f);
  }
}

__global__ void __launch_bounds__(256) gap_fwd_kernel(const uint16_t* __restrict__ x, int N, int HW, int C,
                                                      uint16_t* __restrict__ y16, float* __restrict__ y32) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const uint16_t* xp = x + (int64_t)n * HW * C + c;
  float s = 0.f;
  for (int i = 0; i < HW; ++i) s += bf16_to_f32(xp[(int64_t)i * C]);
  s *= 1.f / (float)HW;
  if (y16) y16[(int64_t)n * C + c] = f32_to_bf16(s);
  if (y32) y32[(int64_t)n * C + c] = s;
}

template <typename TG>
__global__ void __launch_bounds__(256) gap_bwd_kernel(const TG* __restrict__ dy, int N, int HW, int C,
                                                      uint16_t* __restrict__ dx) {
  const int64_t total = (int64_t)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t n = i / ((int64_t)HW * C);
    dx[i] = f32_to_bf16(ld(dy, n * C + c) * inv);
  }
}

// ---------------------------------------------------------------- launchers
void softmax_xent(const void* z, bool z_bf16, int B, int C, const int64_t* lab_idx, const float* lab_dense,
                  bool naive, float gscale, float* loss_rows, float* dz, float* probs, hipStream_t s) {
  dim3 grid((B + 3) / 4);
  if (z_bf16)
    softmax_xent_kernel<uint16_t><<<grid, 256, 0, s>>>((const uint16_t*)z, B, C, lab_idx, lab_dense, naive,
                                                       gscale, loss_rows, dz, probs);
  else
    softmax_xent_kernel<float><<<grid, 256, 0, s>>>((const float*)z, B, C, lab_idx, lab_dense, naive, gscale,
                                                    loss_rows, dz, probs);
}

void softmax_xent_mean(const void* z, bool z_bf16, int B, int C, const int64_t* lab_idx, const float* lab_dense,
                       bool naive, float gscale, float* loss_mean, void* dz, bool dz_bf16, hipStream_t s) {
  if (z_bf16 && dz_bf16)
    softmax_xent_mean_kernel<uint16_t, uint16_t><<<1, 1024, 0, s>>>((const uint16_t*)z, B, C, lab_idx, lab_dense,
                                                                  naive, gscale, loss_mean, (uint16_t*)dz);
  else if (z_bf16)
    softmax_xent_mean_kernel<uint16_t, float><<<1, 1024, 0, s>>>((const uint16_t*)z, B, C, lab_idx, lab_dense,
                                                               naive, gscale, loss_mean, (float*)dz);
  else if (dz_bf16)
    softmax_xent_mean_kernel<float, uint16_t><<<1, 1024, 0, s>>>((const float*)z, B, C, lab_idx, lab_dense, naive,
                                                               gscale, loss_mean, (uint16_t*)dz);
  else
    softmax_xent_mean_kernel<float, float><<<1, 1024, 0, s>>>((const float*)z, B, C, lab_idx, lab_dense, naive,
                                                            gscale, loss_mean, (float*)dz);
}

void accuracy_count(const void* z, bool z_bf16, int B, int C, const int64_t* lab_idx, const float* lab_dense,
                    float* count, hipStream_t s) {
  TFX_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(float), s));
  dim3 grid((B + 3) / 4);
  if (z_bf16)
    accuracy_kernel<uint16_t><<<grid, 256, 0, s>>>((const uint16_t*)z, B, C, lab_idx, lab_dense, count);
  else
    accuracy_kernel<float><<<grid, 256, 0, s>>>((const float*)z, B, C, lab_idx, lab_dense, count);
}

void gap_fwd(const uint16_t* x, int N, int HW, int C, uint16_t* y16, float* y32, hipStream_t s) {
  if (C % 8 == 0 && (int64_t)N * HW * C < (1ll << 31)) {
    gap_fwd_vec_kernel<<<(N * (C / 8) + 255) / 256, 256, 0, s>>>(x, N, HW, C, y16, y32);
    return;
  }
  dim3 grid((C + 255) / 256, N);
  gap_fwd_kernel<<<grid, 256, 0, s>>>(x, N, HW, C, y16, y32);
}

void gap_bwd(const void* dy, bool dy_bf16, int N, int HW, int C, uint16_t* dx, hipStream_t s) {
  const int64_t total = (int64_t)N * HW * C;
  if (C % 8 == 0 && total < (1ll << 31)) {
    const int nvec = (int)(total / 8);
    const int gv = std::min((nvec + 255) / 256, 8192);
    if (dy_bf16)
      gap_bwd_vec_kernel<uint16_t><<<gv, 256, 0, s>>>((const uint16_t*)dy, nvec, HW * (C / 8), C / 8,
                                                      1.f / (float)HW, dx);
    else
      gap_bwd_vec_kernel<float><<<gv, 256, 0, s>>>((const float*)dy, nvec, HW * (C / 8), C / 8, 1.f / (float)HW,
                                                   dx);
    return;
  }
  int g = (int)std::min<int64_t>((total + 1023) / 1024, 4096);
  if (dy_bf16)
    gap_bwd_kernel<uint16_t><<<g, 256, 0, s>>>((const uint16_t*)dy, N, HW, C, dx);
  else
    gap_bwd_kernel<float><<<g, 256, 0, s>>>((const float*)dy, N, HW, C, dx);
}

}  // namespace tfx
