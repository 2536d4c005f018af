// Small fused elementwise / reduction kernels of the reference's parity workloads.
//
// * affine (W * x + b, per-channel W and b broadcast over the leading dims) and its backward
//   (dx = g * W; dW += sum g * x; db += sum g) -- the linear model of R/simple/simple.py:16 and the
//   TF1 Mul / Add gradients behind its minimize (R/simple/simple.py:22-23);
// * sum of squared errors (reduce_sum(square(pred - y)), R/simple/simple.py:20) and its gradient
//   dpred = 2 (pred - y) * g;
// * activation backward fused with the bias column sum: dz = g * y * (1 - y) (TF1 SigmoidGrad) or
//   g * [y > 0] (ReluGrad), and dbias += sum_rows dz -- the MLP's backward of
//   R/distributed/distributed.py:96-98 in one launch instead of an elementwise pass + a reduction;
// * scale by a device scalar (the loss's upstream gradient) with an optional bf16 cast.
//
// These run at tiny sizes (4 elements for simple.py, 100 x 100 for the MLP): one launch each, a
// single block where the whole problem fits one, wave reductions with DPP/shuffles, atomics only
// across blocks.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

__global__ void __launch_bounds__(256) affine_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, int64_t n, int C,
                                                         float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    y[i] = w[c] * x[i] + (b ? b[c] : 0.f);
  }
}

// one block per channel group: thread t accumulates rows r = t/C' ... (C <= 256: channel = t % C)
__global__ void __launch_bounds__(256) affine_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                                         const float* __restrict__ w, int64_t n, int C,
                                                         float* __restrict__ dx, float* __restrict__ dw,
                                                         float* __restrict__ db) {
  const int t = threadIdx.x;
  const int per = 256 / C;  // threads per channel in this block (host: C <= 256)
  const int c = t % C, lane_r = t / C;
  float sw = 0.f, sb = 0.f;
  if (lane_r < per) {
    const int64_t rows = n / C;
    for (int64_t r = (int64_t)blockIdx.x * per + lane_r; r < rows; r += (int64_t)gridDim.x * per) {
      const int64_t i = r * C + c;
      const float gi = g[i];
      sw = fmaf(gi, x[i], sw);
      sb += gi;
      if (dx) dx[i] = gi * w[c];
    }
  }
  __shared__ float rw[256], rb[256];
  rw[t] = sw;
  rb[t] = sb;
  __syncthreads();
  if (t < C) {
    float aw = 0.f, ab = 0.f;
    for (int k = 0; k < per; ++k) {
      aw += rw[t + k * C];
      ab += rb[t + k * C];
    }
    if (gridDim.x == 1) {  // deterministic single-block sum (simple.py: 4 elements)
      if (dw) dw[t] += aw;
      if (db) db[t] += ab;
    } else {
      if (dw) atomicAdd(dw + t, aw);
      if (db) atomicAdd(db + t, ab);
    }
  }
}

// loss[0] = sum (p - y)^2, one block (grid 1) or atomics over blocks (loss pre-zeroed by the host)
__global__ void __launch_bounds__(256) sse_fwd_kernel(const float* __restrict__ p, const float* __restrict__ y,
                                                      int64_t n, float* __restrict__ loss) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float r = p[i] - y[i];
    s = fmaf(r, r, s);
  }
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    if (gridDim.x == 1) loss[0] = tot;
    else atomicAdd(loss, tot);
  }
}

__global__ void __launch_bounds__(256) sse_bwd_kernel(const float* __restrict__ p, const float* __restrict__ y,
                                                      const float* __restrict__ g, int64_t n, float* __restrict__ dp) {
  const float gg = g[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dp[i] = 2.f * (p[i] - y[i]) * gg;
}

// dz = g * act'(y); dbias[c] += sum_rows dz.  Block = 64 columns x 4 row lanes.  T = float, or
// uint16_t for bf16 g / y / dz (the bf16 dense layers: ReLU mask + bias column-sum in one pass;
// dz == nullptr when the caller needs only the column sums).
__device__ __forceinline__ float ld_as_f32(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float ld_as_f32(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
__device__ __forceinline__ void st_from_f32(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st_from_f32(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }

template <int ACT, typename T>
__global__ void __launch_bounds__(256) act_bwd_colsum_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                             int64_t M, int N, T* __restrict__ dz,
                                                             float* __restrict__ dbias) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f;
  if (c < N) {
    for (int64_t r = (int64_t)blockIdx.y * 4 + ty; r < M; r += (int64_t)gridDim.y * 4) {
      const int64_t i = r * N + c;
      float d = ld_as_f32(g, i);
      if (ACT == 1) d = ld_as_f32(y, i) > 0.f ? d : 0.f;
      if (ACT == 2) {
        const float yv = ld_as_f32(y, i);
        d = d * yv * (1.f - yv);  // TF1 SigmoidGrad: dy * y * (1 - y)
      }
      if (dz) st_from_f32(dz, i, d);
      s += d;
    }
  }
  if (!dbias) return;
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (ty == 0 && c < N) {
    const float tot = red[tx] + red[tx + 64] + red[tx + 128] + red[tx + 192];
    if (gridDim.y == 1) dbias[c] += tot;
    else atomicAdd(dbias + c, tot);
  }
}

__global__ void __launch_bounds__(256) scale_scalar_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ scal, int64_t n,
                                                           float* __restrict__ y32, uint16_t* __restrict__ y16) {
  const float s = scal[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i] * s;
    if (y16) y16[i] = f32_to_bf16(v);
    else y32[i] = v;
  }
}

int egrid(int64_t n, int cap = 2048) {
  int64_t g = (n + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

}  // namespace

void affine_fwd(const float* x, const float* w, const float* b, int64_t n, int C, float* y, hipStream_t s) {
  affine_fwd_kernel<<<egrid(n), 256, 0, s>>>(x, w, b, n, C, y);
}

void affine_bwd(const float* g, const float* x, const float* w, int64_t n, int C, float* dx, float* dw, float* db,
                hipStream_t s) {
  const int per = 256 / C;
  const int64_t rows = n / C;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + per - 1) / per, 1024));
  affine_bwd_kernel<<<grid, 256, 0, s>>>(g, x, w, n, C, dx, dw, db);
}

void sse_fwd(const float* p, const float* y, int64_t n, float* loss, hipStream_t s) {
  const int grid = egrid(n, 1024);
  if (grid > 1) TFX_HIP_CHECK(hipMemsetAsync(loss, 0, sizeof(float), s));
  sse_fwd_kernel<<<grid, 256, 0, s>>>(p, y, n, loss);
}

void sse_bwd(const float* p, const float* y, const float* g, int64_t n, float* dp, hipStream_t s) {
  sse_bwd_kernel<<<egrid(n), 256, 0, s>>>(p, y, g, n, dp);
}

template <typename T>
void act_bwd_colsum_t(const T* g, const T* y, int act, int64_t M, int N, T* dz, float* dbias, hipStream_t s) {
  dim3 grid((N + 63) / 64, (unsigned)std::max<int64_t>(1, std::min<int64_t>((M + 63) / 64, 256)));
  if (act == 1) act_bwd_colsum_kernel<1, T><<<grid, 256, 0, s>>>(g, y, M, N, dz, dbias);
  else if (act == 2) act_bwd_colsum_kernel<2, T><<<grid, 256, 0, s>>>(g, y, M, N, dz, dbias);
  else act_bwd_colsum_kernel<0, T><<<grid, 256, 0, s>>>(g, y, M, N, dz, dbias);
}

void act_bwd_colsum(const float* g, const float* y, int act, int64_t M, int N, float* dz, float* dbias,
                    hipStream_t s) {
  act_bwd_colsum_t<float>(g, y, act, M, N, dz, dbias, s);
}

void act_bwd_colsum_bf16(const uint16_t* g, const uint16_t* y, int act, int64_t M, int N, uint16_t* dz,
                         float* dbias, hipStream_t s) {
  act_bwd_colsum_t<uint16_t>(g, y, act, M, N, dz, dbias, s);
}

// ---- backward of a linear layer with few outputs (a classifier head: O <= 64, e.g. ResNet's
// 2048 -> 10 FC): dx = g W, dW += g^T x, db += colsum(g) in ONE launch instead of padded bf16 GEMMs
// plus pad / copy / zero-fill kernels.  Block = 64 input columns x LRB rows (grid.y over the batch):
// the rows' g ([LRB][O], bf16) is staged in LDS as f32; a thread owns one column and LRB/4 rows (dx:
// O FMAs per element) and keeps its column's O partial dW sums in registers; the block's dW / db
// partials go out as f32 atomics (dW, db are accumulated gradients).
constexpr int LRB = 32;
template <int OMAX>
__global__ void __launch_bounds__(256) linear_small_bwd_kernel(const uint16_t* __restrict__ g,
                                                               const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ w, int B, int I, int O,
                                                               uint16_t* __restrict__ dx, float* __restrict__ dw,
                                                               float* __restrict__ db) {
  __shared__ float gs[LRB * OMAX];
  __shared__ float part[4][64][OMAX + 1];
  const int t = threadIdx.x, b0 = blockIdx.y * LRB;
  const int nb = min(LRB, B - b0);
  for (int i = t; i < nb * O; i += 256) gs[i] = bf16_to_f32(g[(int64_t)b0 * O + i]);
  __syncthreads();
  const int c = blockIdx.x * 64 + (t & 63), rq = t >> 6;  // 4 row phases x 64 columns
  float wcol[OMAX], acc[OMAX];
#pragma unroll
  for (int o = 0; o < OMAX; ++o) {
    wcol[o] = (o < O && c < I) ? bf16_to_f32(w[(int64_t)o * I + c]) : 0.f;
    acc[o] = 0.f;
  }
  if (c < I) {
    float xv[LRB / 4];
#pragma unroll
    for (int k = 0; k < LRB / 4; ++k) {
      const int r = rq + 4 * k;
      xv[k] = r < nb ? bf16_to_f32(x[(int64_t)(b0 + r) * I + c]) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < LRB / 4; ++k) {
      const int r = rq + 4 * k;
      if (r < nb) {
        const float* gr = gs + r * O;
        float s = 0.f;
#pragma unroll
        for (int o = 0; o < OMAX; ++o) {
          if (o < O) {
            s = fmaf(gr[o], wcol[o], s);
            acc[o] = fmaf(gr[o], xv[k], acc[o]);
          }
        }
        if (dx) dx[(int64_t)(b0 + r) * I + c] = f32_to_bf16(s);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < OMAX; ++o) part[rq][t & 63][o] = acc[o];
  __syncthreads();
  if (rq == 0 && c < I && dw) {
#pragma unroll
    for (int o = 0; o < OMAX; ++o) {
      if (o < O) atomicAdd(dw + (int64_t)o * I + c, part[0][t][o] + part[1][t][o] + part[2][t][o] + part[3][t][o]);
    }
  }
  if (blockIdx.x == 0 && db && t < O) {
    float s = 0.f;
    for (int r = 0; r < nb; ++r) s += gs[r * O + t];
    atomicAdd(db + t, s);
  }
}

void linear_small_bwd(const uint16_t* g, const uint16_t* x, const uint16_t* w, int B, int I, int O, uint16_t* dx,
                      float* dw, float* db, hipStream_t s) {
  const dim3 grid((I + 63) / 64, (B + LRB - 1) / LRB);
  if (O <= 16) linear_small_bwd_kernel<16><<<grid, 256, 0, s>>>(g, x, w, B, I, O, dx, dw, db);
  else linear_small_bwd_kernel<64><<<grid, 256, 0, s>>>(g, x, w, B, I, O, dx, dw, db);
}

void scale_by_scalar(const float* x, const float* scal, int64_t n, float* y32, uint16_t* y16, hipStream_t s) {
  scale_scalar_kernel<<<egrid(n), 256, 0, s>>>(x, scal, n, y32, y16);
}

}  // namespace tfx
