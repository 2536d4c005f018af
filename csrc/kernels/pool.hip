// NHWC bf16 pooling (LeNet-5 / generic CNNs; BASELINE.json config 2).
//
// max_pool: y[n,p,q,c] = max over the k x k window; the in-window argmax (uint8, first max wins,
//   like tf.nn.max_pool's gradient routing) is stored so the backward routes dy exactly.
// backward: every input element gathers dy from the (at most ceil(k/s)^2) windows that contain it
//   and whose argmax points at it -- no atomics, deterministic, also for overlapping windows.
// Channels are the contiguous axis: a thread handles 8 channels with 16-B loads when C % 8 == 0.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const uint16_t* __restrict__ x, int N, int H, int W, int C,
                                                          int k, int s, int pad, int P, int Q,
                                                          uint16_t* __restrict__ y, uint8_t* __restrict__ arg) {
  const int64_t total = (int64_t)N * P * Q * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float best = -INFINITY;
    int bi = 0;
    for (int dy = 0; dy < k; ++dy) {
      const int h = p * s - pad + dy;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int w = q * s - pad + dx;
        if ((unsigned)w >= (unsigned)W) continue;
        const float v = bf16_to_f32(x[(((int64_t)n * H + h) * W + w) * C + c]);
        if (v > best) {
          best = v;
          bi = dy * k + dx;
        }
      }
    }
    y[i] = f32_to_bf16(best);
    arg[i] = (uint8_t)bi;
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          int N, int H, int W, int C, int k, int s, int pad, int P,
                                                          int Q, uint16_t* __restrict__ dx) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float g = 0.f;
    // windows p with p*s - pad <= h < p*s - pad + k
    const int p0 = max(0, (h + pad - k + s) / s), p1 = min(P - 1, (h + pad) / s);
    const int q0 = max(0, (w + pad - k + s) / s), q1 = min(Q - 1, (w + pad) / s);
    for (int p = p0; p <= p1; ++p) {
      const int dyy = h - (p * s - pad);
      if (dyy < 0 || dyy >= k) continue;
      for (int q = q0; q <= q1; ++q) {
        const int dxx = w - (q * s - pad);
        if (dxx < 0 || dxx >= k) continue;
        const int64_t o = (((int64_t)n * P + p) * Q + q) * C + c;
        if (arg[o] == dyy * k + dxx) g += bf16_to_f32(dy[o]);
      }
    }
    dx[i] = f32_to_bf16(g);
  }
}

// average pool (count excludes padding, like tf.nn.avg_pool with SAME padding)
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const uint16_t* __restrict__ x, int N, int H, int W, int C,
                                                          int k, int s, int pad, int P, int Q, uint16_t* __restrict__ y) {
  const int64_t total = (int64_t)N * P * Q * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float acc = 0.f;
    int cnt = 0;
    for (int dy = 0; dy < k; ++dy) {
      const int h = p * s - pad + dy;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int w = q * s - pad + dx;
        if ((unsigned)w >= (unsigned)W) continue;
        acc += bf16_to_f32(x[(((int64_t)n * H + h) * W + w) * C + c]);
        ++cnt;
      }
    }
    y[i] = f32_to_bf16(cnt ? acc / cnt : 0.f);
  }
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const uint16_t* __restrict__ dy, int N, int H, int W, int C,
                                                          int k, int s, int pad, int P, int Q, uint16_t* __restrict__ dx) {
  const int64_t total = (int64_t)N * H * W * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float g = 0.f;
    const int p0 = max(0, (h + pad - k + s) / s), p1 = min(P - 1, (h + pad) / s);
    const int q0 = max(0, (w + pad - k + s) / s), q1 = min(Q - 1, (w + pad) / s);
    for (int p = p0; p <= p1; ++p) {
      const int hs = p * s - pad;
      if (h < hs || h >= hs + k) continue;
      const int hc = min(hs + k, H) - max(hs, 0);
      for (int q = q0; q <= q1; ++q) {
        const int ws = q * s - pad;
        if (w < ws || w >= ws + k) continue;
        const int wc = min(ws + k, W) - max(ws, 0);
        g += bf16_to_f32(dy[(((int64_t)n * P + p) * Q + q) * C + c]) / (float)(hc * wc);
      }
    }
    dx[i] = f32_to_bf16(g);
  }
}

int pgrid(int64_t total) {
  int64_t g = (total + 1023) / 1024;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}

}  // namespace

void maxpool_fwd(const uint16_t* x, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, uint16_t* y,
                 uint8_t* arg, hipStream_t st) {
  maxpool_fwd_kernel<<<pgrid((int64_t)N * P * Q * C), 256, 0, st>>>(x, N, H, W, C, k, s, pad, P, Q, y, arg);
}
void maxpool_bwd(const uint16_t* dy, const uint8_t* arg, int N, int H, int W, int C, int k, int s, int pad, int P,
                 int Q, uint16_t* dx, hipStream_t st) {
  maxpool_bwd_kernel<<<pgrid((int64_t)N * H * W * C), 256, 0, st>>>(dy, arg, N, H, W, C, k, s, pad, P, Q, dx);
}
void avgpool_fwd(const uint16_t* x, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, uint16_t* y,
                 hipStream_t st) {
  avgpool_fwd_kernel<<<pgrid((int64_t)N * P * Q * C), 256, 0, st>>>(x, N, H, W, C, k, s, pad, P, Q, y);
}
void avgpool_bwd(const uint16_t* dy, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, uint16_t* dx,
                 hipStream_t st) {
  avgpool_bwd_kernel<<<pgrid((int64_t)N * H * W * C), 256, 0, st>>>(dy, N, H, W, C, k, s, pad, P, Q, dx);
}

}  // namespace tfx
