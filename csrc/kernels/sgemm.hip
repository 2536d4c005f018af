// Exact-f32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32) for the fp32 parity models
// (the reference MNIST MLP, R/distributed/distributed.py:96-98, and the CPU-plumbing configs when
// they run on the GPU).  gfx950 has no xf32 path; this instruction is a bitwise f32 fmaf chain.
//
// C[M][N] = act(op(A) op(B) + bias) (+C if accumulate); act: 0 none, 1 relu, 2 sigmoid.
// Tile 64x64x16, 256 threads (4 waves 2x2, 32x32 per wave = 2x2 MFMA 16x16 tiles).
// These shapes are tiny and latency-bound (B=100, K<=784): one pass, no split.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

__global__ void __launch_bounds__(256) sgemm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C, const float* __restrict__ bias, int M,
                                                    int N, int K, int lda, int ldb, int ldc, int transA, int transB,
                                                    int act, int accumulate) {
  __shared__ float As[16][64 + 4];  // [k][m]
  __shared__ float Bs[16][64 + 4];  // [k][n]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = t + 256 * e;  // 0..1023 over a 64x16 tile
      // A tile element: coalesce along the contiguous dimension of the source
      int mm, kk;
      if (transA) { mm = idx & 63; kk = idx >> 6; } else { kk = idx & 15; mm = idx >> 4; }
      const int gm = m0 + mm, gk = k0 + kk;
      float va = 0.f;
      if (gm < M && gk < K) va = transA ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk];
      As[kk][mm] = va;
      int nn, kb;
      if (transB) { kb = idx & 15; nn = idx >> 4; } else { nn = idx & 63; kb = idx >> 6; }
      const int gn = n0 + nn, gkb = k0 + kb;
      float vb = 0.f;
      if (gn < N && gkb < K) vb = transB ? B[(int64_t)gn * ldb + gkb] : B[(int64_t)gkb * ldb + gn];
      Bs[kb][nn] = vb;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 16; ks += 4) {
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[ks + (lane >> 4)][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[ks + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane & 15);
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= M) continue;
        float v = acc[i][j][r];
        if (bias) v += bias[n];
        if (act == 1) v = fmaxf(v, 0.f);
        else if (act == 2) v = 1.f / (1.f + expf(-v));
        float* o = C + (int64_t)m * ldc + n;
        *o = accumulate ? *o + v : v;
      }
    }
}

void sgemm_launch(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
                  int ldb, int ldc, bool transA, bool transB, int act, bool accumulate, hipStream_t s) {
  dim3 grid((N + 63) / 64, (M + 63) / 64);
  sgemm_kernel<<<grid, 256, 0, s>>>(A, B, C, bias, M, N, K, lda, ldb, ldc, transA, transB, act, accumulate);
}

}  // namespace tfx
