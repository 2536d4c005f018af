// Exact-f32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32) for the fp32 models: the reference
// MNIST MLP (R/distributed/distributed.py:96-98) and the word2vec sampled-loss GEMMs
// (neg = E . Ws^T, dE += dn . Ws, dWs = dn^T . E).  gfx950 has no xf32 path; this instruction is a
// bitwise f32 fmaf chain.
//
// C[M][N] = act(op(A) op(B) + bias) (+C if accumulate); act: 0 none, 1 relu, 2 sigmoid.
// Tile 64x64x32, 256 threads (4 waves 2x2, 32x32 per wave = 2x2 MFMA 16x16 tiles).  The next k-tile
// is loaded into registers (16-byte loads along each operand's contiguous dimension when the
// shapes allow, VEC) while the current one is multiplied out of LDS: one barrier-separated LDS
// write per k-tile, its global latency hidden behind the previous tile's MFMAs.
// Split-K (grid.z, opt-in per call): the word2vec weight gradient dWs = dn^T E has M = 64 sampled
// rows, N = 128, K = batch (4096): two output tiles, so without a split two blocks walk all of K
// (the whole step waited on them).  Split blocks add their partials with f32 atomics (no act; bias
// from split 0), so the result is f32 but its summation order varies: the parity MLP never splits.
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

constexpr int SBK = 32;

template <bool TA, bool TB, bool VEC>
__global__ void __launch_bounds__(256) sgemm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C, const float* __restrict__ bias, int M,
                                                    int N, int K, int lda, int ldb, int ldc, int act, int accumulate,
                                                    int kchunk, int atomic_out) {
  __shared__ __attribute__((aligned(16))) float As[SBK][64 + 4];  // [k][m]
  __shared__ __attribute__((aligned(16))) float Bs[SBK][64 + 4];  // [k][n]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // staged k-tile: VEC -> 2 float4 per operand per thread (64 x 32 = 512 float4); else 8 scalars
  float ra[8], rb[8];
  // element (mm, kk) of the A tile / (kk, nn) of the B tile handled by slot e of this thread
  auto a_pos = [&](int e, int& mm, int& kk) {
    if constexpr (VEC) {
      const int idx = t + 256 * e;  // float4 index
      if constexpr (TA) { kk = idx >> 4; mm = (idx & 15) * 4; } else { mm = idx >> 3; kk = (idx & 7) * 4; }
    } else {
      const int idx = t + 256 * e;  // scalar index 0..2047
      if constexpr (TA) { mm = idx & 63; kk = idx >> 6; } else { kk = idx & 31; mm = idx >> 5; }
    }
  };
  auto b_pos = [&](int e, int& kk, int& nn) {
    if constexpr (VEC) {
      const int idx = t + 256 * e;
      if constexpr (TB) { nn = idx >> 3; kk = (idx & 7) * 4; } else { kk = idx >> 4; nn = (idx & 15) * 4; }
    } else {
      const int idx = t + 256 * e;
      if constexpr (TB) { kk = idx & 31; nn = idx >> 5; } else { nn = idx & 63; kk = idx >> 6; }
    }
  };
  auto load = [&](int k0) {
    if constexpr (VEC) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int mm, kk, nn, kb2;
        a_pos(e, mm, kk);
        const int gm = m0 + mm, gk = k0 + kk;
        float4 va = {0.f, 0.f, 0.f, 0.f};
        if (gm < M && gk < ke) va = *reinterpret_cast<const float4*>(TA ? A + (int64_t)gk * lda + gm
                                                                         : A + (int64_t)gm * lda + gk);
        ra[4 * e] = va.x; ra[4 * e + 1] = va.y; ra[4 * e + 2] = va.z; ra[4 * e + 3] = va.w;
        b_pos(e, kb2, nn);
        const int gn = n0 + nn, gkb = k0 + kb2;
        float4 vb = {0.f, 0.f, 0.f, 0.f};
        if (gn < N && gkb < ke) vb = *reinterpret_cast<const float4*>(TB ? B + (int64_t)gn * ldb + gkb
                                                                          : B + (int64_t)gkb * ldb + gn);
        rb[4 * e] = vb.x; rb[4 * e + 1] = vb.y; rb[4 * e + 2] = vb.z; rb[4 * e + 3] = vb.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int mm, kk, nn, kb2;
        a_pos(e, mm, kk);
        const int gm = m0 + mm, gk = k0 + kk;
        ra[e] = (gm < M && gk < ke) ? (TA ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk]) : 0.f;
        b_pos(e, kb2, nn);
        const int gn = n0 + nn, gkb = k0 + kb2;
        rb[e] = (gn < N && gkb < ke) ? (TB ? B[(int64_t)gn * ldb + gkb] : B[(int64_t)gkb * ldb + gn]) : 0.f;
      }
    }
  };
  auto store = [&]() {
    if constexpr (VEC) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int mm, kk, nn, kb2;
        a_pos(e, mm, kk);
        if constexpr (TA) {
          *reinterpret_cast<float4*>(&As[kk][mm]) = make_float4(ra[4 * e], ra[4 * e + 1], ra[4 * e + 2], ra[4 * e + 3]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) As[kk + q][mm] = ra[4 * e + q];
        }
        b_pos(e, kb2, nn);
        if constexpr (TB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) Bs[kb2 + q][nn] = rb[4 * e + q];
        } else {
          *reinterpret_cast<float4*>(&Bs[kb2][nn]) = make_float4(rb[4 * e], rb[4 * e + 1], rb[4 * e + 2], rb[4 * e + 3]);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int mm, kk, nn, kb2;
        a_pos(e, mm, kk);
        As[kk][mm] = ra[e];
        b_pos(e, kb2, nn);
        Bs[kb2][nn] = rb[e];
      }
    }
  };

  load(kb);
  store();
  __syncthreads();
  for (int k0 = kb; k0 < ke; k0 += SBK) {
    const bool more = k0 + SBK < ke;
    if (more) load(k0 + SBK);  // in flight during this tile's MFMAs
#pragma unroll
    for (int ks = 0; ks < SBK; ks += 4) {
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
    if (more) {
      store();
      __syncthreads();
    }
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
        float* o = C + (int64_t)m * ldc + n;
        if (atomic_out) {  // split-K partial (act == 0; the bias comes with split 0)
          if (bias && blockIdx.z == 0) v += bias[n];
          atomicAdd(o, v);
          continue;
        }
        if (bias) v += bias[n];
        if (act == 1) v = fmaxf(v, 0.f);
        else if (act == 2) v = 1.f / (1.f + expf(-v));
        *o = accumulate ? *o + v : v;
      }
    }
}

}  // namespace

void sgemm_launch(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
                  int ldb, int ldc, bool transA, bool transB, int act, bool accumulate, hipStream_t s,
                  bool allow_split) {
  const int tn = (N + 63) / 64, tm = (M + 63) / 64;
  int splits = 1;
  if (allow_split && act == 0 && tn * tm < 128 && K >= 512) {
    splits = std::min((256 + tn * tm - 1) / (tn * tm), K / 128);
    if (splits > 1 && !accumulate) {
      if (ldc != N) splits = 1;  // the zero fill below assumes a dense C
      else TFX_HIP_CHECK(hipMemsetAsync(C, 0, sizeof(float) * (size_t)M * N, s));
    }
  }
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + SBK - 1) / SBK * SBK;
  splits = (K + kchunk - 1) / kchunk;
  if (splits < 1) splits = 1;
  const bool atomic_out = splits > 1;
  const bool aligned = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0;
  const bool vec = aligned && (lda % 4 == 0) && (ldb % 4 == 0) && (M % 4 == 0) && (N % 4 == 0) && (K % 4 == 0);
  dim3 grid(tn, tm, splits);
#define TFX_SG(TA_, TB_)                                                                                   \
  if (vec) sgemm_kernel<TA_, TB_, true><<<grid, 256, 0, s>>>(A, B, C, bias, M, N, K, lda, ldb, ldc, act,   \
                                                              accumulate, kchunk, atomic_out);              \
  else sgemm_kernel<TA_, TB_, false><<<grid, 256, 0, s>>>(A, B, C, bias, M, N, K, lda, ldb, ldc, act,      \
                                                          accumulate, kchunk, atomic_out);
  if (transA) {
    if (transB) { TFX_SG(true, true) } else { TFX_SG(true, false) }
  } else {
    if (transB) { TFX_SG(false, true) } else { TFX_SG(false, false) }
  }
#undef TFX_SG
}

}  // namespace tfx
