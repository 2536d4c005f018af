// Fused classifier head of a training step, for gfx950: global average pool -> FC (O <= 16 classes)
// -> softmax cross-entropy -> the head's input gradient, in ONE launch; its parameter gradients in a
// second, small one.
//
// Layer-wise the head of ResNet-50/CIFAR is five launches (gap_fwd, a 2-block bf16 GEMM that walks
// K = 2048 serially, softmax_xent_mean, linear_small_bwd, gap_bwd: 76 us of a 7.5 ms step,
// profiles/r03_f1/step_trace_conv3.txt).  Forward, one block per sample (rows are independent once
// the batch mean is taken out of the loss gradient: dz = (p - y) / B):
//   f      = bf16(mean_hw x[n])                     (written: the FC weight gradient needs it)
//   z      = bf16(W f + b)                          (DPP row sums, then 16 partials per class in LDS)
//   loss_n = logsumexp(z) - z[label],  dz = bf16((p - onehot) / B)   (dz written for dW / db)
//   dfeat  = bf16(bf16(dz W) / HW) broadcast over the HW pixels      (the unit-seed input gradient)
// with the same roundings as the layer-wise ops, so both paths agree to accumulation order.
// Backward (head_wgrad): dW += dz^T f, db += colsum(dz), one block per 8 channels over every sample.
//
// The batch-mean loss: each block adds ONE 64-bit word -- its row loss as 2^-24 fixed point above a
// 12-bit done count -- with one memory-side atomic.  Integer sums are order-independent, so the mean
// is deterministic; the block that sees count N-1 in the returned word holds the whole sum, writes the
// mean and re-zeroes the word (zero after every launch: graph-replay safe).  The atomic is issued
// before the block's dfeat stores, so its round trip hides behind them; no release/acquire fences
// (atomics complete at the memory side).  A non-finite or huge row loss sets a flag word first: the
// mean is then NaN.
// Reference: R/distributed/distributed.py:96-102 (the loss the reference builds op by op); north-star
// ResNet-50 head (BASELINE.json config 3).
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {
namespace {

constexpr int HEAD_NT = 256;
constexpr int HEAD_CNT_BITS = 12;                        // done count (N <= 4095)
constexpr double HEAD_FIX = 16777216.0;                 // 2^24 per unit of loss
constexpr float HEAD_ROW_MAX = 1e6f;                    // 4095 rows x 1e6 x 2^24 < 2^64 / 2^12

__device__ __forceinline__ void head_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int OMAX>
__global__ void __launch_bounds__(HEAD_NT) head_xent_fwd_kernel(HeadXentArgs a) {
  __shared__ float part[HEAD_NT / 16][OMAX];  // one partial per DPP row (16 lanes)
  __shared__ float dzs[OMAX];
  const int n = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int C8 = a.C >> 3, O = a.O;
  const bool own = t < C8;  // this thread's 8 channels (C <= 8 * HEAD_NT, host check)
  const float inv_hw = 1.f / (float)a.HW;
  const U4* xr = reinterpret_cast<const U4*>(a.x + (int64_t)n * a.HW * a.C);
  const U4 zero = U4{0u, 0u, 0u, 0u};

  // ---- W columns of this thread's channels (L2-resident, independent of x: issued first)
  U4 wraw[OMAX];
#pragma unroll
  for (int j = 0; j < OMAX; ++j) wraw[j] = (j < O && own) ? reinterpret_cast<const U4*>(a.w + (int64_t)j * a.C)[t] : zero;
  // ---- pooled features: 16 pixels' loads in flight per step
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < a.HW; p += 16) {
    U4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = (own && p + q < a.HW) ? xr[(int64_t)(p + q) * C8 + t] : zero;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float e[8];
      unpack8(v[q], e);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += e[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] *= inv_hw;
  const U4 fb = pack8(s);  // the layer-wise gap_fwd output (bf16)
  float f[8];
  unpack8(fb, f);
  if (own) reinterpret_cast<U4*>(a.feat + (int64_t)n * a.C)[t] = fb;

  // ---- logits: per-thread partial dots, DPP row sums, 16 partials per class through LDS
  float w[OMAX][8];
#pragma unroll
  for (int j = 0; j < OMAX; ++j) {
    unpack8(wraw[j], w[j]);
    float d = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) d = fmaf(w[j][k], f[k], d);
    d = row16_sum(d);
    if ((lane & 15) == 0) part[t >> 4][j] = d;
  }
  head_lds_sync();
  unsigned long long prev = 0ull, mine = 0ull;
  float lrow = 0.f;
  if (t == 0) {
    float z[OMAX];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < OMAX; ++j) {
      if (j < O) {
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < HEAD_NT / 16; ++r) acc += part[r][j];
        if (a.b) acc += a.b[j];
        z[j] = bf16_to_f32(f32_to_bf16(acc));  // the layer-wise GEMM's bf16 logits
        m = fmaxf(m, z[j]);
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < OMAX; ++j)
      if (j < O) sum += __expf(z[j] - m);
    const float inv_s = 1.f / sum, lse = m + __logf(sum);
    const int64_t lab = a.labels[n];
#pragma unroll
    for (int j = 0; j < OMAX; ++j) {
      if (j < O) {
        const float y = j == lab ? 1.f : 0.f;
        if (y != 0.f) lrow += lse - z[j];
        const uint16_t d = f32_to_bf16((__expf(z[j] - m) * inv_s - y) * a.gscale);
        a.dz[(int64_t)n * O + j] = d;
        dzs[j] = bf16_to_f32(d);
      }
    }
    // ---- batch mean (see header): the flag (rare) has returned before the word's add is issued
    const bool ok = lrow == lrow && lrow < HEAD_ROW_MAX;
    if (!ok) {
      const unsigned long long r = __hip_atomic_fetch_or(a.state + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("" ::"v"(r) : "memory");
    }
    mine = ((ok ? (unsigned long long)((double)lrow * HEAD_FIX + 0.5) : 0ull) << HEAD_CNT_BITS) | 1ull;
    prev = __hip_atomic_fetch_add(a.state, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  head_lds_sync();
  // ---- dfeat = bf16(bf16(dz W) / HW) over every pixel (the layer-wise linear dx, then gap_bwd)
  float d[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < OMAX; ++j) acc = fmaf(j < O ? dzs[j] : 0.f, w[j][k], acc);
    d[k] = bf16_to_f32(f32_to_bf16(acc)) * inv_hw;
  }
  const U4 o = pack8(d);
  U4* dr = reinterpret_cast<U4*>(a.dfeat + (int64_t)n * a.HW * a.C);
  if (own)
    for (int p = 0; p < a.HW; ++p) dr[(int64_t)p * C8 + t] = o;
  // ---- the last block to count in finishes the mean (its returned word + its own = every row)
  if (t == 0) {
    const unsigned long long tot = prev + mine;
    const unsigned long long cnt = tot & ((1ull << HEAD_CNT_BITS) - 1);
    if (cnt == (unsigned long long)gridDim.x) {
      const unsigned long long bad =
          __hip_atomic_exchange(a.state + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(a.state, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double sum = (double)(tot >> HEAD_CNT_BITS) / HEAD_FIX;
      a.loss[0] = bad ? __builtin_nanf("") : (float)(sum / (double)gridDim.x);
    }
  }
}

// dW [O][C] += dz^T f, db += colsum(dz): block b owns channels 8b .. 8b+7 (plain read-modify-write,
// no atomics: no other block touches them), thread = sample row(s); DPP row sums, then 16 partials
// per (class, channel) through LDS.  Block 0 also reduces db.
template <int OMAX>
__global__ void __launch_bounds__(HEAD_NT) head_wgrad_kernel(const uint16_t* __restrict__ dz,
                                                             const uint16_t* __restrict__ feat, int N, int C, int O,
                                                             float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float part[HEAD_NT / 16][OMAX][9];
  const int t = threadIdx.x, lane = t & 63, cg = blockIdx.x;
  float acc[OMAX][8], accb[OMAX];
#pragma unroll
  for (int j = 0; j < OMAX; ++j) {
    accb[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  }
  for (int r = t; r < N; r += HEAD_NT) {
    float fv[8], g[OMAX];
    unpack8(reinterpret_cast<const U4*>(feat + (int64_t)r * C)[cg], fv);
#pragma unroll
    for (int j = 0; j < OMAX; ++j) g[j] = j < O ? bf16_to_f32(dz[(int64_t)r * O + j]) : 0.f;
#pragma unroll
    for (int j = 0; j < OMAX; ++j) {
      accb[j] += g[j];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[j][k] = fmaf(g[j], fv[k], acc[j][k]);
    }
  }
#pragma unroll
  for (int j = 0; j < OMAX; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float v = row16_sum(acc[j][k]);
      if ((lane & 15) == 0) part[t >> 4][j][k] = v;
    }
    const float vb = row16_sum(accb[j]);
    if ((lane & 15) == 0) part[t >> 4][j][8] = vb;
  }
  __syncthreads();
  if (t < OMAX * 9) {
    const int j = t / 9, k = t % 9;
    if (j < O && (k < 8 || cg == 0)) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < HEAD_NT / 16; ++r) v += part[r][j][k];
      if (k < 8) {
        if (dw) dw[(int64_t)j * C + 8 * cg + k] += v;
      } else if (db) {
        db[j] += v;
      }
    }
  }
}

}  // namespace

bool head_xent_ok(int C, int O, int HW) { return C % 8 == 0 && C <= 8 * HEAD_NT && O >= 1 && O <= 16 && HW >= 1; }

void head_xent_fwd(const HeadXentArgs& args, int N, hipStream_t s) {
  if (args.O <= 10) head_xent_fwd_kernel<10><<<N, HEAD_NT, 0, s>>>(args);  // CIFAR-10
  else head_xent_fwd_kernel<16><<<N, HEAD_NT, 0, s>>>(args);
}

void head_wgrad(const uint16_t* dz, const uint16_t* feat, int N, int C, int O, float* dw, float* db, hipStream_t s) {
  if (O <= 10) head_wgrad_kernel<10><<<C / 8, HEAD_NT, 0, s>>>(dz, feat, N, C, O, dw, db);
  else head_wgrad_kernel<16><<<C / 8, HEAD_NT, 0, s>>>(dz, feat, N, C, O, dw, db);
}

}  // namespace tfx
