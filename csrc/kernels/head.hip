// Fused classifier head of a training step, for gfx950: global average pool -> FC (O <= 16 classes)
// -> softmax cross-entropy -> the head's input gradient, in ONE launch; its parameter gradients in a
// second, small one.
//
// Layer-wise the head of ResNet-50/CIFAR is five launches (gap_fwd, a 2-block bf16 GEMM that walks
// K = 2048 serially, softmax_xent_mean, linear_small_bwd, gap_bwd: 76 us of a 7.5 ms step,
// profiles/r03_f1/step_trace_conv3.txt).  Forward, one block per sample (rows are independent once
// the batch mean is taken out of the loss gradient: dz = (p - y) / B; 1024 threads = 4 pixel groups
// x 256 channel lanes, so a sample's pixels stream in parallel, reduced through LDS):
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
// TAIL: the head's input is the last block's tail BN output, never written -- out = relu(y3 sc + sh + res)
// is formed per pixel while pooling (bf16, exactly the apply pass's values) with its ReLU mask bits
// stored for the BN's backward, and that BN's backward partials (sum g', sum g' xhat over g' = dfeat *
// mask: per channel d * sum_hw mask, d * sum_hw mask xhat, d the pixel-constant input gradient) are
// written as one row per sample (no atomics), summed by head_rows_reduce in the backward -- the apply
// pass and the BN's backward reduction pass disappear.
// Reference: R/distributed/distributed.py:96-102 (the loss the reference builds op by op); north-star
// ResNet-50 head (BASELINE.json config 3).
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {
namespace {

constexpr int HEAD_NT = 256;                             // channel lanes: 8 channels each
constexpr int HEAD_PG = 4;                               // forward: pixel groups of HEAD_NT threads
constexpr int HEAD_FT = HEAD_NT * HEAD_PG;               // forward block
constexpr int HEAD_U = 4;                                // pixels in flight per thread
constexpr int HEAD_UT = 4;                               // ... in TAIL mode (two operands)
constexpr int HEAD_CNT_BITS = 12;                        // done count (N <= 4095)
constexpr double HEAD_FIX = 16777216.0;                 // 2^24 per unit of loss
// a row's fixed-point loss is < HEAD_ROW_MAX x 2^24, and the word holds 64 - 12 = 52 bits of sum:
// 4095 rows x 6.5e4 x 2^24 < 2^52 (2^28 / 4095 = 65552).  A row at or past it (a diverged loss)
// takes the NaN-flag path instead of wrapping the word into a wrong finite mean.
constexpr float HEAD_ROW_MAX = 6.5e4f;

__device__ __forceinline__ void head_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int OMAX, bool TAIL>
__global__ void __launch_bounds__(HEAD_FT) head_xent_fwd_kernel(HeadXentArgs a) {
  __shared__ float part[HEAD_NT / 16][OMAX];  // one partial per DPP row (16 lanes)
  __shared__ float dzs[OMAX];
  // per pixel group: pooled sums (TAIL: + sum_hw mask, sum_hw mask * xhat), [quantity][group][k][t]
  __shared__ float red[TAIL ? 3 : 1][HEAD_PG][8][HEAD_NT];
  __shared__ U4 dlds[HEAD_NT];  // the packed pixel-constant dfeat of each 8-channel group
  __shared__ float bsh[OMAX];
  const int n = blockIdx.x, tt = threadIdx.x, t = tt & (HEAD_NT - 1), pg = tt / HEAD_NT, lane = tt & 63;
  const int C8 = a.C >> 3, O = a.O;
  const bool own = t < C8;   // this thread's 8 channels (C <= 8 * HEAD_NT, host check)
  const bool lead = pg == 0;  // wave-uniform: pixel group 0 computes the logits and dfeat
  const float inv_hw = 1.f / (float)a.HW;
  const U4 zero = U4{0u, 0u, 0u, 0u};
  // every load below is unconditional at a clamped index (a select around a load compiles to a branch
  // that drains the load counter): a thread past C reads channel group 0, a padding pixel the last one
  const int tc = own ? t : 0;
  const int64_t lab = a.labels[n];
  const float bias = ld_f32_or0(a.b, min(tt, O - 1));

  // ---- pooled partials of this pixel group: pixels pg, pg + PG, ... (HEAD_U of them in flight)
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (!TAIL) {
    const U4* xr = reinterpret_cast<const U4*>(a.x + (int64_t)n * a.HW * a.C);
    for (int p = pg; p < a.HW; p += HEAD_PG * HEAD_U) {
      U4 v[HEAD_U];
#pragma unroll
      for (int q = 0; q < HEAD_U; ++q) {
        const int pp = p + HEAD_PG * q;
        v[q] = xr[(int64_t)min(pp, a.HW - 1) * C8 + tc];
      }
#pragma unroll
      for (int q = 0; q < HEAD_U; ++q) {
        if (p + HEAD_PG * q >= a.HW) break;
        float e[8];
        unpack8(v[q], e);
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += e[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[0][pg][k][t] = s[k];
  } else {
    float sc[8], sh[8], mu[8], is[8], cnt[8], sxh[8];  // cnt / sxh: sum_hw mask, sum_hw mask * xhat
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = 8 * tc + k;
      mu[k] = a.save3[c];
      is[k] = a.save3[a.C + c];
      sc[k] = a.save3[2 * a.C + c];
      sh[k] = a.save3[3 * a.C + c];
      cnt[k] = sxh[k] = 0.f;
    }
    const U4* yr = reinterpret_cast<const U4*>(a.y3 + (int64_t)n * a.HW * a.C);
    const U4* rr = reinterpret_cast<const U4*>(a.res + (int64_t)n * a.HW * a.C);
    for (int p = pg; p < a.HW; p += HEAD_PG * HEAD_UT) {
      U4 vy[HEAD_UT], vr[HEAD_UT];
#pragma unroll
      for (int q = 0; q < HEAD_UT; ++q) {
        const int pp = p + HEAD_PG * q;
        const int64_t i = (int64_t)min(pp, a.HW - 1) * C8 + tc;
        vy[q] = yr[i];
        vr[q] = rr[i];
      }
#pragma unroll
      for (int q = 0; q < HEAD_UT; ++q) {
        const int pp = p + HEAD_PG * q;
        if (pp >= a.HW) break;  // a padding pixel would add relu(shift)
        float ey[8], er[8], o[8];
        unpack8(vy[q], ey);
        unpack8(vr[q], er);
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = fmaf(ey[k], sc[k], sh[k]) + er[k];  // bn_apply_vec's math
          const bool on = z > 0.f;
          bits |= (on ? 1u : 0u) << k;
          o[k] = fmaxf(z, 0.f);
          cnt[k] += on ? 1.f : 0.f;
          sxh[k] += on ? (ey[k] - mu[k]) * is[k] : 0.f;
        }
        float ob[8];
        unpack8(pack8(o), ob);  // the bf16 values the apply pass would have written
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += ob[k];
        if (own) a.mask[((int64_t)n * a.HW + pp) * C8 + t] = (uint8_t)bits;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[0][pg][k][t] = s[k];
      red[1][pg][k][t] = cnt[k];
      red[2][pg][k][t] = sxh[k];
    }
  }
  // ---- W columns of this thread's channels (L2-resident; the lead waves only, in flight over the sync)
  // (rows past O read row O-1 and are never used; a thread past C reads real channels, times f = 0)
  U4 wraw[OMAX];
  if (lead) {
#pragma unroll
    for (int j = 0; j < OMAX; ++j) wraw[j] = reinterpret_cast<const U4*>(a.w + (int64_t)min(j, O - 1) * a.C)[tc];
  }
  if (tt < OMAX) bsh[tt] = bias;
  __syncthreads();

  // ---- logits: per-thread partial dots, DPP row sums, 16 partials per class through LDS
  float f[8];
  if (lead) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = red[0][0][k][t];
#pragma unroll
      for (int g = 1; g < HEAD_PG; ++g) v += red[0][g][k][t];
      s[k] = v * inv_hw;
    }
    const U4 fb = pack8(s);  // the layer-wise gap_fwd output (bf16)
    unpack8(fb, f);
    if (!own)
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = 0.f;
    if (own) reinterpret_cast<U4*>(a.feat + (int64_t)n * a.C)[t] = fb;
#pragma unroll
    for (int j = 0; j < OMAX; ++j) {
      float w[8];
      unpack8(wraw[j], w);
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) d = fmaf(w[k], f[k], d);
      d = row16_sum(d);  // classes past O: never read
      if ((lane & 15) == 0) part[t >> 4][j] = d;
    }
  }
  head_lds_sync();
  unsigned long long prev = 0ull, mine = 0ull;
  float lrow = 0.f;
  if (tt == 0) {
    float z[OMAX];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < OMAX; ++j) {
      if (j < O) {
        float acc = 0.f;
#pragma unroll
        for (int r = 0; r < HEAD_NT / 16; ++r) acc += part[r][j];
        acc += bsh[j];
        z[j] = bf16_to_f32(f32_to_bf16(acc));  // the layer-wise GEMM's bf16 logits
        m = fmaxf(m, z[j]);
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < OMAX; ++j)
      if (j < O) sum += __expf(z[j] - m);
    const float inv_s = 1.f / sum, lse = m + __logf(sum);
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
  // ---- dfeat = bf16(bf16(dz W) / HW) (the layer-wise linear dx, then gap_bwd): lead waves form it
  if (lead) {
    float d[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < OMAX; ++j) {
      float w[8];
      unpack8(wraw[j], w);
      const float g = j < O ? dzs[j] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = fmaf(g, w[k], d[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = bf16_to_f32(f32_to_bf16(d[k])) * inv_hw;
    dlds[t] = pack8(d);
  }
  head_lds_sync();
  // ... every pixel group stores its pixels
  U4* dr = reinterpret_cast<U4*>(a.dfeat + (int64_t)n * a.HW * a.C);
  if (own) {
    const U4 o = dlds[t];
    for (int p = pg; p < a.HW; p += HEAD_PG) dr[(int64_t)p * C8 + t] = o;
  }
  if constexpr (TAIL) {
    // the tail BN's backward partials of this sample, g' = dfeat * mask with dfeat pixel-constant:
    // row n of [N][sum g' | sum g' xhat] (plain stores; head_rows_reduce sums the rows)
    float* row = a.bn_rows + (size_t)n * 2 * a.C;
    const uint16_t* dh = reinterpret_cast<const uint16_t*>(dlds);
    for (int v = tt; v < 2 * a.C; v += HEAD_FT) {
      const int kind = v >= a.C ? 1 : 0, c = v - kind * a.C;
      float tot = 0.f;
#pragma unroll
      for (int g = 0; g < HEAD_PG; ++g) tot += red[1 + kind][g][c & 7][c >> 3];
      row[v] = bf16_to_f32(dh[c]) * tot;
    }
  }
  // ---- the last block to count in finishes the mean (its returned word + its own = every row)
  if (tt == 0) {
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

// red[v] = sum_n rows[n][v] over v < 2C ([sum g' | sum g' xhat]); dbeta += red[:C], dgamma += red[C:].
// Block = 64 columns x 4 row groups, 8 rows in flight per thread, LDS sum of the 4 groups.
__global__ void __launch_bounds__(256) head_rows_reduce_kernel(const float* __restrict__ rows, int N, int C,
                                                               float* __restrict__ red, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta) {
  __shared__ float part[4][64];
  const int t = threadIdx.x, col = t & 63, rg = t >> 6;
  const int v = blockIdx.x * 64 + col, V = 2 * C;
  float acc = 0.f;
  if (v < V) {
    int r = rg;
    for (; r + 4 * 7 < N; r += 4 * 8) {
      float x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = rows[(size_t)(r + 4 * q) * V + v];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc += x[q];
    }
    for (; r < N; r += 4) acc += rows[(size_t)r * V + v];
  }
  part[rg][col] = acc;
  __syncthreads();
  if (rg == 0 && v < V) {
    const float tot = ((part[0][col] + part[1][col]) + part[2][col]) + part[3][col];
    red[v] = tot;
    if (v < C) {
      if (dbeta) dbeta[v] += tot;
    } else if (dgamma) {
      dgamma[v - C] += tot;
    }
  }
}

}  // namespace

void head_rows_reduce(const float* rows, int N, int C, float* red, float* dgamma, float* dbeta, hipStream_t s) {
  head_rows_reduce_kernel<<<(2 * C + 63) / 64, 256, 0, s>>>(rows, N, C, red, dgamma, dbeta);
}

bool head_xent_ok(int C, int O, int HW) { return C % 8 == 0 && C <= 8 * HEAD_NT && O >= 1 && O <= 16 && HW >= 1; }

void head_xent_fwd(const HeadXentArgs& args, int N, hipStream_t s) {
  const bool tail = args.y3 != nullptr;
  if (args.O <= 10) {  // CIFAR-10
    if (tail) head_xent_fwd_kernel<10, true><<<N, HEAD_FT, 0, s>>>(args);
    else head_xent_fwd_kernel<10, false><<<N, HEAD_FT, 0, s>>>(args);
  } else {
    if (tail) head_xent_fwd_kernel<16, true><<<N, HEAD_FT, 0, s>>>(args);
    else head_xent_fwd_kernel<16, false><<<N, HEAD_FT, 0, s>>>(args);
  }
}

void head_wgrad(const uint16_t* dz, const uint16_t* feat, int N, int C, int O, float* dw, float* db, hipStream_t s) {
  if (O <= 10) head_wgrad_kernel<10><<<C / 8, HEAD_NT, 0, s>>>(dz, feat, N, C, O, dw, db);
  else head_wgrad_kernel<16><<<C / 8, HEAD_NT, 0, s>>>(dz, feat, N, C, O, dw, db);
}

}  // namespace tfx
