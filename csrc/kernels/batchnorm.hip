// Batch normalisation for NHWC bf16 activations (f32 statistics), with ReLU and the residual add
// of a ResNet bottleneck fused into the apply pass.
//
// Layout: x is [M][C] with M = N*H*W rows (channels-last), C contiguous.
// Forward  : stats -> finalize (mean, invstd, scale = gamma*invstd, shift = beta - mean*scale,
//            running-stat update) -> apply  y = relu?(x*scale + shift (+ res)).
//            The stats normally come for free from the producing conv's epilogue
//            (igemm.hip with a stats workspace); bn_stats is the standalone pass.
// Backward : reduce (sum g', sum g'*xhat with g' = g * [z > 0] recomputed from x/res)
//            -> apply  dx = A*g' + B*x + D per channel (BN backward folded into 3 coefficients),
//            dres = g'.  dgamma / dbeta are accumulated straight into the parameter gradients.
//
// Cross-block reductions go through a PERSISTENT slot workspace [NSLOT][2][C] (one per BN layer):
// block b adds its partial into slot b % NSLOT (<= ~32 adders per address instead of every block
// on one address, which serialises at the memory side: MI355X_MICROARCH.md "Global float
// atomics", contention row).  The consumer (finalize / slot-reduce) zeroes the slots after reading
// them, so the workspace is always zero between uses: no memset launches.
// Elementwise passes give every thread a FIXED 8-channel vector (grid stride is a multiple of
// C/8), so per-channel parameters live in registers; 16 B per lane per access.
#include "tfx_common.h"
#include "tfx_kernels.h"

#include <cstdlib>

namespace tfx {

namespace {

// ------------------------------------------------------------------ stats (vector)
// TPR threads per row (C/8), RPB = 256/TPR rows per block-iteration.
__global__ void __launch_bounds__(256) bn_stats_vec_kernel(const uint16_t* __restrict__ x, int64_t M, int C,
                                                           float* __restrict__ slots) {
  const int tpr = C >> 3;
  const int rpb = 256 / tpr;
  const int t = threadIdx.x;
  const int cv = t % tpr, r0 = t / tpr;
  float s[8] = {0}, q[8] = {0};
  const int64_t stride = (int64_t)gridDim.x * rpb;
  int64_t r = (int64_t)blockIdx.x * rpb + r0;
  for (; r + 3 * stride < M; r += 4 * stride) {
    U4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const U4*>(x + (r + u * stride) * C + cv * 8);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += f[i]; q[i] = fmaf(f[i], f[i], q[i]); }
    }
  }
  for (; r < M; r += stride) {
    float f[8];
    unpack8(*reinterpret_cast<const U4*>(x + r * C + cv * 8), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[i] += f[i]; q[i] = fmaf(f[i], f[i], q[i]); }
  }
  __shared__ float red[256 * 8];
  for (int pass = 0; pass < 2; ++pass) {
    float* v = pass ? q : s;
#pragma unroll
    for (int i = 0; i < 8; ++i) red[i * 256 + t] = v[i];
    __syncthreads();
    for (int h = rpb >> 1; h > 0; h >>= 1) {
      if (r0 < h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) red[i * 256 + t] += red[i * 256 + t + h * tpr];
      }
      __syncthreads();
    }
    __syncthreads();
    // coalesced atomics: consecutive lanes -> consecutive channels (channel c = cv*8 + i lives at
    // red[i*256 + cv]); a lane-per-8-channel pattern would be a 32-B-strided scatter per instruction
    float* slot = slots + (size_t)(blockIdx.x % NSLOT) * 2 * C + pass * C;
    for (int c = t; c < C; c += 256) atomicAdd(slot + c, red[(c & 7) * 256 + (c >> 3)]);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) bn_stats_gen_kernel(const uint16_t* __restrict__ x, int64_t M, int C,
                                                           float* __restrict__ slots) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s = 0.f, q = 0.f;
  if (c < C) {
    for (int64_t r = (int64_t)blockIdx.y * 4 + ty; r < M; r += (int64_t)gridDim.y * 4) {
      const float f = bf16_to_f32(x[r * C + c]);
      s += f;
      q = fmaf(f, f, q);
    }
  }
  __shared__ float rs[256], rq[256];
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  __syncthreads();
  if (ty == 0 && c < C) {
    float* slot = slots + (size_t)((blockIdx.y % NSLOT) * 2) * C;
    atomicAdd(&slot[c], rs[tx] + rs[tx + 64] + rs[tx + 128] + rs[tx + 192]);
    atomicAdd(&slot[C + c], rq[tx] + rq[tx + 64] + rq[tx + 128] + rq[tx + 192]);
  }
}

// Sum the NSLOT slot rows for 16 channels per block (16 slot-lanes x 4 slots each, all loads in
// flight before any store), then zero the consumed slots.  Returns the sums in lanes ty == 0.
__device__ __forceinline__ void slot_sum_consume(float* __restrict__ slots, int C, int c, float& s, float& q) {
  const int ty = threadIdx.x >> 4;  // 0..15
  float vs[NSLOT / 16], vq[NSLOT / 16];
  s = 0.f;
  q = 0.f;
  // loads unconditional at a clamped channel (a branch around them would drain the load counter
  // before the caller's own loads return); the sums of a thread past C are never used
  const int cc = min(c, C - 1);
#pragma unroll
  for (int i = 0; i < NSLOT / 16; ++i) {
    const float* p = slots + (size_t)(ty + 16 * i) * 2 * C;
    vs[i] = p[cc];
    vq[i] = p[C + cc];
  }
#pragma unroll
  for (int i = 0; i < NSLOT / 16; ++i) {
    s += vs[i];
    q += vq[i];
  }
  __shared__ float rs[256], rq[256];
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  // the re-zeroing stores go out after the sums consumed the loads, and the barrier waits for LDS only
  // (__syncthreads' fence would also wait for these stores to complete)
  if (c < C) {
#pragma unroll
    for (int i = 0; i < NSLOT / 16; ++i) {
      float* p = slots + (size_t)(ty + 16 * i) * 2 * C;
      p[c] = 0.f;  // keep the workspace zero for its next use
      p[C + c] = 0.f;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (ty == 0) {
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      s += rs[threadIdx.x + 16 * k];
      q += rq[threadIdx.x + 16 * k];
    }
  }
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(float* __restrict__ slots, int64_t M, int C,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          float eps, float momentum, float* __restrict__ run_mean,
                                                          float* __restrict__ run_var, float* __restrict__ save) {
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  // parameter / running-stat loads issued before the slot reduction: one memory round trip per
  // kernel instead of two (these launches are latency-bound, ~100 of them per ResNet-50 step)
  // (unconditional loads at a clamped channel: no branch around them, see slot_sum_consume)
  const bool own = (threadIdx.x >> 4) == 0 && c < C;
  const int cc = min(c, C - 1);
  const float g0 = ld_f32_or0(gamma, cc), b = ld_f32_or0(beta, cc);
  const float rm = ld_f32_or0(run_mean, cc), rv = ld_f32_or0(run_var, cc);
  const float g = gamma ? g0 : 1.f;
  float sum, sq;
  slot_sum_consume(slots, C, c, sum, sq);
  if (!own) return;
  const float inv_m = 1.f / (float)M;
  const float mean = sum * inv_m;
  const float var = fmaxf(sq * inv_m - mean * mean, 0.f);
  const float invstd = rsqrtf(var + eps);
  const float scale = g * invstd;
  save[c] = mean;
  save[C + c] = invstd;
  save[2 * C + c] = scale;
  save[3 * C + c] = b - mean * scale;
  if (run_mean) {
    const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    run_mean[c] = (1.f - momentum) * rm + momentum * mean;
    run_var[c] = (1.f - momentum) * rv + momentum * unb;
  }
}

// backward: slots -> red[2][C] (= [dbeta | dgamma]); accumulate into the parameter grads
__global__ void __launch_bounds__(256) bn_slot_reduce_kernel(float* __restrict__ slots, int C,
                                                             float* __restrict__ red, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta) {
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool own = (threadIdx.x >> 4) == 0 && c < C;
  const int cc = min(c, C - 1);  // loaded before the slot reduction (one round trip, see finalize)
  const float db = ld_f32_or0(dbeta, cc), dg = ld_f32_or0(dgamma, cc);
  float s, q;
  slot_sum_consume(slots, C, c, s, q);
  if (own) {
    red[c] = s;
    red[C + c] = q;
    if (dbeta) dbeta[c] = db + s;
    if (dgamma) dgamma[c] = dg + q;
  }
}

__global__ void bn_eval_prep_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                    float eps, const float* __restrict__ run_mean,
                                    const float* __restrict__ run_var, float* __restrict__ save) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(run_var[c] + eps);
  const float scale = (gamma ? gamma[c] : 1.f) * invstd;
  save[c] = run_mean[c];
  save[C + c] = invstd;
  save[2 * C + c] = scale;
  save[3 * C + c] = (beta ? beta[c] : 0.f) - run_mean[c] * scale;
}

// ------------------------------------------------------------------ apply (fixed channel vector)
// grid * 256 is a multiple of C/8 (host), so vector i = tid + k*stride always has channel vector
// (tid0 % (C/8)).  Two vectors per iteration for memory-level parallelism.
// With RES && RELU the ReLU mask of the output is also stored, one bit per element (one byte per
// 8-channel vector): the backward then reads 1/16 of the residual tensor's bytes instead of the
// residual itself (twice: reduce and apply).
// RBN: the residual is another BN's INPUT, normalized here on the fly with its rsave -- that BN
// (a ResNet projection shortcut's, used only as this residual) never writes its output.
template <bool RES, bool RELU, bool RBN = false>
__global__ void __launch_bounds__(256) bn_apply_vec_kernel(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ res,
                                                           const float* __restrict__ save, int64_t nvec, int C,
                                                           uint16_t* __restrict__ y, uint8_t* __restrict__ mask,
                                                           const float* __restrict__ rsave = nullptr) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int c0 = (int)(i0 % (C >> 3)) * 8;
  float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = save[2 * C + c0 + k];
    sh[k] = save[3 * C + c0 + k];
    if (RBN) {
      rsc[k] = rsave[2 * C + c0 + k];
      rsh[k] = rsave[3 * C + c0 + k];
    }
  }
  auto one = [&](int64_t i) {
    float f[8], r[8];
    unpack8(reinterpret_cast<const U4*>(x)[i], f);
    if (RES) unpack8(reinterpret_cast<const U4*>(res)[i], r);
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float z = fmaf(f[k], sc[k], sh[k]);
      if (RBN) z += fmaf(r[k], rsc[k], rsh[k]);
      else if (RES) z += r[k];
      bits |= (z > 0.f ? 1u : 0u) << k;
      f[k] = RELU ? fmaxf(z, 0.f) : z;
    }
    reinterpret_cast<U4*>(y)[i] = pack8(f);
    if (RES && RELU && mask) mask[i] = (uint8_t)bits;
  };
  int64_t i = i0;
  for (; i + stride < nvec; i += 2 * stride) {
    one(i);
    one(i + stride);
  }
  if (i < nvec) one(i);
}

template <bool RES, bool RELU>
__global__ void __launch_bounds__(256) bn_apply_gen_kernel(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ res,
                                                           const float* __restrict__ save, int64_t n, int C,
                                                           uint16_t* __restrict__ y) {
  const float* scale = save + 2 * C;
  const float* shift = save + 3 * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    float z = fmaf(bf16_to_f32(x[i]), scale[c], shift[c]);
    if (RES) z += bf16_to_f32(res[i]);
    y[i] = f32_to_bf16(RELU ? fmaxf(z, 0.f) : z);
  }
}

// ------------------------------------------------------------------ backward reduce
// RES && RELU: the ReLU mask comes from the forward's mask bits (``mask``, one byte per vector)
template <bool RES, bool RELU, int U>
__global__ void __launch_bounds__(256) bn_bwd_reduce_vec_kernel(const uint16_t* __restrict__ g,
                                                                const uint16_t* __restrict__ x,
                                                                const uint8_t* __restrict__ mask,
                                                                const float* __restrict__ save, int64_t M, int C,
                                                                float* __restrict__ slots) {
  const int tpr = C >> 3;
  const int rpb = 256 / tpr;
  const int t = threadIdx.x;
  const int cv = t % tpr, r0 = t / tpr;
  float mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = save[cv * 8 + k];
    is[k] = save[C + cv * 8 + k];
    sc[k] = save[2 * C + cv * 8 + k];
    sh[k] = save[3 * C + cv * 8 + k];
  }
  float sg[8] = {0}, sx[8] = {0};
  const int64_t stride = (int64_t)gridDim.x * rpb;
  auto accum = [&](const U4& gv, const U4& xv, uint32_t mb) {
    float gf[8], xf[8];
    unpack8(gv, gf);
    unpack8(xv, xf);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gg = gf[k];
      if (RES && RELU) {
        gg = ((mb >> k) & 1u) ? gg : 0.f;
      } else if (RELU) {
        gg = fmaf(xf[k], sc[k], sh[k]) > 0.f ? gg : 0.f;
      }
      sg[k] += gg;
      sx[k] = fmaf(gg, (xf[k] - mu[k]) * is[k], sx[k]);
    }
  };
  // U independent rows in flight per thread
  const int tprv = C >> 3;
  int64_t r = (int64_t)blockIdx.x * rpb + r0;
  for (; r + (U - 1) * stride < M; r += U * stride) {
    U4 gv[U], xv[U];
    uint32_t mv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (r + u * stride) * C + cv * 8;
      gv[u] = *reinterpret_cast<const U4*>(g + off);
      xv[u] = *reinterpret_cast<const U4*>(x + off);
      mv[u] = (RES && RELU) ? mask[(r + u * stride) * tprv + cv] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) accum(gv[u], xv[u], mv[u]);
  }
  for (; r < M; r += stride) {
    const int64_t off = r * C + cv * 8;
    const uint32_t mb = (RES && RELU) ? mask[r * tprv + cv] : 0u;
    accum(*reinterpret_cast<const U4*>(g + off), *reinterpret_cast<const U4*>(x + off), mb);
  }
  __shared__ float lds[256 * 8];
  for (int pass = 0; pass < 2; ++pass) {
    float* v = pass ? sx : sg;
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[i * 256 + t] = v[i];
    __syncthreads();
    for (int h = rpb >> 1; h > 0; h >>= 1) {
      if (r0 < h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) lds[i * 256 + t] += lds[i * 256 + t + h * tpr];
      }
      __syncthreads();
    }
    __syncthreads();
    float* slot = slots + (size_t)(blockIdx.x % NSLOT) * 2 * C + pass * C;
    for (int c = t; c < C; c += 256) atomicAdd(slot + c, lds[(c & 7) * 256 + (c >> 3)]);
    __syncthreads();
  }
}

template <bool RES, bool RELU>
__global__ void __launch_bounds__(256) bn_bwd_reduce_gen_kernel(const uint16_t* __restrict__ g,
                                                                const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ res,
                                                                const float* __restrict__ save, int64_t M, int C,
                                                                float* __restrict__ slots) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float sg = 0.f, sx = 0.f;
  if (c < C) {
    const float mu = save[c], is = save[C + c], sc = save[2 * C + c], sh = save[3 * C + c];
    for (int64_t r = (int64_t)blockIdx.y * 4 + ty; r < M; r += (int64_t)gridDim.y * 4) {
      const int64_t off = r * C + c;
      float gg = bf16_to_f32(g[off]);
      const float xf = bf16_to_f32(x[off]);
      if (RELU) {
        float z = fmaf(xf, sc, sh);
        if (RES) z += bf16_to_f32(res[off]);
        gg = z > 0.f ? gg : 0.f;
      }
      sg += gg;
      sx = fmaf(gg, (xf - mu) * is, sx);
    }
  }
  __shared__ float a[256], b[256];
  a[threadIdx.x] = sg;
  b[threadIdx.x] = sx;
  __syncthreads();
  if (ty == 0 && c < C) {
    float* slot = slots + (size_t)((blockIdx.y % NSLOT) * 2) * C;
    atomicAdd(&slot[c], a[tx] + a[tx + 64] + a[tx + 128] + a[tx + 192]);
    atomicAdd(&slot[C + c], b[tx] + b[tx + 64] + b[tx + 128] + b[tx + 192]);
  }
}

// ------------------------------------------------------------------ backward apply (fixed channel)
// dx = scale*(g' - sum_g/M - (x-mu)*is*sum_gx/M) = A*g' + B*x + D
// SEC (RES only): the residual input is itself a BN output used nowhere else (the projection
// shortcut's BN of a ResNet block), so its incoming gradient is exactly dres = g'.  While g' is in
// registers, also accumulate that BN's backward partials [sum g' | sum g' xhat2] (xhat2 from its
// input x2 and save2) into its slots2: its separate reduce pass (re-reading dres and x2) goes away.
template <bool RES, bool RELU, bool SEC = false>
__global__ void __launch_bounds__(256) bn_bwd_apply_vec_kernel(const uint16_t* __restrict__ g,
                                                               const uint16_t* __restrict__ x,
                                                               const uint8_t* __restrict__ mask,
                                                               const float* __restrict__ save,
                                                               const float* __restrict__ red, int64_t nvec, int64_t M,
                                                               int C, uint16_t* __restrict__ dx,
                                                               uint16_t* __restrict__ dres,
                                                               const uint16_t* __restrict__ x2 = nullptr,
                                                               const float* __restrict__ save2 = nullptr,
                                                               float* __restrict__ slots2 = nullptr) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int c0 = (int)(i0 % (C >> 3)) * 8;
  const float inv_m = 1.f / (float)M;
  float A[8], B[8], D[8], sc[8], sh[8];
  float mu2[8], is2[8], s2[8], q2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    const float mu = save[c], is = save[C + c];
    sc[k] = save[2 * C + c];
    sh[k] = save[3 * C + c];
    const float kg = red[c] * inv_m, kx = red[C + c] * inv_m * is;
    A[k] = sc[k];
    B[k] = -sc[k] * kx;
    D[k] = sc[k] * (kx * mu - kg);
    if (SEC) {
      mu2[k] = save2[c];
      is2[k] = save2[C + c];
      s2[k] = 0.f;
      q2[k] = 0.f;
    }
  }
  for (int64_t i = i0; i < nvec; i += stride) {
    float gf[8], xf[8], o[8], x2f[8];
    unpack8(reinterpret_cast<const U4*>(g)[i], gf);
    unpack8(reinterpret_cast<const U4*>(x)[i], xf);
    if (SEC) unpack8(reinterpret_cast<const U4*>(x2)[i], x2f);
    const uint32_t mb = (RES && RELU) ? mask[i] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gg = gf[k];
      if (RES && RELU) {
        gg = ((mb >> k) & 1u) ? gg : 0.f;
      } else if (RELU) {
        gg = fmaf(xf[k], sc[k], sh[k]) > 0.f ? gg : 0.f;
      }
      gf[k] = gg;
      o[k] = fmaf(A[k], gg, fmaf(B[k], xf[k], D[k]));
      if (SEC) {
        s2[k] += gg;
        q2[k] = fmaf(gg, (x2f[k] - mu2[k]) * is2[k], q2[k]);
      }
    }
    reinterpret_cast<U4*>(dx)[i] = pack8(o);
    // dres == nullptr: the consumer reads g and the mask bits itself (masked conv addend)
    if (RES && dres) reinterpret_cast<U4*>(dres)[i] = pack8(gf);
  }
  if constexpr (SEC) {
    // threads t and t + k*tpr share channel vector t % tpr (256 % tpr == 0, vec_ok): tree over rows
    const int t = threadIdx.x, tpr = C >> 3, rpb = 256 / tpr, r0 = t / tpr;
    __shared__ float lds[256 * 8];
    for (int pass = 0; pass < 2; ++pass) {
      const float* v = pass ? q2 : s2;
#pragma unroll
      for (int k = 0; k < 8; ++k) lds[k * 256 + t] = v[k];
      __syncthreads();
      for (int h = rpb >> 1; h > 0; h >>= 1) {
        if (r0 < h) {
#pragma unroll
          for (int k = 0; k < 8; ++k) lds[k * 256 + t] += lds[k * 256 + t + h * tpr];
        }
        __syncthreads();
      }
      float* slot = slots2 + (size_t)(blockIdx.x % NSLOT) * 2 * C + pass * C;
      for (int c = t; c < C; c += 256) atomicAdd(slot + c, lds[(c & 7) * 256 + (c >> 3)]);
      __syncthreads();
    }
  }
}

template <bool RES, bool RELU>
__global__ void __launch_bounds__(256) bn_bwd_apply_gen_kernel(const uint16_t* __restrict__ g,
                                                               const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ res,
                                                               const float* __restrict__ save,
                                                               const float* __restrict__ red, int64_t n, int64_t M,
                                                               int C, uint16_t* __restrict__ dx,
                                                               uint16_t* __restrict__ dres) {
  const float inv_m = 1.f / (float)M;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const float mu = save[c], is = save[C + c], sc = save[2 * C + c], sh = save[3 * C + c];
    float gg = bf16_to_f32(g[i]);
    const float xf = bf16_to_f32(x[i]);
    if (RELU) {
      float z = fmaf(xf, sc, sh);
      if (RES) z += bf16_to_f32(res[i]);
      gg = z > 0.f ? gg : 0.f;
    }
    const float xh = (xf - mu) * is;
    dx[i] = f32_to_bf16(sc * (gg - red[c] * inv_m - xh * red[C + c] * inv_m));
    if (RES && dres) dres[i] = f32_to_bf16(gg);
  }
}

// ================================================================== launch helpers
bool vec_ok(int C) { return (C % 8 == 0) && (C / 8) <= 256 && (256 % (C / 8) == 0); }
int grid_for(int64_t work, int per_block, int cap = 2048) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g > cap) g = cap;
  return (int)(g < 1 ? 1 : g);
}
int gcd(int a, int b) { return b ? gcd(b, a % b) : a; }
// vectors per thread of the fixed-channel elementwise passes (TFX_BN_VPT, read once; A/B hook)
static int bn_vpt() {
  static const int v = [] {
    const char* e = getenv("TFX_BN_VPT");
    const int x = e ? atoi(e) : 4;
    return x >= 1 && x <= 64 ? x : 4;
  }();
  return v;
}
// elementwise grid whose stride (grid*256 vectors) is a multiple of C/8
int fixed_channel_grid(int64_t nvec, int C) {
  const int cv = C / 8;
  const int mult = cv / gcd(cv, 256);  // blocks per channel period
  int g = grid_for(nvec, 256 * bn_vpt(), 4096);
  g = (g + mult - 1) / mult * mult;
  return g;
}

#define TFX_DISPATCH_RR(RES, RELU, ...)                              \
  if (RES) {                                                         \
    if (RELU) { constexpr bool R_ = true, L_ = true; __VA_ARGS__; }   \
    else { constexpr bool R_ = true, L_ = false; __VA_ARGS__; }       \
  } else {                                                           \
    if (RELU) { constexpr bool R_ = false, L_ = true; __VA_ARGS__; }  \
    else { constexpr bool R_ = false, L_ = false; __VA_ARGS__; }      \
  }

}  // namespace

void bn_stats(const uint16_t* x, int64_t M, int C, float* slots, hipStream_t s) {
  if (vec_ok(C)) {
    const int rpb = 256 / (C / 8);
    bn_stats_vec_kernel<<<grid_for(M, rpb * 8), 256, 0, s>>>(x, M, C, slots);
  } else {
    dim3 grid((C + 63) / 64, grid_for(M, 64));
    bn_stats_gen_kernel<<<grid, 256, 0, s>>>(x, M, C, slots);
  }
}

// ---- deterministic-reduction test mode
static bool g_det = false;
void set_det_mode(bool on) { g_det = on; }
bool det_mode() { return g_det; }

__global__ void __launch_bounds__(256) zero_f32_kernel(float* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0.f;
}

// The batch statistics of x into the zeroed-first slots with at most NSLOT blocks: block b owns slot b
// alone (one adder per address, onto zero: exact), its rows in a fixed grid-stride order and a fixed LDS
// tree -- the finalize's fixed-order slot sum then gives the same bits on every run.  The producing
// kernels' epilogue statistics (up to 32 adders per slot address, in arrival order) are discarded.
void bn_stats_det(const uint16_t* x, int64_t M, int C, float* slots, hipStream_t s) {
  zero_f32_kernel<<<64, 256, 0, s>>>(slots, (int64_t)NSLOT * 2 * C);
  if (vec_ok(C)) {
    const int rpb = 256 / (C / 8);
    bn_stats_vec_kernel<<<std::min(NSLOT, grid_for(M, rpb * 8)), 256, 0, s>>>(x, M, C, slots);
  } else {
    dim3 grid((C + 63) / 64, std::min(NSLOT, grid_for(M, 64)));
    bn_stats_gen_kernel<<<grid, 256, 0, s>>>(x, M, C, slots);
  }
}

void bn_finalize(float* slots, int64_t M, int C, const float* gamma, const float* beta, float eps, float momentum,
                 float* run_mean, float* run_var, float* save, hipStream_t s) {
  bn_finalize_kernel<<<(C + 15) / 16, 256, 0, s>>>(slots, M, C, gamma, beta, eps, momentum, run_mean, run_var,
                                                   save);
}

void bn_eval_prep(int C, const float* gamma, const float* beta, float eps, const float* run_mean,
                  const float* run_var, float* save, hipStream_t s) {
  bn_eval_prep_kernel<<<(C + 255) / 256, 256, 0, s>>>(C, gamma, beta, eps, run_mean, run_var, save);
}

void bn_apply(const uint16_t* x, const uint16_t* res, const float* save, int64_t M, int C, bool relu, uint16_t* y,
              uint8_t* mask, hipStream_t s) {
  const int64_t n = M * C;
  const bool has_res = res != nullptr;
  if (C % 8 == 0) {
    const int64_t nvec = n / 8;
    const int g = fixed_channel_grid(nvec, C);
    TFX_DISPATCH_RR(has_res, relu, (bn_apply_vec_kernel<R_, L_><<<g, 256, 0, s>>>(x, res, save, nvec, C, y, mask)));
  } else {
    const int g = grid_for(n, 256 * 4);
    TFX_DISPATCH_RR(has_res, relu, (bn_apply_gen_kernel<R_, L_><<<g, 256, 0, s>>>(x, res, save, n, C, y)));
  }
}

void bn_apply_res_bn(const uint16_t* x, const uint16_t* res_x, const float* save, const float* res_save, int64_t M,
                     int C, bool relu, uint16_t* y, uint8_t* mask, hipStream_t s) {
  const int64_t nvec = M * C / 8;
  const int g = fixed_channel_grid(nvec, C);
  if (relu)
    bn_apply_vec_kernel<true, true, true><<<g, 256, 0, s>>>(x, res_x, save, nvec, C, y, mask, res_save);
  else
    bn_apply_vec_kernel<true, false, true><<<g, 256, 0, s>>>(x, res_x, save, nvec, C, y, mask, res_save);
}

void bn_backward(const uint16_t* g, const uint16_t* x, const uint16_t* res, const uint8_t* mask, const float* save,
                 int64_t M, int C, bool relu, float* slots, float* red, float* dgamma, float* dbeta, uint16_t* dx,
                 uint16_t* dres, hipStream_t s) {
  const bool has_res = res != nullptr || mask != nullptr;
  const int64_t n = M * C;
  // the vector kernels take the residual ReLU mask from the forward's mask bits
  if (vec_ok(C) && (!has_res || !relu || mask)) {
    // one row per thread in flight (U = 1): 2 / 4 rows measured no faster (scripts/bn_bench.py)
    const int rpb = 256 / (C / 8);
    const int gr = grid_for(M, rpb * 8);
    TFX_DISPATCH_RR(has_res, relu,
                    (bn_bwd_reduce_vec_kernel<R_, L_, 1><<<gr, 256, 0, s>>>(g, x, mask, save, M, C, slots)));
  } else {
    dim3 grid((C + 63) / 64, grid_for(M, 64));
    TFX_DISPATCH_RR(has_res, relu,
                    (bn_bwd_reduce_gen_kernel<R_, L_><<<grid, 256, 0, s>>>(g, x, res, save, M, C, slots)));
  }
  bn_slot_reduce(slots, C, red, dgamma, dbeta, s);
  bn_backward_apply(g, x, res, mask, save, red, M, C, relu, dx, dres, s);
}

void bn_slot_reduce(float* slots, int C, float* red, float* dgamma, float* dbeta, hipStream_t s) {
  bn_slot_reduce_kernel<<<(C + 15) / 16, 256, 0, s>>>(slots, C, red, dgamma, dbeta);
}

void bn_bwd_reduce(const uint16_t* g, const uint16_t* x, const uint8_t* mask, bool has_res, const float* save,
                   int64_t M, int C, bool relu, float* slots, hipStream_t s) {
  const int rpb = 256 / (C / 8);
  const int gr = grid_for(M, rpb * 8);
  TFX_DISPATCH_RR(has_res, relu,
                  (bn_bwd_reduce_vec_kernel<R_, L_, 1><<<gr, 256, 0, s>>>(g, x, mask, save, M, C, slots)));
}

// bn_backward_apply (vector path, residual input, dres written) that also reduces the residual's
// own BN backward into slots2 (bn_bwd_apply_vec_kernel SEC); the caller finishes it with
// bn_slot_reduce(slots2, ...).  Fewer, fatter blocks than the plain apply: each ends in 2C atomics.
bool bn_backward_apply_sec_ok(int C) { return vec_ok(C); }

void bn_backward_apply_sec(const uint16_t* g, const uint16_t* x, const uint8_t* mask, const float* save,
                           const float* red, int64_t M, int C, bool relu, uint16_t* dx, uint16_t* dres,
                           const uint16_t* x2, const float* save2, float* slots2, hipStream_t s) {
  const int64_t nvec = M * C / 8;
  const int cv = C / 8;
  const int mult = cv / gcd(cv, 256);
  int ga = grid_for(nvec, 256 * 4, 1024);
  ga = (ga + mult - 1) / mult * mult;
  if (relu)
    bn_bwd_apply_vec_kernel<true, true, true><<<ga, 256, 0, s>>>(g, x, mask, save, red, nvec, M, C, dx, dres, x2,
                                                                 save2, slots2);
  else
    bn_bwd_apply_vec_kernel<true, false, true><<<ga, 256, 0, s>>>(g, x, mask, save, red, nvec, M, C, dx, dres,
                                                                  x2, save2, slots2);
}

// the apply half of bn_backward, for a red[] produced elsewhere (a conv dgrad epilogue)
void bn_backward_apply(const uint16_t* g, const uint16_t* x, const uint16_t* res, const uint8_t* mask,
                       const float* save, const float* red, int64_t M, int C, bool relu, uint16_t* dx,
                       uint16_t* dres, hipStream_t s) {
  const bool has_res = res != nullptr || mask != nullptr;
  const int64_t n = M * C;
  // with a residual input dres = g' is produced (the host guarantees dres != nullptr then)
  if (vec_ok(C) && (!has_res || !relu || mask)) {
    const int64_t nvec = n / 8;
    const int ga = fixed_channel_grid(nvec, C);
    TFX_DISPATCH_RR(has_res, relu, (bn_bwd_apply_vec_kernel<R_, L_><<<ga, 256, 0, s>>>(
                                       g, x, mask, save, red, nvec, M, C, dx, dres)));
  } else {
    const int ga = grid_for(n, 256 * 4);
    TFX_DISPATCH_RR(has_res, relu, (bn_bwd_apply_gen_kernel<R_, L_><<<ga, 256, 0, s>>>(
                                       g, x, res, save, red, n, M, C, dx, dres)));
  }
}

}  // namespace tfx
