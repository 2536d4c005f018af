// Fused optimizer updates over FLAT parameter buffers (multi-tensor apply without pointer
// lists: every trainable tensor of a model is a view into one contiguous f32 master buffer,
// its gradient a view into one contiguous grad buffer).  One launch updates the whole model
// and, optionally, refreshes the bf16 compute copy of the weights in the same pass.
//
// Learning rate and step counter live in device memory so a captured hipGraph replays with
// the current schedule value.  Optional global-norm clipping: g *= min(1, max_norm/||g||)
// with ||g||^2 produced on device by sumsq_flat (clip_by_global_norm for the char-LSTM).
// Reference semantics: tf.train.GradientDescentOptimizer -> ApplyGradientDescent
// (R/simple/simple.py:22, R/distributed/distributed.py:107); Momentum/Adam are the north-star
// "fused SGD/Adam" (BASELINE.json).
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

__device__ __forceinline__ float clip_factor(const float* sumsq, float max_norm) {
  if (!sumsq) return 1.f;
  const float nrm = sqrtf(*sumsq);
  return nrm > max_norm ? max_norm / nrm : 1.f;
}

template <typename TG>
__device__ __forceinline__ void load4(const TG* g, int64_t i, float* o);
template <>
__device__ __forceinline__ void load4<float>(const float* g, int64_t i, float* o) {
  float4 v = reinterpret_cast<const float4*>(g)[i];
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
__device__ __forceinline__ void load4<uint16_t>(const uint16_t* g, int64_t i, float* o) {
  uint2 v = reinterpret_cast<const uint2*>(g)[i];
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}

// kind: 0 = SGD, 1 = momentum (heavy ball, TF MomentumOptimizer form), 2 = Nesterov momentum,
//       3 = Adam (bias-corrected, L2 wd added to g), 4 = AdamW (decoupled wd)
template <typename TG, int KIND>
__global__ void __launch_bounds__(256) opt_kernel(float* __restrict__ p, const TG* g,
                                                  float* __restrict__ m, float* __restrict__ v, int64_t n4,
                                                  const float* __restrict__ lr_ptr, float gscale, float wd,
                                                  float b1, float b2, float eps, const float* __restrict__ step_ptr,
                                                  const float* __restrict__ sumsq, float max_norm,
                                                  uint16_t* __restrict__ pbf, const int* __restrict__ skip,
                                                  float* gz) {  // may alias g: no __restrict__ on either
  // gz (optional): the f32 gradient buffer, zeroed in the same pass (the next step's split-K weight
  // gradients accumulate into it with atomics) -- the step then needs no separate gradient fill.  It is
  // g itself on the f32 path; with the bf16 DP wire g is the reduced bf16 twin and gz its f32 source.
  // a nonzero skip word (e.g. the persistent LSTM's sticky health word: this step's gradients came
  // from a launch that gave up on a hand-off) leaves parameters, moments and the shadow untouched --
  // the gradients are still cleared (they are this step's, discarded)
  if (skip && *skip) {
    if (gz)
      for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
        reinterpret_cast<float4*>(gz)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const float lr = *lr_ptr;
  const float gs = gscale * clip_factor(sumsq, max_norm);
  float bc1 = 1.f, bc2 = 1.f;
  if (KIND >= 3) {
    const float t = *step_ptr;
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float pp[4] = {pv.x, pv.y, pv.z, pv.w};
    float gg[4];
    load4<TG>(g, i, gg);
    if (gz) reinterpret_cast<float4*>(gz)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (KIND == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) pp[k] -= lr * fmaf(gg[k], gs, wd * pp[k]);
    } else if (KIND == 1 || KIND == 2) {
      float4 mv = reinterpret_cast<float4*>(m)[i];
      float mm[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = fmaf(gg[k], gs, wd * pp[k]);
        mm[k] = fmaf(b1, mm[k], d);
        pp[k] -= lr * (KIND == 2 ? fmaf(b1, mm[k], d) : mm[k]);
      }
      reinterpret_cast<float4*>(m)[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    } else {
      float4 mv = reinterpret_cast<float4*>(m)[i];
      float4 vv = reinterpret_cast<float4*>(v)[i];
      float mm[4] = {mv.x, mv.y, mv.z, mv.w}, ww[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float d = gg[k] * gs;
        if (KIND == 3) d = fmaf(wd, pp[k], d);
        mm[k] = fmaf(b1, mm[k], (1.f - b1) * d);
        ww[k] = fmaf(b2, ww[k], (1.f - b2) * d * d);
        const float upd = (mm[k] / bc1) / (sqrtf(ww[k] / bc2) + eps);
        pp[k] -= lr * (KIND == 4 ? fmaf(wd, pp[k], upd) : upd);
      }
      reinterpret_cast<float4*>(m)[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
      reinterpret_cast<float4*>(v)[i] = make_float4(ww[0], ww[1], ww[2], ww[3]);
    }
    reinterpret_cast<float4*>(p)[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
    if (pbf) {
      uint2 o;
      o.x = pack_bf16x2(pp[0], pp[1]);
      o.y = pack_bf16x2(pp[2], pp[3]);
      reinterpret_cast<uint2*>(pbf)[i] = o;
    }
  }
}

template <typename TG>
__global__ void __launch_bounds__(256) sumsq_kernel(const TG* __restrict__ g, int64_t n4, float* __restrict__ out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float gg[4];
    load4<TG>(g, i, gg);
#pragma unroll
    for (int k = 0; k < 4; ++k) s = fmaf(gg[k], gg[k], s);
  }
  s = wave_sum(s);
  __shared__ float r[4];
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, r[0] + r[1] + r[2] + r[3]);
}

// f32 -> bf16 copy (weights refresh, DP bf16 gradient buckets) and bf16 -> f32
__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ x, int64_t n,
                                                            uint16_t* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = f32_to_bf16(x[i]);
}

// 8 elements per thread: two 16-B loads, one 16-B store (16-B aligned x and y, n8 = n / 8)
__global__ void __launch_bounds__(256) cast_f32_bf16_vec_kernel(const float4* __restrict__ x, int64_t n8,
                                                                U4* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const float4 a = x[2 * i], b = x[2 * i + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    y[i] = pack8(f);
  }
}

static inline int ogrid(int64_t n4) {
  int64_t g = (n4 + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

void optimizer_apply(int kind, float* p, const void* g, bool g_bf16, float* m, float* v, int64_t n,
                     const float* lr, float gscale, float wd, float b1, float b2, float eps, const float* step,
                     const float* sumsq, float max_norm, uint16_t* pbf, const int* skip, float* gz,
                     hipStream_t s) {
  const int64_t n4 = n / 4;  // host wrapper pads flat buffers to a multiple of 4 elements
  const int grid = ogrid(n4);
#define TFX_OPT(K)                                                                                     \
  if (g_bf16)                                                                                          \
    opt_kernel<uint16_t, K><<<grid, 256, 0, s>>>(p, (const uint16_t*)g, m, v, n4, lr, gscale, wd, b1, b2, \
                                                 eps, step, sumsq, max_norm, pbf, skip, gz);           \
  else                                                                                                 \
    opt_kernel<float, K><<<grid, 256, 0, s>>>(p, (const float*)g, m, v, n4, lr, gscale, wd, b1, b2, eps, \
                                              step, sumsq, max_norm, pbf, skip, gz);
  switch (kind) {
    case 0: TFX_OPT(0); break;
    case 1: TFX_OPT(1); break;
    case 2: TFX_OPT(2); break;
    case 3: TFX_OPT(3); break;
    default: TFX_OPT(4); break;
  }
#undef TFX_OPT
}

void sumsq_flat(const void* g, bool g_bf16, int64_t n, float* out, hipStream_t s) {
  TFX_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(float), s));
  const int64_t n4 = n / 4;
  const int grid = std::min(ogrid(n4), 1024);
  if (g_bf16)
    sumsq_kernel<uint16_t><<<grid, 256, 0, s>>>((const uint16_t*)g, n4, out);
  else
    sumsq_kernel<float><<<grid, 256, 0, s>>>((const float*)g, n4, out);
}

void cast_f32_bf16(const float* x, int64_t n, uint16_t* y, hipStream_t s) {
  if (n % 8 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0) {
    const int64_t n8 = n / 8;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n8 + 1023) / 1024, 4096));
    cast_f32_bf16_vec_kernel<<<grid, 256, 0, s>>>(reinterpret_cast<const float4*>(x), n8, reinterpret_cast<U4*>(y));
    return;
  }
  cast_f32_bf16_kernel<<<ogrid(n), 256, 0, s>>>(x, n, y);
}

}  // namespace tfx
