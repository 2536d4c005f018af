// Shared device helpers for the gfx950 (CDNA4) kernels of tensorflow_examples_amd.
// Wave = 64 lanes everywhere; bf16 is handled as raw 16-bit payloads and
// vectorised as 16-byte loads (8 x bf16) per lane (cdna_hip_programming.md G13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TFX_WAVE 64

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8_t __attribute__((ext_vector_type(8)));

struct alignas(16) U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even; a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 and keeps NaNs.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}
__device__ __forceinline__ void unpack8(const U4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ U4 pack8(const float* f) {
  U4 r;
  r.x = pack_bf16x2(f[0], f[1]);
  r.y = pack_bf16x2(f[2], f[3]);
  r.z = pack_bf16x2(f[4], f[5]);
  r.w = pack_bf16x2(f[6], f[7]);
  return r;
}

// Sum over each 16-lane DPP row (lanes 16k..16k+15), result in every lane of the row: 4 VALU
// adds with DPP source modifiers (quad_perm xor 1, xor 2, row_half_mirror, row_mirror) instead of
// ds_bpermute round trips through the LDS crossbar.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5, T1):
// blocks b and b+8 share an XCD's L2 under round-robin dispatch, so hand each XCD a
// contiguous run of logical tiles.  Pure speed: correctness never depends on placement.
// p[i], or 0 for a null p, as a buffer load whose resource has no records when p is null: no branch
// around the load (a branch -- even on a uniform condition -- makes the waitcnt pass drain the load
// counter at its join, serialising the loads behind it)
__device__ __forceinline__ float ld_f32_or0(const float* p, int i) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, p ? 0x7fffffff : 0, 0x00020000);
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)i * 4u, 0, 0));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx) return bid;
  const int q = nwg / nx, r = nwg % nx, xcd = bid % nx, idx = bid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

#define TFX_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, \
              __LINE__);                                                           \
      abort();                                                                     \
    }                                                                              \
  } while (0)
