// Shared pieces of the persistent pointwise-conv kernels (pw_bwd.hip, pw_fwd.hip): 512-thread
// blocks over 32-row m-tiles, LDS image layouts and fragment reads (kernel-private: anonymous namespace).
#pragma once
#include "tfx_common.h"
#include "tfx_kernels.h"

#include <type_traits>
#include <utility>

namespace tfx {
namespace {

constexpr int PW_NT = 512;   // threads per block
constexpr int PW_BM = 32;    // rows (pixels) per m-tile

typedef short pw_s4 __attribute__((ext_vector_type(4)));
typedef short pw_s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) pw_s4 pw_lds_s4;
typedef __attribute__((address_space(3))) char pw_lds_char;
typedef __attribute__((address_space(3))) bf16x8_t pw_lds_bf16x8;
typedef unsigned int pw_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int pw_u32x2 __attribute__((ext_vector_type(2)));

// K-major image of 64-channel rows (128 B): 16-B chunk c of row r at r*128 + ((c ^ (r&7)) << 4)
__device__ __forceinline__ int pw_kmaj(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }
// MN-major image of COLS-element rows (as igemm_impl.h mn_off): XOR swizzle per row length
template <int COLS>
__device__ __forceinline__ int pw_mn(int r, int c) {
  int swz;
  if constexpr (COLS >= 128) swz = ((r & 3) << 2) | ((r >> 2) & 3);
  else swz = (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;
  return r * (COLS * 2) + ((c ^ swz) << 4);
}

// A fragment (16 rows x 32 k) of a K-major image: lane holds row rb + (l&15), k = 8(l>>4) + j
__device__ __forceinline__ bf16x8_t pw_frag_kmaj(const char* img, int off, int rb, int kc, int lane) {
  return *(const pw_lds_bf16x8*)((pw_lds_char*)img + off + pw_kmaj(rb + (lane & 15), kc + (lane >> 4)));
}
// Transposed fragment of a row-major image: lane holds X[col = cb + (l&15)][k = 8(l>>4) + j], where the
// image rows are k and its columns the fragment's M (or N) index; OFF(r, c16) = byte offset of 16-B
// chunk c16 of row r (ds_read_b64_tr_b16, cdna_hip_programming.md T10)
template <typename OFF>
__device__ __forceinline__ bf16x8_t pw_frag_tr(const char* img, int off, int cb, int lane, OFF offf) {
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, p = ii & 3;
  const int chunk = (cb >> 3) + (p >> 1);
  pw_s4 v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kr = 8 * g + 4 * h + q;
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_s4*)((pw_lds_char*)img + off + offf(kr, chunk) + (p & 1) * 8));
  }
  pw_s8 r = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pw_rsrc(const void* p, int64_t bytes) {
  const int n = bytes > 0x7fffffff ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, n, 0x00020000);
}

// Copy N16 16-byte pieces global -> LDS (a block's resident weight image) with every load in flight
// before the first LDS store.  The plain `for (q = t; q < N16; q += PW_NT)` loop waits for each piece's
// load before its store: one memory round trip per iteration, 4-16 of them before the main loop.
// src(q) / dst(q): the piece's global source / LDS destination.  Pieces past N16 re-copy the last one
// (identical duplicate writes: no branch around the loads).
template <int N16, typename DST, typename SRC>
__device__ __forceinline__ void pw_resident_copy(int t, DST dst, SRC src) {
  constexpr int NPT = (N16 + PW_NT - 1) / PW_NT;
  pw_u32x4 v[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) v[i] = *src(min(t + PW_NT * i, N16 - 1));
#pragma unroll
  for (int i = 0; i < NPT; ++i) *dst(min(t + PW_NT * i, N16 - 1)) = v[i];
}

template <int... I, typename F>
__device__ __forceinline__ void pw_sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void pw_sfor(F&& f) {
  pw_sfor_impl(f, std::make_integer_sequence<int, N>{});
}

}  // namespace
}  // namespace tfx
