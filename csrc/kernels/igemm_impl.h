// Implicit-GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16) for gfx950 -- kernel template and host
// launch helpers, included by the per-mode translation units igemm_*.hip (compiled in parallel).
//
// One template covers every matmul-shaped op of the framework.  An operand is described by its
// KIND (how its tile is gathered from global memory) and is staged either K-major or MN-major:
//   K-major kinds  (LDS image [rows][64 k], fragments by ds_read_b128):
//     KM_DENSE     A[m*ld + k]
//     KM_FWD_X     im2col(X) of an NHWC conv forward, gathered on the fly
//     KM_FWD_XT    the same when C % 64 == 0 (every 64-deep k-tile inside one filter tap): the tap /
//                  channel decode is uniform per k-tile (scalar), a row's padding test one bit of a
//                  per-row tap-validity mask built at the block's start
//     KM_DGRAD_DY  gather of dY for the conv data-gradient (stride via parity test)
//   MN-major kinds (LDS image [64 k][cols], fragments by ds_read_b64_tr_b16, no transpose pass):
//     MN_DENSE     A[k*ld + m]                (also dY^T for the weight gradient)
//     MN_DGRAD_W   W[ko][r][s][c] read as B(k=(r,s,ko), n=c)
//     MN_WGRAD_X   im2col(X) rows j=(n,p,q), columns (r,s,c)
//     MN_WGRAD_XT  the same when a 64-pixel k-tile is whole output rows of one image or whole images
//                  (P*Q % 64 == 0 and 64 % Q == 0, or 64 % (P*Q) == 0): each k-row's (p, q) offset
//                  inside the tile is a per-thread constant, so per k-tile only the tile's (n0, p0) --
//                  scalar -- and one bound test per piece remain
// Ops: conv FWD = <KM_FWD_X, KM_DENSE>, DGRAD = <KM_DGRAD_DY, MN_DGRAD_W>,
//      WGRAD = <MN_DENSE(dY), MN_WGRAD_X> or transposed <MN_WGRAD_X, MN_DENSE(dY)> (+trans_out),
//      GEMM = any K/MN-major dense pair.
//
// Block = 256 threads = 4 waves (2x2), tile BM x BN x 64 with (BM,BN) in {128x128, 256x64, 128x64}.
// Loads are UNCONDITIONAL buffer_load_dwordx4 through a buffer resource: padding / out-of-range
// elements get an offset past num_records and the hardware returns zeros, so hipcc never branches
// around a load and can count vmcnt statically (cdna_hip_programming.md §5 item 4(c)).
// Pipeline: two register stage sets (tiles t+1, t+2 in flight) feeding two LDS stages, one
// barrier per k-tile; each load has ~2 tiles of MFMA work to land.
// LDS swizzles: K-major 128-B rows chunk c ^ (r&7) (conflict-free ds_read_b128, T2); MN-major rows
// XOR-swizzled so the transposed reads of a 32-lane half hit 8 distinct 32-B slots (T10).
// blockIdx is remapped XCD-aware (T1).  Reference: the matmuls of R/distributed/distributed.py:96-98
// and their TF1 gradients; conv/FC layers of the north-star models (BASELINE.json configs 2-5).
#pragma once
#include "tfx_common.h"
#include "tfx_kernels.h"
#include "igemm_entry.h"

#include <cstdio>
#include <utility>
#include <cstdlib>

namespace tfx {

namespace {

enum { KM_DENSE = 0, KM_FWD_X = 1, KM_DGRAD_DY = 2, KM_FWD_XT = 3, MN_DENSE = 10, MN_DGRAD_W = 11,
       MN_WGRAD_X = 12, MN_DGRAD_W2 = 13, MN_WGRAD_XT = 14 };
enum { EPI_PLAIN = 0, EPI_STATS = 1, EPI_BNB = 2 };
constexpr uint32_t BAD = 0x80000000u;  // byte offset beyond any num_records -> loads return 0
constexpr int NT = 256, BKT = 64;

typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4_t lds_s4;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr bool is_kmaj(int kind) { return kind < 10; }

__device__ __forceinline__ int kmaj_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }
// MN-major image, rows of `COLS` bf16; swizzle chosen per row length (see header)
template <int COLS>
__device__ __forceinline__ int mn_swz(int r) {
  if constexpr (COLS >= 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;
}
template <int COLS>
__device__ __forceinline__ int mn_off(int r, int c) {
  return r * (COLS * 2) + ((c ^ mn_swz<COLS>(r)) << 4);
}

// Fragment reads address LDS as (array base, integer byte offset) with ONE pointer step: LDS
// lowering attaches the array's alias scope only to accesses within a few GEPs of the array, and a
// read without a scope makes the waitcnt pass wait for every LDS-DMA in flight (vmcnt(0)).
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) bf16x8_t lds_bf16x8;
__device__ __forceinline__ bf16x8_t lds_read_kmaj(const char* img, int img_off, int row, int chunk) {
  return *(const lds_bf16x8*)((lds_char*)img + (img_off + kmaj_off(row, chunk)));
}

// fragment of an MN-major image: lane needs X[col = cb + (l&15)][k = 32kk + 8(l>>4) + j], j = 0..7
template <int COLS>
__device__ __forceinline__ bf16x8_t lds_read_mn(const char* img, int img_off, int cb, int kk, int lane) {
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, p = ii & 3;
  const int chunk = (cb >> 3) + (p >> 1);
  s4_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kr = 32 * kk + 8 * g + 4 * h + q;
    const int off = img_off + mn_off<COLS>(kr, chunk) + (p & 1) * 8;
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)((lds_char*)img + off));
  }
  s8_t r = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

// ------------------------------------------------------------------ operand loaders
// ROWS = tile extent of this operand (BM for A, BN for B).  K-major: thread covers chunk t&7 of rows
// (t>>3) + 32*i.  MN-major: thread covers ONE k-row, t>>2, and chunks (t&3) + 4*j of it -- the k
// decode (pixel n,p,q for the weight gradient, (r,s,ko) for the data gradient's weights) is done once
// per k-tile, not once per load; the 4-apart chunks keep the swizzled ds_write_b128 conflict-free.
// Address math is split into a per-row part precomputed once (init) and a per-k-tile part shared by
// all of a thread's rows, with 24-bit multiplies (v_mul_u32_u24, full rate; the host guarantees
// pixel counts < 2^24) instead of quarter-rate 32-bit ones: the K loop's VALU issue competes with
// the MFMAs for the SIMD (MI355X_MICROARCH.md 'vector-instruction ISSUE cost').
// zero the bf16 halves of an 8 x bf16 vector whose bit in `bits` (element k = bit k) is clear:
// each 32-bit word gets a mask from two sign-extended 1-bit fields (v_bfe_i32), no selects
__device__ __forceinline__ U4 mask_bf16x8(const U4& v, uint32_t bits) {
  auto wmask = [&](int s) -> uint32_t {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)bits, s, 1) & 0xffffu;
    const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)bits, s + 1, 1) << 16;
    return lo | hi;
  };
  U4 r;
  r.x = v.x & wmask(0);
  r.y = v.y & wmask(2);
  r.z = v.z & wmask(4);
  r.w = v.w & wmask(6);
  return r;
}

__device__ __forceinline__ int mul24(int a, int b) { return (int)__umul24((unsigned)a, (unsigned)b); }

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt fields left at their maxima): the counted wait of the
// LDS-DMA ring, which lets N LDS-DMA pieces stay in flight across the next barrier.
template <int V>
struct IC {
  static constexpr int value = V;
};

template <int... I, typename F>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(IC<I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// GL (LDS-DMA staging, buffer_load ... lds): every 16-B piece goes straight from global memory to
// LDS, and one wave-instruction writes 64 x 16 B = 1 KB CONTIGUOUSLY (lane-linear destination,
// cdna_hip_programming.md §5 Caveat).  The LDS images keep their XOR swizzles by permuting the
// SOURCE instead (rule 21): the lane that lands at chunk position p of row r loads logical chunk
// p ^ swz(r).  K-major: a wave-instruction covers 8 full 128-B rows, so only the chunk index
// changes (c0).  MN-major: a wave-instruction covers 1 KB / (2 ROWS) k-rows with every lane on a
// FIXED chunk position; the k-row (and, through the swizzle, the logical column chunk) changes per
// instruction, so the per-chunk column decode is precomputed per instruction at init and the k
// decode runs once per instruction and k-tile.
template <int KIND, int ROWS, bool GL = false>
struct Loader {
  static constexpr bool KM = is_kmaj(KIND);
  static constexpr int NP = ROWS / 32;          // 16-B loads per thread per tile
  static constexpr int CH = ROWS / 8;           // MN-major chunks per k-row
  static constexpr int RPI = 512 / ROWS;        // GL MN-major: k-rows per wave-instruction
  static_assert(KM || CH == 4 * NP, "MN-major: 4 threads per k-row");
  int c0;        // K-major: element offset of chunk in k (8*kc)
  int r0;        // K-major: first row; MN-major: the k-row
  int ctx0[NP], ctx1[NP], ctx2[NP], base[NP];
  int col[NP];                     // MN-major: column of chunk j (-1: out of range)
  int cr[NP], cs[NP], cc[NP];      // MN_WGRAD_X column decode per chunk
  int rk[NP];                      // GL MN-major: k-row of instruction j
  int t3_;                         // MN-major: first chunk (t & 3) of the k-row

  __device__ __forceinline__ void init(const IgemmArgs& a, int base0, int lim, int ld, int t) {
    if constexpr (KM) {
      // GL: the lane at chunk position t&7 of row r (r&7 == (t>>3)&7) loads chunk (t&7) ^ (r&7)
      c0 = GL ? 8 * ((t & 7) ^ ((t >> 3) & 7)) : 8 * (t & 7);
      r0 = t >> 3;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int row = base0 + r0 + 32 * i;
        const bool ok = row < lim;
        if constexpr (KIND == KM_DENSE) {
          ctx0[i] = ok ? 0 : -1;
          base[i] = row * ld;
        } else {
          constexpr bool IM2COL = KIND == KM_FWD_X || KIND == KM_FWD_XT;
          const int GY = IM2COL ? a.P : a.H, GX = IM2COL ? a.Q : a.W;
          int n = row / (GY * GX), yx = row - n * GY * GX, y = yx / GX, x = yx - y * GX;
          // rows past M get a y far out of range: every bounds test below then fails (no flag register)
          constexpr int FAR = -(1 << 28);
          if constexpr (IM2COL) {
            ctx1[i] = ok ? y * a.sh - a.ph : FAR;
            ctx2[i] = x * a.sw - a.pw;
            // element offset of (n, iy0, ix0, 0): may be negative (padding), only used when in range
            base[i] = ((n * a.H + y * a.sh - a.ph) * a.W + ctx2[i]) * a.C;
            if constexpr (KIND == KM_FWD_XT) {
              // bit (r*S + s) = tap (r, s) of this row is inside the image (rows past M: none)
              uint32_t vm = 0;
              for (int r = 0; r < a.R; ++r) {
                const bool yin = (unsigned)(ctx1[i] + r * a.dh) < (unsigned)a.H;
                for (int s2 = 0; s2 < a.S; ++s2) {
                  const bool xin = (unsigned)(ctx2[i] + s2 * a.dw) < (unsigned)a.W;
                  vm |= (yin && xin ? 1u : 0u) << (r * a.S + s2);
                }
              }
              ctx0[i] = (int)vm;
              base[i] += c0;  // the thread's channel chunk is fixed: fold it into the row base
              // opaque from here: hipcc otherwise re-derives base + dk per k-tile as
              // ((nH + iy) W + ix) C -- two quarter-rate v_mul_lo_u32 per piece
              asm volatile("" : "+v"(base[i]), "+v"(ctx0[i]));
            }
          } else {
            ctx1[i] = ok ? y + a.ph : FAR;
            ctx2[i] = x + a.pw;
            base[i] = n * a.P;
          }
        }
      }
    } else if constexpr (GL) {
      const int w = t >> 6, l = t & 63;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int r = RPI * (w * NP + j) + l / CH;           // k-row of this lane in instruction j
        rk[j] = r;
        const int cj = base0 + 8 * ((l % CH) ^ mn_swz<ROWS>(r));
        col[j] = cj < lim ? cj : -1;
        if constexpr (KIND == MN_DENSE) base[j] = r * ld + cj;
        if constexpr (KIND == MN_WGRAD_X || KIND == MN_WGRAD_XT) {
          const int rs = cj < lim ? cj / a.C : 0;
          cc[j] = cj - rs * a.C;
          cr[j] = rs / a.S;
          cs[j] = rs - cr[j] * a.S;
        }
        if constexpr (KIND == MN_WGRAD_XT) xt_init(a, j, r, cj < lim);
      }
    } else {
      r0 = t >> 2;
      t3_ = t & 3;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int cj = base0 + 8 * ((t & 3) + 4 * j);
        col[j] = cj < lim ? cj : -1;
        if constexpr (KIND == MN_DENSE) base[j] = r0 * ld + cj;
        if constexpr (KIND == MN_WGRAD_X || KIND == MN_WGRAD_XT) {
          const int rs = cj < lim ? cj / a.C : 0;
          cc[j] = cj - rs * a.C;
          cr[j] = rs / a.S;
          cs[j] = rs - cr[j] * a.S;
        }
        if constexpr (KIND == MN_WGRAD_XT) {
          rk[j] = r0;
          xt_init(a, j, r0, cj < lim);
        }
      }
    }
  }

  // MN_WGRAD_XT: k-row r of a tile = pixel k0 + r with k0 % 64 == 0; under the kind's condition its
  // image is n0 + r / PQ and its (p, q) = (p0 + (r % PQ) / Q, (r % PQ) % Q), with (n0, p0) uniform per
  // k-tile.  base[j] = the element offset of (r / PQ, iy - p0 sh, ix, c) relative to image n0;
  // cr[j] = that row's iy without the tile's p0 sh (FAR when the column or ix is out of range).
  __device__ __forceinline__ void xt_init(const IgemmArgs& a, int j, int r, bool colok) {
    const int PQ = a.P * a.Q;
    const int nr = r / PQ, pq = r - nr * PQ, p = pq / a.Q, q = pq - p * a.Q;
    const int iyc = p * a.sh - a.ph + cr[j] * a.dh, ix = q * a.sw - a.pw + cs[j] * a.dw;
    const bool ok = colok && (unsigned)ix < (unsigned)a.W;
    base[j] = ((nr * a.H + iyc) * a.W + ix) * a.C + cc[j];
    cr[j] = ok ? iyc : -(1 << 28);
    asm volatile("" : "+v"(base[j]), "+v"(cr[j]));  // keep them as values (no re-derivation per k-tile)
  }

  // byte offsets of this thread's NP 16-B pieces of k-tile k0 (BAD = zero fill)
  // All predicates are combined with bitwise & and resolved by a select: no branches in the
  // load path, so hipcc can count vmcnt statically.  kend = end of this block's K range.
  __device__ __forceinline__ void offsets(const IgemmArgs& a, int ld, int k0, int kend, uint32_t* off) const {
    if constexpr (KM) {
      const int k = k0 + c0;
      const bool kok = k < kend;
      if constexpr (KIND == KM_DENSE) {
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const uint32_t o = (uint32_t)(base[i] + k) * 2u;
          off[i] = (kok & (ctx0[i] >= 0)) ? o : BAD;
        }
      } else if constexpr (KIND == KM_FWD_XT) {
        // one tap per k-tile (C % 64 == 0): tap, channel base and the tap's element offset are uniform --
        // scalar math on k0; per piece a mask bit and one add (K % 64 == 0: the k bound is uniform too)
        const int tap = a.fd_C.div(k0), cb = k0 - tap * a.C, r = a.fd_S.div(tap), s = tap - r * a.S;
        const int dk = ((r * a.dh) * a.W + s * a.dw) * a.C + cb;
        const bool kok0 = k0 < kend;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const bool ok = kok0 & (((uint32_t)ctx0[i] >> tap) & 1u);
          off[i] = ok ? (uint32_t)(base[i] + dk) * 2u : BAD;
        }
      } else if constexpr (KIND == KM_FWD_X) {
        const int rs = a.fd_C.div(k), c = k - mul24(rs, a.C), r = a.fd_S.div(rs), s = rs - mul24(r, a.S);
        const int rdh = mul24(r, a.dh), sdw = mul24(s, a.dw);
        const int dk = mul24(mul24(rdh, a.W) + sdw, a.C) + c;  // (r*dh*W + s*dw)*C + c
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int iy = ctx1[i] + rdh, ix = ctx2[i] + sdw;
          const bool ok = kok & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W);
          const uint32_t o = (uint32_t)(base[i] + dk) * 2u;
          off[i] = ok ? o : BAD;
        }
      } else {  // KM_DGRAD_DY: k = (r, s, ko)
        const int rs = a.fd_Ko.div(k), ko = k - mul24(rs, a.Ko), r = a.fd_S.div(rs), s = rs - mul24(r, a.S);
        const int rdh = mul24(r, a.dh), sdw = mul24(s, a.dw);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int ty = ctx1[i] - rdh, tx = ctx2[i] - sdw;
          const int p = ty >> a.sh_log2, q = tx >> a.sw_log2;
          const bool ok = kok & (ty >= 0) & (tx >= 0) & ((p << a.sh_log2) == ty) &
                          ((q << a.sw_log2) == tx) & (p < a.P) & (q < a.Q);
          const uint32_t o = (uint32_t)(mul24(mul24(base[i] + p, a.Q) + q, a.Ko) + ko) * 2u;
          off[i] = ok ? o : BAD;
        }
      }
    } else if constexpr (GL) {
      // one k-row per instruction: decoded once per instruction and k-tile
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int k = k0 + rk[j];
        const bool ok = (k < kend) & (col[j] >= 0);
        if constexpr (KIND == MN_DENSE) {
          off[j] = ok ? (uint32_t)(k0 * ld + base[j]) * 2u : BAD;
        } else if constexpr (KIND == MN_DGRAD_W) {
          const int rs = a.fd_Ko.div(k), ko = k - mul24(rs, a.Ko);
          const int e0 = mul24(ko, a.R * a.S * a.C) + mul24(rs, a.C);
          off[j] = ok ? (uint32_t)(e0 + col[j]) * 2u : BAD;
        } else if constexpr (KIND == MN_DGRAD_W2) {
          const int rs = a.fd_Ko.div(k), ko = k - mul24(rs, a.Ko);
          const int ri = a.fd_S.div(rs), si = rs - mul24(ri, a.S);
          const int tap = mul24(a.cr0 + 2 * ri, a.wS) + a.cs0 + 2 * si;
          const int e0 = mul24(ko, a.wR * a.wS * a.C) + mul24(tap, a.C);
          off[j] = ok ? (uint32_t)(e0 + col[j]) * 2u : BAD;
        } else if constexpr (KIND == MN_WGRAD_XT) {
          const int n0 = a.fd_PQ.div(k0), p0 = a.fd_Q.div(k0 - n0 * a.P * a.Q);  // uniform
          const int dys = p0 * a.sh, U = (n0 * a.H + dys) * a.W * a.C;
          const int iy = cr[j] + dys;
          const bool in = (k < kend) & ((unsigned)iy < (unsigned)a.H);
          off[j] = in ? (uint32_t)(base[j] + U) * 2u : BAD;
        } else {  // MN_WGRAD_X
          const int PQ = a.P * a.Q;
          const int n = a.fd_PQ.div(k), pq = k - mul24(n, PQ), p = a.fd_Q.div(pq), q = pq - mul24(p, a.Q);
          const int iy = mul24(p, a.sh) - a.ph + mul24(cr[j], a.dh), ix = mul24(q, a.sw) - a.pw + mul24(cs[j], a.dw);
          const bool in = ok & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W);
          const int e = mul24(mul24(mul24(n, a.H) + iy, a.W) + ix, a.C) + cc[j];
          off[j] = in ? (uint32_t)e * 2u : BAD;
        }
      }
    } else {
      const int k = k0 + r0;  // this thread's k-row: decoded once per k-tile
      const bool kok = k < kend;
      if constexpr (KIND == MN_DENSE) {
        const int k0ld = k0 * ld;
#pragma unroll
        for (int j = 0; j < NP; ++j) off[j] = (kok & (col[j] >= 0)) ? (uint32_t)(k0ld + base[j]) * 2u : BAD;
      } else if constexpr (KIND == MN_DGRAD_W) {
        const int rs = a.fd_Ko.div(k), ko = k - mul24(rs, a.Ko);
        const int e0 = mul24(ko, a.R * a.S * a.C) + mul24(rs, a.C);  // ((ko*R + r)*S + s)*C
#pragma unroll
        for (int j = 0; j < NP; ++j) off[j] = (kok & (col[j] >= 0)) ? (uint32_t)(e0 + col[j]) * 2u : BAD;
      } else if constexpr (KIND == MN_DGRAD_W2) {
        // parity-class taps: k = (ri, si, ko) -> full-filter tap (cr0 + 2 ri, cs0 + 2 si)
        const int rs = a.fd_Ko.div(k), ko = k - mul24(rs, a.Ko);
        const int ri = a.fd_S.div(rs), si = rs - mul24(ri, a.S);
        const int tap = mul24(a.cr0 + 2 * ri, a.wS) + a.cs0 + 2 * si;
        const int e0 = mul24(ko, a.wR * a.wS * a.C) + mul24(tap, a.C);
#pragma unroll
        for (int j = 0; j < NP; ++j) off[j] = (kok & (col[j] >= 0)) ? (uint32_t)(e0 + col[j]) * 2u : BAD;
      } else if constexpr (KIND == MN_WGRAD_XT) {
        const int n0 = a.fd_PQ.div(k0), p0 = a.fd_Q.div(k0 - n0 * a.P * a.Q);  // uniform
        const int dys = p0 * a.sh, U = (n0 * a.H + dys) * a.W * a.C;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const int iy = cr[j] + dys;
          const bool in = kok & ((unsigned)iy < (unsigned)a.H);
          off[j] = in ? (uint32_t)(base[j] + U) * 2u : BAD;
        }
      } else {  // MN_WGRAD_X: pixel (n, p, q) of k, then per chunk its (r, s, c) tap
        const int PQ = a.P * a.Q;
        const int n = a.fd_PQ.div(k), pq = k - mul24(n, PQ), p = a.fd_Q.div(pq), q = pq - mul24(p, a.Q);
        const int iy0 = mul24(p, a.sh) - a.ph, ix0 = mul24(q, a.sw) - a.pw, nH = mul24(n, a.H);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const int iy = iy0 + mul24(cr[j], a.dh), ix = ix0 + mul24(cs[j], a.dw);
          const bool ok = kok & (col[j] >= 0) & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W);
          const int e = mul24(mul24(nH + iy, a.W) + ix, a.C) + cc[j];
          off[j] = ok ? (uint32_t)e * 2u : BAD;
        }
      }
    }
  }

  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rsrc, const uint32_t* off, u32x4_t* r) const {
#pragma unroll
    for (int i = 0; i < NP; ++i) r[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off[i], 0, 0);
  }

  // GL: NP LDS-DMA wave-instructions into the operand image at `img` (wave-uniform destinations:
  // K-major rows 8w + 32i, MN-major 1-KB block w*NP + i).  Out-of-range pieces (BAD) land as zeros.
  __device__ __forceinline__ void load_lds(__amdgpu_buffer_rsrc_t rsrc, const uint32_t* off, char* img, int img_off,
                                           int w) const {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int dst = img_off + (KM ? (8 * w + 32 * i) * 128 : (w * NP + i) * 1024);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)((lds_char*)img + dst),
                                               16, off[i], 0, 0, 0);
    }
  }

  __device__ __forceinline__ void store(char* img, const u32x4_t* r) const {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      int o;
      if constexpr (KM) o = kmaj_off(r0 + 32 * i, c0 >> 3);
      else o = mn_off<ROWS>(r0, (t3_ + 4 * i));
      *reinterpret_cast<u32x4_t*>(img + o) = r[i];
    }
  }
};

template <int KIND, int ROWS>
__device__ __forceinline__ bf16x8_t frag(const char* img, int img_off, int rowbase, int kk, int lane) {
  if constexpr (is_kmaj(KIND)) return lds_read_kmaj(img, img_off, rowbase + (lane & 15), 4 * kk + (lane >> 4));
  else return lds_read_mn<ROWS>(img, img_off, rowbase, kk, lane);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
  const int n = bytes > 0x7fffffff ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, n, 0x00020000);
}

// (the anonymous namespace continues: kernels get internal linkage per translation unit)

// SWAP: compute the transposed tile (MFMA operands exchanged) so each lane holds 4 CONSECUTIVE
// output columns of one row: bf16 outputs leave as one 8-byte store per 16x16 tile per lane, and
// transposed f32 outputs (dW^T) as 16-lane contiguous runs.  Plain f32 atomics keep SWAP=false
// (4 rows x 16 contiguous columns per instruction).
// STG = LDS stages: 2 for the pipelined K loop; 1 for single-k-tile GEMMs (K <= 64: the 1x1 convs
// of 64-channel layers), which then fit 4 blocks per CU -- those are memory-bound, and occupancy is
// what keeps enough loads and stores in flight.
// EPI: compile-time epilogue extras (so the plain GEMM / wgrad kernels carry none of their code or
// registers): EPI_STATS = fused BN statistics of a conv forward.
//
// sr_block: bn_slot_reduce_kernel's math for channels [16 sb, 16 sb + 16) of the sr_* layer, 256 threads:
// 16 slot-lanes x 4 slots each per channel, all loads in flight before the re-zeroing stores, then an
// LDS reduction over the 16 slot-lanes.  dbeta / dgamma are loaded before the slot round trip.
__device__ __forceinline__ void sr_block(float* __restrict__ slots, float* __restrict__ red, float* __restrict__ dgamma,
                                         float* __restrict__ dbeta, int C, int sb, float* red2) {
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = sb * 16 + tx;
  const bool own = ty == 0 && c < C;
  // every load unconditional (clamped channel; null dgamma / dbeta through record-less resources): a
  // branch around a load makes the waitcnt pass drain the load counter at its join -- two round trips
  const int cc = min(c, C - 1);
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(dgamma, dgamma ? 0x7fffffff : 0);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(dbeta, dbeta ? 0x7fffffff : 0);
  const float db = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, (uint32_t)cc * 4u, 0, 0));
  const float dg = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, (uint32_t)cc * 4u, 0, 0));
  float s = 0.f, q = 0.f;
  float vs[NSLOT / 16], vq[NSLOT / 16];
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
  red2[threadIdx.x] = s;
  red2[256 + threadIdx.x] = q;
  if (c < C) {
#pragma unroll
    for (int i = 0; i < NSLOT / 16; ++i) {
      float* p = slots + (size_t)(ty + 16 * i) * 2 * C;
      p[c] = 0.f;  // the workspace is zero again for its next use
      p[C + c] = 0.f;
    }
  }
  // LDS-only barrier (a fence would wait for the zeroing stores); the waves still running: threads
  // >= 256 of an 8-wave block have exited
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (own) {
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      s += red2[threadIdx.x + 16 * k];
      q += red2[256 + threadIdx.x + 16 * k];
    }
    red[c] = s;
    red[C + c] = q;
    if (dbeta) dbeta[c] = db + s;
    if (dgamma) dgamma[c] = dg + q;
  }
}

// EPI_BNB = fused BN-backward partials of a conv data gradient.
// KS = 2: in-block split-K for the f32-atomic weight gradients.  512 threads = two 4-wave groups
// on the SAME output tile, each running the pipelined K loop over half of the block's k-tiles in its
// own LDS stages; group 1 hands its accumulators to group 0 through LDS and only group 0 issues the
// atomics.  Twice the loads in flight per CU (these GEMMs are latency-bound at one 4-wave block per
// CU) for the SAME atomic bytes -- splitting across blocks instead doubles the f32 atomic traffic,
// which runs at ~1.3 TB/s chip-wide (MI355X_MICROARCH.md "Global float atomics").
// GLS = LDS-DMA ring depth (0: the register-staged pipeline above; 1: single k-tile; >= 2: GLS LDS
// stages, GLS - 1 k-tiles in flight).  The ring: prologue issues tiles 0 .. GLS-2; iteration it waits
// vmcnt((GLS-2) tiles' pieces) -- its own pieces of tile it have landed, later tiles stay in flight --
// then ONE raw s_barrier (every wave's pieces of tile it are in LDS, and every wave has finished
// reading the stage of tile it-1), issues tile it+GLS-1 into that freed stage, and computes tile it.
// No __syncthreads() in the loop: its fence would drain vmcnt(0) (§5 'Pipelining across barriers').
constexpr int gl_waves(int BM, int BN, int KS, int GLS) {
  const int stage = (BM + BN) * BKT * 2 * KS * (GLS > 1 ? GLS : 1);
  int blocks = 163840 / stage;
  blocks = blocks < 1 ? 1 : (blocks > 4 ? 4 : blocks);
  return blocks * KS;  // waves per SIMD
}
constexpr int igemm_waves(int BM, int BN, int STG, int EPI, int KS, int GLS) {
  return GLS > 0 ? gl_waves(BM, BN, KS, GLS)
                 : (KS == 2 ? 1 : ((STG == 1 && EPI != EPI_BNB) ? (BM * BN >= 128 * 128 ? 3 : 4) : 2));
}

template <int AKIND, int BKIND, int BM, int BN, bool SWAP, int STG, int EPI, int KS = 1, int GLS = 0>
__global__ void __launch_bounds__(256 * KS, igemm_waves(BM, BN, STG, EPI, KS, GLS)) igemm_kernel(IgemmArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * BKT * 2, STAGE = (BM + BN) * BKT * 2;
  constexpr bool GL = GLS > 0;
  constexpr int NSTG = GL ? GLS : STG;  // LDS stages per 4-wave group
  static_assert(KS == 1 || (KS == 2 && (STG == 2 || GLS >= 2)), "in-block split-K: pipelined kernels");
  static_assert(KS == 1 || TM * TN * 4096 <= NSTG * STAGE, "accumulator hand-off must fit its LDS region");
  static_assert(!GL || (A_BYTES % 4096 == 0 && (STAGE - A_BYTES) % 4096 == 0), "hand-off pairs tile the arrays");
  static_assert(KS * NSTG * STAGE <= 163840, "LDS budget");
  static_assert(GLS <= 6 && (KS == 1 || GLS <= 3), "ring depth: <= 6 stages (<= 3 per group with in-block split-K)");
  // GL: one __shared__ array per ring stage.  LDS lowering gives each array its own alias scope, so
  // the waitcnt pass can prove that a fragment read of stage s does not alias the LDS-DMA in flight
  // into another stage; with every stage in one array hipcc waits vmcnt(0) before each read and the
  // ring degenerates to one tile in flight.  Stage indices are therefore compile-time (the loop is
  // unrolled by GLS).
  // The A and B images of a stage are separate arrays too (a B read addressed off the A image's base
  // loses its scope), and so are the two 4-wave groups' rings of the in-block split-K (a runtime group
  // offset adds a GEP level, and LDS lowering stops annotating after a few).
  constexpr int BBY = STAGE - A_BYTES;
  constexpr int GA = GL ? A_BYTES : 16, GB = GL ? BBY : 16;
  constexpr int HA = (GL && KS == 2) ? A_BYTES : 16, HB = (GL && KS == 2) ? BBY : 16;
  __shared__ __attribute__((aligned(16))) char smem_all[GL ? 16 : KS * NSTG * STAGE];
  __shared__ __attribute__((aligned(16))) char ga0[GA];
  __shared__ __attribute__((aligned(16))) char gb0[GB];
  __shared__ __attribute__((aligned(16))) char ga1[GLS >= 2 ? GA : 16];
  __shared__ __attribute__((aligned(16))) char gb1[GLS >= 2 ? GB : 16];
  __shared__ __attribute__((aligned(16))) char ga2[GLS >= 3 ? GA : 16];
  __shared__ __attribute__((aligned(16))) char gb2[GLS >= 3 ? GB : 16];
  // deep rings (KS = 1: up to 6 stages, GLS - 1 k-tiles in flight in one block's LDS)
  __shared__ __attribute__((aligned(16))) char ga3[GLS >= 4 ? GA : 16];
  __shared__ __attribute__((aligned(16))) char gb3[GLS >= 4 ? GB : 16];
  __shared__ __attribute__((aligned(16))) char ga4[GLS >= 5 ? GA : 16];
  __shared__ __attribute__((aligned(16))) char gb4[GLS >= 5 ? GB : 16];
  __shared__ __attribute__((aligned(16))) char ga5[GLS >= 6 ? GA : 16];
  __shared__ __attribute__((aligned(16))) char gb5[GLS >= 6 ? GB : 16];
  __shared__ __attribute__((aligned(16))) char ha0[HA];
  __shared__ __attribute__((aligned(16))) char hb0[HB];
  __shared__ __attribute__((aligned(16))) char ha1[GLS >= 2 ? HA : 16];
  __shared__ __attribute__((aligned(16))) char hb1[GLS >= 2 ? HB : 16];
  __shared__ __attribute__((aligned(16))) char ha2[GLS >= 3 ? HA : 16];
  __shared__ __attribute__((aligned(16))) char hb2[GLS >= 3 ? HB : 16];
  const int grp = KS == 2 ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 8) : 0;
  // GL: epilogue scratch = group 0's A image of stage 0 (>= 8 KB + flag for every tile shape)
  char* smem = GL ? ga0 : smem_all + grp * (NSTG * STAGE);
  auto img_a0 = [&](auto S) -> char* {
    constexpr int st = decltype(S)::value;
    if constexpr (st == 0) return ga0;
    else if constexpr (st == 1) return ga1;
    else if constexpr (st == 2) return ga2;
    else if constexpr (st == 3) return ga3;
    else if constexpr (st == 4) return ga4;
    else return ga5;
  };
  auto img_b0 = [&](auto S) -> char* {
    constexpr int st = decltype(S)::value;
    if constexpr (st == 0) return gb0;
    else if constexpr (st == 1) return gb1;
    else if constexpr (st == 2) return gb2;
    else if constexpr (st == 3) return gb3;
    else if constexpr (st == 4) return gb4;
    else return gb5;
  };
  const int t = threadIdx.x & 255, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;

  // tail blocks past the GEMM's grid: another BN layer's backward slot reduction (IgemmArgs sr_*)
  const int nsr1 = a.sr_C ? (a.sr_C + 15) / 16 : 0, nsr2 = a.sr2_C ? (a.sr2_C + 15) / 16 : 0;
  const int gemm_blocks = (int)gridDim.x - nsr1 - nsr2;
  if ((int)blockIdx.x >= gemm_blocks) {
    if (threadIdx.x < 256) {
      float* scratch = reinterpret_cast<float*>(GL ? ga0 : smem_all);  // >= 2 KB, unused by this block
      const int sb = (int)blockIdx.x - gemm_blocks;
      if (sb < nsr1) sr_block(a.sr_slots, a.sr_red, a.sr_dgamma, a.sr_dbeta, a.sr_C, sb, scratch);
      else sr_block(a.sr2_slots, a.sr2_red, a.sr2_dgamma, a.sr2_dbeta, a.sr2_C, sb - nsr1, scratch);
    }
    return;
  }
  const int bid = xcd_remap(blockIdx.x, gemm_blocks);
  const int tiles_mn = a.tiles_m * a.tiles_n;
  const int split = bid / tiles_mn;
  const int rem = bid - split * tiles_mn;
  const int tm = rem / a.tiles_n, tn = rem - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nkt = (a.K + BKT - 1) / BKT;
  const int kt0_blk = split * a.kps;
  const int kt1 = min(nkt, kt0_blk + a.kps);
  if (kt0_blk >= kt1) return;
  // this group's k-tiles [kt0, kt0 + kh): the SAME trip count for both groups (their barriers are
  // block-wide); tiles past kt1 are zero-filled through kend
  const int kh = KS == 2 ? (kt1 - kt0_blk + 1) / 2 : kt1 - kt0_blk;
  const int kt0 = kt0_blk + grp * kh;

  using LA = Loader<AKIND, BM, GL>;
  using LB = Loader<BKIND, BN, GL>;
  LA la;
  LB lb;
  la.init(a, m0, a.M, a.lda, t);
  lb.init(a, n0, a.N, a.ldb, t);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.A, a.a_bytes), rb = make_rsrc(a.B, a.b_bytes);

  uint32_t oa[LA::NP], ob[LB::NP];

  // tiles at or past kt1 are zero-filled (every offset BAD), so an odd tile count can run the
  // even/odd loop to completion: the extra step multiplies zeros.
  const int kend = min(a.K, min(kt1, kt0 + kh) * BKT);
  u32x4_t sa0[GL ? 1 : LA::NP], sb0[GL ? 1 : LB::NP];
  u32x4_t sa1[GL ? 1 : LA::NP], sb1[GL ? 1 : LB::NP];
  auto issue = [&](int kt, u32x4_t* sa, u32x4_t* sb) {
    const int k0 = kt * BKT;
    la.offsets(a, a.lda, k0, kend, oa);
    lb.offsets(a, a.ldb, k0, kend, ob);
    la.load(ra, oa, sa);
    lb.load(rb, ob, sb);
  };
  auto stage_store = [&](int st, const u32x4_t* sa, const u32x4_t* sb) {
    char* img = smem + st * STAGE;
    la.store(img, sa);
    lb.store(img + A_BYTES, sb);
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto compute_ab = [&](const char* ia, int ia_off, const char* ib, int ib_off) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag<AKIND, BM>(ia, ia_off, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag<BKIND, BN>(ib, ib_off, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (SWAP) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    }
  };
  auto compute = [&](int st) { compute_ab(smem, st * STAGE, smem, st * STAGE + A_BYTES); };

  // ---- epilogue-operand prefetch (fused BN-backward data gradients).  The epilogue reads, per
  // output element, the BN input x, its ReLU mask bits and the residual-branch addend: as much as
  // the GEMM itself moves on the memory-bound 1x1 layers.  Issued in the epilogue they cost one
  // exposed memory round trip per block after the last MFMA (measured: conv_dgrad_bn 92 us vs
  // conv_dgrad 30 us at M 262144, N 256, K 64 -- scripts/operand_major_bench.py).  They do not
  // depend on the GEMM, so PF issues them while the last k-tile(s) compute: in place of the final
  // (zero-tile) refill of the LDS-DMA ring or of the register pipeline, or with the single tile.  Kept to tiles whose per-lane set fits (<= 4 rows x 8 columns, 40 VGPRs;
  // 8 on the single-tile path).
  // Epilogue operands are read through buffer resources with 32-bit offsets (no 64-bit address
  // math per row).  A null operand gets a zero-extent resource: its loads return 0 without a memory
  // access, so every load is unconditional -- a load under a runtime flag makes hipcc branch around
  // it and drain vmcnt(0) at the join (cdna_hip_programming.md "Projection GEMM" item 4(c)).
  struct EpiRes {
    __amdgpu_buffer_rsrc_t ad, am, x, m;
  };
  auto epi_res = [&]() {
    EpiRes r;
    r.ad = make_rsrc(a.addend, a.addend ? 0x7fffffff : 0);
    r.am = make_rsrc(a.addend_mask, a.addend_mask ? 0x7fffffff : 0);
    r.x = make_rsrc(a.bnb_x, a.bnb_x ? 0x7fffffff : 0);
    r.m = make_rsrc(a.bnb_mask, a.bnb_mask ? 0x7fffffff : 0);
    return r;
  };
  // element offset o (bf16 elements) of the output / addend / BN-input tensors
  // addend element offset of output pixel `row`, column nl (BAD bytes -> zeros: an odd pixel of a
  // stride-2 compact addend)
  auto addend_off = [&](int row, int nl) -> uint32_t {
    if (!a.addend_s2) return ((uint32_t)row * (uint32_t)a.ldc + (uint32_t)nl) * 2u;
    const int HW = a.H * a.W;
    const int nn = a.fd_s2HW.div(row), yx = row - nn * HW, y = a.fd_s2W.div(yx), x = yx - y * a.W;
    const uint32_t o = ((uint32_t)((nn * a.s2_P + (y >> 1)) * a.s2_Q + (x >> 1)) * (uint32_t)a.ldc + nl) * 2u;
    return ((y | x) & 1) ? BAD : o;
  };
  auto epi_load = [&](const EpiRes& r, uint32_t o, uint32_t oa, U4& ad, uint32_t& am, U4& xv, uint32_t& mb) {
    ad = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(r.ad, oa, 0, 0));
    am = a.addend_mask ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r.am, o >> 3, 0, 0) : 0xffu;
    if constexpr (EPI == EPI_BNB) {
      xv = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(r.x, o * 2u, 0, 0));
      mb = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r.m, o >> 3, 0, 0);
    }
  };
  constexpr int NPF = SWAP ? (TN / 2) * TM : 1;
  constexpr bool PF = EPI == EPI_BNB && SWAP && (NPF <= 4 || (STG == 1 && !GL && NPF <= 8));
  U4 pf_ad[PF ? NPF : 1], pf_x[PF ? NPF : 1];
  uint32_t pf_am[PF ? NPF : 1], pf_m[PF ? NPF : 1];
  auto epi_prefetch = [&]() {
    if constexpr (PF) {
      if (KS == 2 && grp != 0) return;  // group 1 only hands its accumulators over
      const EpiRes er = epi_res();
      const int mb0 = m0 + wm * WM, nb0 = n0 + wn * WN;
      const bool odd = (lane >> 4) & 1;
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        const int n = nb0 + (j + (odd ? 1 : 0)) * 16 + ((lane >> 5) << 3);
        const int nl = min(n, a.N - 8);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = min(mb0 + i * 16 + (lane & 15), a.M - 1);
          int row = m;
          if (a.cls) {
            const int nn = a.fd_cHW.div(m), yx = m - nn * a.H * a.W, y = a.fd_cW.div(yx), x = yx - y * a.W;
            row = (nn * a.out_H + 2 * y + a.cph) * a.out_W + 2 * x + a.cpw;
          }
          const uint32_t o = (uint32_t)row * (uint32_t)a.ldc + (uint32_t)nl;
          const int e = (j / 2) * TM + i;
          epi_load(er, o, addend_off(row, nl), pf_ad[e], pf_am[e], pf_x[e], pf_m[e]);
        }
      }
    }
  };

  if constexpr (GL) {
    constexpr int NPT = LA::NP + LB::NP;  // LDS-DMA pieces per thread per k-tile
    // the wave index as a scalar: every LDS-DMA destination (M0) is then computed once in SGPRs
    // instead of a v_readfirstlane per piece and k-tile
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // stage images of group G, stage S (compile-time: each read / DMA names its array directly)
    auto img_a = [&](auto G, auto S) -> char* {
      constexpr int g = decltype(G)::value, st = decltype(S)::value;
      if constexpr (g == 0) {
        return img_a0(S);
      } else {
        if constexpr (st == 0) return ha0;
        else if constexpr (st == 1) return ha1;
        else return ha2;
      }
    };
    auto img_b = [&](auto G, auto S) -> char* {
      constexpr int g = decltype(G)::value, st = decltype(S)::value;
      if constexpr (g == 0) {
        return img_b0(S);
      } else {
        if constexpr (st == 0) return hb0;
        else if constexpr (st == 1) return hb1;
        else return hb2;
      }
    };
    auto issue_gl = [&](int kt, auto G, auto S) {
      const int k0 = kt * BKT;
      la.offsets(a, a.lda, k0, kend, oa);
      lb.offsets(a, a.ldb, k0, kend, ob);
      la.load_lds(ra, oa, img_a(G, S), 0, wv);
      lb.load_lds(rb, ob, img_b(G, S), 0, wv);
    };
    auto ring = [&](auto G) {
      if constexpr (GLS == 1) {  // host guarantees a single k-tile
        issue_gl(kt0, G, IC<0>{});
        epi_prefetch();
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        compute_ab(img_a(G, IC<0>{}), 0, img_b(G, IC<0>{}), 0);
      } else {
        // one ring step: tile `it` sits in stage S; tile it+GLS-1 goes into the stage tile it-1 used
        auto body = [&](auto S, int it) {
          constexpr int st = decltype(S)::value;
          constexpr int ist = (st + GLS - 1) % GLS;
          wait_vmcnt<NPT * (GLS - 2)>();
          __builtin_amdgcn_s_barrier();
          issue_gl(kt0 + it + GLS - 1, G, IC<ist>{});
          __builtin_amdgcn_sched_barrier(0);
          compute_ab(img_a(G, IC<st>{}), 0, img_b(G, IC<st>{}), 0);
          __builtin_amdgcn_sched_barrier(0);
        };
        // PF: the last step's ring refill would be a zero tile -- the epilogue operands go out
        // instead (nothing after that step waits on a count, only the final drain).  Peeled so the
        // operand registers are live only from there on.
        auto last = [&](auto S) {
          constexpr int st = decltype(S)::value;
          wait_vmcnt<NPT * (GLS - 2)>();
          __builtin_amdgcn_s_barrier();
          epi_prefetch();
          __builtin_amdgcn_sched_barrier(0);
          compute_ab(img_a(G, IC<st>{}), 0, img_b(G, IC<st>{}), 0);
          __builtin_amdgcn_sched_barrier(0);
        };
        // prologue: tiles 0 .. GLS-2 into stages 0 .. GLS-2
        static_for<GLS - 1>([&](auto P) { issue_gl(kt0 + decltype(P)::value, G, P); });
        int it = 0;
        if constexpr (PF) {
          for (; it + GLS < kh; it += GLS) static_for<GLS>([&](auto S) { body(S, it + decltype(S)::value); });
          const int rem = kh - it;  // 1 .. GLS steps left, the final one peeled
          static_for<GLS>([&](auto R) {
            constexpr int r = decltype(R)::value;
            if (rem == r + 1) {
              static_for<r>([&](auto S) { body(S, it + decltype(S)::value); });
              last(R);
            }
          });
        } else {
          for (; it + GLS <= kh; it += GLS) static_for<GLS>([&](auto S) { body(S, it + decltype(S)::value); });
          const int rem = kh - it;  // < GLS
          static_for<GLS - 1>([&](auto S) {
            if (rem > decltype(S)::value) body(S, it + decltype(S)::value);
          });
        }
      }
    };
    // both groups run the same number of ring steps, so their block-wide barriers pair up
    if constexpr (KS == 2) {
      if (grp == 1) ring(IC<1>{});
      else ring(IC<0>{});
    } else {
      ring(IC<0>{});
    }
    // drain the ring (the zero-filled pieces issued past the last tile too) before the epilogue
    // reuses LDS or the workgroup exits with LDS writes in flight
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  } else if constexpr (STG == 1) {  // host guarantees a single k-tile
    issue(kt0, sa0, sb0);
    epi_prefetch();
    if constexpr (AKIND == KM_DENSE && EPI == EPI_STATS) {
      // consumer-applied ReLU BN (IgemmArgs a_scale): the thread's chunk is channels c0 .. c0+7 of the
      // single k-tile; rows past M stay zero (their loads returned zeros, not the BN of zero)
      if (a.a_scale) {
        // two 16-B loads each, unconditional (a per-element guard compiles to branches that drain
        // vmcnt); K < 64: chunks past K read the last 8 entries -- their A values meet zero-filled B
        const int cc = min(la.c0, a.K - 8);
        const float4 s0 = *reinterpret_cast<const float4*>(a.a_scale + cc);
        const float4 s1 = *reinterpret_cast<const float4*>(a.a_scale + cc + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(a.a_shift + cc);
        const float4 h1 = *reinterpret_cast<const float4*>(a.a_shift + cc + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < LA::NP; ++i) {
          float f[8];
          unpack8(__builtin_bit_cast(U4, sa0[i]), f);
#pragma unroll
          for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], sc[k], sh[k]), 0.f);
          const uint32_t keep = la.ctx0[i] >= 0 ? 0xffffffffu : 0u;  // bit mask, not a select: no branch
          U4 p = pack8(f);
          p.x &= keep; p.y &= keep; p.z &= keep; p.w &= keep;
          sa0[i] = __builtin_bit_cast(u32x4_t, p);
        }
      }
    }
    stage_store(0, sa0, sb0);
    __syncthreads();
    compute(0);
  } else {
  // prologue: tile kt0 -> stage 0, tile kt0+1 in flight in set 1
  issue(kt0, sa0, sb0);
  issue(kt0 + 1, sa1, sb1);
  stage_store(0, sa0, sb0);
  __syncthreads();
  if (kh == 1) {
    epi_prefetch();
    compute(0);
  } else if constexpr (PF) {
    // as below, with the final pair peeled: its two tiles are already staged / in flight, so the
    // epilogue operands go out in place of the (zero-filled) prefetches past the end
    const int ktend = kt0 + kh;
    int kt = kt0;
    for (; kt + 2 < ktend; kt += 2) {
      issue(kt + 2, sa0, sb0);
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      stage_store(1, sa1, sb1);
      __syncthreads();
      issue(kt + 3, sa1, sb1);
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      stage_store(0, sa0, sb0);
      __syncthreads();
    }
    epi_prefetch();
    __builtin_amdgcn_sched_barrier(0);
    compute(0);
    __builtin_amdgcn_sched_barrier(0);
    stage_store(1, sa1, sb1);  // tile kt + 1 (zero-filled when kh is odd)
    __syncthreads();
    compute(1);
  } else {
    // single exit at the bottom: every path into the loop header has set 1 in flight and set 0
    // free, so the vmcnt bookkeeping is identical on both edges (no conservative vmcnt(0)).
    // sched_barrier(0) pins the order issue -> MFMAs -> LDS write: without it hipcc hoists the
    // stage write (and its vmcnt wait on the previous tile's loads) above the MFMAs.
    const int ktend = kt0 + kh;
    for (int kt = kt0; kt < ktend; kt += 2) {
      issue(kt + 2, sa0, sb0);  // even: stage 0 holds kt, set 1 holds kt+1
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      stage_store(1, sa1, sb1);
      __syncthreads();
      issue(kt + 3, sa1, sb1);  // odd: stage 1 holds kt+1, set 0 holds kt+2
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      stage_store(0, sa0, sb0);
      __syncthreads();
    }
  }
  }

  if constexpr (KS == 2) {
    // group 1's accumulators -> its (now free) LDS stages -> summed into group 0's, conflict-free
    // [element][thread] layout; group 1 is done after the hand-off
    __syncthreads();  // kh == 1 leaves compute(0) without a trailing barrier
    // register path: group 1's stage space.  GL: group 0's stage arrays in order (both groups are past
    // the drain); accumulator pair (i, j) = 4 KB goes to array xk(p) at xo(p)
    auto xrow = [&](auto P) -> float* {
      constexpr int pr = decltype(P)::value;
      if constexpr (!GL) {
        return reinterpret_cast<float*>(smem_all + NSTG * STAGE) + pr * 1024;
      } else {
        constexpr int pa = A_BYTES / 4096, pb = BBY / 4096;  // pairs per A / B array
        constexpr int q = pr % (pa + pb), st = pr / (pa + pb);
        char* base = q < pa ? img_a0(IC<st>{}) : img_b0(IC<st>{});
        return reinterpret_cast<float*>(base) + (q < pa ? q : q - pa) * 1024;
      }
    };
    if (grp == 1) {
      static_for<TM * TN>([&](auto P) {
        constexpr int pr = decltype(P)::value, i = pr / TN, j = pr % TN;
        float* x = xrow(P);
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r * 256 + t] = acc[i][j][r];
      });
    }
    __syncthreads();
    if (grp == 1) return;
    static_for<TM * TN>([&](auto P) {
      constexpr int pr = decltype(P)::value, i = pr / TN, j = pr % TN;
      const float* x = xrow(P);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] += x[r * 256 + t];
    });
    // the fused-BN epilogues reuse this LDS for their partials: every group-0 wave must be past its
    // hand-off reads first (group 1 has exited; s_barrier waits only on the surviving waves)
    if constexpr (EPI != EPI_PLAIN) __syncthreads();
  }

  // Element (m, n) of lane's acc[i][j][r]:
  //   SWAP : m = mb + i*16 + (lane&15),        n = nb + j*16 + (lane>>4)*4 + r
  //   !SWAP: m = mb + i*16 + (lane>>4)*4 + r,  n = nb + j*16 + (lane&15)
  const int mb = m0 + wm * WM, nb = n0 + wn * WN;

  // ---------------- fused BN statistics of the bf16-rounded output (per column n, this tile's rows)
  if constexpr (STG == 1 && !GL) {
    // single-k-tile variant: no barrier after compute(0) -- other waves may still be reading the
    // stage that the epilogue's LDS partials overwrite (the GL paths end on a drain + barrier)
    if constexpr (EPI != EPI_PLAIN) __syncthreads();
  }
  static_assert(EPI == EPI_PLAIN || SWAP, "fused-BN epilogues use the SWAP (16-byte store) orientation");

  // ---------------- epilogue (mode tested once per block, bias preloaded: no loads in the store loops)
  if constexpr (SWAP) {
    float bias[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[j][r] = 0.f;
    if (a.bias) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + j * 16 + (lane >> 4) * 4 + r;
          bias[j][r] = a.bias[min(n, a.N - 1)];
        }
    }
    const bool relu = a.relu != 0;
    // element offset of output row m (MODE_DGRAD_CLS: class sub-grid pixel -> full-grid pixel)
    int64_t rowoff[TM];
    int rowpix[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = min(mb + i * 16 + (lane & 15), a.M - 1);
      int row = m;
      if (a.cls) {
        const int n = a.fd_cHW.div(m), yx = m - n * a.H * a.W, y = a.fd_cW.div(yx), x = yx - y * a.W;
        row = (n * a.out_H + 2 * y + a.cph) * a.out_W + 2 * x + a.cpw;
      }
      rowoff[i] = (int64_t)row * a.ldc;
      rowpix[i] = row;
    }
    // fused-BN variants only ever take the 16-byte path (igemm_launch checks): compile only that one
    if (EPI != EPI_PLAIN ||
        (a.out_mode == OUT_BF16 && !a.trans_out && (a.ldc & 7) == 0 && (a.N & 7) == 0 && (TN % 2) == 0)) {
      // 16-byte stores: lanes l and l^16 hold 4-column halves of the same row in tiles j and j+1;
      // swapping one half (4 floats over __shfl_xor 16) gives each lane 8 consecutive columns --
      // the even lane of tile j, the odd lane of tile j+1 -- i.e. half the store instructions.
      uint16_t* Cb = reinterpret_cast<uint16_t*>(a.Cp);
      const bool odd = (lane >> 4) & 1;
      constexpr bool bnb = EPI == EPI_BNB;    // fused BN-backward partials of this output
      constexpr bool sts = EPI == EPI_STATS;  // fused BN statistics of this (bf16-rounded) output
      float* red = reinterpret_cast<float*>(smem);  // [2 wm][BN cols][2] partials (LDS free after the loop)
      // BN-backward ReLU mask source, decided once: 2 = the residual layer's bits, 1 = recomputed
      // from x*scale+shift, 0 = none
      const int bnb_mode = !a.bnb_relu ? 0 : (a.bnb_mask ? 2 : 1);
      const EpiRes er = epi_res();
      const __amdgpu_buffer_rsrc_t r_out = make_rsrc(a.Cp, 0x7fffffff);
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        const int n = nb + (j + (odd ? 1 : 0)) * 16 + ((lane >> 5) << 3);
        // per-column BN parameters of this lane's 8 columns (mean, invstd, scale, shift)
        float mu[8], is[8], sc[8], sh[8], bs[8], bq[8];
        if constexpr (bnb || sts) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            bs[k] = 0.f;
            bq[k] = 0.f;
          }
        }
        float nmi[8];  // -mean * invstd
        if constexpr (bnb) {
          const int nc = min(n, a.N - 8);
#pragma unroll
          for (int q = 0; q < 2; ++q) {  // nc and N are multiples of 8: 16-byte loads
            const float4 m4 = *reinterpret_cast<const float4*>(a.bnb_save + nc + 4 * q);
            const float4 i4 = *reinterpret_cast<const float4*>(a.bnb_save + a.N + nc + 4 * q);
            const float4 c4 = *reinterpret_cast<const float4*>(a.bnb_save + 2 * a.N + nc + 4 * q);
            const float4 h4 = *reinterpret_cast<const float4*>(a.bnb_save + 3 * a.N + nc + 4 * q);
            mu[4 * q] = m4.x; mu[4 * q + 1] = m4.y; mu[4 * q + 2] = m4.z; mu[4 * q + 3] = m4.w;
            is[4 * q] = i4.x; is[4 * q + 1] = i4.y; is[4 * q + 2] = i4.z; is[4 * q + 3] = i4.w;
            sc[4 * q] = c4.x; sc[4 * q + 1] = c4.y; sc[4 * q + 2] = c4.z; sc[4 * q + 3] = c4.w;
            sh[4 * q] = h4.x; sh[4 * q + 1] = h4.y; sh[4 * q + 2] = h4.z; sh[4 * q + 3] = h4.w;
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) nmi[k] = -mu[k] * is[k];
        }
        // The epilogue's global reads (addend, BN input, ReLU mask bits) of IC rows are issued
        // together BEFORE the rows' stores: the compiler cannot hoist a load over a store it may
        // alias (the addend IS the output when summed in place), so a row-by-row loop would run one
        // full memory latency per row.  Loads use an in-range column; out-of-range rows / columns
        // are dropped at the store.
        constexpr int IC = TM < 4 ? TM : 4;
        const int nl = min(n, a.N - 8);
#pragma unroll
        for (int i0 = 0; i0 < TM; i0 += IC) {
          U4 adv[IC], xvv[IC];
          uint32_t mbv[IC], amv[IC];
#pragma unroll
          for (int ii = 0; ii < IC; ++ii) {
            if constexpr (PF) {  // issued during the last k-tile(s): see epi_prefetch
              const int e = (j / 2) * TM + i0 + ii;
              adv[ii] = pf_ad[e];
              amv[ii] = pf_am[e];
              xvv[ii] = pf_x[e];
              mbv[ii] = pf_m[e];
              continue;
            }
            // BN-backward kernels load unconditionally (null operands read zeros); the others only
            // ever read an addend, under its (uniform) flag
            if (bnb || a.addend)
              epi_load(er, (uint32_t)rowoff[i0 + ii] + (uint32_t)nl, addend_off(rowpix[i0 + ii], nl), adv[ii],
                       amv[ii], xvv[ii], mbv[ii]);
          }
#pragma unroll
          for (int ii = 0; ii < IC; ++ii) {
            const int i = i0 + ii;
            const int m = mb + i * 16 + (lane & 15);
            float v0[4], v1[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v0[r] = acc[i][j][r] + bias[j][r];
              v1[r] = acc[i][j + 1][r] + bias[j + 1][r];
              if (relu) {
                v0[r] = fmaxf(v0[r], 0.f);
                v1[r] = fmaxf(v1[r], 0.f);
              }
            }
            float o[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              // v_permlane16_swap: odd 16-lane rows of v0 <-> even rows of v1.  Even lanes end with
              // [own v0 | partner v0], odd lanes with [partner v1 | own v1] (no LDS round trip)
              const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(v0[r]), __float_as_uint(v1[r]),
                                                               false, false);
              o[r] = __uint_as_float(sw[0]);
              o[4 + r] = __uint_as_float(sw[1]);
            }
            if (m < a.M && n < a.N) {
              if (a.addend) {  // fused residual-branch gradient sum (dX = dgrad + other branch)
                // the addend's ReLU mask bits (0xff when unmasked) zero its bf16 halves before the
                // unpack: straight-line bit ops, no per-element select on a runtime flag
                float ad[8];
                unpack8(mask_bf16x8(adv[ii], amv[ii]), ad);
#pragma unroll
                for (int r = 0; r < 8; ++r) o[r] += ad[r];
              }
              const U4 packed = pack8(o);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, packed), r_out,
                                                     ((uint32_t)rowoff[i] + (uint32_t)n) * 2u, 0, 0);
              if constexpr (sts) {
                // per-column sum / sum of squares of exactly the bf16 values the BN will read
                float g[8];
                unpack8(packed, g);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                  bs[k] += g[k];
                  bq[k] = fmaf(g[k], g[k], bq[k]);
                }
              }
              if constexpr (bnb) {
                // g' = bf16(out) * relu mask; xhat = x * invstd - mean * invstd from the BN input x
                // (same NHWC position).  The mask comes from the residual layer's bits or from
                // x*scale+shift > 0, chosen once per kernel (bnb_mode), and is applied to the bf16
                // words before the unpack.
                float xv[8];
                unpack8(xvv[ii], xv);
                uint32_t on8 = 0xffu;
                if (bnb_mode == 2) {
                  on8 = mbv[ii];
                } else if (bnb_mode == 1) {
                  on8 = 0;
#pragma unroll
                  for (int k = 0; k < 8; ++k) on8 |= (fmaf(xv[k], sc[k], sh[k]) > 0.f ? 1u : 0u) << k;
                }
                float g[8];
                unpack8(mask_bf16x8(packed, on8), g);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                  bs[k] += g[k];
                  bq[k] = fmaf(g[k], fmaf(xv[k], is[k], nmi[k]), bq[k]);
                }
              }
            }
          }
        }
        if constexpr (bnb || sts) {
          // the 16 rows of this DPP row share the lane's 8 columns: reduce them in registers
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            bs[k] = row16_sum(bs[k]);
            bq[k] = row16_sum(bq[k]);
          }
          if ((lane & 15) == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const int col = n - n0 + k;
              red[(wm * BN + col) * 2 + 0] = bs[k];
              red[(wm * BN + col) * 2 + 1] = bq[k];
            }
          }
        }
      }
      if constexpr (bnb || sts) {
        __syncthreads();
        if (t < BN) {
          const int nn = n0 + t;
          if (nn < a.N) {
            float* slot = (bnb ? a.bnb_slots : a.stats) + (size_t)(tm % (bnb ? NSLOT : a.stat_slots)) * 2 * a.N;
            atomicAdd(&slot[nn], red[t * 2] + red[(BN + t) * 2]);
            atomicAdd(&slot[a.N + nn], red[t * 2 + 1] + red[(BN + t) * 2 + 1]);
          }
        }
      }
    } else if (a.out_mode == OUT_BF16 && !a.trans_out && (a.ldc & 3) == 0 && (a.N & 3) == 0) {
      uint16_t* Cb = reinterpret_cast<uint16_t*>(a.Cp);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = nb + j * 16 + (lane >> 4) * 4;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[i][j][r] + bias[j][r];
            if (relu) v[r] = fmaxf(v[r], 0.f);
          }
          if (m < a.M && n < a.N) {
            if (a.addend) {  // fused residual-branch gradient sum (dX = dgrad + other branch)
              const uint2 o2 = *reinterpret_cast<const uint2*>(a.addend + rowoff[i] + n);
              v[0] += __uint_as_float(o2.x << 16);
              v[1] += __uint_as_float(o2.x & 0xffff0000u);
              v[2] += __uint_as_float(o2.y << 16);
              v[3] += __uint_as_float(o2.y & 0xffff0000u);
            }
            uint2 w2;
            w2.x = pack_bf16x2(v[0], v[1]);
            w2.y = pack_bf16x2(v[2], v[3]);
            *reinterpret_cast<uint2*>(Cb + rowoff[i] + n) = w2;
          }
        }
      }
    } else if (a.out_mode == OUT_F32_ATOMIC && a.trans_out) {
      float* Cf = reinterpret_cast<float*>(a.Cp);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = nb + j * 16 + (lane >> 4) * 4 + r;
            if (m < a.M && n < a.N) atomicAdd(Cf + (int64_t)n * a.ldc + m, acc[i][j][r]);
          }
      }
    } else {  // generic (ragged N, other modes): element stores
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = nb + j * 16 + (lane >> 4) * 4 + r;
            if (m >= a.M || n >= a.N) continue;
            float v = acc[i][j][r] + bias[j][r];
            if (relu) v = fmaxf(v, 0.f);
            const int64_t o = a.trans_out ? (int64_t)n * a.ldc + m : rowoff[i] + n;
            if (a.addend) v += bf16_to_f32(a.addend[o]);
            if (a.out_mode == OUT_BF16) reinterpret_cast<uint16_t*>(a.Cp)[o] = f32_to_bf16(v);
            else if (a.out_mode == OUT_F32) reinterpret_cast<float*>(a.Cp)[o] = v;
            else if (a.out_mode == OUT_F32_ADD) reinterpret_cast<float*>(a.Cp)[o] += v;
            else atomicAdd(reinterpret_cast<float*>(a.Cp) + o, v);
          }
      }
    }
  } else {
    float bias[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bias[j] = a.bias ? a.bias[min(nb + j * 16 + (lane & 15), a.N - 1)] : 0.f;
    if (a.out_mode == OUT_F32_ATOMIC && !a.trans_out) {
      float* Cf = reinterpret_cast<float*>(a.Cp);
      // Row-contiguous atomics: an accumulator register as it stands is 4 rows x 64 B per
      // wave-instruction; the wave parks its WM x WN tile in a private LDS region and adds it back row
      // by row -- two 128-B rows per instruction (WN 32), an f32 atomic shape that
      // runs at the full memory-side rate (MI355X_MICROARCH.md "Global float atomics").
      constexpr int RB = WM * WN * 4;  // region bytes per wave
      constexpr bool GLR = GL && GLS >= 2 && (BBY >= RB || A_BYTES >= 2 * RB);
      constexpr bool REGR = !GL && 4 * RB <= KS * NSTG * STAGE;
      // (measured: 1x1 weight gradients, WN 32, 8-17 % faster; the 128x128-tile 3x3 ones, WN 64, 3-11 %
      // slower -- their atomics overlap the other blocks' main loops -- and keep the direct form)
      if constexpr ((GLR || REGR) && WN == 32) {
        float* T;
        if constexpr (GLR) {
          if constexpr (BBY >= RB) T = reinterpret_cast<float*>(w == 0 ? ga0 : w == 1 ? gb0 : w == 2 ? ga1 : gb1);
          else T = reinterpret_cast<float*>(w == 0 ? ga0 : w == 1 ? ga0 + RB : w == 2 ? ga1 : ga1 + RB);
        } else {
          T = reinterpret_cast<float*>(smem_all) + w * (WM * WN);
        }
        // every wave is past its last fragment / hand-off read of this LDS (LDS-only barrier)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // column chunk XOR (bit 2 of the row -> bit 4 of the column): the 4-row register layout
        // writes conflict-free; a row read is a permutation within the row
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = i * 16 + (lane >> 4) * 4 + r, col = j * 16 + (lane & 15);
              T[row * WN + (col ^ (((row >> 2) & 1) << 4))] = acc[i][j][r] + bias[j];
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back only its own region
        constexpr int RPI = 64 / WN;  // rows per instruction
#pragma unroll
        for (int q = 0; q < WM / RPI; ++q) {
          const int row = q * RPI + lane / WN, col = lane % WN;
          const float v = T[row * WN + (col ^ (((row >> 2) & 1) << 4))];
          const int m = mb + row, n = nb + col;
          if (m < a.M && n < a.N) atomicAdd(Cf + (int64_t)m * a.ldc + n, v);
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = nb + j * 16 + (lane & 15);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int m = mb + i * 16 + (lane >> 4) * 4 + r;
              if (m < a.M && n < a.N) atomicAdd(Cf + (int64_t)m * a.ldc + n, acc[i][j][r] + bias[j]);
            }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = nb + j * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = mb + i * 16 + (lane >> 4) * 4 + r;
            if (m >= a.M || n >= a.N) continue;
            float v = acc[i][j][r] + bias[j];
            if (a.relu) v = fmaxf(v, 0.f);
            const int64_t o = a.trans_out ? (int64_t)n * a.ldc + m : (int64_t)m * a.ldc + n;
            if (a.out_mode == OUT_BF16) reinterpret_cast<uint16_t*>(a.Cp)[o] = f32_to_bf16(v);
            else if (a.out_mode == OUT_F32) reinterpret_cast<float*>(a.Cp)[o] = v;
            else if (a.out_mode == OUT_F32_ADD) reinterpret_cast<float*>(a.Cp)[o] += v;
            else atomicAdd(reinterpret_cast<float*>(a.Cp) + o, v);
          }
      }
    }
  }
}

// ============================================================ host launcher

// LDS-DMA ring depth for the main loop: 0 = register-staged pipeline (the default: in the full
// training step the ring's 1-block-per-CU occupancy left no room for the overlapping kernels,
// bench.py 9.334 vs 9.266 ms/step, profiles/r02_glds/step_ab.txt), 2 or 3 = ring depth, capped per
// tile shape by the LDS budget -- chosen per layer by the measured launch table (TuneCfg.gls).
// launch configuration of the current launch_shape call (igemm_tune_lookup), read by launch_t
thread_local TuneCfg g_tc;

int pick_splits(int tiles, int nkt, int want_blocks, int min_kps = 4) {
  if (tiles >= want_blocks) return 1;
  // floor: never more blocks than the target (1 or 2 per CU) -- a few CUs holding an extra block
  // would set the kernel's time (e.g. 36 tiles x 8 splits = 288 blocks on 256 CUs)
  int s = want_blocks / tiles;
  if (s * tiles < want_blocks * 3 / 4) s = (want_blocks + tiles - 1) / tiles;  // floor under-fills: round up
  const int max_s = std::max(1, nkt / min_kps);  // keep >= min_kps (default 4) k-tiles per split
  return std::max(1, std::min(s, max_s));
}

template <int AK, int BK, int BM, int BN, int EPI = EPI_PLAIN, int KS = 1>
void launch_t(IgemmArgs& a, hipStream_t s, int want_mult = 1, int min_kps = 4) {
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  const int nkt = (a.K + BKT - 1) / BKT;
  const int tiles = a.tiles_m * a.tiles_n;
  int splits = 1;
  constexpr int want = 256;  // one block per CU: measured best (fewer f32 atomic partials)
  const int want_blocks = g_tc.want > 0 ? g_tc.want : want * want_mult;
  // (deterministic mode: one block per output tile, its single atomic add per element onto the zeroed
  // gradient is exact)
  if (a.out_mode == OUT_F32_ATOMIC && !det_mode()) splits = pick_splits(tiles, nkt, want_blocks, min_kps);
  a.kps = (nkt + splits - 1) / splits;
  if constexpr (KS == 2) {
    // each 4-wave group takes kps/2 k-tiles: a multiple of 4 keeps both halves even (no zero step).
    // An 8-wave block holds its CU's LDS alone, so more blocks than CUs would run a second wave
    // (e.g. 144 tiles x 2 splits): the 4-wave form fits those at two blocks per CU.
    if (a.kps < 4 || tiles * splits > (g_tc.want > 0 ? g_tc.want : want))
      return launch_t<AK, BK, BM, BN, EPI, 1>(a, s, want_mult, min_kps);
    a.kps = (a.kps + 3) & ~3;
  } else if (splits > 1) {
    a.kps += a.kps & 1;  // even k-tiles per split: no zero step in the loop
  }
  splits = (nkt + a.kps - 1) / a.kps;
  if (tiles * splits == 0) return;
  const int grid = tiles * splits + (a.sr_C ? (a.sr_C + 15) / 16 : 0) +
                   (a.sr2_C ? (a.sr2_C + 15) / 16 : 0);  // + slot-reduce tail blocks
  // transposed MFMA orientation for bf16 outputs and transposed stores (see kernel comment)
  const bool swap = a.out_mode == OUT_BF16 || a.trans_out;
  constexpr int STAGE_B = (BM + BN) * BKT * 2;
  constexpr int G3 = KS * 3 * STAGE_B <= 163840 ? 3 : 2;
  const int gls = (g_tc.gls >= 0 && !a.a_scale) ? g_tc.gls : 0;  // the A transform is register-path only
  // the general im2col gathers (C % 64 != 0 / pixel tiles crossing image rows: LeNet, odd stems) run the
  // register pipeline only
  if constexpr (AK != KM_FWD_X && AK != MN_WGRAD_X && BK != MN_WGRAD_X) {
  if (gls > 0) {
    // LDS-DMA ring: single k-tile -> GLS 1; otherwise the deepest ring (<= 3) that fits the LDS
    const bool single = nkt == 1 && splits == 1;
    // (the kernel takes rings of up to 6 stages at KS = 1; deep rings -- one 4-wave block per CU holding
    // 4-6 stages -- lost at every ResNet-50 conv pass, profiles/r05_deep, and are not instantiated)
#define TFX_GL_LAUNCH(SW)                                                                              \
    if constexpr (KS == 1) {                                                                           \
      if (single) { igemm_kernel<AK, BK, BM, BN, SW, 1, EPI, 1, 1><<<grid, NT, 0, s>>>(a); return; }   \
    }                                                                                                  \
    if (gls == 2 || G3 == 2) igemm_kernel<AK, BK, BM, BN, SW, 2, EPI, KS, 2><<<grid, KS * NT, 0, s>>>(a); \
    else igemm_kernel<AK, BK, BM, BN, SW, 2, EPI, KS, G3><<<grid, KS * NT, 0, s>>>(a);
    if constexpr (EPI != EPI_PLAIN) {
      TFX_GL_LAUNCH(true)
    } else {
      if (swap) { TFX_GL_LAUNCH(true) } else { TFX_GL_LAUNCH(false) }
    }
#undef TFX_GL_LAUNCH
    return;
  }
  }
  if constexpr (KS == 2) {
    if constexpr (EPI != EPI_PLAIN) {
      igemm_kernel<AK, BK, BM, BN, true, 2, EPI, 2><<<grid, 2 * NT, 0, s>>>(a);
    } else {
      if (swap) igemm_kernel<AK, BK, BM, BN, true, 2, EPI_PLAIN, 2><<<grid, 2 * NT, 0, s>>>(a);
      else igemm_kernel<AK, BK, BM, BN, false, 2, EPI_PLAIN, 2><<<grid, 2 * NT, 0, s>>>(a);
    }
    return;
  }
  if constexpr (EPI != EPI_PLAIN) {  // fused-BN epilogues: bf16 outputs only (SWAP orientation)
    if (nkt == 1 && splits == 1) igemm_kernel<AK, BK, BM, BN, true, 1, EPI><<<grid, NT, 0, s>>>(a);
    else igemm_kernel<AK, BK, BM, BN, true, 2, EPI><<<grid, NT, 0, s>>>(a);
  } else if (nkt == 1 && splits == 1) {
    if (swap) igemm_kernel<AK, BK, BM, BN, true, 1, EPI><<<grid, NT, 0, s>>>(a);
    else igemm_kernel<AK, BK, BM, BN, false, 1, EPI><<<grid, NT, 0, s>>>(a);
  } else {
    if (swap) igemm_kernel<AK, BK, BM, BN, true, 2, EPI><<<grid, NT, 0, s>>>(a);
    else igemm_kernel<AK, BK, BM, BN, false, 2, EPI><<<grid, NT, 0, s>>>(a);
  }
}

// tile choice: narrow N -> 256x64 (if M is large) or 128x64; otherwise 128x128, unless that leaves
// the chip under-filled (fewer than 2 blocks per CU: the small late-stage convs), then 128x64 --
// twice the blocks for the same K loop.
// Weight gradients (split-K, f32 atomics): in-block split-K (8-wave blocks, KS = 2) by default;
// 128x64 tiles for the dense (1x1) pair -- half the atomic bytes of the 2-blocks-per-CU 128x64 form
// -- and 128x128 for the im2col-gathered ones (measured: profiles/r01_v10, r02_bigtile).
// min k-tiles per split for the skinny GEMM path
constexpr int kSkinnyMinKps = 2;

template <int AK, int BK, bool ALLOW256 = true, int EPI = EPI_PLAIN>
void launch_shape(IgemmArgs& a, hipStream_t s, int fam = -1) {
  TuneCfg tc;
  const bool tuned = igemm_tune_lookup(fam, a.M, a.N, a.K, &tc);
  g_tc = tuned ? tc : TuneCfg{};
  if (tuned && tc.tile > 0) {
    if constexpr (!ALLOW256) {
      if (tc.ks == 2 || tc.ks == 0) {
        if (tc.tile == 2) return launch_t<AK, BK, 128, 64, EPI, 2>(a, s);
        return launch_t<AK, BK, 128, 128, EPI, 2>(a, s);
      }
      if (tc.tile == 2) return launch_t<AK, BK, 128, 64, EPI>(a, s, 2);
      return launch_t<AK, BK, 128, 128, EPI>(a, s);
    } else {
      // ks 2 on a bf16-output family: 8-wave blocks, two 4-wave groups splitting the tile's K (twice the
      // loads in flight per CU for the under-filled late-stage layers); group 0 runs the epilogue
      if (tc.ks == 2 && tc.tile != 3) {
        if (tc.tile == 2) return launch_t<AK, BK, 128, 64, EPI, 2>(a, s);
        return launch_t<AK, BK, 128, 128, EPI, 2>(a, s);
      }
      if (tc.tile == 3) return launch_t<AK, BK, 256, 64, EPI>(a, s);
      if (tc.tile == 2) return launch_t<AK, BK, 128, 64, EPI>(a, s);
      return launch_t<AK, BK, 128, 128, EPI>(a, s);
    }
  }
  if constexpr (!ALLOW256) {
    const bool dense_pair = (AK == MN_DENSE && BK == MN_DENSE) || (a.R == 1 && a.S == 1);  // 1x1 (any stride)
    const bool ks2 = tuned && tc.ks > 0 ? tc.ks == 2 : true;
    if (ks2) {
      if (a.N <= 64 || dense_pair) return launch_t<AK, BK, 128, 64, EPI, 2>(a, s);
      return launch_t<AK, BK, 128, 128, EPI, 2>(a, s);
    }
    if (a.N > 64 && dense_pair) return launch_t<AK, BK, 128, 64, EPI>(a, s, 2);
  }
  if (a.N <= 64) {
    if constexpr (ALLOW256) {
      if (a.M >= 256 * 256) return launch_t<AK, BK, 256, 64, EPI>(a, s);
    }
    launch_t<AK, BK, 128, 64, EPI>(a, s);
  } else {
    const long tiles128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128);
    if constexpr (ALLOW256) {
      if (tiles128 < 512) return launch_t<AK, BK, 128, 64, EPI>(a, s);
    }
    launch_t<AK, BK, 128, 128, EPI>(a, s);
  }
}


template <int AK, int BK, int EPI_ON>
void launch_epi(IgemmArgs& a, hipStream_t s, int fam) {
  if (a.stats || a.bnb_x) launch_shape<AK, BK, true, EPI_ON>(a, s, fam);
  else launch_shape<AK, BK, true, EPI_PLAIN>(a, s, fam);
}

}  // namespace

}  // namespace tfx
