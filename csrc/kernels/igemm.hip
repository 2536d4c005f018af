// Implicit-GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16) for gfx950.
//
// One template covers every matmul-shaped op of the framework.  An operand is described by its
// KIND (how its tile is gathered from global memory) and is staged either K-major or MN-major:
//   K-major kinds  (LDS image [rows][64 k], fragments by ds_read_b128):
//     KM_DENSE     A[m*ld + k]
//     KM_FWD_X     im2col(X) of an NHWC conv forward, gathered on the fly
//     KM_DGRAD_DY  gather of dY for the conv data-gradient (stride via parity test)
//   MN-major kinds (LDS image [64 k][cols], fragments by ds_read_b64_tr_b16, no transpose pass):
//     MN_DENSE     A[k*ld + m]                (also dY^T for the weight gradient)
//     MN_DGRAD_W   W[ko][r][s][c] read as B(k=(r,s,ko), n=c)
//     MN_WGRAD_X   im2col(X) rows j=(n,p,q), columns (r,s,c)
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
#include "tfx_common.h"
#include "tfx_kernels.h"

#include <cstdio>
#include <cstdlib>

namespace tfx {

namespace {

enum { KM_DENSE = 0, KM_FWD_X = 1, KM_DGRAD_DY = 2, MN_DENSE = 10, MN_DGRAD_W = 11, MN_WGRAD_X = 12,
       MN_DGRAD_W2 = 13 };
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

__device__ __forceinline__ bf16x8_t lds_read_kmaj(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(img + kmaj_off(row, chunk));
}

// fragment of an MN-major image: lane needs X[col = cb + (l&15)][k = 32kk + 8(l>>4) + j], j = 0..7
template <int COLS>
__device__ __forceinline__ bf16x8_t lds_read_mn(const char* img, int cb, int kk, int lane) {
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, p = ii & 3;
  const int chunk = (cb >> 3) + (p >> 1);
  s4_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kr = 32 * kk + 8 * g + 4 * h + q;
    const int off = mn_off<COLS>(kr, chunk) + (p & 1) * 8;
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)((__attribute__((address_space(3))) char*)img + off));
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
__device__ __forceinline__ int mul24(int a, int b) { return (int)__umul24((unsigned)a, (unsigned)b); }

template <int KIND, int ROWS>
struct Loader {
  static constexpr bool KM = is_kmaj(KIND);
  static constexpr int NP = ROWS / 32;          // 16-B loads per thread per tile
  static constexpr int CH = ROWS / 8;           // MN-major chunks per k-row
  static_assert(KM || CH == 4 * NP, "MN-major: 4 threads per k-row");
  int c0;        // K-major: element offset of chunk in k (8*kc)
  int r0;        // K-major: first row; MN-major: the k-row
  int ctx0[NP], ctx1[NP], ctx2[NP], base[NP];
  int col[NP];                     // MN-major: column of chunk j (-1: out of range)
  int cr[NP], cs[NP], cc[NP];      // MN_WGRAD_X column decode per chunk
  int t3_;                         // MN-major: first chunk (t & 3) of the k-row

  __device__ __forceinline__ void init(const IgemmArgs& a, int base0, int lim, int ld, int t) {
    if constexpr (KM) {
      c0 = 8 * (t & 7);
      r0 = t >> 3;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int row = base0 + r0 + 32 * i;
        const bool ok = row < lim;
        if constexpr (KIND == KM_DENSE) {
          ctx0[i] = ok ? 0 : -1;
          base[i] = row * ld;
        } else {
          const int GY = KIND == KM_FWD_X ? a.P : a.H, GX = KIND == KM_FWD_X ? a.Q : a.W;
          int n = row / (GY * GX), yx = row - n * GY * GX, y = yx / GX, x = yx - y * GX;
          // rows past M get a y far out of range: every bounds test below then fails (no flag register)
          constexpr int FAR = -(1 << 28);
          if constexpr (KIND == KM_FWD_X) {
            ctx1[i] = ok ? y * a.sh - a.ph : FAR;
            ctx2[i] = x * a.sw - a.pw;
            // element offset of (n, iy0, ix0, 0): may be negative (padding), only used when in range
            base[i] = ((n * a.H + y * a.sh - a.ph) * a.W + ctx2[i]) * a.C;
          } else {
            ctx1[i] = ok ? y + a.ph : FAR;
            ctx2[i] = x + a.pw;
            base[i] = n * a.P;
          }
        }
      }
    } else {
      r0 = t >> 2;
      t3_ = t & 3;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int cj = base0 + 8 * ((t & 3) + 4 * j);
        col[j] = cj < lim ? cj : -1;
        if constexpr (KIND == MN_DENSE) base[j] = r0 * ld + cj;
        if constexpr (KIND == MN_WGRAD_X) {
          const int rs = cj < lim ? cj / a.C : 0;
          cc[j] = cj - rs * a.C;
          cr[j] = rs / a.S;
          cs[j] = rs - cr[j] * a.S;
        }
      }
    }
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
__device__ __forceinline__ bf16x8_t frag(const char* img, int rowbase, int kk, int lane) {
  if constexpr (is_kmaj(KIND)) return lds_read_kmaj(img, rowbase + (lane & 15), 4 * kk + (lane >> 4));
  else return lds_read_mn<ROWS>(img, rowbase, kk, lane);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
  const int n = bytes > 0x7fffffff ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, n, 0x00020000);
}

// ------------------------------------------------------------------ fused-BN last arriver
// Every block of column tile tn has added its per-column partials into the slots.  The payload is
// written ONLY by agent-scope atomics (performed past the XCD L2, which drops the line), so the
// hand-off needs no L2 writeback (MI355X_MICROARCH.md "Correctness boundaries", sc1 table row 1):
// every wave drains vmcnt, barrier, ONE lane bumps the tile's counter; the block whose add returns
// tiles_m - 1 is last and its waves read the slots with sc1 loads after a barrier.  An agent release
// (buffer_wbl2) per block here would write back the freshly stored output tile of every block on the
// XCD: measured 2-6x slower conv kernels.  The host only fuses when the tile's slot columns are whole
// 128-B lines (N % 32 == 0), so no block ever loads a line holding another tile's pending sums.
// The last arriver sums the NSLOT slot rows of the tile's columns, re-zeroes them (sc1 stores: the
// lines leave the L2 again) and resets the counter, so the workspace is zero between uses.
// FWD: finalize the BN of the columns (bn_finalize_kernel's math); BWD: red + dgamma / dbeta.
template <int BN, bool BWD>
__device__ __forceinline__ void bn_tile_reduce(const IgemmArgs& a, int tn, int n0, char* smem, int t) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* flag = reinterpret_cast<unsigned*>(smem + 8192);  // past the [2][BN][2] f32 partials
  if (t == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.bn_cnt + tn, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == (unsigned)(a.tiles_m - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (*flag == 0) return;
  constexpr int NPH = 256 / BN;  // slot phases per column
  const int cl = t % BN, ph = t / BN, c = n0 + cl;
  float* slots = BWD ? a.bnb_slots : a.stats;
  float s = 0.f, q = 0.f;
  if (c < a.N) {
    // 8 slot rows in flight per step (bounded registers: this runs in every fused-BN kernel)
    constexpr int CH = NSLOT / NPH < 8 ? NSLOT / NPH : 8;
    for (int k0 = 0; k0 < NSLOT / NPH; k0 += CH) {
      float vs[CH], vq[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        float* row = slots + (size_t)(ph + (k0 + k) * NPH) * 2 * a.N;
        vs[k] = __hip_atomic_load(row + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vq[k] = __hip_atomic_load(row + a.N + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        s += vs[k];
        q += vq[k];
        float* row = slots + (size_t)(ph + (k0 + k) * NPH) * 2 * a.N;
        __hip_atomic_store(row + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(row + a.N + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  float* part = reinterpret_cast<float*>(smem);
  part[(ph * BN + cl) * 2] = s;
  part[(ph * BN + cl) * 2 + 1] = q;
  __syncthreads();
  if (t < BN && c < a.N) {
    s = 0.f;
    q = 0.f;
#pragma unroll
    for (int k = 0; k < NPH; ++k) {
      s += part[(k * BN + t) * 2];
      q += part[(k * BN + t) * 2 + 1];
    }
    const int C = a.N;
    if constexpr (BWD) {
      a.bnb_red[c] = s;
      a.bnb_red[C + c] = q;
      if (a.bnb_dbeta) a.bnb_dbeta[c] += s;
      if (a.bnb_dgamma) a.bnb_dgamma[c] += q;
    } else {
      const float inv_m = 1.f / (float)a.M;
      const float mean = s * inv_m;
      const float var = fmaxf(q * inv_m - mean * mean, 0.f);
      const float invstd = rsqrtf(var + a.bn_eps);
      const float scale = (a.bn_gamma ? a.bn_gamma[c] : 1.f) * invstd;
      a.bn_save[c] = mean;
      a.bn_save[C + c] = invstd;
      a.bn_save[2 * C + c] = scale;
      a.bn_save[3 * C + c] = (a.bn_beta ? a.bn_beta[c] : 0.f) - mean * scale;
      if (a.bn_rmean) {
        const float unb = a.M > 1 ? var * (float)a.M / (float)(a.M - 1) : var;
        a.bn_rmean[c] = (1.f - a.bn_momentum) * a.bn_rmean[c] + a.bn_momentum * mean;
        a.bn_rvar[c] = (1.f - a.bn_momentum) * a.bn_rvar[c] + a.bn_momentum * unb;
      }
    }
  }
  if (t == 0) __hip_atomic_store(a.bn_cnt + tn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// SWAP: compute the transposed tile (MFMA operands exchanged) so each lane holds 4 CONSECUTIVE
// output columns of one row: bf16 outputs leave as one 8-byte store per 16x16 tile per lane, and
// transposed f32 outputs (dW^T) as 16-lane contiguous runs.  Plain f32 atomics keep SWAP=false
// (4 rows x 16 contiguous columns per instruction).
// STG = LDS stages: 2 for the pipelined K loop; 1 for single-k-tile GEMMs (K <= 64: the 1x1 convs
// of 64-channel layers), which then fit 4 blocks per CU -- those are memory-bound, and occupancy is
// what keeps enough loads and stores in flight.
// EPI: compile-time epilogue extras (so the plain GEMM / wgrad kernels carry none of their code or
// registers): EPI_STATS = fused BN statistics (+ last-arriver finalize) of a conv forward,
// EPI_BNB = fused BN-backward partials (+ last-arriver reduce) of a conv data gradient.
// KS = 2: in-block split-K for the f32-atomic weight gradients.  512 threads = two 4-wave groups
// on the SAME output tile, each running the pipelined K loop over half of the block's k-tiles in its
// own LDS stages; group 1 hands its accumulators to group 0 through LDS and only group 0 issues the
// atomics.  Twice the loads in flight per CU (these GEMMs are latency-bound at one 4-wave block per
// CU) for the SAME atomic bytes -- splitting across blocks instead doubles the f32 atomic traffic,
// which runs at ~1.3 TB/s chip-wide (MI355X_MICROARCH.md "Global float atomics").
template <int AKIND, int BKIND, int BM, int BN, bool SWAP, int STG, int EPI, int KS = 1>
__global__ void __launch_bounds__(256 * KS, KS == 2 ? 1 : ((STG == 1 && EPI != EPI_BNB) ? (BM * BN >= 128 * 128 ? 3 : 4) : 2)) igemm_kernel(IgemmArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * BKT * 2, STAGE = (BM + BN) * BKT * 2;
  static_assert(KS == 1 || (KS == 2 && EPI == EPI_PLAIN && STG == 2), "in-block split-K: plain pipelined kernels");
  static_assert(KS == 1 || TM * TN * 4 * 256 * 4 <= STG * STAGE, "accumulator hand-off must fit a group's stages");
  __shared__ __attribute__((aligned(16))) char smem_all[KS * STG * STAGE];
  const int grp = KS == 2 ? (int)(threadIdx.x >> 8) : 0;
  char* smem = smem_all + grp * (STG * STAGE);
  const int t = threadIdx.x & 255, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
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

  Loader<AKIND, BM> la;
  Loader<BKIND, BN> lb;
  la.init(a, m0, a.M, a.lda, t);
  lb.init(a, n0, a.N, a.ldb, t);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.A, a.a_bytes), rb = make_rsrc(a.B, a.b_bytes);

  u32x4_t sa0[Loader<AKIND, BM>::NP], sb0[Loader<BKIND, BN>::NP];
  u32x4_t sa1[Loader<AKIND, BM>::NP], sb1[Loader<BKIND, BN>::NP];
  uint32_t oa[Loader<AKIND, BM>::NP], ob[Loader<BKIND, BN>::NP];

  // tiles at or past kt1 are zero-filled (every offset BAD), so an odd tile count can run the
  // even/odd loop to completion: the extra step multiplies zeros.
  const int kend = min(a.K, min(kt1, kt0 + kh) * BKT);
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

  auto compute = [&](int st) {
    const char* ia = smem + st * STAGE;
    const char* ib = ia + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag<AKIND, BM>(ia, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag<BKIND, BN>(ib, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (SWAP) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    }
  };

  if constexpr (STG == 1) {  // host guarantees a single k-tile
    issue(kt0, sa0, sb0);
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
    compute(0);
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
    float* xch = reinterpret_cast<float*>(smem_all + STG * STAGE);
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) xch[((i * TN + j) * 4 + r) * 256 + t] = acc[i][j][r];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += xch[((i * TN + j) * 4 + r) * 256 + t];
  }

  // Element (m, n) of lane's acc[i][j][r]:
  //   SWAP : m = mb + i*16 + (lane&15),        n = nb + j*16 + (lane>>4)*4 + r
  //   !SWAP: m = mb + i*16 + (lane>>4)*4 + r,  n = nb + j*16 + (lane&15)
  const int mb = m0 + wm * WM, nb = n0 + wn * WN;

  // ---------------- fused BN statistics of the bf16-rounded output (per column n, this tile's rows)
  if constexpr (STG == 1) {
    // single-k-tile variant: no barrier after compute(0) -- other waves may still be reading the
    // stage that the epilogue's LDS partials overwrite
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
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = min(mb + i * 16 + (lane & 15), a.M - 1);
      int row = m;
      if (a.cls) {
        const int n = a.fd_cHW.div(m), yx = m - n * a.H * a.W, y = a.fd_cW.div(yx), x = yx - y * a.W;
        row = (n * a.out_H + 2 * y + a.cph) * a.out_W + 2 * x + a.cpw;
      }
      rowoff[i] = (int64_t)row * a.ldc;
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
        if constexpr (bnb) {
          const int nc = min(n, a.N - 8);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            mu[k] = a.bnb_save[nc + k];
            is[k] = a.bnb_save[a.N + nc + k];
            sc[k] = a.bnb_save[2 * a.N + nc + k];
            sh[k] = a.bnb_save[3 * a.N + nc + k];
          }
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
            const int64_t o = rowoff[i0 + ii] + nl;
            if (a.addend) {
              adv[ii] = *reinterpret_cast<const U4*>(a.addend + o);
              amv[ii] = a.addend_mask ? a.addend_mask[o >> 3] : 0xffu;
            }
            if constexpr (bnb) {
              xvv[ii] = *reinterpret_cast<const U4*>(a.bnb_x + o);
              mbv[ii] = a.bnb_mask ? a.bnb_mask[o >> 3] : 0xffu;
            }
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
              uint16_t* dst = Cb + rowoff[i] + n;
              if (a.addend) {  // fused residual-branch gradient sum (dX = dgrad + other branch)
                float ad[8];
                unpack8(adv[ii], ad);
#pragma unroll
                for (int r = 0; r < 8; ++r) o[r] += ((amv[ii] >> r) & 1u) ? ad[r] : 0.f;
              }
              const U4 packed = pack8(o);
              *reinterpret_cast<U4*>(dst) = packed;
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
                // g' = bf16(out) * relu mask; xhat from the BN input x (same NHWC position)
                float g[8], xv[8];
                unpack8(packed, g);
                unpack8(xvv[ii], xv);
                const uint32_t mbits = mbv[ii];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                  bool on = true;
                  if (a.bnb_relu) on = a.bnb_mask ? ((mbits >> k) & 1u) != 0 : fmaf(xv[k], sc[k], sh[k]) > 0.f;
                  const float gg = on ? g[k] : 0.f;
                  bs[k] += gg;
                  bq[k] = fmaf(gg, (xv[k] - mu[k]) * is[k], bq[k]);
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
            float* slot = (bnb ? a.bnb_slots : a.stats) + (size_t)(tm % NSLOT) * 2 * a.N;
            atomicAdd(&slot[nn], red[t * 2] + red[(BN + t) * 2]);
            atomicAdd(&slot[a.N + nn], red[t * 2 + 1] + red[(BN + t) * 2 + 1]);
          }
        }
        if (a.bn_final) bn_tile_reduce<BN, bnb>(a, tn, n0, smem, t);
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
namespace {

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
  static const int want = [] {
    const char* e = getenv("TFX_SPLITK_BLOCKS");
    return e ? atoi(e) : 256;  // one block per CU: measured best (fewer f32 atomic partials)
  }();
  if (a.out_mode == OUT_F32_ATOMIC) splits = pick_splits(tiles, nkt, want * want_mult, min_kps);
  a.kps = (nkt + splits - 1) / splits;
  if constexpr (KS == 2) {
    // each 4-wave group takes kps/2 k-tiles: a multiple of 4 keeps both halves even (no zero step).
    // An 8-wave block holds its CU's LDS alone, so more blocks than CUs would run a second wave
    // (e.g. 144 tiles x 2 splits): the 4-wave form fits those at two blocks per CU.
    if (a.kps < 4 || tiles * splits > want) return launch_t<AK, BK, BM, BN, EPI, 1>(a, s, want_mult, min_kps);
    a.kps = (a.kps + 3) & ~3;
  } else if (splits > 1) {
    a.kps += a.kps & 1;  // even k-tiles per split: no zero step in the loop
  }
  splits = (nkt + a.kps - 1) / a.kps;
  const int grid = tiles * splits;
  if (grid == 0) return;
  // transposed MFMA orientation for bf16 outputs and transposed stores (see kernel comment)
  const bool swap = a.out_mode == OUT_BF16 || a.trans_out;
  if constexpr (KS == 2) {
    if (swap) igemm_kernel<AK, BK, BM, BN, true, 2, EPI_PLAIN, 2><<<grid, 2 * NT, 0, s>>>(a);
    else igemm_kernel<AK, BK, BM, BN, false, 2, EPI_PLAIN, 2><<<grid, 2 * NT, 0, s>>>(a);
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
// twice the blocks for the same K loop.  TFX_TILE_POLICY=0 disables the under-fill rule (A/B).
int tile_policy() {
  static const int p = [] {
    const char* e = getenv("TFX_TILE_POLICY");
    return e ? atoi(e) : 1;
  }();
  return p;
}

// weight gradients (split-K, f32 atomics): 128x64 tiles at twice the block target keep the same
// splits (same atomic traffic) but put two blocks on each CU for latency hiding.  Measured: -25 %
// on the 1x1 (dense x dense) weight gradients, +3..8 % on the im2col-gathered 3x3 ones, so the
// default (0 = auto) uses it for the dense pair only; TFX_WGRAD_TILE=64/128 forces one (A/B).
int wgrad_tile() {
  static const int t = [] {
    const char* e = getenv("TFX_WGRAD_TILE");
    return e ? atoi(e) : 0;
  }();
  return t;
}

// in-block split-K for the weight gradients (TFX_WGRAD_KS=1 restores one 4-wave group per block)
int wgrad_ks() {
  static const int k = [] {
    const char* e = getenv("TFX_WGRAD_KS");
    return e ? atoi(e) : 2;
  }();
  return k;
}

// min k-tiles per split for the skinny GEMM path (TFX_SKINNY_KPS; 0 disables the path)
int skinny_min_kps() {
  static const int k = [] {
    const char* e = getenv("TFX_SKINNY_KPS");
    return e ? atoi(e) : 2;
  }();
  return k;
}

template <int AK, int BK, bool ALLOW256 = true, int EPI = EPI_PLAIN>
void launch_shape(IgemmArgs& a, hipStream_t s) {
  if constexpr (!ALLOW256) {
    const bool dense_pair = (AK == MN_DENSE && BK == MN_DENSE) || (a.R == 1 && a.S == 1);  // 1x1 (any stride)
    if (wgrad_ks() == 2) {
      // 8-wave blocks, one per CU: 128x64 tiles for the dense pair (half the atomic bytes of the
      // 2-blocks-per-CU 128x64 form), 128x128 for the im2col-gathered ones
      if (a.N <= 64 || (dense_pair && wgrad_tile() != 128) || wgrad_tile() == 64)
        return launch_t<AK, BK, 128, 64, EPI, 2>(a, s);
      return launch_t<AK, BK, 128, 128, EPI, 2>(a, s);
    }
    if (a.N > 64 && (wgrad_tile() == 64 || (wgrad_tile() == 0 && dense_pair))) return launch_t<AK, BK, 128, 64, EPI>(a, s, 2);
  }
  if (a.N <= 64) {
    if constexpr (ALLOW256) {
      if (a.M >= 256 * 256) return launch_t<AK, BK, 256, 64, EPI>(a, s);
    }
    launch_t<AK, BK, 128, 64, EPI>(a, s);
  } else {
    const long tiles128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128);
    if constexpr (ALLOW256) {
      if (tile_policy() >= 1 && tiles128 < 512) return launch_t<AK, BK, 128, 64, EPI>(a, s);
    }
    launch_t<AK, BK, 128, 128, EPI>(a, s);
  }
}

}  // namespace

template <int AK, int BK, int EPI_ON>
void launch_epi(IgemmArgs& a, hipStream_t s) {
  if (a.stats || a.bnb_x) launch_shape<AK, BK, true, EPI_ON>(a, s);
  else launch_shape<AK, BK, true, EPI_PLAIN>(a, s);
}

void igemm_launch(IgemmArgs a, int mode, hipStream_t s) {
  if (a.out_mode == OUT_F32_ATOMIC && a.zero_out) {
    const size_t rows = a.trans_out ? a.N : a.M;
    TFX_HIP_CHECK(hipMemsetAsync(a.Cp, 0, sizeof(float) * rows * a.ldc, s));
  }
  // a masked addend is applied only by the bf16 16-byte-store epilogue path
  if (a.addend_mask && !(a.addend && a.out_mode == OUT_BF16 && !a.trans_out && (a.ldc & 7) == 0 && (a.N & 7) == 0)) {
    fprintf(stderr, "igemm_launch: masked addend needs a bf16 output with 8-aligned columns\n");
    abort();
  }
  // fused-BN epilogues live in the bf16 16-byte-store path of the forward / data-gradient kernels
  if (a.stats || a.bnb_x) {
    if (!(a.out_mode == OUT_BF16 && !a.trans_out && (a.ldc & 7) == 0 && (a.N & 7) == 0 &&
          (mode == MODE_FWD || (a.bnb_x && mode == MODE_DGRAD)) && (a.stats == nullptr || a.bnb_x == nullptr))) {
      fprintf(stderr, "igemm_launch: unsupported fused-BN epilogue configuration\n");
      abort();
    }
  }
  // 1x1 stride-1 unpadded convs (two thirds of ResNet-50's) are plain GEMMs over the NHWC rows:
  // dense loaders instead of the im2col / parity gathers -- no per-row address decode at all.
  const bool pointwise = mode != MODE_GEMM && a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 &&
                         a.pw == 0;
  if (pointwise) {
    switch (mode) {
      case MODE_FWD:  // X[M][C] . W[Ko][C]^T
        a.lda = a.C; a.ldb = a.C;
        launch_epi<KM_DENSE, KM_DENSE, EPI_STATS>(a, s);
        return;
      case MODE_DGRAD:  // dY[M][Ko] . W[Ko][C]
        a.lda = a.Ko; a.ldb = a.C;
        launch_epi<KM_DENSE, MN_DENSE, EPI_BNB>(a, s);
        return;
      case MODE_WGRAD:  // dY^T[Ko][pix] . X[pix][C]
        a.lda = a.Ko; a.ldb = a.C;
        launch_shape<MN_DENSE, MN_DENSE, false>(a, s);
        return;
      case MODE_WGRAD_T:  // X^T[C][pix] . dY[pix][Ko]
        a.lda = a.C; a.ldb = a.Ko;
        launch_shape<MN_DENSE, MN_DENSE, false>(a, s);
        return;
      case MODE_DGRAD_CLS:
        // single-tap class aligned with dY (1x1 stride-2 even pixels, 3x3 stride-2 (even, even)):
        // dY[M][Ko] . W[:, tap, :] -- dense operands, the tap folded into B's base; rows remapped
        if (a.H == a.P && a.W == a.Q) {
          const int64_t tap_off = (int64_t)(a.cr0 * a.wS + a.cs0) * a.C;
          a.B += tap_off;
          a.b_bytes -= tap_off * 2;
          a.lda = a.Ko; a.ldb = a.wR * a.wS * a.C;
          launch_shape<KM_DENSE, MN_DENSE>(a, s);
          return;
        }
        break;
    }
  }
  switch (mode) {
    case MODE_FWD: launch_epi<KM_FWD_X, KM_DENSE, EPI_STATS>(a, s); break;
    case MODE_DGRAD: launch_epi<KM_DGRAD_DY, MN_DGRAD_W, EPI_BNB>(a, s); break;
    case MODE_DGRAD_CLS: launch_shape<KM_DGRAD_DY, MN_DGRAD_W2>(a, s); break;
    case MODE_WGRAD: launch_shape<MN_DENSE, MN_WGRAD_X, false>(a, s); break;
    case MODE_WGRAD_T: launch_shape<MN_WGRAD_X, MN_DENSE, false>(a, s); break;
    default:
      // skinny f32-accumulated GEMMs (the recurrent h @ W_hh^T / dgates @ W_hh of an LSTM step:
      // M = batch <= 128, a few thousand columns): latency-bound, so cut them into many short
      // blocks -- 128x64 tiles, split-K down to min_kps k-tiles per block
      if (a.out_mode == OUT_F32_ATOMIC && a.M <= 128 && skinny_min_kps() > 0) {
        const int mk = skinny_min_kps();
        if (a.a_kmajor && a.b_kmajor) launch_t<KM_DENSE, KM_DENSE, 128, 64>(a, s, 1, mk);
        else if (a.a_kmajor) launch_t<KM_DENSE, MN_DENSE, 128, 64>(a, s, 1, mk);
        else if (a.b_kmajor) launch_t<MN_DENSE, KM_DENSE, 128, 64>(a, s, 1, mk);
        else launch_t<MN_DENSE, MN_DENSE, 128, 64>(a, s, 1, mk);
        return;
      }
      if (a.a_kmajor && a.b_kmajor) launch_t<KM_DENSE, KM_DENSE, 128, 128>(a, s);
      else if (a.a_kmajor) launch_t<KM_DENSE, MN_DENSE, 128, 128>(a, s);
      else if (a.b_kmajor) launch_t<MN_DENSE, KM_DENSE, 128, 128>(a, s);
      else launch_t<MN_DENSE, MN_DENSE, 128, 128>(a, s);
  }
}

}  // namespace tfx
