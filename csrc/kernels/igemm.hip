// Implicit-GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16) for gfx950.
//
// One template covers every matmul-shaped op of the framework:
//   MODE_GEMM : C[M][N] = sum_k A(m,k) B(k,n), A/B each K-major or MN-major (dense, any ld)
//   MODE_FWD  : NHWC conv forward     A = im2col(X) gathered on the fly, B = W [Ko][R*S*C]
//   MODE_DGRAD: NHWC conv data-grad   A = gather(dY) (stride handled by parity test),
//                                     B = W read MN-major (no weight transpose pass)
//   MODE_WGRAD: NHWC conv weight-grad A = dY^T (MN-major), B = im2col(X) MN-major, split-K
//                                     over N*P*Q with f32 atomic accumulation into dW
//
// Block tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 MFMA tiles.
// LDS images (two stages, 64 KiB):
//   K-major operand  [128 rows][64 k]  128-B rows, 16-B chunk c of row r at c ^ (r&7)
//                    -> fragment reads are ds_read_b128, conflict-free (T2 swizzle)
//   MN-major operand [64 k][128 cols] 256-B rows, chunk c of row r at c ^ f(r),
//                    f(r) = ((r&3)<<2)|((r>>2)&3) -> fragments via ds_read_b64_tr_b16 (T10),
//                    conflict-free per 32-lane half.
// Register-staged double buffer: the next tile's global loads are issued before the MFMAs of
// the current tile and written to the other LDS stage after them (T14), one barrier per tile.
// blockIdx is remapped XCD-aware (T1).  Reference: the matmuls of R/distributed/distributed.py:96-98
// and their TF1 gradients; conv/FC layers of the north-star models (BASELINE.json configs 2-5).
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

constexpr int BM = 128, BN = 128, BKT = 64, NT = 256;
constexpr int STAGE_BYTES = 2 * 16384;  // A + B image per stage

typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4;

__device__ __forceinline__ int kmaj_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }
__device__ __forceinline__ int mnmaj_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int mnmaj_off(int r, int c) { return r * 256 + ((c ^ mnmaj_swz(r)) << 4); }

__device__ __forceinline__ bf16x8_t lds_read_kmaj(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8_t*>(img + kmaj_off(row, chunk));
}

// fragment of the MN-major image: lane needs X[col = cb + (l&15)][k = 32kk + 8(l>>4) + j], j=0..7
__device__ __forceinline__ bf16x8_t lds_read_mnmaj(const char* img, int cb, int kk, int lane) {
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, p = ii & 3;
  const int chunk = (cb >> 3) + (p >> 1);
  s4_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kr = 32 * kk + 8 * g + 4 * h + q;
    const int off = kr * 256 + ((chunk ^ mnmaj_swz(kr)) << 4) + (p & 1) * 8;
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)((__attribute__((address_space(3))) char*)img + off));
  }
  typedef short s8_t __attribute__((ext_vector_type(8)));
  s8_t r = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

__device__ __forceinline__ U4 ldg16(const uint16_t* p, bool ok) {
  if (ok) return *reinterpret_cast<const U4*>(p);
  U4 z = {0u, 0u, 0u, 0u};
  return z;
}

}  // namespace

template <int MODE, bool AK, bool BK>
__global__ void __launch_bounds__(256, 2) igemm_kernel(IgemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_mn = a.tiles_m * a.tiles_n;
  const int split = bid / tiles_mn;
  const int rem = bid - split * tiles_mn;
  const int tm = rem / a.tiles_n, tn = rem - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nkt = (a.K + BKT - 1) / BKT;
  const int kt0 = split * a.kps;
  const int kt1 = min(nkt, kt0 + a.kps);
  if (kt0 >= kt1) return;

  // ---------------- per-thread loader context (fixed for the whole block)
  // K-major tiles: chunk c = t&7, rows (t>>3) + 32*i ; MN-major tiles: chunk c = t&15, rows (t>>4) + 16*i
  const int kc = t & 7, kr = t >> 3;
  const int mc = t & 15, mr = t >> 4;
  // A context
  int64_t a_row[4];  // GEMM K-major: element offset of row; FWD/DGRAD: packed n (or -1)
  int a_y[4], a_x[4];
  if constexpr (AK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + kr + 32 * i;
      if constexpr (MODE == MODE_GEMM) {
        a_row[i] = m < a.M ? (int64_t)m * a.lda : -1;
      } else {
        // m -> (n, oy, ox) over the GEMM-M spatial grid: FWD uses (P,Q), DGRAD uses (H,W)
        const int GY = MODE == MODE_FWD ? a.P : a.H, GX = MODE == MODE_FWD ? a.Q : a.W;
        if (m < a.M) {
          const int n = m / (GY * GX), yx = m - n * GY * GX, y = yx / GX, x = yx - y * GX;
          a_row[i] = n;
          if constexpr (MODE == MODE_FWD) {
            a_y[i] = y * a.sh - a.ph;
            a_x[i] = x * a.sw - a.pw;
          } else {
            a_y[i] = y + a.ph;
            a_x[i] = x + a.pw;
          }
        } else {
          a_row[i] = -1;
          a_y[i] = a_x[i] = 0;
        }
      }
    }
  }
  // A MN-major: column chunk fixed
  const int a_col = m0 + 8 * mc;
  const bool a_col_ok = a_col < a.M;
  // B K-major: rows n
  int64_t b_row[4];
  if constexpr (BK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + kr + 32 * i;
      b_row[i] = n < a.N ? (int64_t)n * a.ldb : -1;
    }
  }
  // B MN-major: column chunk fixed
  const int b_col = n0 + 8 * mc;
  const bool b_col_ok = b_col < a.N;
  int b_r = 0, b_s = 0, b_c = 0;
  if constexpr (MODE == MODE_WGRAD) {
    if (b_col_ok) {
      const int rs = b_col / a.C;
      b_c = b_col - rs * a.C;
      b_r = rs / a.S;
      b_s = rs - b_r * a.S;
    }
  }

  U4 ra[4], rb[4];

  auto load_tile = [&](int kt) {
    const int k0 = kt * BKT;
    // ---------------- A
    if constexpr (AK) {
      const int k = k0 + 8 * kc;
      const bool kok = k < a.K;
      if constexpr (MODE == MODE_GEMM) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[i] = ldg16(a.A + a_row[i] + k, kok && a_row[i] >= 0);
      } else if constexpr (MODE == MODE_FWD) {
        const int rs = a.fd_C.div(k), cc = k - rs * a.C, r = a.fd_S.div(rs), s = rs - r * a.S;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int iy = a_y[i] + r * a.dh, ix = a_x[i] + s * a.dw;
          const bool ok = kok && a_row[i] >= 0 && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
          const int64_t off = ok ? (((int64_t)a_row[i] * a.H + iy) * a.W + ix) * a.C + cc : 0;
          ra[i] = ldg16(a.A + off, ok);
        }
      } else {  // DGRAD: A = dY[n][p][q][ko], k = (r,s,ko)
        const int rs = a.fd_Ko.div(k), ko = k - rs * a.Ko, r = a.fd_S.div(rs), s = rs - r * a.S;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ty = a_y[i] - r * a.dh, tx = a_x[i] - s * a.dw;
          bool ok = kok && a_row[i] >= 0 && ty >= 0 && tx >= 0;
          int p = 0, q = 0;
          if (ok) {  // strides are powers of two (checked on the host)
            p = ty >> a.sh_log2;
            q = tx >> a.sw_log2;
            ok = ((p << a.sh_log2) == ty) && ((q << a.sw_log2) == tx) && p < a.P && q < a.Q;
          }
          const int64_t off = ok ? (((int64_t)a_row[i] * a.P + p) * a.Q + q) * a.Ko + ko : 0;
          ra[i] = ldg16(a.A + off, ok);
        }
      }
    } else {
      // MN-major A: rows are k
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + mr + 16 * i;
        const bool ok = a_col_ok && k < a.K;
        // GEMM: A[k*lda + m]; WGRAD: dY[j*Ko + ko] (lda = Ko)
        ra[i] = ldg16(a.A + (ok ? (int64_t)k * a.lda + a_col : 0), ok);
      }
    }
    // ---------------- B
    if constexpr (BK) {
      const int k = k0 + 8 * kc;
      const bool kok = k < a.K;
#pragma unroll
      for (int i = 0; i < 4; ++i) rb[i] = ldg16(a.B + b_row[i] + k, kok && b_row[i] >= 0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + mr + 16 * i;
        bool ok = b_col_ok && k < a.K;
        int64_t off = 0;
        if constexpr (MODE == MODE_GEMM) {
          off = (int64_t)k * a.ldb + b_col;
        } else if constexpr (MODE == MODE_DGRAD) {
          // B(k=(r,s,ko), c) = W[ko][r][s][c]
          const int rs = a.fd_Ko.div(k), ko = k - rs * a.Ko, r = a.fd_S.div(rs), s = rs - r * a.S;
          off = (((int64_t)ko * a.R + r) * a.S + s) * a.C + b_col;
        } else if constexpr (MODE == MODE_WGRAD) {
          // B(k=j=(n,p,q), col=(r,s,c)) = X[n][p*sh-ph+r*dh][q*sw-pw+s*dw][c]
          const int PQ = a.P * a.Q;
          const int n = a.fd_PQ.div(k), pq = k - n * PQ, p = a.fd_Q.div(pq), q = pq - p * a.Q;
          const int iy = p * a.sh - a.ph + b_r * a.dh, ix = q * a.sw - a.pw + b_s * a.dw;
          ok = ok && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
          off = (((int64_t)n * a.H + iy) * a.W + ix) * a.C + b_c;
        }
        rb[i] = ldg16(a.B + (ok ? off : 0), ok);
      }
    }
  };

  auto store_tile = [&](int stage) {
    char* ia = smem + stage * STAGE_BYTES;
    char* ib = ia + 16384;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (AK) *reinterpret_cast<U4*>(ia + kmaj_off(kr + 32 * i, kc)) = ra[i];
      else *reinterpret_cast<U4*>(ia + mnmaj_off(mr + 16 * i, mc)) = ra[i];
      if constexpr (BK) *reinterpret_cast<U4*>(ib + kmaj_off(kr + 32 * i, kc)) = rb[i];
      else *reinterpret_cast<U4*>(ib + mnmaj_off(mr + 16 * i, mc)) = rb[i];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  load_tile(kt0);
  store_tile(0);
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const int stage = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) load_tile(kt + 1);
    const char* ia = smem + stage * STAGE_BYTES;
    const char* ib = ia + 16384;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (AK) fa[i] = lds_read_kmaj(ia, wm * 64 + i * 16 + (lane & 15), 4 * kk + (lane >> 4));
        else fa[i] = lds_read_mnmaj(ia, wm * 64 + i * 16, kk, lane);
        if constexpr (BK) fb[i] = lds_read_kmaj(ib, wn * 64 + i * 16 + (lane & 15), 4 * kk + (lane >> 4));
        else fb[i] = lds_read_mnmaj(ib, wn * 64 + i * 16, kk, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_tile(stage ^ 1);
    __syncthreads();
  }

  // ---------------- fused BN statistics of the bf16-rounded output (per column, this tile's rows)
  if (a.stats) {
    float cs[4], cq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[j] = 0.f;
      cq[j] = 0.f;
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      const float bias = (a.bias && n < a.N) ? a.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          v = bf16_to_f32(f32_to_bf16(v));
          if (m < a.M) {
            cs[j] += v;
            cq[j] = fmaf(v, v, cq[j]);
          }
        }
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    float* red = reinterpret_cast<float*>(smem);  // [2 wm][128 cols][2]; LDS is free after the loop
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + lane;
        red[(wm * 128 + col) * 2 + 0] = cs[j];
        red[(wm * 128 + col) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (t < 128) {
      const int n = n0 + t;
      if (n < a.N) {
        float* slot = a.stats + (size_t)(tm % NSLOT) * 2 * a.N;
        atomicAdd(&slot[n], red[t * 2] + red[(128 + t) * 2]);
        atomicAdd(&slot[a.N + n], red[t * 2 + 1] + red[(128 + t) * 2 + 1]);
      }
    }
  }

  // ---------------- epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each 16x16 tile
  const int col_l = lane & 15, row_l = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + col_l;
    if (n >= a.N) continue;
    const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + row_l + r;
        if (m >= a.M) continue;
        float v = acc[i][j][r] + bias;
        if (a.relu) v = fmaxf(v, 0.f);
        const int64_t o = (int64_t)m * a.ldc + n;
        if (a.out_mode == OUT_BF16) reinterpret_cast<uint16_t*>(a.Cp)[o] = f32_to_bf16(v);
        else if (a.out_mode == OUT_F32) reinterpret_cast<float*>(a.Cp)[o] = v;
        else if (a.out_mode == OUT_F32_ADD) reinterpret_cast<float*>(a.Cp)[o] += v;
        else atomicAdd(reinterpret_cast<float*>(a.Cp) + o, v);
      }
    }
  }
}

// ============================================================ host launcher
static int pick_splits(int tiles, int nkt, int want_blocks) {
  if (tiles >= want_blocks) return 1;
  int s = (want_blocks + tiles - 1) / tiles;
  const int max_s = std::max(1, nkt / 4);  // keep >= 4 k-tiles per split
  return std::max(1, std::min(s, max_s));
}

void igemm_launch(IgemmArgs a, int mode, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  const int nkt = (a.K + BKT - 1) / BKT;
  const int tiles = a.tiles_m * a.tiles_n;
  int splits = 1;
  if (a.out_mode == OUT_F32_ATOMIC) splits = pick_splits(tiles, nkt, 1024);
  a.kps = (nkt + splits - 1) / splits;
  splits = (nkt + a.kps - 1) / a.kps;
  if (a.out_mode == OUT_F32_ATOMIC && a.zero_out)
    TFX_HIP_CHECK(hipMemsetAsync(a.Cp, 0, sizeof(float) * (size_t)a.M * a.ldc, s));
  const int grid = tiles * splits;
  if (grid == 0) return;
  switch (mode) {
    case MODE_FWD: igemm_kernel<MODE_FWD, true, true><<<grid, NT, 0, s>>>(a); break;
    case MODE_DGRAD: igemm_kernel<MODE_DGRAD, true, false><<<grid, NT, 0, s>>>(a); break;
    case MODE_WGRAD: igemm_kernel<MODE_WGRAD, false, false><<<grid, NT, 0, s>>>(a); break;
    default:
      if (a.a_kmajor && a.b_kmajor) igemm_kernel<MODE_GEMM, true, true><<<grid, NT, 0, s>>>(a);
      else if (a.a_kmajor) igemm_kernel<MODE_GEMM, true, false><<<grid, NT, 0, s>>>(a);
      else if (a.b_kmajor) igemm_kernel<MODE_GEMM, false, true><<<grid, NT, 0, s>>>(a);
      else igemm_kernel<MODE_GEMM, false, false><<<grid, NT, 0, s>>>(a);
  }
}

}  // namespace tfx
