// Persistent implicit GEMM for the 1x1 convolutions' forward (X[M][C] . W[Ko][C]^T, + fused BN statistics):
// one resident block per CU slot walks its output tiles back to back through ONE continuous LDS-DMA ring.
//
// Why: these GEMMs are short in K (256-1024: 4-16 k-tiles per 128x128 tile) and long in tiles (512-2048).
// The one-tile-per-block kernel (igemm_impl.h) pays, per tile, the ring fill (the first k-tiles' L2/MALL
// latency, nothing to overlap it with at one block per CU), the epilogue (bf16 stores + statistics
// atomics) with no loads in flight, and the block start/exit -- at the many-tile stage-1/2 shapes a
// large part of the tile's time (profiles/r05_persist).  Here the ring's step index runs
// over (tile, k-tile) pairs of ALL the block's tiles: the next tile's first k-tiles are already landing
// while the current tile's epilogue runs, and the only fill is the block's first.
//
// Ring: GLS stages, one __shared__ array per stage and operand (compile-time stage index per unrolled
// body: the waitcnt pass then proves fragment reads and in-flight DMAs of other stages disjoint, see
// igemm_impl.h), GLS - 1 steps in flight, one barrier per step.  A tile's epilogue runs at the top of the
// next tile's first step, after that step's barrier and BEFORE the step's DMA issue, so its stores and
// atomics are older than every DMA the later counted waits leave in flight (vmcnt counts loads, stores,
// atomics and LDS-DMA in issue order).  Operand offsets of a tile = the tile-0 offsets + a per-tile scalar:
// the host only routes shapes with M % BM == N % BN == K % 64 == 0 here, so no row or column is ragged.
// Reference: the matmuls of R/distributed/distributed.py:96-98 (conv forward of the north-star ResNet-50,
// BASELINE.json config 3).
#include "igemm_impl.h"

namespace tfx {
namespace {

// BNA: the A operand is a plain ReLU BN's input, applied on load -- A[m][k] -> relu(A a_scale[k] +
// a_shift[k]) -- in registers, after each fragment's LDS read (the ring stays a raw LDS-DMA copy).  The
// per-channel coefficients are staged in LDS once per block (K <= BNA_KMAX).
constexpr int BNA_KMAX = 1024;  // 8 KB of coefficients: 128x128 tiles keep 2 blocks per CU

template <int BM, int BN, int GLS, bool STATS, bool BNA = false>
__global__ void __launch_bounds__(256) igemm_persist_kernel(IgemmArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2;
  static_assert(GLS == 2 || GLS == 3, "ring depth");
  static_assert(TN % 2 == 0, "16-byte epilogue pairs column tiles");
  __shared__ __attribute__((aligned(16))) char ga0[A_BYTES];
  __shared__ __attribute__((aligned(16))) char gb0[B_BYTES];
  __shared__ __attribute__((aligned(16))) char ga1[A_BYTES];
  __shared__ __attribute__((aligned(16))) char gb1[B_BYTES];
  __shared__ __attribute__((aligned(16))) char ga2[GLS >= 3 ? A_BYTES : 16];
  __shared__ __attribute__((aligned(16))) char gb2[GLS >= 3 ? B_BYTES : 16];
  __shared__ __attribute__((aligned(16))) float red[STATS ? 2 * BN * 2 : 4];  // [wm][col][sum | sumsq]
  __shared__ __attribute__((aligned(16))) float bsc[BNA ? BNA_KMAX : 4];     // a_scale, a_shift
  __shared__ __attribute__((aligned(16))) float bsh[BNA ? BNA_KMAX : 4];
  auto img_a = [&](auto S) __attribute__((always_inline)) -> char* {
    constexpr int st = decltype(S)::value;
    if constexpr (st == 0) return ga0;
    else if constexpr (st == 1) return ga1;
    else return ga2;
  };
  auto img_b = [&](auto S) __attribute__((always_inline)) -> char* {
    constexpr int st = decltype(S)::value;
    if constexpr (st == 0) return gb0;
    else if constexpr (st == 1) return gb1;
    else return gb2;
  };
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int grid = (int)gridDim.x;
  const int bid = xcd_remap(blockIdx.x, grid);
  const int tiles_n = a.tiles_n, ntiles = a.tiles_m * a.tiles_n;
  const int nkt = a.K / BKT;
  const int my = (ntiles - bid + grid - 1) / grid;  // >= 1: the host sizes grid <= ntiles
  const int total = my * nkt;

  // tile-0 loaders (every row / column valid: M % BM == N % BN == 0); a tile's offsets add a scalar
  using LA = Loader<KM_DENSE, BM, true>;
  using LB = Loader<KM_DENSE, BN, true>;
  LA la;
  LB lb;
  la.init(a, 0, BM, a.lda, t);
  lb.init(a, 0, BN, a.ldb, t);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.A, a.a_bytes), rb = make_rsrc(a.B, a.b_bytes);
  constexpr int NPT = LA::NP + LB::NP;
  uint32_t oa[LA::NP], ob[LB::NP];

  auto tile_of = [&](int ti) __attribute__((always_inline)) { return bid + ti * grid; };
  // step s of this block = k-tile (s mod nkt) of its tile (s div nkt); s >= total: zero pieces (BAD)
  auto issue = [&](int s, auto S) __attribute__((always_inline)) {
    const int ti = s / nkt, kt = s - ti * nkt;
    const int tile = tile_of(ti), tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int kend = s < total ? a.K : 0;
    la.offsets(a, a.lda, kt * BKT, kend, oa);
    lb.offsets(a, a.ldb, kt * BKT, kend, ob);
    // BAD (0x80000000) + a tile offset (< 2^31) stays past num_records: still a zero fill
    const uint32_t aoff = (uint32_t)(tm * BM) * (uint32_t)a.lda * 2u, boff = (uint32_t)(tn * BN) * (uint32_t)a.ldb * 2u;
#pragma unroll
    for (int i = 0; i < LA::NP; ++i) oa[i] += aoff;
#pragma unroll
    for (int i = 0; i < LB::NP; ++i) ob[i] += boff;
    la.load_lds(ra, oa, img_a(S), 0, wv);
    lb.load_lds(rb, ob, img_b(S), 0, wv);
  };

  f32x4_t acc[TM][TN];
  auto zero = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  };
  // kbase: the k-tile's first channel (BNA coefficients)
  auto compute = [&](const char* ia, const char* ib, int kbase) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag<KM_DENSE, BM>(ia, 0, wm * WM + i * 16, kk, lane);
      if constexpr (BNA) {
        // the lane's 8 channels of this 32-deep half: kbase + 32 kk + 8 (lane >> 4) + 0..7
        const int c = kbase + 32 * kk + 8 * (lane >> 4);
        const float4 s0 = *reinterpret_cast<const float4*>(&bsc[c]), s1 = *reinterpret_cast<const float4*>(&bsc[c + 4]);
        const float4 h0 = *reinterpret_cast<const float4*>(&bsh[c]), h1 = *reinterpret_cast<const float4*>(&bsh[c + 4]);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float f[8];
          unpack8(__builtin_bit_cast(U4, fa[i]), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f);
          fa[i] = __builtin_bit_cast(bf16x8_t, pack8(f));
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag<KM_DENSE, BN>(ib, 0, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  // epilogue of tile `tile`: bf16 16-byte stores (lanes l, l^16 pair their column halves through
  // v_permlane16_swap) + the BN statistics of the stored values (per column: the tile's rows reduced in
  // registers, then across the two wave rows in LDS, one atomic pair per column into row tm % stat_slots)
  const __amdgpu_buffer_rsrc_t r_out = make_rsrc(a.Cp, 0x7fffffff);
  auto epilogue = [&](int tile) __attribute__((always_inline)) {
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN, mb = m0 + wm * WM, nb = n0 + wn * WN;
    const bool odd = (lane >> 4) & 1;
#pragma unroll
    for (int j = 0; j < TN; j += 2) {
      const int n = nb + (j + (odd ? 1 : 0)) * 16 + ((lane >> 5) << 3);
      float bs[8], bq[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) bs[k] = bq[k] = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + (lane & 15);
        float o[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][r]), __float_as_uint(acc[i][j + 1][r]),
                                                           false, false);
          o[r] = __uint_as_float(sw[0]);
          o[4 + r] = __uint_as_float(sw[1]);
        }
        const U4 packed = pack8(o);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, packed), r_out,
                                               ((uint32_t)m * (uint32_t)a.ldc + (uint32_t)n) * 2u, 0, 0);
        if constexpr (STATS) {
          float g[8];
          unpack8(packed, g);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            bs[k] += g[k];
            bq[k] = fmaf(g[k], g[k], bq[k]);
          }
        }
      }
      if constexpr (STATS) {
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
    if constexpr (STATS) {
      // LDS-only barrier: a __syncthreads() fence would drain the ring's DMAs in flight (vmcnt(0))
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t < BN) {
        float* slot = a.stats + (size_t)(tm % a.stat_slots) * 2 * a.N;
        atomicAdd(&slot[n0 + t], red[t * 2] + red[(BN + t) * 2]);
        atomicAdd(&slot[a.N + n0 + t], red[t * 2 + 1] + red[(BN + t) * 2 + 1]);
      }
      // the next epilogue's red writes come after at least one ring barrier (nkt >= 1 steps later)
    }
  };

  if constexpr (BNA) {
    // the coefficients into LDS before the ring starts (its loads are the only ones outstanding later)
    for (int i = t; i < a.K; i += 256) {
      bsc[i] = a.a_scale[i];
      bsh[i] = a.a_shift[i];
    }
    __syncthreads();
  }
  zero();
  issue(0, IC<0>{});
  if constexpr (GLS >= 3) issue(1, IC<1>{});
  for (int s = 0; s < total; s += GLS) {
    static_for<GLS>([&](auto S) __attribute__((always_inline)) {
      constexpr int st_ = decltype(S)::value;
      const int st = s + st_;
      if (st < total) {
        wait_vmcnt<NPT * (GLS - 2)>();
        __builtin_amdgcn_s_barrier();
        if (st > 0 && st % nkt == 0) {  // the previous tile is complete: its epilogue, before the next DMA
          epilogue(tile_of(st / nkt - 1));
          zero();
        }
        issue(st + GLS - 1, IC<(st_ + GLS - 1) % GLS>{});
        __builtin_amdgcn_sched_barrier(0);
        compute(img_a(S), img_b(S), (st % nkt) * BKT);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  }
  // drain the ring (zero pieces past the end) before the last epilogue and the exit
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  epilogue(tile_of(my - 1));
}

int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}

// TFX_IGEMM_PERSIST: 0 = off (the one-tile-per-block kernel), 2 / 3 = ring depth (default 2); tests and
// A/B runs switch it at run time (igemm_persist_set)
int g_persist = [] {
  const char* e = getenv("TFX_IGEMM_PERSIST");
  if (!e) return 2;
  const int v = atoi(e);
  return v == 0 || v == 2 || v == 3 ? v : 2;
}();
int persist_mode() { return g_persist; }

template <int BM, int BN, int GLS, bool STATS, bool BNA = false>
void launch_p(IgemmArgs& a, hipStream_t s) {
  a.tiles_m = a.M / BM;
  a.tiles_n = a.N / BN;
  const int ntiles = a.tiles_m * a.tiles_n;
  constexpr int lds = (BM + BN) * BKT * 2 * GLS + (BNA ? 2 * BNA_KMAX * 4 : 0);
  constexpr int bpc = 163840 / lds < 4 ? 163840 / lds : 4;  // resident blocks per CU (4 waves each)
  const int grid = std::min(ntiles, num_cus() * bpc);
  igemm_persist_kernel<BM, BN, GLS, STATS, BNA><<<grid, 256, 0, s>>>(a);
}

}  // namespace

int igemm_persist_set(int mode) {
  const int prev = g_persist;
  if (mode == 0 || mode == 2 || mode == 3) g_persist = mode;
  return prev;
}

// Routed only where a block gets >= 2 tiles at the resident grid (>= 4 tiles per CU) and K >= 128: with
// fewer tiles the per-tile kernel's split-K over two wave groups keeps more of the chip busy, and at
// K = 64 (one k-tile per tile) it loses 1 us of 40 (the A/B over the ResNet-50 1x1 shapes,
// profiles/r05_persist/README.md).
static bool persist_shape_ok(const IgemmArgs& a) {
  return a.out_mode == OUT_BF16 && !a.trans_out && !a.bias && !a.relu && !a.addend && !a.bnb_x && a.M > 0 &&
         a.M % 128 == 0 && a.N % 64 == 0 && a.K % BKT == 0 && a.K >= 2 * BKT && a.ldc == a.N && a.lda % 8 == 0 &&
         a.ldb % 8 == 0 && (a.stats == nullptr || a.stat_slots > 0);
}

bool igemm_fwd_persist_ok(const IgemmArgs& a) {
  if (a.a_scale) return igemm_fwd_persist_bna_ok(a);
  const int bn = a.N % 128 == 0 ? 128 : 64;
  return persist_mode() != 0 && (int64_t)(a.M / 128) * (a.N / bn) >= 4 * num_cus() && persist_shape_ok(a);
}

// the A-operand BN transform (a plain ReLU BN applied on load by this 1x1 conv): any tile count (it
// replaces a whole BN apply pass), K <= BNA_KMAX channels of coefficients in LDS
bool igemm_fwd_persist_bna_ok(const IgemmArgs& a) {
  return a.a_scale && a.a_shift && a.stats && a.K <= BNA_KMAX && persist_shape_ok(a);
}

bool igemm_fwd_bna_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && M % 128 == 0 && N % 64 == 0 && K % BKT == 0 && K >= 2 * BKT && K <= BNA_KMAX;
}

// X[M][C] . W[Ko][C]^T (A = X rows, B = W rows, both K-major; + BN statistics when a.stats)
void igemm_fwd_persist(IgemmArgs& a, hipStream_t s) {
  const bool st = a.stats != nullptr;
  if (a.a_scale) {  // BN on load: ring depth 2 (the coefficient arrays take 16 KB of LDS)
    if (a.N % 128 == 0) launch_p<128, 128, 2, true, true>(a, s);
    else launch_p<128, 64, 2, true, true>(a, s);
    return;
  }
  const int gls = persist_mode();
  if (a.N % 128 == 0) {
    if (gls == 3) { st ? launch_p<128, 128, 3, true>(a, s) : launch_p<128, 128, 3, false>(a, s); }
    else { st ? launch_p<128, 128, 2, true>(a, s) : launch_p<128, 128, 2, false>(a, s); }
  } else {
    if (gls == 3) { st ? launch_p<128, 64, 3, true>(a, s) : launch_p<128, 64, 3, false>(a, s); }
    else { st ? launch_p<128, 64, 2, true>(a, s) : launch_p<128, 64, 2, false>(a, s); }
  }
}

}  // namespace tfx
