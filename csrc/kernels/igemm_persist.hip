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

// EPI: EPI_STATS = the forward's BN statistics of the output (stat_slots rows); EPI_PLAIN = stores only.
// (Measured and removed, git history: a fused-BN data-gradient form of this schedule and BN applied on
// load to the A operand -- both slower than the per-tile kernel / the apply pass, profiles/r05_persist,
// profiles/r05_bna.)
template <int BM, int BN, int GLS, int EPI>
__global__ void __launch_bounds__(256) igemm_persist_kernel(IgemmArgs a) {
  static_assert(EPI == EPI_STATS || EPI == EPI_PLAIN, "forward epilogues");
  constexpr bool STATS = EPI == EPI_STATS;
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
  __shared__ __attribute__((aligned(16))) float red[EPI != EPI_PLAIN ? 2 * BN * 2 : 4];  // [wm][col][2 sums]
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
    const uint32_t aoff = (uint32_t)(tm * BM) * (uint32_t)a.lda * 2u;
    // B: the tile's rows (K-major) -- every one valid (N % BN == 0)
    const uint32_t boff = (uint32_t)(tn * BN) * (uint32_t)a.ldb * 2u;
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
  auto compute = [&](const char* ia, const char* ib) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag<KM_DENSE, BM>(ia, 0, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag<KM_DENSE, BN>(ib, 0, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  // epilogue of tile `tile`: bf16 16-byte stores (lanes l, l^16 pair their column halves through
  // v_permlane16_swap), plus STATS: the BN statistics of the stored values (per column: the tile's rows
  // reduced in registers, then across the two wave rows in LDS, one atomic pair per column into row
  // tm % stat_slots)
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
      if constexpr (EPI != EPI_PLAIN) {
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
    if constexpr (EPI != EPI_PLAIN) {
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
        compute(img_a(S), img_b(S));
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

template <int BM, int BN, int GLS, int EPI>
void launch_p(IgemmArgs& a, hipStream_t s) {
  a.tiles_m = a.M / BM;
  a.tiles_n = a.N / BN;
  const int ntiles = a.tiles_m * a.tiles_n;
  // resident blocks per CU as the occupancy calculator sees them (LDS and VGPRs): a persistent grid
  // larger than what is resident would run its extra blocks after the others -- a second wave
  static const int bpc = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, igemm_persist_kernel<BM, BN, GLS, EPI>, 256, 0) !=
            hipSuccess || n <= 0) {
      constexpr int lds = (BM + BN) * BKT * 2 * GLS;
      n = 163840 / lds < 2 ? 163840 / lds : 2;
    }
    return n;
  }();
  const int grid = std::min(ntiles, num_cus() * bpc);
  igemm_persist_kernel<BM, BN, GLS, EPI><<<grid, 256, 0, s>>>(a);
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
  return a.out_mode == OUT_BF16 && !a.trans_out && !a.bias && !a.relu && !a.addend && !a.bnb_x && !a.cls && a.M > 0 &&
         a.M % 128 == 0 && a.N % 64 == 0 && a.K % BKT == 0 && a.K >= 2 * BKT && a.ldc == a.N && a.lda % 8 == 0 &&
         a.ldb % 8 == 0 && (a.stats == nullptr || a.stat_slots > 0);
}

bool igemm_fwd_persist_ok(const IgemmArgs& a) {
  if (a.a_scale) return false;  // the A-operand transform is the single-k-tile register path's
  const int bn = a.N % 128 == 0 ? 128 : 64;
  return persist_mode() != 0 && (int64_t)(a.M / 128) * (a.N / bn) >= 4 * num_cus() && persist_shape_ok(a);
}

// X[M][C] . W[Ko][C]^T (A = X rows, B = W rows, both K-major; + BN statistics when a.stats)
void igemm_fwd_persist(IgemmArgs& a, hipStream_t s) {
  const bool st = a.stats != nullptr;
  constexpr int S = EPI_STATS, P = EPI_PLAIN;
  const int gls = persist_mode();
  if (a.N % 128 == 0) {
    if (gls == 3) { st ? launch_p<128, 128, 3, S>(a, s) : launch_p<128, 128, 3, P>(a, s); }
    else { st ? launch_p<128, 128, 2, S>(a, s) : launch_p<128, 128, 2, P>(a, s); }
  } else {
    if (gls == 3) { st ? launch_p<128, 64, 3, S>(a, s) : launch_p<128, 64, 3, P>(a, s); }
    else { st ? launch_p<128, 64, 2, S>(a, s) : launch_p<128, 64, 2, P>(a, s); }
  }
}

}  // namespace tfx
