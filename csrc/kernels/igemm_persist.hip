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
// a_shift[k]).  1 = in registers, after each fragment's LDS read (every wave of a wave row transforms
// the rows it reads); 2 = in LDS, once per element: when a stage has landed, the block rewrites its A
// image in place (4 16-byte chunks per thread) before an LDS-only barrier and the MFMAs.  The ring stays
// a raw LDS-DMA copy either way.  The per-channel coefficients are staged in LDS once per block
// (K <= BNA_KMAX).
constexpr int BNA_KMAX = 1024;  // 8 KB of coefficients: 128x128 tiles keep 2 blocks per CU

// EPI: EPI_STATS = the forward's BN statistics of the output (stat_slots rows); EPI_BNB = a data
// gradient's fused BN-backward partials (the BN feeding this conv: sum g', sum g' xhat into its NSLOT
// slots), with the residual-branch addend (and its ReLU mask bits) summed in; EPI_PLAIN = stores only.
// BKIND: the B operand's layout -- KM_DENSE (forward: W[Ko][C], K-major rows) or MN_DENSE (1x1 data
// gradient: W[Ko][C] with k = Ko rows and the output channels as columns).
template <int BM, int BN, int GLS, int EPI, int BNA = 0, int BKIND = KM_DENSE>
__global__ void __launch_bounds__(256) igemm_persist_kernel(IgemmArgs a) {
  constexpr bool STATS = EPI == EPI_STATS, BNB = EPI == EPI_BNB;
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
  using LB = Loader<BKIND, BN, true>;
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
    // B: the tile's rows (K-major) or columns (MN-major) -- every one valid (N % BN == 0)
    const uint32_t boff = is_kmaj(BKIND) ? (uint32_t)(tn * BN) * (uint32_t)a.ldb * 2u : (uint32_t)(tn * BN) * 2u;
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
      if constexpr (BNA == 1) {
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
      for (int j = 0; j < TN; ++j) fb[j] = frag<BKIND, BN>(ib, 0, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  // epilogue of tile `tile`: bf16 16-byte stores (lanes l, l^16 pair their column halves through
  // v_permlane16_swap), plus
  //  STATS: the BN statistics of the stored values (per column: the tile's rows reduced in registers,
  //         then across the two wave rows in LDS, one atomic pair per column into row tm % stat_slots);
  //  BNB:   the residual addend summed in, then the BN-backward partials of the stored gradient g' =
  //         bf16(out) * relu mask against xhat of the BN input x (same reductions, slot tm % NSLOT).
  // BNB's global operands (addend, its mask bits, x, the BN's mask bits) of a tile are prefetched into
  // registers during the tile's last k-step (epi_prefetch), so the epilogue does not wait a memory
  // round trip per tile.
  const __amdgpu_buffer_rsrc_t r_out = make_rsrc(a.Cp, 0x7fffffff);
  constexpr int NPF = BNB ? (TN / 2) * TM : 1;
  U4 pf_ad[NPF], pf_x[NPF];
  uint32_t pf_am[NPF], pf_mb[NPF];
  const __amdgpu_buffer_rsrc_t r_ad = make_rsrc(a.addend, a.addend ? 0x7fffffff : 0),
                               r_am = make_rsrc(a.addend_mask, a.addend_mask ? 0x7fffffff : 0),
                               r_x = make_rsrc(a.bnb_x, a.bnb_x ? 0x7fffffff : 0),
                               r_mb = make_rsrc(a.bnb_mask, a.bnb_mask ? 0x7fffffff : 0);
  auto epi_prefetch = [&](int tile) __attribute__((always_inline)) {
    if constexpr (BNB) {
      const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
      const int mb = tm * BM + wm * WM, nb = tn * BN + wn * WN;
      const bool odd = (lane >> 4) & 1;
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        const int n = nb + (j + (odd ? 1 : 0)) * 16 + ((lane >> 5) << 3);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint32_t o = (uint32_t)(mb + i * 16 + (lane & 15)) * (uint32_t)a.ldc + (uint32_t)n;
          const int e = (j / 2) * TM + i;
          // null operands read zeros through zero-extent resources: every load unconditional
          pf_ad[e] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(r_ad, o * 2u, 0, 0));
          pf_am[e] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r_am, o >> 3, 0, 0);
          pf_x[e] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(r_x, o * 2u, 0, 0));
          pf_mb[e] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r_mb, o >> 3, 0, 0);
        }
      }
    }
  };
  // BN-backward ReLU mask source: 2 = the residual layer's bits, 1 = recomputed from x*scale+shift
  const int bnb_mode = !a.bnb_relu ? 0 : (a.bnb_mask ? 2 : 1);
  const bool has_am = a.addend_mask != nullptr;
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
      // BNB: this lane's 8 columns of the BN's [mean | invstd | scale | shift]
      float is[8], nmi[8], sc[8], sh[8];
      if constexpr (BNB) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float4 m4 = *reinterpret_cast<const float4*>(a.bnb_save + n + 4 * q);
          const float4 i4 = *reinterpret_cast<const float4*>(a.bnb_save + a.N + n + 4 * q);
          const float4 c4 = *reinterpret_cast<const float4*>(a.bnb_save + 2 * a.N + n + 4 * q);
          const float4 h4 = *reinterpret_cast<const float4*>(a.bnb_save + 3 * a.N + n + 4 * q);
          const float mu4[4] = {m4.x, m4.y, m4.z, m4.w}, is4[4] = {i4.x, i4.y, i4.z, i4.w};
          const float sc4[4] = {c4.x, c4.y, c4.z, c4.w}, sh4[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            is[4 * q + k] = is4[k];
            nmi[4 * q + k] = -mu4[k] * is4[k];
            sc[4 * q + k] = sc4[k];
            sh[4 * q + k] = sh4[k];
          }
        }
      }
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
        if constexpr (BNB) {
          // the residual-branch gradient (its ReLU mask bits zero the masked bf16 halves; no addend: zeros)
          const int e = (j / 2) * TM + i;
          float ad[8];
          unpack8(mask_bf16x8(pf_ad[e], has_am ? pf_am[e] : 0xffu), ad);
#pragma unroll
          for (int r = 0; r < 8; ++r) o[r] += ad[r];
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
        if constexpr (BNB) {
          const int e = (j / 2) * TM + i;
          float xv[8];
          unpack8(pf_x[e], xv);
          uint32_t on8 = 0xffu;
          if (bnb_mode == 2) {
            on8 = pf_mb[e];
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
        float* slot = BNB ? a.bnb_slots + (size_t)(tm % NSLOT) * 2 * a.N
                          : a.stats + (size_t)(tm % a.stat_slots) * 2 * a.N;
        atomicAdd(&slot[n0 + t], red[t * 2] + red[(BN + t) * 2]);
        atomicAdd(&slot[a.N + n0 + t], red[t * 2 + 1] + red[(BN + t) * 2 + 1]);
      }
      // the next epilogue's red writes come after at least one ring barrier (nkt >= 1 steps later)
    }
  };

  // BNA 2: the landed A image of one stage, transformed in place (physical chunk p of row r holds
  // logical k-chunk p ^ (r & 7): kmaj_off's swizzle), then an LDS-only barrier before any fragment read
  auto bn_in_lds = [&](char* ia, int kbase) __attribute__((always_inline)) {
    static_assert(BM * BKT * 2 == 4 * 256 * 16, "4 chunks per thread");
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = t + 256 * u, r = q >> 3, pc = q & 7, c = kbase + 8 * (pc ^ (r & 7));
      lds_bf16x8* ptr = (lds_bf16x8*)((lds_char*)ia + (r * 128 + (pc << 4)));
      const float4 s0 = *reinterpret_cast<const float4*>(&bsc[c]), s1 = *reinterpret_cast<const float4*>(&bsc[c + 4]);
      const float4 h0 = *reinterpret_cast<const float4*>(&bsh[c]), h1 = *reinterpret_cast<const float4*>(&bsh[c + 4]);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
      float f[8];
      unpack8(__builtin_bit_cast(U4, *ptr), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f);
      *ptr = __builtin_bit_cast(bf16x8_t, pack8(f));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  if constexpr (BNA != 0) {
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
        // a tile's last k-step: its epilogue operands, behind this step's DMA (the next step's counted
        // wait then covers both)
        if constexpr (BNB) {
          if (st % nkt == nkt - 1) epi_prefetch(tile_of(st / nkt));
        }
        if constexpr (BNA == 2) bn_in_lds(img_a(S), (st % nkt) * BKT);
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

template <int BM, int BN, int GLS, int EPI, int BNA = 0, int BKIND = KM_DENSE>
void launch_p(IgemmArgs& a, hipStream_t s) {
  a.tiles_m = a.M / BM;
  a.tiles_n = a.N / BN;
  const int ntiles = a.tiles_m * a.tiles_n;
  // resident blocks per CU as the occupancy calculator sees them (LDS and VGPRs): a persistent grid
  // larger than what is resident would run its extra blocks after the others -- a second wave
  static const int bpc = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, igemm_persist_kernel<BM, BN, GLS, EPI, BNA, BKIND>, 256, 0) !=
            hipSuccess || n <= 0) {
      constexpr int lds = (BM + BN) * BKT * 2 * GLS + (BNA ? 2 * BNA_KMAX * 4 : 0);
      n = 163840 / lds < 2 ? 163840 / lds : 2;
    }
    return n;
  }();
  const int grid = std::min(ntiles, num_cus() * bpc);
  igemm_persist_kernel<BM, BN, GLS, EPI, BNA, BKIND><<<grid, 256, 0, s>>>(a);
}

}  // namespace

// the A-operand BN transform's form (TFX_BNA_MODE / igemm_bna_mode_set): 1 = registers, 2 = in LDS
int g_bna_mode = [] {
  const char* e = getenv("TFX_BNA_MODE");
  return e && atoi(e) == 2 ? 2 : 1;
}();

int igemm_bna_mode_set(int mode) {
  const int prev = g_bna_mode;
  if (mode == 1 || mode == 2) g_bna_mode = mode;
  return prev;
}

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
  constexpr int S = EPI_STATS, P = EPI_PLAIN;
  if (a.a_scale) {  // BN on load: ring depth 2 (the coefficient arrays take 8 KB of LDS)
    if (g_bna_mode == 2) {
      if (a.N % 128 == 0) launch_p<128, 128, 2, S, 2>(a, s);
      else launch_p<128, 64, 2, S, 2>(a, s);
    } else {
      if (a.N % 128 == 0) launch_p<128, 128, 2, S, 1>(a, s);
      else launch_p<128, 64, 2, S, 1>(a, s);
    }
    return;
  }
  const int gls = persist_mode();
  if (a.N % 128 == 0) {
    if (gls == 3) { st ? launch_p<128, 128, 3, S>(a, s) : launch_p<128, 128, 3, P>(a, s); }
    else { st ? launch_p<128, 128, 2, S>(a, s) : launch_p<128, 128, 2, P>(a, s); }
  } else {
    if (gls == 3) { st ? launch_p<128, 64, 3, S>(a, s) : launch_p<128, 64, 3, P>(a, s); }
    else { st ? launch_p<128, 64, 2, S>(a, s) : launch_p<128, 64, 2, P>(a, s); }
  }
}

// The fused-BN 1x1 data gradient dY[M][Ko] . W[Ko][C] (A = dY rows, K-major; B = W, MN-major) with the
// BN-backward partials of the BN that produced this conv's input and the residual addend: 128x64 tiles
// (the epilogue's prefetched operands: 40 VGPRs), ring depth 2.  OPT-IN (igemm_persist_dgrad_set,
// TFX_IGEMM_PERSIST_DGRAD=1): 11-20 % slower than the one-tile-per-block register-path kernel at every
// ResNet-50 shape it could take (profiles/r05_persist/README.md), so the model does not route here.
int g_persist_dgrad = [] {
  const char* e = getenv("TFX_IGEMM_PERSIST_DGRAD");
  return e && atoi(e) != 0 ? 1 : 0;
}();

int igemm_persist_dgrad_set(int on) {
  const int prev = g_persist_dgrad;
  g_persist_dgrad = on ? 1 : 0;
  return prev;
}

bool igemm_dgrad_persist_ok(const IgemmArgs& a) {
  return g_persist_dgrad && a.bnb_x && a.bnb_save && a.bnb_slots && a.out_mode == OUT_BF16 && !a.trans_out &&
         !a.bias && !a.relu && !a.addend_s2 && !a.cls && !a.stats && !a.a_scale && a.M > 0 && a.M % 128 == 0 &&
         a.N % 64 == 0 && a.K % BKT == 0 && a.K >= 2 * BKT && a.ldc == a.N && a.lda % 8 == 0 && a.ldb % 8 == 0 &&
         (int64_t)(a.M / 128) * (a.N / 64) >= 4 * num_cus();
}

void igemm_dgrad_persist(IgemmArgs& a, hipStream_t s) { launch_p<128, 64, 2, EPI_BNB, false, MN_DENSE>(a, s); }

}  // namespace tfx
