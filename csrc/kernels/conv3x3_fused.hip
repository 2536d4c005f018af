// Stage-1 3x3 convolution of a ResNet bottleneck (conv2: 64 -> 64 channels, stride 1, pad 1, 32-pixel
// rows) as persistent halo-tiled kernels with its BN layers fused, for gfx950.
//
// Forward, layer-wise: bn_apply (a1 = relu(y1 sc1 + sh1), written) then the implicit-GEMM conv, which
// re-reads every a1 pixel once per tap (9 k-tiles of 64 channels, one tap each) through L2.  Here each
// 128-pixel output tile (4 image rows) loads its (4+2) x (32+2)-pixel input halo ONCE, applies BN1 +
// ReLU in registers (padding stays exactly zero), and runs all 9 taps from that LDS image against the
// 9 x 64 x 64 weights resident in LDS for the whole launch: a1 never exists in HBM and the input is read
// ~1.6x (the halo overlap) instead of 9x.  The epilogue stores y2 and accumulates BN2's statistics
// (igemm.hip EPI_STATS math); the op finalizes them.
// Pipeline: 512 threads (8 waves), one block per CU, a register staging ring of two tiles' halos, LDS
// halo images double-buffered, one barrier per tile.
// Reference: the reference has no ResNet; this is the north-star ResNet-50 config (BASELINE.json config 3,
// SURVEY §2.7's "fuse the unfused op chain" of /root/reference/distributed/distributed.py:96-102).
// Why stage 1 only (C = K = 64, width 32): the kernel's premise is the whole 9 x C x K filter resident
// in LDS for the launch (9 x 64 x 64 x 2 B = 72 KB beside two 26 KB halo images).  Stage 2's 128 x 128
// filter is 288 KB and stage 3's 1.2 MB -- more than the 160 KB LDS -- so those convs must stream their
// weights per k-tile, which is the generic implicit GEMM (igemm_impl.h, KM_FWD_XT tap-uniform operand);
// their halo-operand variant inside the igemm was measured ~2x slower (profiles/r03_halo/README.md).
#include "pw_common.h"

namespace tfx {
namespace {

// Geometry: C = K = 64 channels, image width IW = 32, TR = 4 output rows per tile (128 pixels).
constexpr int C3_C = 64, C3_IW = 32, C3_TR = 4, C3_BM = C3_TR * C3_IW;
constexpr int C3_HW = C3_IW + 2, C3_HH = C3_TR + 2, C3_HP = C3_HH * C3_HW;   // halo: 6 x 34 = 204 pixels
constexpr int C3_HBYTES = C3_HP * 128;                                      // halo image (K-major rows)
constexpr int C3_WTAP = C3_C * 128;                                         // one tap's weight image
constexpr int C3_PIECES = C3_HP * 8;                                        // 16-B halo pieces
constexpr int C3_PPT = (C3_PIECES + PW_NT - 1) / PW_NT;                     // per thread (4)

// v zeroed where !keep, as a bit mask on the packed words: a per-element `keep ? x : 0` on the staged
// halo compiles to one exec-masked branch per element, and every such branch makes the waitcnt pass
// wait for the loads at its join (the next tile's halo included) -- padding pixels are zeroed after
// the BN transform (relu(0 sc + sh) is not 0) with straight-line code instead
__device__ __forceinline__ U4 mask_u4(U4 v, bool keep) {
  const uint32_t m = 0u - (uint32_t)keep;
  v.x &= m; v.y &= m; v.z &= m; v.w &= m;
  return v;
}

__global__ void __launch_bounds__(PW_NT, 1) conv3x3_fwd_fused_kernel(Conv3Args a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * C3_HBYTES + 9 * C3_WTAP];
  char* wimg = smem + 2 * C3_HBYTES;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int tiles_img = a.H / C3_TR, ntiles = a.N * tiles_img;

  // ---- W [K][3][3][C] -> per-tap K-major images (row = output channel), resident
  pw_resident_copy<9 * C3_C * 8>(
      t,
      [&](int q) {
        const int co = q / 72, rem = q % 72, tap = rem / 8, ch = rem % 8;
        return reinterpret_cast<pw_u32x4*>(wimg + tap * C3_WTAP + pw_kmaj(co, ch));
      },
      [&](int q) { return reinterpret_cast<const pw_u32x4*>(a.w) + q; });
  // this thread's halo pieces: chunk t % 8 (fixed), halo pixels t / 8 + 64 i
  const int hch = t & 7;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = a.save_in[2 * C3_C + 8 * hch + k];
    sh[k] = a.save_in[3 * C3_C + 8 * hch + k];
  }
  const __amdgpu_buffer_rsrc_t rx = pw_rsrc(a.x, (int64_t)a.N * a.H * C3_IW * C3_C * 2);
  const __amdgpu_buffer_rsrc_t ry = pw_rsrc(a.y, (int64_t)a.N * a.H * C3_IW * C3_C * 2);

  struct Stage {
    pw_u32x4 v[C3_PPT];
  };
  Stage st0, st1;
  auto issue = [&](Stage& s, int tile) {
    const bool ok = tile < ntiles;
    const int n = tile / tiles_img, y0 = (tile % tiles_img) * C3_TR;
#pragma unroll
    for (int i = 0; i < C3_PPT; ++i) {
      // pieces past the halo re-load its last pixel (identical duplicate writes): no branch in the
      // load path, so hipcc keeps the counted waits instead of draining vmcnt at a join
      const int hp = min((t >> 3) + 64 * i, C3_HP - 1), hy = hp / C3_HW, hx = hp % C3_HW;
      const int iy = y0 + hy - 1, ix = hx - 1;
      const bool in = ok & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)C3_IW);
      const uint32_t off = in ? (uint32_t)(((n * a.H + iy) * C3_IW + ix) * C3_C + 8 * hch) * 2u : 0x80000000u;
      s.v[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
    }
  };
  // BN1 + ReLU of the staged halo into the LDS image; padding pixels stay zero (not relu(shift))
  auto stage = [&](const Stage& s, char* img, int tile) {
    const int y0 = (tile % tiles_img) * C3_TR;
#pragma unroll
    for (int i = 0; i < C3_PPT; ++i) {
      const int hp = min((t >> 3) + 64 * i, C3_HP - 1), hy = hp / C3_HW, hx = hp % C3_HW;
      const bool in = ((unsigned)(y0 + hy - 1) < (unsigned)a.H) & ((unsigned)(hx - 1) < (unsigned)C3_IW);
      float f[8];
      unpack8(__builtin_bit_cast(U4, s.v[i]), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], sc[k], sh[k]), 0.f);
      *reinterpret_cast<U4*>(img + pw_kmaj(hp, hch)) = mask_u4(pack8(f), in);
    }
  };
  // wave tile: output row r = wv & 3 of the tile (32 pixels = 2 m-tiles), 32 output channels (wv >> 2)
  const int wr = wv & 3, wcb = 32 * (wv >> 2);
  // BN statistics of the lane's 8 output channels (after the epilogue's lane pairing, below)
  float bs[8], bq[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) bs[k] = bq[k] = 0.f;
  const int ecol = wcb + 16 * ((lane >> 4) & 1) + 8 * (lane >> 5);
  auto mfma = [&](const char* img, f32x4_t (&acc)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int hp = (wr + ky) * C3_HW + 16 * i + (lane & 15) + kx;
          fa[i] = *(const pw_lds_bf16x8*)((pw_lds_char*)img + pw_kmaj(hp, 4 * kk + (lane >> 4)));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[j] = pw_frag_kmaj(wimg, tap * C3_WTAP, wcb + 16 * j, 4 * kk, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    }
  };
  // epilogue: y (bf16) + BN statistics of the stored values.  v_permlane16_swap pairs the lane's two
  // 16-column tiles so each lane holds 8 consecutive channels of one pixel: one 16-byte store per pixel
  // group (16 pixels x 64 contiguous bytes per wave-instruction) instead of two 8-byte ones
  auto epi = [&](const f32x4_t (&acc)[2][2], int tile) {
    const int n = tile / tiles_img, y0 = (tile % tiles_img) * C3_TR;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pix = (n * a.H + y0 + wr) * C3_IW + 16 * i + (lane & 15);
      float o[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][0][r]), __float_as_uint(acc[i][1][r]),
                                                         false, false);
        o[r] = __uint_as_float(sw[0]);
        o[4 + r] = __uint_as_float(sw[1]);
      }
      const U4 packed = pack8(o);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pw_u32x4, packed), ry,
                                             (uint32_t)(pix * C3_C + ecol) * 2u, 0, 0);
      float v[8];
      unpack8(packed, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bs[k] += v[k];
        bq[k] = fmaf(v[k], v[k], bq[k]);
      }
    }
  };
  // (measured: waves 4-7 running each tile's epilogue one tile late, beside their partners' MFMAs, was
  // 4 % slower than this lockstep order -- profiles/r05_conv3)
  auto compute = [&](const char* img, int tile) {
    f32x4_t acc[2][2];
    mfma(img, acc);
    epi(acc, tile);
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  const int tile0 = blockIdx.x, tstep = gridDim.x;
  issue(st0, tile0);
  issue(st1, tile0 + tstep);
  __syncthreads();  // weight images written
  for (int tile = tile0; tile < ntiles; tile += 2 * tstep) {
    stage(st0, smem, tile);
    issue(st0, tile + 2 * tstep);
    sync();
    compute(smem, tile);
    const int t1 = tile + tstep;
    if (t1 >= ntiles) break;
    stage(st1, smem + C3_HBYTES, t1);
    issue(st1, t1 + 2 * tstep);
    sync();
    compute(smem + C3_HBYTES, t1);
  }
  // ---- BN statistics: sum the 16 rows of each DPP row, one atomic pair per column per wave
  float* slots = a.slots + (size_t)(blockIdx.x % NSLOT) * 2 * C3_C;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float s = row16_sum(bs[k]), q = row16_sum(bq[k]);
    if ((lane & 15) == 0) {
      atomicAdd(slots + ecol + k, s);
      atomicAdd(slots + C3_C + ecol + k, q);
    }
  }
}

// ---------------------------------------------------------------------------------------- backward
// Layer-wise: bn_bwd_apply (dy2 = A2 (g2 relu2) + B2 y2 + D2, written), the data gradient (a flipped-tap
// implicit GEMM over dy2, + BN1's backward partials in its epilogue) and the weight gradient (an
// implicit GEMM over dy2 and a materialised a1 = relu(y1 sc1 + sh1)).  Here per 128-pixel tile the
// block loads the g2 / y2 / y1 halos once and forms, in LDS, the dy2 halo (the data gradient's A
// operand, shifted per tap; its interior is the weight gradient's A^T) and the a1 halo (the weight
// gradient's B, shifted per tap); the raw y1 interior serves BN1's partials.  dA1 is stored; BN1's
// partials go to its slots; the weight gradient accumulates in registers over the block's tiles
// (64 x 576, 72 per thread) and leaves through a per-block slab (pw_bwd.hip pw_slab_reduce, map 2).
// LDS: weights (MN images per tap, 72 KB) + dy2 halo + a1 halo + y1 interior + coefficient tables
// (141 KB): the halos are single-buffered, the next tile's raw halos wait in registers.
constexpr int C3_YBYTES = C3_BM * 128;  // raw y1 interior, K-major rows

__global__ void __launch_bounds__(PW_NT, 1) conv3x3_bwd_fused_kernel(Conv3BwdArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[9 * C3_WTAP + 2 * C3_HBYTES + C3_YBYTES + 16 + 9 * C3_C * 4];
  __shared__ float bnacc[2 * C3_C];  // BN1 backward partials of the block (sum g', sum g' xhat)
  char* wimg = smem;
  char* timg = wimg + 9 * C3_WTAP;   // dy2 halo
  char* aimg = timg + C3_HBYTES;     // a1 halo
  char* yimg = aimg + C3_HBYTES;     // raw y1, tile interior
  float* coef = reinterpret_cast<float*>(yimg + C3_YBYTES + 16);  // (+ the 16-B trash slot)
  // coef: [A2 | B2 | D2 | sc2 | sh2 | sc1 | sh1 | is1 | -mu1 is1] x 64
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int tiles_img = a.H / C3_TR, ntiles = a.N * tiles_img;

  if (t < 2 * C3_C) bnacc[t] = 0.f;
  if (t < C3_C) {
    const float inv_m = 1.f / ((float)a.N * a.H * C3_IW);
    const float mu = a.save2[t], is = a.save2[C3_C + t], sc = a.save2[2 * C3_C + t];
    const float kg = a.red2[t] * inv_m, kx = a.red2[C3_C + t] * inv_m * is;
    coef[t] = sc;
    coef[C3_C + t] = -sc * kx;
    coef[2 * C3_C + t] = sc * (kx * mu - kg);
    coef[3 * C3_C + t] = sc;
    coef[4 * C3_C + t] = a.save2[3 * C3_C + t];
    const float is1 = a.save1[C3_C + t];
    coef[5 * C3_C + t] = a.save1[2 * C3_C + t];
    coef[6 * C3_C + t] = a.save1[3 * C3_C + t];
    coef[7 * C3_C + t] = is1;
    coef[8 * C3_C + t] = -a.save1[t] * is1;
  }
  // ---- W [K][3][3][C] -> per-tap MN images (row = output channel co, columns = ci), resident
  pw_resident_copy<9 * C3_C * 8>(
      t,
      [&](int q) {
        const int co = q / 72, rem = q % 72, tap = rem / 8, ch = rem % 8;
        return reinterpret_cast<pw_u32x4*>(wimg + tap * C3_WTAP + pw_mn<64>(co, ch));
      },
      [&](int q) { return reinterpret_cast<const pw_u32x4*>(a.w) + q; });
  const int64_t bytes = (int64_t)a.N * a.H * C3_IW * C3_C * 2;
  const __amdgpu_buffer_rsrc_t rg = pw_rsrc(a.g2, bytes), ry2 = pw_rsrc(a.y2, bytes), ry1 = pw_rsrc(a.y1, bytes);
  const __amdgpu_buffer_rsrc_t rdx = pw_rsrc(a.dx, bytes);

  // halo pieces of this thread: chunk t % 8 (fixed), halo pixels t / 8 + 64 i
  const int hch = t & 7;
  struct Stage {
    pw_u32x4 g[C3_PPT], y2[C3_PPT], y1[C3_PPT];
  };
  Stage st;
  auto issue = [&](int tile) {
    const bool ok = tile < ntiles;
    const int n = tile / tiles_img, y0 = (tile % tiles_img) * C3_TR;
#pragma unroll
    for (int i = 0; i < C3_PPT; ++i) {
      // pieces past the halo re-load its last pixel (identical duplicate writes): no branch in the
      // load path, so hipcc keeps the counted waits instead of draining vmcnt at a join
      const int hp = min((t >> 3) + 64 * i, C3_HP - 1), hy = hp / C3_HW, hx = hp % C3_HW;
      const int iy = y0 + hy - 1, ix = hx - 1;
      const bool in = ok & ((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)C3_IW);
      const uint32_t off = in ? (uint32_t)(((n * a.H + iy) * C3_IW + ix) * C3_C + 8 * hch) * 2u : 0x80000000u;
      st.g[i] = __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 0);
      st.y2[i] = __builtin_amdgcn_raw_buffer_load_b128(ry2, off, 0, 0);
      st.y1[i] = __builtin_amdgcn_raw_buffer_load_b128(ry1, off, 0, 0);
    }
  };
  // dy2 halo (BN2 backward apply), a1 halo (BN1 + ReLU), raw y1 interior; padding stays zero
  auto stage = [&](int tile) {
    const int y0 = (tile % tiles_img) * C3_TR;
    // two passes (dy2, then a1 + raw y1) keep only one coefficient set live
    {
      float cA[8], cB[8], cD[8], s2[8], h2[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = 8 * hch + k;
        cA[k] = coef[c]; cB[k] = coef[C3_C + c]; cD[k] = coef[2 * C3_C + c];
        s2[k] = coef[3 * C3_C + c]; h2[k] = coef[4 * C3_C + c];
      }
#pragma unroll
      for (int i = 0; i < C3_PPT; ++i) {
        const int hp = min((t >> 3) + 64 * i, C3_HP - 1), hy = hp / C3_HW, hx = hp % C3_HW;
        const bool in = ((unsigned)(y0 + hy - 1) < (unsigned)a.H) & ((unsigned)(hx - 1) < (unsigned)C3_IW);
        float g[8], y2[8];
        unpack8(__builtin_bit_cast(U4, st.g[i]), g);
        unpack8(__builtin_bit_cast(U4, st.y2[i]), y2);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gg = fmaf(y2[k], s2[k], h2[k]) > 0.f ? g[k] : 0.f;
          g[k] = fmaf(cA[k], gg, fmaf(cB[k], y2[k], cD[k]));
        }
        *reinterpret_cast<U4*>(timg + pw_kmaj(hp, hch)) = mask_u4(pack8(g), in);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    {
      float s1[8], h1[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s1[k] = coef[5 * C3_C + 8 * hch + k];
        h1[k] = coef[6 * C3_C + 8 * hch + k];
      }
#pragma unroll
      for (int i = 0; i < C3_PPT; ++i) {
        const int hp = min((t >> 3) + 64 * i, C3_HP - 1), hy = hp / C3_HW, hx = hp % C3_HW;
        const bool in = ((unsigned)(y0 + hy - 1) < (unsigned)a.H) & ((unsigned)(hx - 1) < (unsigned)C3_IW);
        float y1[8];
        unpack8(__builtin_bit_cast(U4, st.y1[i]), y1);
#pragma unroll
        for (int k = 0; k < 8; ++k) y1[k] = fmaxf(fmaf(y1[k], s1[k], h1[k]), 0.f);
        *reinterpret_cast<U4*>(aimg + pw_kmaj(hp, hch)) = mask_u4(pack8(y1), in);
        // raw y1 of the tile interior; border pixels go to a trash slot past the image (no branch)
        const bool inner = ((unsigned)(hy - 1) < (unsigned)C3_TR) & ((unsigned)(hx - 1) < (unsigned)C3_IW);
        *reinterpret_cast<pw_u32x4*>(yimg + (inner ? pw_kmaj((hy - 1) * C3_IW + hx - 1, hch) : C3_YBYTES)) = st.y1[i];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // dgrad wave tile: output row wr = wv & 3 (2 m-tiles of 16 pixels), 32 input channels (wv >> 2); SWAP
  const int wr = wv & 3, dcb = 32 * (wv >> 2);
  // wgrad wave tile: output channels 32 (wv & 1: 2 m-tiles), (tap, 16-ci) column tiles 9 (wv >> 1) * 9 + nn
  const int wco = 32 * (wv & 1), wng = 9 * (wv >> 1);
  f32x4_t accw[2][9];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 9; ++nn) accw[m][nn] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // ---- data gradient: dA1[px][ci] = sum over taps of dy2(px + (1 - ky, 1 - kx)) . W[:, tap, ci]
  auto dgrad_mfma = [&](f32x4_t (&acc)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int tap = 3 * ky + kx;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int hp = (wr + 2 - ky) * C3_HW + 16 * i + (lane & 15) + 2 - kx;
          fa[i] = *(const pw_lds_bf16x8*)((pw_lds_char*)timg + pw_kmaj(hp, 4 * kk + (lane >> 4)));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[j] = pw_frag_tr(wimg, tap * C3_WTAP + 32 * kk * 128, dcb + 16 * j, lane,
                             [](int r, int c) { return pw_mn<64>(r, c); });
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    }
  };
  // epilogue: dA1 (bf16) + BN1 backward partials (ReLU mask from y1 sc1 + sh1 > 0).  v_permlane16_swap
  // pairs the lane's two 16-column tiles so each lane holds 8 CONSECUTIVE channels of one pixel: one
  // 16-byte store per pixel group (a wave-instruction writes 16 pixels x 64 contiguous bytes) instead of
  // two 8-byte ones.  The partials are sum g' and sum g' y1 (xhat is affine in y1: centred and scaled
  // once per block, below) -- two coefficients per channel live here instead of four.
  auto dgrad_epi = [&](const f32x4_t (&acc)[2][2], int tile) {
    {
      const int n = tile / tiles_img, y0 = (tile % tiles_img) * C3_TR;
      const int g = lane >> 4, col = dcb + 16 * (g & 1) + 8 * (g >> 1);
      float bs[8], bq[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) bs[k] = bq[k] = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int lpx = wr * C3_IW + 16 * i + (lane & 15);
        const int pix = (n * a.H + y0 + wr) * C3_IW + 16 * i + (lane & 15);
        float o[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][0][r]), __float_as_uint(acc[i][1][r]),
                                                           false, false);
          o[r] = __uint_as_float(sw[0]);
          o[4 + r] = __uint_as_float(sw[1]);
        }
        const U4 packed = pack8(o);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pw_u32x4, packed), rdx,
                                               (uint32_t)(pix * C3_C + col) * 2u, 0, 0);
        float y1[8], gv[8];
        unpack8(*reinterpret_cast<const U4*>(yimg + pw_kmaj(lpx, col >> 3)), y1);
        unpack8(packed, gv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int c = col + k;
          const float gp = fmaf(y1[k], coef[5 * C3_C + c], coef[6 * C3_C + c]) > 0.f ? gv[k] : 0.f;
          bs[k] += gp;
          bq[k] = fmaf(gp, y1[k], bq[k]);
        }
      }
      // the 16 rows of each DPP row share columns: reduce, one LDS float atomic per column and wave
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float sv = row16_sum(bs[k]), qv = row16_sum(bq[k]);
        if ((lane & 15) == 0) {
          atomicAdd(&bnacc[col + k], sv);
          atomicAdd(&bnacc[C3_C + col + k], qv);
        }
      }
    }
  };
  // ---- weight gradient: dW[co][tap][ci] += sum over the tile's pixels of dy2[px][co] a1[px + tap - 1][ci]
  auto wgrad = [&]() {
#pragma unroll 1
    for (int r = 0; r < C3_TR; ++r) {  // k-step = one output row (32 pixels)
      const int hp0 = (r + 1) * C3_HW + 1;
      bf16x8_t fa[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
        fa[m] = pw_frag_tr(timg, 0, wco + 16 * m, lane, [hp0](int kr, int c) { return pw_kmaj(hp0 + kr, c); });
      // B fragments two column tiles ahead (a 3-slot register ring): each transposed LDS read has two
      // iterations of MFMAs to land behind instead of stalling the one right after it
      auto fbld = [&](int nn) {
        const int idx = wng + nn, tap = idx >> 2, cit = idx & 3, ky = tap / 3, kx = tap % 3;
        const int hb0 = (r + ky) * C3_HW + kx;
        return pw_frag_tr(aimg, 0, 16 * cit, lane, [hb0](int kr, int c) { return pw_kmaj(hb0 + kr, c); });
      };
      bf16x8_t fbq[3];
      fbq[0] = fbld(0);
      fbq[1] = fbld(1);
#pragma unroll
      for (int nn = 0; nn < 9; ++nn) {
        if (nn + 2 < 9) fbq[(nn + 2) % 3] = fbld(nn + 2);
        __builtin_amdgcn_sched_barrier(0);  // the prefetch issues before this step's MFMAs
#pragma unroll
        for (int m = 0; m < 2; ++m)
          accw[m][nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fbq[nn % 3], accw[m][nn], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // bound the fragment reads hoisted ahead
      }
    }
  };
  // (measured: placing the epilogue of waves 4-7 after half the weight-gradient k-steps, so SIMD partners
  // reach it at different times, was 3 % slower than this lockstep order -- profiles/r05_conv3)
  auto compute = [&](int tile) {
    f32x4_t acc[2][2];
    dgrad_mfma(acc);
    dgrad_epi(acc, tile);
    wgrad();
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  const int tile0 = blockIdx.x, tstep = gridDim.x;
  issue(tile0);
  __syncthreads();  // weight images, coefficient tables written
  if (tile0 < ntiles) {
    stage(tile0);
    issue(tile0 + tstep);
    sync();
  }
  for (int tile = tile0; tile < ntiles; tile += tstep) {
    compute(tile);
    const int nt = tile + tstep;
    if (nt >= ntiles) break;
    sync();  // every wave is done with this tile's halos
    stage(nt);
    issue(nt + tstep);
    sync();
  }

  // ---- weight-gradient accumulators -> this block's slab, register order (coalesced 16-B stores)
  float* slab = a.slab + (size_t)blockIdx.x * (C3_C * 576);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 9; ++nn)
      *reinterpret_cast<f32x4_t*>(slab + ((size_t)(m * 9 + nn) * PW_NT + t) * 4) = accw[m][nn];
  // ---- BN1 partials of the block -> its slot (one global atomic per value); the block summed g' and
  // g' y1, so sum g' xhat = is1 (sum g' y1) - mu1 is1 (sum g')
  __syncthreads();
  if (t < 2 * C3_C) {
    const int c = t & (C3_C - 1);
    const float v = t < C3_C ? bnacc[t] : fmaf(coef[7 * C3_C + c], bnacc[t], coef[8 * C3_C + c] * bnacc[c]);
    atomicAdd(a.slots1 + (size_t)(blockIdx.x % NSLOT) * 2 * C3_C + t, v);
  }
}

}  // namespace

bool conv3x3_fused_ok(int N, int H, int W, int C, int K) {
  return C == C3_C && K == C3_C && W == C3_IW && H % C3_TR == 0 && N > 0 && (int64_t)N * H * W * C < (1ll << 30);
}

void conv3x3_fwd_fused(const Conv3Args& a, hipStream_t s) {
  const int ntiles = a.N * (a.H / C3_TR);
  conv3x3_fwd_fused_kernel<<<std::min(256, ntiles), PW_NT, 0, s>>>(a);
}

int conv3x3_bwd_fused_grid(int N, int H) { return std::min(256, N * (H / C3_TR)); }

void conv3x3_bwd_fused(const Conv3BwdArgs& a, int nblocks, hipStream_t s) {
  conv3x3_bwd_fused_kernel<<<nblocks, PW_NT, 0, s>>>(a);
}

}  // namespace tfx
