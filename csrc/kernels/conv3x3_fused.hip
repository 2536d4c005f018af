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
// Reference: the conv2 / BN layers of the R/cnn ResNet bottleneck; north-star ResNet-50
// (BASELINE.json config 3).
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

__global__ void __launch_bounds__(PW_NT, 1) conv3x3_fwd_fused_kernel(Conv3Args a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * C3_HBYTES + 9 * C3_WTAP];
  char* wimg = smem + 2 * C3_HBYTES;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int tiles_img = a.H / C3_TR, ntiles = a.N * tiles_img;

  // ---- W [K][3][3][C] -> per-tap K-major images (row = output channel), resident
  for (int q = t; q < 9 * C3_C * 8; q += PW_NT) {
    const int co = q / 72, rem = q % 72, tap = rem / 8, ch = rem % 8;
    *reinterpret_cast<pw_u32x4*>(wimg + tap * C3_WTAP + pw_kmaj(co, ch)) =
        *reinterpret_cast<const pw_u32x4*>(a.w + (int64_t)co * 576 + tap * 64 + ch * 8);
  }
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
      const int hp = (t >> 3) + 64 * i, hy = hp / C3_HW, hx = hp % C3_HW;
      const int iy = y0 + hy - 1, ix = hx - 1;
      const bool in = ok && hp < C3_HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)C3_IW;
      const uint32_t off = in ? (uint32_t)(((n * a.H + iy) * C3_IW + ix) * C3_C + 8 * hch) * 2u : 0x80000000u;
      s.v[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
    }
  };
  // BN1 + ReLU of the staged halo into the LDS image; padding pixels stay zero (not relu(shift))
  auto stage = [&](const Stage& s, char* img, int tile) {
    const int y0 = (tile % tiles_img) * C3_TR;
#pragma unroll
    for (int i = 0; i < C3_PPT; ++i) {
      const int hp = (t >> 3) + 64 * i, hy = hp / C3_HW, hx = hp % C3_HW;
      if (hp < C3_HP) {
        const int iy = y0 + hy - 1, ix = hx - 1;
        const bool in = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)C3_IW;
        float f[8];
        unpack8(__builtin_bit_cast(U4, s.v[i]), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = in ? fmaxf(fmaf(f[k], sc[k], sh[k]), 0.f) : 0.f;
        *reinterpret_cast<U4*>(img + pw_kmaj(hp, hch)) = pack8(f);
      }
    }
  };
  // wave tile: output row r = wv & 3 of the tile (32 pixels = 2 m-tiles), 32 output channels (wv >> 2)
  const int wr = wv & 3, wcb = 32 * (wv >> 2);
  float bs[2][4], bq[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs[j][r] = bq[j][r] = 0.f;
  auto compute = [&](const char* img, int tile) {
    f32x4_t acc[2][2];
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
    // epilogue: y (bf16, 8-byte stores) + BN statistics of the stored values
    const int n = tile / tiles_img, y0 = (tile % tiles_img) * C3_TR;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pix = (n * a.H + y0 + wr) * C3_IW + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wcb + 16 * j + (lane >> 4) * 4;
        const uint32_t lo = pack_bf16x2(acc[i][j][0], acc[i][j][1]), hi = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
        __builtin_amdgcn_raw_buffer_store_b64((pw_u32x2){lo, hi}, ry, (uint32_t)(pix * C3_C + col) * 2u, 0, 0);
        const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u), __uint_as_float(hi << 16),
                            __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bs[j][r] += v[r];
          bq[j][r] = fmaf(v[r], v[r], bq[j][r]);
        }
      }
    }
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
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = row16_sum(bs[j][r]), q = row16_sum(bq[j][r]);
      if ((lane & 15) == 0) {
        const int c = wcb + 16 * j + (lane >> 4) * 4 + r;
        atomicAdd(slots + c, s);
        atomicAdd(slots + C3_C + c, q);
      }
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

}  // namespace tfx
