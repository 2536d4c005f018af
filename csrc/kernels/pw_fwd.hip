// Fused forward of a ResNet bottleneck's block tail and the NEXT block's squeezing 1x1 conv, for gfx950.
//
// Layer-wise, the boundary between two bottlenecks is two passes over the wide (CI-channel) tensor:
//   tail apply   out = relu(y3 * sc3 + sh3 + res)       reads y3, res      writes out, ReLU mask bits
//   next conv1   y1  = out . W1^T  (+ BN1 statistics)  reads out          writes y1 (CO channels)
// Here ONE persistent launch reads y3 and the residual once, forms `out` (bf16, exactly the values
// the apply pass would write) in registers, stores it (the next tail's residual and conv1's
// weight-gradient input still need it) together with the mask bits, and feeds the same registers --
// through LDS -- to conv1's MFMAs with W1 resident in LDS for the whole launch.  The read of `out`
// by conv1 disappears (ResNet-50/CIFAR stage 1: 134 MB per block boundary) and a launch with it.
// RBN: the residual is a projection shortcut's BN output that was never written (its input ysc is
// normalised on the fly with that BN's scale / shift, as bn_apply_res_bn does).
// The epilogue stores y1 and accumulates BN1's statistics (sum, sum of squares of the bf16-rounded
// y1: igemm.hip's EPI_STATS math) over the whole launch: one atomic pair per column per block into
// BN1's slot workspace; the op runs bn_finalize after it, as conv_fwd_bn does.
// Pipeline: as pw_bwd.hip -- 512 threads, one block per CU, a register staging ring of two 32-row
// m-tiles, one barrier per step.
// Reference: no ResNet in the reference; SURVEY §2.7 asks the framework to fuse the reference's
// unfused per-op chain (/root/reference/distributed/distributed.py:96-102) -- here at the north-star
// ResNet-50 scale (BASELINE.json config 3).
#include "pw_common.h"

namespace tfx {
namespace {

// CI = wide input channels (the tail's width), CO = conv1's output channels, BM = rows per m-tile
// (32; 16 when W1 is 128 KB -- ResNet-50 stage 2, 512 -> 128: two 16 KB tile slots + W1 = all 160 KB)
template <int CI, int CO>
struct PwSqueezeCfg {
  static constexpr int BM = CI * CO * 2 > 64 * 1024 ? 16 : PW_BM;
  static constexpr int RG = BM / 16;                   // 16-row groups per tile
  static constexpr int NCH = CI / 64;                  // 64-channel chunks of the wide tile
  static constexpr int TPR = CI / 8;                   // threads per wide row (16-B chunks)
  static constexpr int LPT = BM * TPR / PW_NT;         // wide 16-B loads per thread per tensor per tile
  static constexpr int RSTEP = PW_NT / TPR;            // rows between a thread's loads
  static constexpr int T_BYTES = NCH * BM * 128;       // `out` tile, K-major in 64-channel chunks
  static constexpr int W_BYTES = NCH * CO * 128;       // W1 image (rows = output channel), resident
  static constexpr int DCOLS = CO * RG / 8;            // columns per wave (RG row groups x 8/RG col groups)
  static constexpr int DTN = DCOLS / 16;
  static_assert(LPT >= 1 && BM * TPR % PW_NT == 0, "wide tile mapping");
  static_assert(DTN >= 1 && DCOLS % 16 == 0, "column mapping");
  static_assert(2 * T_BYTES + W_BYTES <= 160 * 1024, "LDS budget");
};

template <int CI, int CO, bool RBN>
__global__ void __launch_bounds__(PW_NT, 1) pw_fwd_squeeze_kernel(PwSqueezeArgs a) {
  using C = PwSqueezeCfg<CI, CO>;
  constexpr int NCH = C::NCH, LPT = C::LPT, TPR = C::TPR, BM = C::BM;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::T_BYTES + C::W_BYTES];
  char* wimg = smem + 2 * C::T_BYTES;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ntiles = a.M / BM;

  // ---- per-thread wide-channel group (fixed for the launch) and the tail's affine maps
  const int chc = t % TPR, c0 = 8 * chc, r0 = t / TPR;
  float sc[8], sh[8], rsc[RBN ? 8 : 1], rsh[RBN ? 8 : 1];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = a.save3[2 * CI + c0 + k];
    sh[k] = a.save3[3 * CI + c0 + k];
    if constexpr (RBN) {
      rsc[k] = a.save_r[2 * CI + c0 + k];
      rsh[k] = a.save_r[3 * CI + c0 + k];
    }
  }
  // ---- W1 [CO][CI] -> K-major image (row = output channel, 64-channel chunks), resident
  pw_resident_copy<CO * CI / 8>(
      t,
      [&](int q) {
        const int n = q / TPR, cc = q % TPR;
        return reinterpret_cast<pw_u32x4*>(wimg + (cc >> 3) * (CO * 128) + pw_kmaj(n, cc & 7));
      },
      [&](int q) { return reinterpret_cast<const pw_u32x4*>(a.w) + q; });

  const int64_t wide = (int64_t)a.M * CI * 2;
  const __amdgpu_buffer_rsrc_t ry = pw_rsrc(a.y3, wide), rr = pw_rsrc(a.res, wide);
  const __amdgpu_buffer_rsrc_t ro = pw_rsrc(a.out, wide), rm = pw_rsrc(a.mask, (int64_t)a.M * CI / 8);
  const __amdgpu_buffer_rsrc_t r1 = pw_rsrc(a.y1, (int64_t)a.M * CO * 2);

  // wave tile: rows 16 (wv % RG), columns DCOLS (wv / RG); SWAP orientation -> lane holds row
  // (lane & 15), columns cb + (lane >> 4) * 4 + r of each 16-col tile
  const int rb = 16 * (wv % C::RG), cb = C::DCOLS * (wv / C::RG);
  float bs[C::DTN][4], bq[C::DTN][4];  // BN1 statistics of this lane's columns, whole launch
#pragma unroll
  for (int j = 0; j < C::DTN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs[j][r] = bq[j][r] = 0.f;

  struct Stage {
    pw_u32x4 y[LPT], r[LPT];
  };
  Stage st0, st1;
  const int tile0 = blockIdx.x, tstep = gridDim.x;
  auto issue = [&](Stage& s, int tile) {
    const bool ok = tile < ntiles;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int row = tile * BM + r0 + C::RSTEP * i;
      const uint32_t off = ok ? (uint32_t)(row * CI + c0) * 2u : 0x80000000u;
      s.y[i] = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
      s.r[i] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
    }
  };
  // tail apply of the staged tile: `out` + mask bits to memory, `out` into the LDS slot
  auto stage = [&](const Stage& s, char* slot, int tile) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      float yf[8], rf[8];
      unpack8(__builtin_bit_cast(U4, s.y[i]), yf);
      unpack8(__builtin_bit_cast(U4, s.r[i]), rf);
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float z = fmaf(yf[k], sc[k], sh[k]);
        if constexpr (RBN) z += fmaf(rf[k], rsc[k], rsh[k]);
        else z += rf[k];
        bits |= (z > 0.f ? 1u : 0u) << k;
        yf[k] = fmaxf(z, 0.f);
      }
      const U4 o = pack8(yf);
      const int lrow = r0 + C::RSTEP * i, row = tile * BM + lrow;
      *reinterpret_cast<U4*>(slot + (chc >> 3) * (BM * 128) + pw_kmaj(lrow, chc & 7)) = o;
      if (tile < ntiles) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pw_u32x4, o), ro, (uint32_t)(row * CI + c0) * 2u, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bits, rm, (uint32_t)(row * TPR + chc), 0, 0);
      }
    }
  };
  auto compute = [&](const char* slot, int tile) {
    f32x4_t acc[C::DTN];
#pragma unroll
    for (int j = 0; j < C::DTN; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < CI / 32; ++kc) {  // 32-deep k-steps over the wide channels
      const bf16x8_t fa = pw_frag_kmaj(slot, (kc >> 1) * (BM * 128), rb, 4 * (kc & 1), lane);
#pragma unroll
      for (int j = 0; j < C::DTN; ++j) {
        const bf16x8_t fb = pw_frag_kmaj(wimg, (kc >> 1) * (CO * 128), cb + 16 * j, 4 * (kc & 1), lane);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa, acc[j], 0, 0, 0);  // SWAP
      }
    }
    const int row = tile * BM + rb + (lane & 15);
#pragma unroll
    for (int j = 0; j < C::DTN; ++j) {
      const int col = cb + 16 * j + (lane >> 4) * 4;
      const uint32_t lo = pack_bf16x2(acc[j][0], acc[j][1]), hi = pack_bf16x2(acc[j][2], acc[j][3]);
      __builtin_amdgcn_raw_buffer_store_b64((pw_u32x2){lo, hi}, r1, (uint32_t)(row * CO + col) * 2u, 0, 0);
      // statistics of exactly the bf16 values BN1 will read
      const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u), __uint_as_float(hi << 16),
                          __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bs[j][r] += v[r];
        bq[j][r] = fmaf(v[r], v[r], bq[j][r]);
      }
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  // ---- main loop over this block's m-tiles (tile0, tile0 + tstep, ...): staged two ahead
  issue(st0, tile0);
  issue(st1, tile0 + tstep);
  __syncthreads();  // W1 image written
  for (int tile = tile0; tile < ntiles; tile += 2 * tstep) {
    stage(st0, smem, tile);
    issue(st0, tile + 2 * tstep);
    sync();
    compute(smem, tile);
    const int t1 = tile + tstep;
    if (t1 >= ntiles) break;
    stage(st1, smem + C::T_BYTES, t1);
    issue(st1, t1 + 2 * tstep);
    sync();
    compute(smem + C::T_BYTES, t1);
  }

  // ---- BN1 statistics: sum the 16 rows of each DPP row (same columns), one atomic pair per column
  float* slots = a.slots1 + (size_t)(blockIdx.x % NSLOT) * 2 * CO;
#pragma unroll
  for (int j = 0; j < C::DTN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = row16_sum(bs[j][r]), q = row16_sum(bq[j][r]);
      if ((lane & 15) == 0) {
        const int c = cb + 16 * j + (lane >> 4) * 4 + r;
        atomicAdd(slots + c, s);
        atomicAdd(slots + CO + c, q);
      }
    }
}

}  // namespace

bool pw_fwd_squeeze_ok(int CI, int CO, int64_t M) {
  const bool s1 = CI == 256 && (CO == 64 || CO == 128), s2 = CI == 512 && CO == 128;
  const int bm = s2 ? PwSqueezeCfg<512, 128>::BM : PW_BM;
  return (s1 || s2) && M % bm == 0 && M > 0 && (int64_t)M * CI < (1ll << 30);
}

int pw_fwd_squeeze_grid(int CI, int CO, int64_t M) {
  const int bm = (CI == 512 && CO == 128) ? PwSqueezeCfg<512, 128>::BM : PW_BM;
  return (int)std::min<int64_t>(256, M / bm);
}

void pw_fwd_squeeze(const PwSqueezeArgs& args, int nblocks, hipStream_t s) {
  const bool rbn = args.save_r != nullptr;
#define TFX_PWF(CI_, CO_)                                                                             \
  if (rbn) pw_fwd_squeeze_kernel<CI_, CO_, true><<<nblocks, PW_NT, 0, s>>>(args);                     \
  else pw_fwd_squeeze_kernel<CI_, CO_, false><<<nblocks, PW_NT, 0, s>>>(args);
  if (args.CI == 256 && args.CO == 64) {
    TFX_PWF(256, 64)
  } else if (args.CI == 256 && args.CO == 128) {
    TFX_PWF(256, 128)
  } else if (args.CI == 512 && args.CO == 128) {
    TFX_PWF(512, 128)
  } else {
    abort();
  }
#undef TFX_PWF
}

}  // namespace tfx
