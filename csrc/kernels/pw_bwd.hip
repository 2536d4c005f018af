// Fused backward of a ResNet bottleneck's EXPANDING 1x1 conv (conv3: narrow width CN -> wide CW = 4 CN)
// together with the block-tail BN's backward apply, for gfx950.
//
// The layer-wise backward of an identity block's tail is three passes over wide (CW-channel) tensors:
//   bn_bwd_apply   dy3 = A (g * relu_mask) + B y3 + D          reads g, y3, mask   writes dy3
//   conv3 dgrad    dA2 = dy3 . W3        (+ BN2-backward partials of dA2 in the epilogue)   reads dy3
//   conv3 wgrad    dW3 += dy3^T . a2                                                         reads dy3
// Here ONE persistent launch reads g, y3 and the mask bits once, forms dy3 (bf16, as the apply pass
// would have written it) straight into LDS, and runs BOTH GEMMs from that tile: per 32-row m-tile
//   dgrad  acc_d[32 x CN]  += T[32 x CW] . W3[CW x CN]      (W3 resident in LDS for the whole launch)
//   wgrad  acc_w[CW x CN]  += T^T[CW x 32] . A2[32 x CN]    (accumulated in registers over every
//                                                            m-tile of the block)
// so dy3 never exists in HBM: two wide passes and a launch fewer per block (ResNet-50/CIFAR stage 1:
// 134 MB each).  The dgrad epilogue stores dA2 and accumulates the BN2 backward partials (sum g',
// sum g' xhat with g' = bf16(dA2) * [y2 scale + shift > 0]) -- igemm.hip's EPI_BNB math.  Each block
// leaves its wgrad accumulator in a per-block f32 slab (plain coalesced stores, no f32 atomics:
// MI355X_MICROARCH.md "Global float atomics" runs those at ~1.3 TB/s); pw_slab_reduce then sums the
// slabs into dW3 and, in tail blocks of the same launch, reduces BN2's slots.
//
// Pipeline: 512 threads (8 waves), one block per CU, register staging ring of two m-tiles: at step i
// tile i's staged registers are transformed into LDS slot i%2, then tile i+2 is issued into the same
// registers -- two m-tiles (~90 KB) in flight per CU while tile i computes.  One barrier per step
// (two LDS slots: a slot is rewritten two steps after it was read, behind the barrier between).
// Reference: the unfused chain of R/distributed/distributed.py:96-102 that SURVEY §2.7 says the
// framework fuses; north-star ResNet-50 (BASELINE.json configs 3).
#include "pw_common.h"

namespace tfx {
namespace {

// ---------------------------------------------------------------------------------- F3 (expand)
// CN = narrow width (conv3 input channels), CW = 4 CN (conv3 output channels).
template <int CN>
struct PwExpandCfg {
  static constexpr int CW = 4 * CN;
  static constexpr int NCH = CW / 64;                  // 64-channel chunks of the wide tile
  static constexpr int TPR = CW / 8;                   // threads per wide row (16-B chunks)
  static constexpr int LPT = PW_BM * TPR / PW_NT;      // wide-tensor 16-B loads per thread per tile
  static constexpr int RSTEP = PW_NT / TPR;            // rows between a thread's loads
  static constexpr int NTPR = CN / 8;                  // threads per narrow row
  static constexpr int NLD = PW_BM * NTPR;             // threads that load one narrow chunk
  static constexpr int T_BYTES = NCH * PW_BM * 128;    // dy3 tile (K-major, 64-channel chunks)
  static constexpr int A2_BYTES = PW_BM * CN * 2;      // a2 tile (row-major, MN image)
  static constexpr int SLOT = T_BYTES + A2_BYTES;
  static constexpr int W_BYTES = CW * CN * 2;          // W3 image, resident
  static constexpr int WCOLS = CN / 2;                 // wgrad: columns per wave (2 column groups)
  static constexpr int WTN = WCOLS / 16;               // wgrad: 16-col tiles per wave per chunk
  static constexpr int DCOLS = CN / 4;                 // dgrad: columns per wave (2 x 4 waves)
  static constexpr int DTN = DCOLS / 16;
  static_assert(LPT >= 1 && PW_BM * TPR % PW_NT == 0, "wide tile mapping");
  static_assert(NLD <= PW_NT, "narrow tile mapping");
  static_assert(2 * SLOT + W_BYTES <= 160 * 1024, "LDS budget");
};

// SEC (a projection block's tail): the residual was the shortcut BN's output, used only there, so its
// output gradient is the same g' = g * mask -- accumulate that BN's sum g' * ysc per channel while g'
// is in registers (pw_slab_reduce turns it into sum g' * xhat_sc); its sum g' equals red3's.
template <int CN, bool SEC>
__global__ void __launch_bounds__(PW_NT, 1) pw_bwd_expand_kernel(PwExpandArgs a) {
  using C = PwExpandCfg<CN>;
  constexpr int CW = C::CW, NCH = C::NCH, LPT = C::LPT, TPR = C::TPR;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::SLOT + C::W_BYTES + (SEC ? 8 * 4 * PW_NT : 0)];
  char* wimg = smem + 2 * C::SLOT;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ntiles = a.M / PW_BM;

  // ---- per-thread wide-channel group (fixed for the whole launch) and its BN3 backward coefficients
  const int chc = t % TPR, c0 = 8 * chc, r0 = t / TPR;
  float A[8], B[8], D[8];
  {
    const float inv_m = 1.f / (float)a.M;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      const float mu = a.save3[c], is = a.save3[CW + c], sc = a.save3[2 * CW + c];
      const float kg = a.red3[c] * inv_m, kx = a.red3[CW + c] * inv_m * is;
      A[k] = sc;
      B[k] = -sc * kx;
      D[k] = sc * (kx * mu - kg);
    }
  }
  // ---- W3 [CW][CN] -> MN image (rows = k = wide channel), resident
  pw_resident_copy<CW * CN / 8>(
      t, [&](int q) { return reinterpret_cast<pw_u32x4*>(wimg + pw_mn<CN>(q / (CN / 8), q % (CN / 8))); },
      [&](int q) { return reinterpret_cast<const pw_u32x4*>(a.w) + q; });

  const __amdgpu_buffer_rsrc_t rg = pw_rsrc(a.g, (int64_t)a.M * CW * 2), ry = pw_rsrc(a.y3, (int64_t)a.M * CW * 2);
  const __amdgpu_buffer_rsrc_t rm = pw_rsrc(a.mask3, (int64_t)a.M * CW / 8);
  const __amdgpu_buffer_rsrc_t ra = pw_rsrc(a.a2, (int64_t)a.M * CN * 2);
  const __amdgpu_buffer_rsrc_t rx2 = pw_rsrc(a.y2, a.y2 ? (int64_t)a.M * CN * 2 : 0);
  const __amdgpu_buffer_rsrc_t rsc = pw_rsrc(a.ysc, SEC ? (int64_t)a.M * CW * 2 : 0);
  // SEC: sum g' * ysc per channel of this thread, accumulated in a private LDS column qcol[k][PW_NT]
  // (registers are full); the tail turns it into sum g' * xhat_sc = is_sc * (S - mu_sc * sum g') with
  // red3's sum g'.  ysc is staged ONE tile ahead in a single register buffer (the ring is two deep).
  float* qcol = reinterpret_cast<float*>(smem + 2 * C::SLOT + C::W_BYTES);
  if constexpr (SEC) {
#pragma unroll
    for (int k = 0; k < 8; ++k) qcol[k * PW_NT + t] = 0.f;
  }
  pw_u32x4 ysb[SEC ? LPT : 1];
  auto issue_ys = [&](int tile) {
    if constexpr (SEC) {
      const bool ok = tile < ntiles;
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int row = tile * PW_BM + r0 + C::RSTEP * i;
        ysb[i] = __builtin_amdgcn_raw_buffer_load_b128(rsc, ok ? (uint32_t)(row * CW + c0) * 2u : 0x80000000u, 0, 0);
      }
    }
  };

  // a2_save: conv3's input is relu(BN2(y2)) formed on load from y2 (a.a2 holds y2); this thread's
  // narrow chunk is channels 8 (t % NTPR) .. +7.  Scale / shift live in an LDS table, read per tile:
  // held in registers (16 per lane) they pushed the SEC variant past 256 VGPRs into scratch, and every
  // scratch reload inside the loop waited vmcnt(0) -- draining the next tiles' loads with it.
  const bool a2_bn = a.a2_save != nullptr;
  __shared__ float a2tab[2 * CN];
  for (int c = t; c < CN; c += PW_NT) {
    a2tab[c] = a2_bn ? a.a2_save[2 * CN + c] : 1.f;
    a2tab[CN + c] = a2_bn ? a.a2_save[3 * CN + c] : 0.f;
  }
  // dgrad wave tile: rows 16 (wv & 1), columns DCOLS (wv >> 1); SWAP orientation -> lane holds row
  // (lane & 15), columns dcb + (lane >> 4) * 4 + r of each 16-col tile
  const int drb = 16 * (wv & 1), dcb = C::DCOLS * (wv >> 1);
  // BN2 backward partials of this lane's 4 * DTN columns (accumulated over the whole launch)
  float bs[C::DTN][4], bq[C::DTN][4], mu2[C::DTN][4], is2[C::DTN][4], sc2[C::DTN][4], sh2[C::DTN][4];
#pragma unroll
  for (int j = 0; j < C::DTN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = dcb + 16 * j + (lane >> 4) * 4 + r;
      bs[j][r] = bq[j][r] = 0.f;
      mu2[j][r] = a.y2 ? a.save2[c] : 0.f;
      is2[j][r] = a.y2 ? a.save2[CN + c] : 0.f;
      sc2[j][r] = a.y2 ? a.save2[2 * CN + c] : 0.f;
      sh2[j][r] = a.y2 ? a.save2[3 * CN + c] : 0.f;
    }
  // wgrad wave tile: chunk rows 16 (wv & 3) of every chunk, columns WCOLS (wv >> 2)
  const int wrb = 16 * (wv & 3), wcb = C::WCOLS * (wv >> 2);
  f32x4_t accw[NCH][C::WTN];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int n = 0; n < C::WTN; ++n) accw[j][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // ---- register staging ring (two tiles)
  struct Stage {
    pw_u32x4 g[LPT], y[LPT];
    uint32_t m[LPT];
    pw_u32x4 a2;
    pw_u32x2 x2[C::DTN];
  };
  Stage st0, st1;
  const int tile0 = blockIdx.x, tstep = gridDim.x;
  auto issue = [&](Stage& s, int tile) {
    const bool ok = tile < ntiles;
    const int row0 = tile * PW_BM;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int row = row0 + r0 + C::RSTEP * i;
      const uint32_t off = ok ? (uint32_t)(row * CW + c0) * 2u : 0x80000000u;
      s.g[i] = __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 0);
      s.y[i] = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
      s.m[i] = __builtin_amdgcn_raw_buffer_load_b8(rm, ok ? (uint32_t)(row * TPR + chc) : 0x80000000u, 0, 0);
    }
    {
      const int row = row0 + t / C::NTPR, cc = t % C::NTPR;
      const bool aok = ok && t < C::NLD;
      s.a2 = __builtin_amdgcn_raw_buffer_load_b128(ra, aok ? (uint32_t)(row * CN + 8 * cc) * 2u : 0x80000000u, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < C::DTN; ++j) {
      const int row = row0 + drb + (lane & 15), col = dcb + 16 * j + (lane >> 4) * 4;
      s.x2[j] = __builtin_amdgcn_raw_buffer_load_b64(rx2, ok ? (uint32_t)(row * CN + col) * 2u : 0x80000000u, 0, 0);
    }
  };
  // transform tile (registers) -> LDS slot; the epilogue's y2 values move to `x2` (the staging
  // registers are re-issued before the tile computes)
  pw_u32x2 x2[C::DTN];
  auto stage = [&](const Stage& s, char* slot, int next_tile) {
#pragma unroll
    for (int j = 0; j < C::DTN; ++j) x2[j] = s.x2[j];
    float q[SEC ? 8 : 1];
    if constexpr (SEC) {
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = qcol[k * PW_NT + t];
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      float gf[8], yf[8], o[8];
      unpack8(__builtin_bit_cast(U4, s.g[i]), gf);
      unpack8(__builtin_bit_cast(U4, s.y[i]), yf);
      float sf[SEC ? 8 : 1];
      if constexpr (SEC) unpack8(__builtin_bit_cast(U4, ysb[i]), sf);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gg = ((s.m[i] >> k) & 1u) ? gf[k] : 0.f;
        o[k] = fmaf(A[k], gg, fmaf(B[k], yf[k], D[k]));
        if constexpr (SEC) q[k] = fmaf(gg, sf[k], q[k]);
      }
      const int row = r0 + C::RSTEP * i;
      *reinterpret_cast<U4*>(slot + (chc >> 3) * (PW_BM * 128) + pw_kmaj(row, chc & 7)) = pack8(o);
    }
    if constexpr (SEC) {
#pragma unroll
      for (int k = 0; k < 8; ++k) qcol[k * PW_NT + t] = q[k];
      issue_ys(next_tile);
    }
    if (t < C::NLD) {
      const int row = t / C::NTPR, cc = t % C::NTPR;
      pw_u32x4 v = s.a2;
      if (a2_bn) {  // uniform: BN2 + ReLU of the staged y2 piece (rows past M are never stored)
        float f[8];
        unpack8(__builtin_bit_cast(U4, v), f);
        const float4 s0 = *reinterpret_cast<const float4*>(a2tab + 8 * cc);
        const float4 s1 = *reinterpret_cast<const float4*>(a2tab + 8 * cc + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(a2tab + CN + 8 * cc);
        const float4 h1 = *reinterpret_cast<const float4*>(a2tab + CN + 8 * cc + 4);
        const float a2s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float a2h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], a2s[k], a2h[k]), 0.f);
        v = __builtin_bit_cast(pw_u32x4, pack8(f));
      }
      *reinterpret_cast<pw_u32x4*>(slot + C::T_BYTES + pw_mn<CN>(row, cc)) = v;
    }
  };
  auto compute = [&](const char* slot, int tile) {
    // dgrad: acc_d[32 x CN] = T[32 x CW] . W3
    f32x4_t accd[C::DTN];
#pragma unroll
    for (int j = 0; j < C::DTN; ++j) accd[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < CW / 32; ++kc) {  // 32-deep k-steps over the wide channels
      const bf16x8_t fa = pw_frag_kmaj(slot, (kc >> 1) * (PW_BM * 128), drb, 4 * (kc & 1), lane);
#pragma unroll
      for (int j = 0; j < C::DTN; ++j) {
        const bf16x8_t fb = pw_frag_tr(wimg, 32 * kc * CN * 2, dcb + 16 * j, lane,
                                       [](int r, int c) { return pw_mn<CN>(r, c); });
        accd[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa, accd[j], 0, 0, 0);  // SWAP
      }
    }
    // wgrad: acc_w[CW x CN] += T^T . A2 (k = the tile's 32 rows)
    bf16x8_t fb2[C::WTN];
#pragma unroll
    for (int n = 0; n < C::WTN; ++n)
      fb2[n] = pw_frag_tr(slot + C::T_BYTES, 0, wcb + 16 * n, lane, [](int r, int c) { return pw_mn<CN>(r, c); });
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const bf16x8_t fa = pw_frag_tr(slot + j * (PW_BM * 128), 0, wrb, lane, [](int r, int c) { return pw_kmaj(r, c); });
#pragma unroll
      for (int n = 0; n < C::WTN; ++n) accw[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb2[n], accw[j][n], 0, 0, 0);
    }
    // dgrad epilogue: dA2 (bf16, 8-byte stores) + BN2 backward partials
    const int row = tile * PW_BM + drb + (lane & 15);
#pragma unroll
    for (int j = 0; j < C::DTN; ++j) {
      const int col = dcb + 16 * j + (lane >> 4) * 4;
      const uint32_t lo = pack_bf16x2(accd[j][0], accd[j][1]), hi = pack_bf16x2(accd[j][2], accd[j][3]);
      *reinterpret_cast<pw_u32x2*>(a.dA2 + (int64_t)row * CN + col) = (pw_u32x2){lo, hi};
      if (a.y2) {
        const float gv[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                             __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
        const float xv[4] = {__uint_as_float(x2[j][0] << 16), __uint_as_float(x2[j][0] & 0xffff0000u),
                             __uint_as_float(x2[j][1] << 16), __uint_as_float(x2[j][1] & 0xffff0000u)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gp = (!a.relu2 || fmaf(xv[r], sc2[j][r], sh2[j][r]) > 0.f) ? gv[r] : 0.f;
          bs[j][r] += gp;
          bq[j][r] = fmaf(gp, (xv[r] - mu2[j][r]) * is2[j][r], bq[j][r]);
        }
      }
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  // ---- main loop over this block's m-tiles (tile0, tile0 + tstep, ...): staged two ahead
  // ysc first: in the loop it is issued before the next tiles' loads, so the waitcnt pass (which merges
  // the prologue's and the back edge's outstanding loads at the loop header) sees the same order here --
  // issued last, its wait at the header drained every load in flight
  issue_ys(tile0);
  issue(st0, tile0);
  issue(st1, tile0 + tstep);
  __syncthreads();  // W3 image written
  for (int tile = tile0; tile < ntiles; tile += 2 * tstep) {
    stage(st0, smem, tile + tstep);
    issue(st0, tile + 2 * tstep);
    sync();
    compute(smem, tile);
    const int t1 = tile + tstep;
    if (t1 >= ntiles) break;
    stage(st1, smem + C::SLOT, t1 + tstep);
    issue(st1, t1 + 2 * tstep);
    sync();
    compute(smem + C::SLOT, t1);
  }

  // ---- wgrad accumulators -> this block's slab, in register order (coalesced 16-B stores)
  float* slab = a.slab + (size_t)blockIdx.x * (CW * CN);
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int n = 0; n < C::WTN; ++n)
      *reinterpret_cast<f32x4_t*>(slab + ((size_t)(j * C::WTN + n) * PW_NT + t) * 4) = accw[j][n];
  // ---- SEC partials: threads t, t + TPR, ... share channel group chc -> sum their LDS columns,
  // one atomic per channel
  if constexpr (SEC) {
    __syncthreads();
    const float* red = qcol;
    if (t < TPR) {
      float* slots = a.slots_sc + (size_t)(blockIdx.x % NSLOT) * 2 * CW;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float q = 0.f;
        for (int r = 0; r < PW_NT / TPR; ++r) q += red[k * PW_NT + r * TPR + t];
        atomicAdd(slots + CW + c0 + k, q);
      }
    }
  }
  // ---- BN2 partials: sum the 16 rows of each DPP row (same columns), one atomic per column
  if (a.y2) {
    float* slots = a.slots2 + (size_t)(blockIdx.x % NSLOT) * 2 * CN;
#pragma unroll
    for (int j = 0; j < C::DTN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = row16_sum(bs[j][r]), q = row16_sum(bq[j][r]);
        if ((lane & 15) == 0) {
          const int c = dcb + 16 * j + (lane >> 4) * 4 + r;
          atomicAdd(slots + c, s);
          atomicAdd(slots + CN + c, q);
        }
      }
  }
}

// zero the bf16 halves of 8 x bf16 whose bit in `bits` is clear (as igemm_impl.h mask_bf16x8)
__device__ __forceinline__ U4 mask_bf16x8_pw(const U4& v, uint32_t bits) {
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

// ---------------------------------------------------------------------------------- F1 (squeeze)
// Backward of an identity bottleneck's SQUEEZING 1x1 conv1 (CI wide -> CO narrow) fused with BN1's
// backward apply.  Layer-wise: bn_bwd_apply (dy1, narrow), conv1 dgrad (dx, wide: + the residual
// branch's masked gradient + the previous tail BN's backward partials in its epilogue), conv1 wgrad.
// Here per 32-row m-tile:
//   T1 = A1 (g1 * relu1) + B1 y1 + D1        (relu1 from y1 sc1 + sh1 > 0; bf16, LDS only)
//   dgrad  dx [32 x CI] = T1 . W1 + addend * amask     (W1 resident as an MN image: rows = co)
//          epilogue: dx stored; previous tail BN partials (sum g', sum g' xhat), g' = bf16(dx) * pmask
//   wgrad  dW1 [CO x CI] += T1^T . X                   (X = conv1's input tile, MN image)
// dy1 never exists in HBM and dx's tensors are read once: the launch moves g1, y1, X, the addend and
// its mask, the previous tail's input and mask, and writes dx (ResNet-50/CIFAR stage 1: ~610 MB).
// wide-column split of the F1 kernel per narrow width (see PwSqueezeBwdCfg)
constexpr int pw_squeeze_split(int CO) { return CO == 128 ? 4 : 1; }

// Wide columns split over S blocks (stage 2, CI = 512 / CO = 128: W1 is 128 KB, too big to sit in LDS
// beside the tiles, and a CO x CI/2 wgrad accumulator spills at 256 VGPRs; S = 4 blocks each keep a
// CO x CI/4 slice resident and take the same m-tiles' other columns -- the narrow g1 / y1 pieces are
// read by all four, ~30 % of the launch's bytes).  Block b runs one part over m-tiles t0, t0 + grid / S,
// ... (mapping in the kernel); its wgrad slab is slab part * grid / S + t0.
template <int CI, int CO, int S>
struct PwSqueezeBwdCfg {
  static constexpr int CIH = CI / S;                   // wide columns per block
  static constexpr int NPC = CO * PW_BM / PW_NT;       // narrow channels per thread piece (4 or 8)
  static constexpr int NTPR = CO / NPC;                // threads per narrow row
  static constexpr int TPR = CIH / 8;                  // threads per wide row (16-B pieces)
  static constexpr int RSTEP = PW_NT / TPR;            // rows between a thread's wide pieces
  static constexpr int LPT = PW_BM * TPR / PW_NT;      // wide pieces per thread per tensor per tile
  static constexpr int T_BYTES = PW_BM * CO * 2;       // T1 tile: CO / 64 K-major images of 64-channel rows
  static constexpr int X_BYTES = PW_BM * CIH * 2;      // X tile, MN image
  static constexpr int SLOT = T_BYTES + X_BYTES;
  static constexpr int W_BYTES = CO * CIH * 2;         // W1 slice MN image (rows = co), resident
  static constexpr int D_BYTES = PW_BM * CIH * 4;      // dgrad accumulator tile (f32), epilogue hand-off
  static constexpr int DCOLS = CIH / 4;                // dgrad columns per wave (2 row x 4 col groups)
  static constexpr int DTN = DCOLS / 16;
  static constexpr int WROWS = CO / 2;                 // wgrad: co rows per wave (2 groups)
  static constexpr int WTM = WROWS / 16;
  static constexpr int WCOLS = CIH / 4;                // wgrad: ci columns per wave (4 groups)
  static constexpr int WTN = WCOLS / 16;
  static_assert(CO % 64 == 0 && (NPC == 4 || NPC == 8), "T1: 64-channel K-major chunks, 8 / 16-B pieces");
  static_assert(PW_BM * NTPR == PW_NT, "narrow tile mapping");
  static_assert(LPT >= 1 && PW_BM * TPR % PW_NT == 0, "wide tile mapping");
  static_assert(2 * SLOT + W_BYTES + D_BYTES + (2 * CIH + 5 * CO) * 4 <= 160 * 1024, "LDS budget");
  static_assert(16 * PW_NT * 4 <= 2 * SLOT, "previous tail partials tree in the (free) slot area");
};
// byte offset of 16-B chunk c (8 narrow channels) of row r in the T1 image (64-channel K-major images)
__device__ __forceinline__ int pw_toff(int r, int c) { return (c >> 3) * (PW_BM * 128) + pw_kmaj(r, c & 7); }

// D tile (f32 [32][CI]): 16-B chunk q of row r at r * CI * 4 + ((q ^ (r & 7)) << 4)  (the SWAP writers put
// 16 rows x 4 consecutive columns per instruction; the row-contiguous readers take 32 B of one row)
template <int CI>
__device__ __forceinline__ int pw_doff(int r, int q) { return r * CI * 4 + ((q ^ (r & 7)) << 4); }

template <int CI, int CO, int S>
__global__ void __launch_bounds__(PW_NT, 1) pw_bwd_squeeze_kernel(PwSqueezeBwdArgs a) {
  using C = PwSqueezeBwdCfg<CI, CO, S>;
  constexpr int LPT = C::LPT, CIH = C::CIH, NPC = C::NPC;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::SLOT + C::W_BYTES + C::D_BYTES + (2 * CIH + 5 * CO) * 4];
  char* wimg = smem + 2 * C::SLOT;
  char* dimg = wimg + C::W_BYTES;
  // previous tail BN's [invstd | -mean invstd] per wide channel; BN1's [A | B | D | scale | shift]
  float* pcoef = reinterpret_cast<float*>(dimg + C::D_BYTES);
  float* ncoef = pcoef + 2 * CIH;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ntiles = a.M / PW_BM;
  // column part and first m-tile of this block.  With the grid a multiple of 8 S the split is XCD-aware:
  // blocks are dispatched round-robin over the 8 XCDs (b % 8), and the S parts of one m-tile stride take
  // consecutive slots of ONE XCD, so the narrow g1 / y1 pieces they all read are shared through that
  // XCD's L2 instead of being fetched once per XCD.  Other grids: part b % S, tile b / S.
  const int b = (int)blockIdx.x;
  const bool xcd_split = S > 1 && (int)gridDim.x % (8 * S) == 0;
  const int part = S == 1 ? 0 : xcd_split ? (b / 8) % S : b % S, col0 = part * CIH;  // this block's wide columns
  const int tile0 = S == 1 ? b : xcd_split ? (b % 8) + 8 * (b / (8 * S)) : b / S;

  for (int c = t; c < CIH; c += PW_NT) {
    const float is = a.psave[CI + col0 + c];
    pcoef[c] = is;
    pcoef[CIH + c] = -a.psave[col0 + c] * is;
  }
  if (t < CO) {
    const float inv_m = 1.f / (float)a.M;
    const float mu = a.save1[t], is = a.save1[CO + t], sc = a.save1[2 * CO + t];
    const float kg = a.red1[t] * inv_m, kx = a.red1[CO + t] * inv_m * is;
    ncoef[t] = sc;
    ncoef[CO + t] = -sc * kx;
    ncoef[2 * CO + t] = sc * (kx * mu - kg);
    ncoef[3 * CO + t] = sc;
    ncoef[4 * CO + t] = a.save1[3 * CO + t];
  }
  // ---- W1 [CO][col0 .. col0 + CIH) -> MN image (row = co), resident
  pw_resident_copy<CO * CIH / 8>(
      t, [&](int q) { return reinterpret_cast<pw_u32x4*>(wimg + pw_mn<CIH>(q / (CIH / 8), q % (CIH / 8))); },
      [&](int q) {
        return reinterpret_cast<const pw_u32x4*>(a.w) + (q / (CIH / 8)) * (CI / 8) + col0 / 8 + q % (CIH / 8);
      });
  const int64_t wide = (int64_t)a.M * CI * 2, narrow = (int64_t)a.M * CO * 2;
  const __amdgpu_buffer_rsrc_t rg = pw_rsrc(a.g1, narrow), ry = pw_rsrc(a.y1, narrow), rx = pw_rsrc(a.x, wide);
  const __amdgpu_buffer_rsrc_t rad = pw_rsrc(a.addend, wide), ram = pw_rsrc(a.amask, (int64_t)a.M * CI / 8);
  const __amdgpu_buffer_rsrc_t rpx = pw_rsrc(a.px, wide), rpm = pw_rsrc(a.pmask, (int64_t)a.M * CI / 8);
  const __amdgpu_buffer_rsrc_t rdx = pw_rsrc(a.dx, wide);

  // narrow piece (g1 / y1 -> T1): row t / NTPR, channels nc0 .. nc0 + NPC - 1
  const int nrow = t / C::NTPR, nc0 = NPC * (t % C::NTPR);
  // wide pieces (X, addend, previous tail input, masks; the dx epilogue): rows r0 + RSTEP i, channels
  // 8 chc .. 8 chc + 7 -- fixed for the launch, so the previous tail BN's partials stay per thread
  const int chc = t % C::TPR, r0 = t / C::TPR;
  float bs[8], bq[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) bs[k] = bq[k] = 0.f;
  // dgrad wave tile: rows 16 (wv & 1), columns DCOLS (wv >> 1); SWAP
  const int drb = 16 * (wv & 1), dcb = C::DCOLS * (wv >> 1);
  // wgrad wave tile: co rows WROWS (wv & 1), ci columns WCOLS (wv >> 1); !SWAP
  const int wrb = C::WROWS * (wv & 1), wcb = C::WCOLS * (wv >> 1);
  f32x4_t accw[C::WTM][C::WTN];
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int n = 0; n < C::WTN; ++n) accw[i][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // ---- register staging ring (two tiles): every operand of a tile, coalesced 8 / 16-B pieces
  using NV = std::conditional_t<NPC == 4, pw_u32x2, pw_u32x4>;
  struct Stage {
    NV g, y;
    pw_u32x4 x[LPT], ad[LPT], px[LPT];
    uint32_t mk[LPT];  // addend mask byte | previous tail mask byte << 8
  };
  Stage st0, st1;
  const int tstep = (int)gridDim.x / S;
  auto issue = [&](Stage& s, int tile) {
    const bool ok = tile < ntiles;
    const uint32_t no = ok ? (uint32_t)((tile * PW_BM + nrow) * CO + nc0) * 2u : 0x80000000u;
    if constexpr (NPC == 4) {
      s.g = __builtin_amdgcn_raw_buffer_load_b64(rg, no, 0, 0);
      s.y = __builtin_amdgcn_raw_buffer_load_b64(ry, no, 0, 0);
    } else {
      s.g = __builtin_amdgcn_raw_buffer_load_b128(rg, no, 0, 0);
      s.y = __builtin_amdgcn_raw_buffer_load_b128(ry, no, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int row = tile * PW_BM + r0 + C::RSTEP * i;
      const uint32_t o = ok ? (uint32_t)(row * CI + col0 + 8 * chc) * 2u : 0x80000000u;
      const uint32_t ob = ok ? (uint32_t)(row * (CI / 8) + col0 / 8 + chc) : 0x80000000u;
      s.x[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0);
      s.ad[i] = __builtin_amdgcn_raw_buffer_load_b128(rad, o, 0, 0);
      s.px[i] = __builtin_amdgcn_raw_buffer_load_b128(rpx, o, 0, 0);
      s.mk[i] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(ram, ob, 0, 0) |
                ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rpm, ob, 0, 0) << 8);
    }
  };
  // epilogue operands of the tile being staged move to `ep` (the staging registers are re-issued
  // before the tile's epilogue runs)
  pw_u32x4 ead[LPT], epx[LPT];
  uint32_t emk[LPT];
  auto stage = [&](const Stage& s, char* slot) {
    float gf[NPC], yf[NPC], o[NPC];
#pragma unroll
    for (int h = 0; h < NPC / 2; ++h) {
      gf[2 * h] = __uint_as_float(s.g[h] << 16);
      gf[2 * h + 1] = __uint_as_float(s.g[h] & 0xffff0000u);
      yf[2 * h] = __uint_as_float(s.y[h] << 16);
      yf[2 * h + 1] = __uint_as_float(s.y[h] & 0xffff0000u);
    }
#pragma unroll
    for (int q = 0; q < NPC / 4; ++q) {
      const int c = nc0 + 4 * q;
      const float4 A4 = *reinterpret_cast<const float4*>(ncoef + c);
      const float4 B4 = *reinterpret_cast<const float4*>(ncoef + CO + c);
      const float4 D4 = *reinterpret_cast<const float4*>(ncoef + 2 * CO + c);
      const float4 S4 = *reinterpret_cast<const float4*>(ncoef + 3 * CO + c);
      const float4 H4 = *reinterpret_cast<const float4*>(ncoef + 4 * CO + c);
      const float A[4] = {A4.x, A4.y, A4.z, A4.w}, B[4] = {B4.x, B4.y, B4.z, B4.w}, D[4] = {D4.x, D4.y, D4.z, D4.w};
      const float sc[4] = {S4.x, S4.y, S4.z, S4.w}, sh[4] = {H4.x, H4.y, H4.z, H4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gg = fmaf(yf[4 * q + k], sc[k], sh[k]) > 0.f ? gf[4 * q + k] : 0.f;
        o[4 * q + k] = fmaf(A[k], gg, fmaf(B[k], yf[4 * q + k], D[k]));
      }
    }
    if constexpr (NPC == 4) {
      *reinterpret_cast<pw_u32x2*>(slot + pw_toff(nrow, nc0 >> 3) + ((nc0 >> 2) & 1) * 8) =
          (pw_u32x2){pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
    } else {
      *reinterpret_cast<pw_u32x4*>(slot + pw_toff(nrow, nc0 >> 3)) =
          (pw_u32x4){pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]),
                     pack_bf16x2(o[6], o[7])};
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      *reinterpret_cast<pw_u32x4*>(slot + C::T_BYTES + pw_mn<CIH>(r0 + C::RSTEP * i, chc)) = s.x[i];
      ead[i] = s.ad[i];
      epx[i] = s.px[i];
      emk[i] = s.mk[i];
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  auto compute = [&](const char* slot, int tile) {
    // dgrad: acc_d[32 x CIH] = T1[32 x CO] . W1 slice -> D tile (f32, LDS)
    {
      f32x4_t accd[C::DTN];
#pragma unroll
      for (int j = 0; j < C::DTN; ++j) accd[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < CO / 32; ++kc) {
        const bf16x8_t fa = pw_frag_kmaj(slot, ((4 * kc) >> 3) * (PW_BM * 128), drb, (4 * kc) & 7, lane);
#pragma unroll
        for (int j = 0; j < C::DTN; ++j) {
          const bf16x8_t fb = pw_frag_tr(wimg, 32 * kc * CIH * 2, dcb + 16 * j, lane,
                                         [](int r, int c) { return pw_mn<CIH>(r, c); });
          accd[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa, accd[j], 0, 0, 0);  // SWAP
        }
      }
      const int drow = drb + (lane & 15);
#pragma unroll
      for (int j = 0; j < C::DTN; ++j)
        *reinterpret_cast<f32x4_t*>(dimg + pw_doff<CIH>(drow, (dcb + 16 * j) / 4 + (lane >> 4))) = accd[j];
    }
    // wgrad: acc_w[CO x CIH] += T1^T . X (k = the tile's 32 rows)
    bf16x8_t fx[C::WTN];
#pragma unroll
    for (int n = 0; n < C::WTN; ++n)
      fx[n] = pw_frag_tr(slot + C::T_BYTES, 0, wcb + 16 * n, lane, [](int r, int c) { return pw_mn<CIH>(r, c); });
#pragma unroll
    for (int i = 0; i < C::WTM; ++i) {
      const bf16x8_t ft = pw_frag_tr(slot, 0, wrb + 16 * i, lane, [](int r, int c) { return pw_toff(r, c); });
#pragma unroll
      for (int n = 0; n < C::WTN; ++n) accw[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ft, fx[n], accw[i][n], 0, 0, 0);
    }
    sync();  // D tile complete
    // dx epilogue, row-contiguous: + masked addend -> bf16 16-B stores; previous tail BN partials
    const float4 pi0 = *reinterpret_cast<const float4*>(pcoef + 8 * chc);
    const float4 pi1 = *reinterpret_cast<const float4*>(pcoef + 8 * chc + 4);
    const float4 pn0 = *reinterpret_cast<const float4*>(pcoef + CIH + 8 * chc);
    const float4 pn1 = *reinterpret_cast<const float4*>(pcoef + CIH + 8 * chc + 4);
    const float pis[8] = {pi0.x, pi0.y, pi0.z, pi0.w, pi1.x, pi1.y, pi1.z, pi1.w};
    const float pnm[8] = {pn0.x, pn0.y, pn0.z, pn0.w, pn1.x, pn1.y, pn1.z, pn1.w};
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int lrow = r0 + C::RSTEP * i;
      const f32x4_t v0 = *reinterpret_cast<const f32x4_t*>(dimg + pw_doff<CIH>(lrow, 2 * chc));
      const f32x4_t v1 = *reinterpret_cast<const f32x4_t*>(dimg + pw_doff<CIH>(lrow, 2 * chc + 1));
      float ad[8], xv[8], v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      unpack8(mask_bf16x8_pw(__builtin_bit_cast(U4, ead[i]), emk[i] & 0xffu), ad);
      unpack8(__builtin_bit_cast(U4, epx[i]), xv);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += ad[k];
      const U4 packed = pack8(v);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pw_u32x4, packed), rdx,
                                             (uint32_t)((tile * PW_BM + lrow) * CI + col0 + 8 * chc) * 2u, 0, 0);
      float gv[8];
      unpack8(mask_bf16x8_pw(packed, emk[i] >> 8), gv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bs[k] += gv[k];
        bq[k] = fmaf(gv[k], fmaf(xv[k], pis[k], pnm[k]), bq[k]);
      }
    }
  };

  issue(st0, tile0);
  issue(st1, tile0 + tstep);
  __syncthreads();  // W1 image, coefficient tables written
  for (int tile = tile0; tile < ntiles; tile += 2 * tstep) {
    stage(st0, smem);
    issue(st0, tile + 2 * tstep);
    sync();  // also: every thread is past the previous tile's D reads
    compute(smem, tile);
    const int t1 = tile + tstep;
    if (t1 >= ntiles) break;
    stage(st1, smem + C::SLOT);
    issue(st1, t1 + 2 * tstep);
    sync();
    compute(smem + C::SLOT, t1);
  }

  // ---- wgrad accumulators -> this block's slab, in register order (coalesced 16-B stores); the slabs
  // of one column part are contiguous
  float* slab = a.slab + (size_t)(part * tstep + tile0) * (CO * CIH);
#pragma unroll
  for (int i = 0; i < C::WTM; ++i)
#pragma unroll
    for (int n = 0; n < C::WTN; ++n)
      *reinterpret_cast<f32x4_t*>(slab + ((size_t)(i * C::WTN + n) * PW_NT + t) * 4) = accw[i][n];
  // ---- previous tail BN partials: threads t, t + TPR, ... share channels 8 chc .. 8 chc + 7 -> LDS
  // (the staging slots, free now) tree over the RSTEP row groups, one atomic pair per channel
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [16][RSTEP][TPR]
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[(k * C::RSTEP + r0) * C::TPR + chc] = bs[k];
    red[((8 + k) * C::RSTEP + r0) * C::TPR + chc] = bq[k];
  }
  __syncthreads();
  for (int e = t; e < 16 * C::TPR; e += PW_NT) {
    const int kk = e / C::TPR, ch = e % C::TPR;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < C::RSTEP; ++r) v += red[(kk * C::RSTEP + r) * C::TPR + ch];
    const int c = 8 * ch + (kk & 7);
    atomicAdd(a.pslots + (size_t)(tile0 % NSLOT) * 2 * CI + (kk >> 3) * CI + col0 + c, v);
  }
}

// F1 slab element e = ((i * WTN + n) * NT + t) * 4 + r of column part p  ->  dW1 [co][ci]: lane = t & 63,
// wave = t >> 6; co = WROWS (wave & 1) + 16 i + (lane >> 4) * 4 + r,
// ci = p CIH + WCOLS (wave >> 1) + 16 n + (lane & 15)
template <int CI, int CO, int S>
__device__ __forceinline__ int pw_slab_to_dw1(int e, int p) {
  using C = PwSqueezeBwdCfg<CI, CO, S>;
  const int r = e & 3, t = (e >> 2) % PW_NT, in = (e >> 2) / PW_NT;
  const int i = in / C::WTN, n = in % C::WTN;
  const int lane = t & 63, wv = t >> 6;
  const int co = C::WROWS * (wv & 1) + 16 * i + (lane >> 4) * 4 + r;
  const int ci = p * C::CIH + C::WCOLS * (wv >> 1) + 16 * n + (lane & 15);
  return co * CI + ci;
}

// Slab element e = ((j * WTN + n) * NT + t) * 4 + r  ->  dW3 (row = wide channel, col = narrow):
// lane = t & 63, wave = t >> 6; row = 64 j + 16 (wave & 3) + (lane >> 4) * 4 + r,
// col = WCOLS (wave >> 2) + 16 n + (lane & 15)   (the !SWAP accumulator layout)
template <int CN>
__device__ __forceinline__ int pw_slab_to_dw(int e) {
  using C = PwExpandCfg<CN>;
  const int r = e & 3, t = (e >> 2) % PW_NT, jn = (e >> 2) / PW_NT;
  const int j = jn / C::WTN, n = jn % C::WTN;
  const int lane = t & 63, wv = t >> 6;
  const int row = 64 * j + 16 * (wv & 3) + (lane >> 4) * 4 + r;
  const int col = C::WCOLS * (wv >> 2) + 16 * n + (lane & 15);
  return row * CN + col;
}

// dW3 += sum over the nslab slabs; grid.x = elements / 256 column groups x PW_RG slab groups (f32
// atomics of the partial sums: nslab / PW_RG-fold fewer than per-block atomics).  Blocks past that
// grid reduce a BN layer's backward slots (bn_slot_reduce's math), 16 channels each.
constexpr int PW_RG = 8;
// SEC tail (sec_C > 0): the shortcut BN's reduction -- red_sc = [red3's sum g' | sum of the q slots]
// (its slots' first halves are never written), dbeta_sc / dgamma_sc +=, q slots re-zeroed.
// conv3x3_fused.hip backward slab element e = ((m * 9 + nn) * NT + t) * 4 + r  ->  dW [co][tap][ci]:
// lane = t & 63, wave = t >> 6; co = 32 (wave & 1) + 16 m + (lane >> 4) * 4 + r; column tile
// idx = 9 (wave >> 1) + nn: tap = idx / 4, ci = 16 (idx % 4) + (lane & 15)
__device__ __forceinline__ int pw_slab_to_dw_c3(int e) {
  const int r = e & 3, t = (e >> 2) % PW_NT, mn = (e >> 2) / PW_NT;
  const int m = mn / 9, nn = mn % 9, lane = t & 63, wv = t >> 6;
  const int co = 32 * (wv & 1) + 16 * m + (lane >> 4) * 4 + r;
  const int idx = 9 * (wv >> 1) + nn;
  return co * 576 + (idx >> 2) * 64 + 16 * (idx & 3) + (lane & 15);
}

// MAP: the slab's register-order layout -- 0 = F3's dW3 (CW x CN), 1 = F1's dW1 (CO = CN x CI = 4 CN),
// 2 = the stage-1 3x3 conv's dW (64 x 9 x 64)
template <int CN, int MAP>
__global__ void __launch_bounds__(256) pw_slab_reduce_kernel(const float* __restrict__ slab, int nslab,
                                                             float* __restrict__ dw, float* __restrict__ sr_slots,
                                                             int sr_C, float* __restrict__ sr_red,
                                                             float* __restrict__ sr_dgamma,
                                                             float* __restrict__ sr_dbeta, PwSecReduce sec, int rg) {
  constexpr int E = MAP == 2 ? 64 * 576 : 4 * CN * CN;
  const int ngemm = (E / 256) * rg;
  const int nsr = sr_C ? (sr_C + 15) / 16 : 0;
  if ((int)blockIdx.x >= ngemm + nsr) {
    // SEC: 16 channels per block, 16 slot-lanes x NSLOT/16 slots each (q halves only)
    const int sb = blockIdx.x - ngemm - nsr, C = sec.C;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4, c = sb * 16 + tx;
    __shared__ float redq[256];
    float q = 0.f;
    if (c < C) {
      float vq[NSLOT / 16];
#pragma unroll
      for (int i = 0; i < NSLOT / 16; ++i) vq[i] = sec.slots[(size_t)(ty + 16 * i) * 2 * C + C + c];
#pragma unroll
      for (int i = 0; i < NSLOT / 16; ++i) {
        q += vq[i];
        sec.slots[(size_t)(ty + 16 * i) * 2 * C + C + c] = 0.f;
      }
    }
    redq[threadIdx.x] = q;
    __syncthreads();
    if (ty == 0 && c < C) {
#pragma unroll
      for (int k = 1; k < 16; ++k) q += redq[threadIdx.x + 16 * k];
      const float sg = sec.red3[c];
      q = sec.save[C + c] * (q - sec.save[c] * sg);
      sec.red[c] = sg;
      sec.red[C + c] = q;
      if (sec.dbeta) sec.dbeta[c] += sg;
      if (sec.dgamma) sec.dgamma[c] += q;
    }
    return;
  }
  if ((int)blockIdx.x >= ngemm) {
    // BN slot reduction: 16 channels per block, 16 slot-lanes x NSLOT/16 slots each
    const int sb = blockIdx.x - ngemm;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4, c = sb * 16 + tx;
    __shared__ float red2[512];
    float s = 0.f, q = 0.f;
    if (c < sr_C) {
      float vs[NSLOT / 16], vq[NSLOT / 16];
#pragma unroll
      for (int i = 0; i < NSLOT / 16; ++i) {
        const float* p = sr_slots + (size_t)(ty + 16 * i) * 2 * sr_C;
        vs[i] = p[c];
        vq[i] = p[sr_C + c];
      }
#pragma unroll
      for (int i = 0; i < NSLOT / 16; ++i) {
        s += vs[i];
        q += vq[i];
        float* p = sr_slots + (size_t)(ty + 16 * i) * 2 * sr_C;
        p[c] = 0.f;
        p[sr_C + c] = 0.f;
      }
    }
    red2[threadIdx.x] = s;
    red2[256 + threadIdx.x] = q;
    __syncthreads();
    if (ty == 0 && c < sr_C) {
#pragma unroll
      for (int k = 1; k < 16; ++k) {
        s += red2[threadIdx.x + 16 * k];
        q += red2[256 + threadIdx.x + 16 * k];
      }
      sr_red[c] = s;
      sr_red[sr_C + c] = q;
      if (sr_dbeta) sr_dbeta[c] += s;
      if (sr_dgamma) sr_dgamma[c] += q;
    }
    return;
  }
  // F1 with its wide columns split over S blocks: S groups of nslab / S slabs of E / S elements each
  constexpr int S = MAP == 1 ? pw_squeeze_split(CN) : 1, EH = E / S;
  const int eg = (blockIdx.x % (E / 256)) * 256 + threadIdx.x, grp = blockIdx.x / (E / 256);
  const int part = eg / EH, e = eg % EH, nper = nslab / S;
  const float* sl = slab + (size_t)part * nper * EH;
  float acc = 0.f;
  int b = grp;
  for (; b + 3 * rg < nper; b += 4 * rg) {
    const float v0 = sl[(size_t)b * EH + e], v1 = sl[(size_t)(b + rg) * EH + e];
    const float v2 = sl[(size_t)(b + 2 * rg) * EH + e], v3 = sl[(size_t)(b + 3 * rg) * EH + e];
    acc += (v0 + v1) + (v2 + v3);
  }
  for (; b < nper; b += rg) acc += sl[(size_t)b * EH + e];
  if constexpr (MAP == 0) atomicAdd(dw + pw_slab_to_dw<CN>(e), acc);
  else if constexpr (MAP == 1) atomicAdd(dw + pw_slab_to_dw1<4 * CN, CN, S>(e, part), acc);
  else atomicAdd(dw + pw_slab_to_dw_c3(e), acc);
}

}  // namespace

bool pw_bwd_expand_ok(int CN, int64_t M) { return (CN == 64) && M % PW_BM == 0 && M > 0 && M < (1 << 24); }

int pw_bwd_expand_grid(int CN, int64_t M) {
  (void)CN;
  const int64_t tiles = M / PW_BM;
  return (int)std::min<int64_t>(256, tiles);
}

void pw_bwd_expand(const PwExpandArgs& args, int nblocks, hipStream_t s) {
  switch (args.CN) {
    case 64:
      if (args.ysc) pw_bwd_expand_kernel<64, true><<<nblocks, PW_NT, 0, s>>>(args);
      else pw_bwd_expand_kernel<64, false><<<nblocks, PW_NT, 0, s>>>(args);
      break;
    default: abort();
  }
}

bool pw_bwd_squeeze_ok(int CI, int CO, int64_t M) {
  return ((CI == 256 && CO == 64) || (CI == 512 && CO == 128)) && M % PW_BM == 0 && M > 0 &&
         (int64_t)M * CI < (1ll << 30);
}

// one block per CU: S column parts x up to 256 / S m-tile strides
int pw_bwd_squeeze_grid(int CI, int CO, int64_t M) {
  (void)CI;
  const int S = pw_squeeze_split(CO);
  return S * (int)std::min<int64_t>(256 / S, M / PW_BM);
}

int64_t pw_bwd_squeeze_slab_floats(int CI, int CO, int nblocks) { return (int64_t)nblocks * CO * CI / pw_squeeze_split(CO); }

void pw_bwd_squeeze(const PwSqueezeBwdArgs& args, int nblocks, hipStream_t s) {
  if (args.CI == 256 && args.CO == 64) pw_bwd_squeeze_kernel<256, 64, 1><<<nblocks, PW_NT, 0, s>>>(args);
  else if (args.CI == 512 && args.CO == 128) pw_bwd_squeeze_kernel<512, 128, pw_squeeze_split(128)><<<nblocks, PW_NT, 0, s>>>(args);
  else abort();
}

void pw_slab_reduce(const float* slab, int nslab, int CN, float* dw, float* sr_slots, int sr_C, float* sr_red,
                    float* sr_dgamma, float* sr_dbeta, const PwSecReduce& sec, hipStream_t s, int map) {
  const int E = map == 2 ? 64 * 576 : 4 * CN * CN;
  const int nsr = sr_slots ? (sr_C + 15) / 16 : 0;
  const int rg = det_mode() ? 1 : PW_RG;  // one adder per dW element in the deterministic mode
  const int grid = (E / 256) * rg + nsr + (sec.C ? (sec.C + 15) / 16 : 0);
  switch (CN) {
    case 64:
      if (map == 0)
        pw_slab_reduce_kernel<64, 0><<<grid, 256, 0, s>>>(slab, nslab, dw, sr_slots, sr_slots ? sr_C : 0, sr_red,
                                                          sr_dgamma, sr_dbeta, sec, rg);
      else if (map == 1)
        pw_slab_reduce_kernel<64, 1><<<grid, 256, 0, s>>>(slab, nslab, dw, sr_slots, sr_slots ? sr_C : 0, sr_red,
                                                          sr_dgamma, sr_dbeta, sec, rg);
      else
        pw_slab_reduce_kernel<64, 2><<<grid, 256, 0, s>>>(slab, nslab, dw, sr_slots, sr_slots ? sr_C : 0, sr_red,
                                                          sr_dgamma, sr_dbeta, sec, rg);
      break;
    case 128:
      if (map != 1) abort();
      pw_slab_reduce_kernel<128, 1><<<grid, 256, 0, s>>>(slab, nslab, dw, sr_slots, sr_slots ? sr_C : 0, sr_red,
                                                         sr_dgamma, sr_dbeta, sec, rg);
      break;
    default: abort();
  }
}

}  // namespace tfx
