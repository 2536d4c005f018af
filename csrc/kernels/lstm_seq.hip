// Persistent whole-sequence LSTM recurrence for gfx950 (char-LSTM, BASELINE.json config 5).
//
// The reference unrolls BasicLSTMCell with dynamic_rnn: per time step one [B, In+H] x [In+H, 4H]
// MatMul and the gate ops, i.e. T dependent kernel chains per layer and direction
// (SURVEY.md §2 char-LSTM row).  On MI355X the per-step work at the PTB shape (B = 64, H = 512)
// is a 64 x 2048 x 512 GEMM -- under a microsecond of MFMA time -- so a kernel per step is pure
// launch/boundary cost (~1.5 us per dependent boundary, x2 kernels, x T, x layers, x fwd+bwd).
// Here ONE launch runs all T steps of a layer:
//
//   grid (H/16, B/16) workgroups, one per CU (96 KB dynamic LDS pins residency); workgroup
//   (ub, rb) owns batch rows r0 = 16 rb .. +16 and hidden units u0 = 16 ub .. +16.
//   forward, per step t:   wave w = K quarter [w H/4, (w+1) H/4) of the recurrent GEMM
//                          z[16 x 4 gates x 16] = h_{t-1}[rows, :] . W_hh[gate rows, :]^T
//                          (v_mfma_f32_16x16x32_bf16, W_hh slice resident in VGPRs for the
//                          whole sequence), partials reduced through LDS; one thread per
//                          (row, unit) adds gx[t] (the hoisted input projection + bias), runs
//                          the cell with c in a register, writes act / c (for backward) and
//                          h_t as bf16.
//   backward, t = T-1..0:  wave q = gate q's K block of  dh_rec = dg_{t+1}[rows, :] . W_hh[:, units]
//                          (W_hh^T slice in VGPRs), + dH_out[t]; the cell backward carries dc in
//                          a register and writes dg_t (bf16) for the recurrence AND for the
//                          batched weight-gradient GEMMs that follow the launch.
//
// Inter-workgroup hand-off of h_t / dg_t: every handed-off byte is written ONCE per launch (hbuf
// and dg keep one slot per time step) with 16-byte write-through (sc1) buffer stores and read
// ONLY with sc1 buffer loads (cdna_hip_programming.md §6 Guideline 16).  Protocol: every storing
// wave drains vmcnt, a workgroup barrier, ONE lane adds 1 to the row block's counter (agent-scope
// atomic); a consumer lane polls the counter relaxed, a workgroup barrier, then the sc1 loads
// (MI355X_MICROARCH.md "Valid forms" table row 1).  (Rejected alternatives, measured slower and
// removed: data-as-flag sentinel slots, 2.13 vs 1.79 ms/step; per-producer flag words --
// profiles/r02_lstm.)
//
// A row block depends only on its own 16 rows.  Every spin is bounded: on expiry the status word
// is set and the whole grid drains (no hang).  The host reads the status word asynchronously
// (ops/rnn.py: a pinned copy checked at the next log / sync point) and raises.
#include "tfx_common.h"
#include "tfx_kernels.h"

#include <algorithm>
#include <cstdio>

namespace tfx {
namespace {

constexpr int LS_LDS = 96 * 1024;      // > 80 KB: one workgroup per CU (160 KB LDS)
constexpr int LS_STRIDE = 32;          // u32 words per counter (own 128-B line)
constexpr unsigned LS_SPIN_LIMIT = 1u << 20;

typedef __attribute__((address_space(1))) unsigned gu32;
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
template <int NK>
constexpr int H_of() { return NK * 32; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ls_rsrc(const void* p, int64_t bytes) {
  const int n = bytes > 0x7fffffff ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, n, 0x00020000);
}
// 16-byte write-through (sc1) load / store
__device__ __forceinline__ bf16x8_t ld_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int off, u32x4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

__device__ __forceinline__ float ls_sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// One lane: wait until *ctr >= target.  false = gave up (status word set).
__device__ __forceinline__ bool ls_wait(gu32* ctr, unsigned target, gu32* status, unsigned limit) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v >= target) return true;
    if (spins >= limit) {
      __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Block-wide: lane 0 waits; everyone learns the outcome after the barrier.
__device__ __forceinline__ bool ls_block_wait(gu32* ctr, unsigned target, gu32* status, int* flag,
                                              unsigned limit) {
  if (threadIdx.x == 0) {
    const bool ok = ls_wait(ctr, target, status, limit);
    *flag = ok ? 1 : 0;
  }
  __syncthreads();
  return *flag != 0;
}

// Publish: every storing wave drains, barrier, one lane bumps the counter.
__device__ __forceinline__ void ls_publish(gu32* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ forward
template <int NK>
__global__ void __launch_bounds__(256, 1)
    lstm_seq_fwd_kernel(const float* __restrict__ gx, const uint16_t* __restrict__ whh, int T, int B,
                        uint16_t* hbuf, float* __restrict__ cbuf, float* __restrict__ act, float* __restrict__ hT,
                        unsigned* sync, unsigned* status_word, unsigned limit) {
  constexpr int H = NK * 32, NKW = NK / 4, KQ = H / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);                    // [wave][gate][lane][4]  16 KB
  uint16_t* hs = reinterpret_cast<uint16_t*>(smem + 16384);      // [row][unit] bf16       512 B
  int* flag = reinterpret_cast<int*>(smem + 16384 + 512);         // [0] wait result, [1] abort
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nub = gridDim.x, u0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  gu32* ctr = (gu32*)(sync + blockIdx.y * nub * LS_STRIDE);  // row block's counter / flag lines
  gu32* status = (gu32*)status_word;  // sticky health word: set on a bounded wait's expiry
  if (tid == 0) flag[1] = 0;

  // W_hh rows (gate q, unit u0 + lane%16), this wave's K quarter: B operand, resident all sequence
  bf16x8_t w[4][NKW];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int kk = 0; kk < NKW; ++kk)
      w[q][kk] = *reinterpret_cast<const bf16x8_t*>(whh + (int64_t)(q * H + u0 + (lane & 15)) * H + wave * KQ +
                                                   kk * 32 + (lane >> 4) * 8);
  const int cr = tid >> 4, cu = tid & 15;  // cell thread: row, unit within the tile
  const int64_t cidx = (int64_t)(r0 + cr) * H + u0 + cu;
  const int64_t BH = (int64_t)B * H;
  float c = cbuf[cidx];
  const int aoff = ((lane & 15) * H + wave * KQ + (lane >> 4) * 8) * 2;  // byte offset in a row tile
  const int rl = (cr >> 2) * 16 + cu, ri = cr & 3;                      // (lane, reg) holding (cr, cu)
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const float* g = gx + (int64_t)t * 4 * BH + (int64_t)(r0 + cr) * 4 * H + u0 + cu;
    const float z0 = g[0], z1 = g[H], z2 = g[2 * H], z3 = g[3 * H];  // hoisted projection, pre-launch data
    const __amdgpu_buffer_rsrc_t hr = ls_rsrc(hbuf + t * BH + (int64_t)r0 * H, 16 * H * 2);
    bf16x8_t a[NKW];
    if (t > 0 && !ls_block_wait(ctr, (unsigned)(t * nub), status, flag, limit)) return;
#pragma unroll
    for (int kk = 0; kk < NKW; ++kk) a[kk] = ld_sc1(hr, aoff + kk * 64);
    __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first MFMA waits
    f32x4_t acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < NKW; ++kk)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk], w[q][kk], acc[q], 0, 0, 0);
    // acc[q][i] = partial z of (row (lane/16)*4 + i, unit lane%16, gate q)
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4_t*>(red + ((wave * 4 + q) * 64 + lane) * 4) = acc[q];
    __syncthreads();
    float z[4] = {z0, z1, z2, z3};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) z[q] += red[((w2 * 4 + q) * 64 + rl) * 4 + ri];
    const float ig = ls_sigm(z[0]), fg = ls_sigm(z[1]), gg = tanhf(z[2]), og = ls_sigm(z[3]);
    c = fmaf(fg, c, ig * gg);
    const float h = og * tanhf(c);
    float* ap = act + (int64_t)t * 4 * BH + (int64_t)(r0 + cr) * 4 * H + u0 + cu;
    ap[0] = ig;
    ap[H] = fg;
    ap[2 * H] = gg;
    ap[3 * H] = og;
    cbuf[(t + 1) * BH + cidx] = c;
    if (t == T - 1) hT[cidx] = h;
    hs[cr * 16 + cu] = f32_to_bf16(h);
    __syncthreads();
    if (tid < 32) {
      const int row = tid >> 1, half = tid & 1;
      const u32x4v v = *reinterpret_cast<const u32x4v*>(hs + row * 16 + half * 8);
      const __amdgpu_buffer_rsrc_t hw = ls_rsrc(hbuf + (t + 1) * BH + (int64_t)r0 * H, 16 * H * 2);
      st_sc1(hw, (row * H + u0 + half * 8) * 2, v);
    }
    ls_publish(ctr);
  }
}

// ------------------------------------------------------------------ backward
// dH (bf16, optional): gradient of every h_t from outside the recurrence; dhT / dc_in (f32,
// optional): gradients of h_T / c_T; dbias (optional): += sum over t and rows of dgates (f32).
template <int NK>
__global__ void __launch_bounds__(256, 1)
    lstm_seq_bwd_kernel(const float* __restrict__ act, const float* __restrict__ cbuf,
                        const uint16_t* __restrict__ dH, const float* __restrict__ dhT,
                        const float* __restrict__ dc_in, const uint16_t* __restrict__ whh, int T, int B, uint16_t* dg,
                        float* __restrict__ dc_out, float* __restrict__ dbias, unsigned* sync, unsigned* status_word,
                        unsigned limit) {
  constexpr int H = NK * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);                    // [wave][lane][4]  4 KB
  uint16_t* ds = reinterpret_cast<uint16_t*>(smem + 4096);       // [row][gate][unit] bf16  2 KB
  int* flag = reinterpret_cast<int*>(smem + 4096 + 2048);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nub = gridDim.x, u0 = blockIdx.x * 16, r0 = blockIdx.y * 16;
  gu32* ctr = (gu32*)(sync + blockIdx.y * nub * LS_STRIDE);
  gu32* status = (gu32*)status_word;  // sticky health word: set on a bounded wait's expiry
  if (tid == 0) flag[1] = 0;

  // W_hh^T slice: B operand k = gate column q*H + kk*32 + (lane/16)*8 + e, n = unit u0 + lane%16
  bf16x8_t w[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u16x8_t v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = whh[(int64_t)(wave * H + kk * 32 + (lane >> 4) * 8 + e) * H + u0 + (lane & 15)];
    w[kk] = __builtin_bit_cast(bf16x8_t, v);
  }
  const int cr = tid >> 4, cu = tid & 15;
  const int64_t cidx = (int64_t)(r0 + cr) * H + u0 + cu;
  const int64_t BH = (int64_t)B * H;
  float dc = dc_in ? dc_in[cidx] : 0.f;
  float cn = cbuf[T * BH + cidx];
  float db0 = 0.f, db1 = 0.f, db2 = 0.f, db3 = 0.f;
  const int aoff = ((lane & 15) * 4 * H + wave * H + (lane >> 4) * 8) * 2;
  const int rl = (cr >> 2) * 16 + cu, ri = cr & 3;
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = T - 1 - s;
    const float* ap = act + (int64_t)t * 4 * BH + (int64_t)(r0 + cr) * 4 * H + u0 + cu;
    const float ig = ap[0], fg = ap[H], gg = ap[2 * H], og = ap[3 * H];
    const float cp = cbuf[t * BH + cidx];
    float dhv = dH ? bf16_to_f32(dH[t * BH + cidx]) : 0.f;
    if (s == 0 && dhT) dhv += dhT[cidx];
    if (s > 0) {
      const __amdgpu_buffer_rsrc_t gr = ls_rsrc(dg + (t + 1) * 4 * BH + (int64_t)r0 * 4 * H, 16 * 4 * H * 2);
      bf16x8_t a[NK];
      if (!ls_block_wait(ctr, (unsigned)(s * nub), status, flag, limit)) return;
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) a[kk] = ld_sc1(gr, aoff + kk * 64);
      __builtin_amdgcn_sched_barrier(0);
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; kk += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk], w[kk], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk + 1], w[kk + 1], acc1, 0, 0, 0);
      }
      *reinterpret_cast<f32x4_t*>(red + (wave * 64 + lane) * 4) = acc0 + acc1;
      __syncthreads();
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2) dhv += red[(w2 * 64 + rl) * 4 + ri];
    }
    const float tc = tanhf(cn);
    dc = fmaf(dhv * og, 1.f - tc * tc, dc);
    const float d0 = dc * gg * ig * (1.f - ig), d1 = dc * cp * fg * (1.f - fg);
    const float d2 = dc * ig * (1.f - gg * gg), d3 = dhv * tc * og * (1.f - og);
    db0 += d0;
    db1 += d1;
    db2 += d2;
    db3 += d3;
    dc *= fg;
    cn = cp;
    uint16_t* dp = ds + cr * 64 + cu;
    dp[0] = f32_to_bf16(d0);
    dp[16] = f32_to_bf16(d1);
    dp[32] = f32_to_bf16(d2);
    dp[48] = f32_to_bf16(d3);
    __syncthreads();
    if (tid < 128) {
      const int row = tid >> 3, q = (tid >> 1) & 3, half = tid & 1;
      const u32x4v v = *reinterpret_cast<const u32x4v*>(ds + row * 64 + q * 16 + half * 8);
      const __amdgpu_buffer_rsrc_t gw = ls_rsrc(dg + t * 4 * BH + (int64_t)r0 * 4 * H, 16 * 4 * H * 2);
      st_sc1(gw, (row * 4 * H + q * H + u0 + half * 8) * 2, v);
    }
    ls_publish(ctr);
  }
  if (dc_out) dc_out[cidx] = dc;
  if (dbias) {
    // bias gradient: this tile's sum over its 16 rows, one f32 atomic per (gate, unit)
    __syncthreads();
    float* bsum = red;  // [gate][row][unit]
    bsum[(0 * 16 + cr) * 16 + cu] = db0;
    bsum[(1 * 16 + cr) * 16 + cu] = db1;
    bsum[(2 * 16 + cr) * 16 + cu] = db2;
    bsum[(3 * 16 + cr) * 16 + cu] = db3;
    __syncthreads();
    if (tid < 64) {
      const int q = tid >> 4, u = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) v += bsum[(q * 16 + r) * 16 + u];
      atomicAdd(dbias + q * H + u0 + u, v);
    }
  }
}

template <typename K>
void ls_prepare(K k) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, LS_LDS);
}

// Workgroups of kernel k that can be resident at once on the whole device (occupancy API at the
// launch's block size and dynamic LDS, x CUs).  The 96 KB of LDS caps it at one per CU, so the API's
// known over-count at high SGPR use (MI355X_MICROARCH.md, correctness boundaries) cannot apply.
template <typename K>
int ls_resident(K k, int cus) {
  ls_prepare(k);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k), 256, LS_LDS) !=
      hipSuccess)
    return 0;
  return std::min(per_cu, 1) * cus;
}

// Co-residency of the grid is required (workgroups wait on each other): outside a graph capture the
// launch is cooperative (the runtime refuses a grid that cannot be co-resident instead of starting
// it); inside a capture -- where a cooperative launch is not recorded -- a plain launch, guarded by
// the occupancy check of lstm_seq_supported and the bounded waits.
template <typename K>
void ls_launch(K k, dim3 grid, void** args, hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cs);
  if (cs == hipStreamCaptureStatusNone) {
    const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k), grid, dim3(256), args,
                                                    LS_LDS, s);
    if (e == hipSuccess) return;
    (void)hipGetLastError();  // clear it: the plain launch below reports its own errors
    fprintf(stderr, "lstm_seq: cooperative launch refused (%s); plain launch with bounded waits\n",
            hipGetErrorString(e));
  }
  TFX_HIP_CHECK(hipLaunchKernel(reinterpret_cast<const void*>(k), grid, dim3(256), args, LS_LDS, s));
}

template <int NK>
void fwd_launch(dim3 grid, const float* gx, const uint16_t* whh, int T, int B, uint16_t* hbuf, float* cbuf,
                float* act, float* hT, unsigned* sync, unsigned* status, unsigned limit, hipStream_t s) {
  static bool once = (ls_prepare(lstm_seq_fwd_kernel<NK>), true);
  (void)once;
  (void)hipMemsetAsync(sync, 0, (size_t)lstm_seq_sync_words(B, H_of<NK>()) * 4, s);
  void* args[] = {&gx, &whh, &T, &B, &hbuf, &cbuf, &act, &hT, &sync, &status, &limit};
  ls_launch(lstm_seq_fwd_kernel<NK>, grid, args, s);
}

template <int NK>
void bwd_launch(dim3 grid, const float* act, const float* cbuf, const uint16_t* dH, const float* dhT,
                const float* dc_in, const uint16_t* whh, int T, int B, uint16_t* dg, float* dc_out, float* dbias,
                unsigned* sync, unsigned* status, unsigned limit, hipStream_t s) {
  static bool once = (ls_prepare(lstm_seq_bwd_kernel<NK>), true);
  (void)once;
  (void)hipMemsetAsync(sync, 0, (size_t)lstm_seq_sync_words(B, H_of<NK>()) * 4, s);
  void* args[] = {&act, &cbuf, &dH, &dhT, &dc_in, &whh, &T, &B, &dg, &dc_out, &dbias, &sync, &status, &limit};
  ls_launch(lstm_seq_bwd_kernel<NK>, grid, args, s);
}

template <int NK>
void residency(int cus, int* f, int* b) {
  *f = ls_resident(lstm_seq_fwd_kernel<NK>, cus);
  *b = ls_resident(lstm_seq_bwd_kernel<NK>, cus);
}

}  // namespace

int lstm_seq_sync_words(int B, int H) { return ((B / 16) * (H / 16) + 1) * LS_STRIDE; }

void lstm_seq_residency(int B, int H, int num_cus, int* fwd, int* bwd) {
  *fwd = *bwd = 0;
  switch (H) {
    case 128: residency<4>(num_cus, fwd, bwd); break;
    case 256: residency<8>(num_cus, fwd, bwd); break;
    case 512: residency<16>(num_cus, fwd, bwd); break;
    case 1024: residency<32>(num_cus, fwd, bwd); break;
    default: break;
  }
}

bool lstm_seq_supported(int B, int H, int num_cus) {
  if (B <= 0 || B % 16 != 0) return false;
  if (H != 128 && H != 256 && H != 512 && H != 1024) return false;
  // every workgroup resident at once: the occupancy API's count for both kernels, not just grid <= CUs
  int f = 0, b = 0;
  lstm_seq_residency(B, H, num_cus, &f, &b);
  const int64_t grid = (int64_t)(B / 16) * (H / 16);
  return grid <= num_cus && grid <= f && grid <= b;
}

void lstm_seq_fwd(const float* gx, const uint16_t* whh, int T, int B, int H, uint16_t* hbuf, float* cbuf, float* act,
                  float* hT, unsigned* sync, unsigned* status, unsigned spin_limit, hipStream_t s) {
  const dim3 grid(H / 16, B / 16);
  if (status == nullptr) status = sync + (B / 16) * (H / 16) * LS_STRIDE;
  const unsigned lim = spin_limit ? spin_limit : LS_SPIN_LIMIT;
  switch (H) {
    case 128: fwd_launch<4>(grid, gx, whh, T, B, hbuf, cbuf, act, hT, sync, status, lim, s); break;
    case 256: fwd_launch<8>(grid, gx, whh, T, B, hbuf, cbuf, act, hT, sync, status, lim, s); break;
    case 512: fwd_launch<16>(grid, gx, whh, T, B, hbuf, cbuf, act, hT, sync, status, lim, s); break;
    default: fwd_launch<32>(grid, gx, whh, T, B, hbuf, cbuf, act, hT, sync, status, lim, s); break;
  }
}

void lstm_seq_bwd(const float* act, const float* cbuf, const uint16_t* dH, const float* dhT, const float* dc_in,
                  const uint16_t* whh, int T, int B, int H, uint16_t* dg, float* dc_out, float* dbias, unsigned* sync,
                  unsigned* status, unsigned spin_limit, hipStream_t s) {
  const dim3 grid(H / 16, B / 16);
  if (status == nullptr) status = sync + (B / 16) * (H / 16) * LS_STRIDE;
  const unsigned lim = spin_limit ? spin_limit : LS_SPIN_LIMIT;
  switch (H) {
    case 128: bwd_launch<4>(grid, act, cbuf, dH, dhT, dc_in, whh, T, B, dg, dc_out, dbias, sync, status, lim, s); break;
    case 256: bwd_launch<8>(grid, act, cbuf, dH, dhT, dc_in, whh, T, B, dg, dc_out, dbias, sync, status, lim, s); break;
    case 512: bwd_launch<16>(grid, act, cbuf, dH, dhT, dc_in, whh, T, B, dg, dc_out, dbias, sync, status, lim, s); break;
    default: bwd_launch<32>(grid, act, cbuf, dH, dhT, dc_in, whh, T, B, dg, dc_out, dbias, sync, status, lim, s); break;
  }
}

}  // namespace tfx
