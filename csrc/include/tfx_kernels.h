// Host-callable launchers of every HIP kernel in csrc/kernels (torch-free; raw pointers +
// hipStream_t).  The TORCH_LIBRARY bindings in csrc/torch_ops validate shapes and call these.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace tfx {

// Cross-block reduction slots for per-channel statistics ([NSLOT][2][C] f32, see batchnorm.hip)
constexpr int NSLOT = 64;

// Division by a runtime-invariant divisor via multiply-high (valid for n < 2^31).
struct FastDiv {
  uint32_t d = 1, m = 0, s = 0;
  FastDiv() = default;
  explicit FastDiv(uint32_t dd) : d(dd) {
    s = 0;
    while ((1u << s) < d) ++s;
    m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  }
#ifdef __HIPCC__
  // valid for n < 2^31 (then t + n < 2^32): every index the kernels divide is < 2^31
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t t = __umulhi(n, m);
    return (t + n) >> s;
  }
#endif
  uint32_t div_host(uint32_t n) const {
    const uint32_t t = (uint32_t)(((uint64_t)n * m) >> 32);
    return (uint32_t)(((uint64_t)t + n) >> s);
  }
};

// ---------------------------------------------------------------- implicit GEMM
// MODE_DGRAD_FLIP: a 3x3 stride-1 data gradient posed as the forward conv of dY with the flipped,
// transposed filter (args built as that forward: A = dY, B = Wf [C][3][3][Ko]; igemm_dgrad_flip.hip)
enum { MODE_GEMM = 0, MODE_FWD = 1, MODE_DGRAD = 2, MODE_WGRAD = 3, MODE_WGRAD_T = 4, MODE_DGRAD_CLS = 5,
       MODE_DGRAD_FLIP = 6 };
enum { OUT_BF16 = 0, OUT_F32 = 1, OUT_F32_ADD = 2, OUT_F32_ATOMIC = 3 };

struct IgemmArgs {
  const uint16_t* A = nullptr;
  const uint16_t* B = nullptr;
  int64_t a_bytes = 0, b_bytes = 0;  // extents of A/B (buffer-resource bounds; must be < 2 GiB)
  int trans_out = 0;                 // store C[m][n] at Cp[n*ldc + m]
  const uint16_t* addend = nullptr;  // bf16 outputs: C = acc + addend (same layout as C; may alias Cp)
  // optional ReLU-mask bits of the addend (1 bit per element, one byte per 8 channels): C = acc +
  // addend * mask -- a residual BN's masked output gradient consumed without materialising it
  const uint8_t* addend_mask = nullptr;
  // addend_s2: the addend holds only the even-(y, x) pixels of the output grid, compact
  // [Nb][s2_P][s2_Q][ldc] (the data gradient of a 1x1 stride-2 projection shortcut): odd pixels add
  // nothing.  Output rows decode as pixel (n, y, x) of an H x W grid (fd_s2HW / fd_s2W).
  int addend_s2 = 0, s2_P = 0, s2_Q = 0;
  FastDiv fd_s2HW, fd_s2W;
  void* Cp = nullptr;
  const float* bias = nullptr;
  int M = 0, N = 0, K = 0;
  int lda = 0, ldb = 0, ldc = 0;
  int a_kmajor = 1, b_kmajor = 1;
  // conv geometry (NHWC input [Nb][H][W][C], weight [Ko][R][S][C], output [Nb][P][Q][Ko])
  int Nb = 0, H = 0, W = 0, C = 0, Ko = 0, R = 1, S = 1, P = 0, Q = 0;
  int sh = 1, sw = 1, ph = 0, pw = 0, dh = 1, dw = 1;
  int sh_log2 = 0, sw_log2 = 0;
  int out_mode = OUT_BF16;
  int relu = 0;
  // optional per-column BN statistics of the (bf16-rounded) output: [NSLOT][2][N] f32, pre-zeroed
  float* stats = nullptr;
  // rows of `stats` the epilogue adds into (tile row tm -> row tm % stat_slots)
  int stat_slots = NSLOT;
  FastDiv fd_C, fd_S, fd_Ko, fd_PQ, fd_Q;
  int zero_out = 1;
  // MODE_DGRAD_CLS: one output-parity class (cph, cpw) of a stride-2 data gradient.  The GEMM rows
  // are the class's sub-grid pixels (H x W above = the class grid), its k = (ri, si, ko) runs over
  // the taps r = cr0 + 2 ri, s = cs0 + 2 si of the full wR x wS filter only, and row m is stored at
  // pixel (n, 2y + cph, 2x + cpw) of the out_H x out_W gradient (fd_cHW / fd_cW decode m).
  int cls = 0, cph = 0, cpw = 0, cr0 = 0, cs0 = 0, wR = 1, wS = 1, out_H = 0, out_W = 0;
  FastDiv fd_cHW, fd_cW;
  // ---- fused batch-norm epilogues (per output column c; the BN layer's workspace holds the
  // [NSLOT][2][N] slots, zero between uses: the finalize / slot-reduce that consumes them re-zeroes)
  // backward partials of the BN whose OUTPUT gradient this dgrad produces: g' = bf16(out) * relu
  // mask (from x*scale+shift > 0, or the residual layer's mask bits), accumulated per column:
  // sum g' and sum g' * (x - mean) * invstd into bnb_slots
  const uint16_t* bnb_x = nullptr;
  const float* bnb_save = nullptr;
  const uint8_t* bnb_mask = nullptr;
  int bnb_relu = 0;
  float* bnb_slots = nullptr;
  // optional tail blocks (weight-gradient launches): reduce ANOTHER BN layer's backward slots
  // ([NSLOT][2][sr_C], filled by an earlier data-gradient epilogue) into sr_red = [sum g' | sum g'
  // xhat] and dgamma / dbeta += -- bn_slot_reduce folded into this launch (16 channels per block,
  // after the GEMM's blocks: they fill CUs the GEMM's tail leaves idle).  sr_C == 0: none.
  float* sr_slots = nullptr;
  float* sr_red = nullptr;
  float* sr_dgamma = nullptr;
  float* sr_dbeta = nullptr;
  int sr_C = 0;
  // a second such reduction in the same tail (blocks after the first one's)
  float* sr2_slots = nullptr;
  float* sr2_red = nullptr;
  float* sr2_dgamma = nullptr;
  float* sr2_dbeta = nullptr;
  int sr2_C = 0;
  // optional A-operand transform on load: A[m][k] -> relu(A * a_scale[k] + a_shift[k]) (a plain ReLU
  // BN applied by its consumer: the BN output is never written).  1x1 stride-1 forward convs with a
  // single k-tile (K <= 64) on the register-staged pipeline only (igemm_launch checks).
  const float* a_scale = nullptr;
  const float* a_shift = nullptr;
  // im2col (KM_FWD_X) operand with C % 64 == 0 and R*S <= 32 (set by igemm_launch): every 64-deep
  // k-tile lies in ONE filter tap, so the tap / channel decode is uniform (scalar) per k-tile and a
  // row's padding test is one bit of a per-row tap-validity mask precomputed at the block's start
  int tapmask = 0;
  // filled by the launcher
  int kps = 0, tiles_m = 0, tiles_n = 0;
};
void igemm_launch(IgemmArgs a, int mode, hipStream_t s);
// persistent 1x1-forward mode (igemm_persist.hip): 0 off, 2 / 3 ring depth; returns the previous mode
int igemm_persist_set(int mode);

// ---------------------------------------------------------------- fused pointwise-conv backward (pw_bwd.hip)
// Backward of a bottleneck's expanding 1x1 conv (CN -> CW = 4 CN) fused with the block-tail BN's
// backward apply: dy3 = A (g * mask) + B y3 + D formed on load, dA2 = dy3 . W3 (+ BN2 backward
// partials into slots2 when y2 != null), dW3 partials into slab[grid][CW * CN] (pw_slab_reduce).
struct PwExpandArgs {
  const uint16_t* g = nullptr;      // [M][CW] output gradient of the block
  const uint16_t* y3 = nullptr;     // [M][CW] tail BN input (conv3 output)
  const uint8_t* mask3 = nullptr;   // [M][CW / 8] tail ReLU mask bits
  const float* save3 = nullptr;     // [4][CW] mean | invstd | scale | shift
  const float* red3 = nullptr;      // [2][CW] sum g' | sum g' xhat
  const uint16_t* a2 = nullptr;     // [M][CN] conv3 input
  const uint16_t* w = nullptr;      // [CW][CN] conv3 weight
  uint16_t* dA2 = nullptr;          // [M][CN] out
  // a2_save set: a2 holds BN2's INPUT y2 and conv3's input is relu(y2 * scale + shift) with BN2's
  // [4][CN] save -- formed on load (the forward applied BN2 on load too: a2 was never written)
  const float* a2_save = nullptr;
  const uint16_t* y2 = nullptr;     // [M][CN] BN2 input (null: no BN2 partials)
  const float* save2 = nullptr;     // [4][CN]
  int relu2 = 0;
  float* slots2 = nullptr;          // [NSLOT][2][CN]
  float* slab = nullptr;            // [grid][CW * CN] f32
  // projection-block tail (optional): the shortcut BN's input ysc [M][CW]; partial sums g' * ysc go
  // to the second halves of slots_sc [NSLOT][2][CW] (pw_slab_reduce centres and scales them)
  const uint16_t* ysc = nullptr;
  float* slots_sc = nullptr;
  int M = 0, CN = 0;
};
// Fused block tail + next squeezing 1x1 conv forward (pw_fwd.hip): out = relu(y3 sc3 + sh3 + res')
// (res' = res, or res * sc_r + sh_r when save_r is set: a never-written shortcut BN output), out and its
// mask bits stored, y1 = out . W1^T stored with BN1's statistics added into slots1 [NSLOT][2][CO].
struct PwSqueezeArgs {
  const uint16_t* y3 = nullptr;    // [M][CI] tail BN input
  const float* save3 = nullptr;    // [4][CI]
  const uint16_t* res = nullptr;   // [M][CI] residual (or the shortcut BN's input)
  const float* save_r = nullptr;   // [4][CI] shortcut BN (null: plain residual)
  const uint16_t* w = nullptr;     // [CO][CI]
  uint16_t* out = nullptr;         // [M][CI]
  uint8_t* mask = nullptr;         // [M][CI / 8]
  uint16_t* y1 = nullptr;          // [M][CO]
  float* slots1 = nullptr;         // [NSLOT][2][CO]
  int M = 0, CI = 0, CO = 0;
};
bool pw_fwd_squeeze_ok(int CI, int CO, int64_t M);
int pw_fwd_squeeze_grid(int CI, int CO, int64_t M);
void pw_fwd_squeeze(const PwSqueezeArgs& args, int nblocks, hipStream_t s);
// Stage-1 3x3 conv (64 -> 64, stride 1, pad 1, width 32) with its BN layers fused (conv3x3_fused.hip).
// Forward: y = conv(relu(x sc_in + sh_in)) with BN statistics of y added into slots [NSLOT][2][64].
struct Conv3Args {
  const uint16_t* x = nullptr;      // [N][H][32][64] input BN's input (y1)
  const float* save_in = nullptr;   // [4][64] input BN's [mean | invstd | scale | shift]
  const uint16_t* w = nullptr;      // [64][3][3][64]
  uint16_t* y = nullptr;            // [N][H][32][64]
  float* slots = nullptr;           // [NSLOT][2][64] output BN statistics
  int N = 0, H = 0;
};
bool conv3x3_fused_ok(int N, int H, int W, int C, int K);
void conv3x3_fwd_fused(const Conv3Args& a, hipStream_t s);
// Backward: dy2 = BN2's backward apply (g2, y2, save2, red2) formed on load; dx = dgrad(dy2) with BN1's
// backward partials (y1, save1; ReLU mask recomputed) into slots1; dW into per-block slabs [grid][64 * 576].
struct Conv3BwdArgs {
  const uint16_t* g2 = nullptr;
  const uint16_t* y2 = nullptr;
  const float* save2 = nullptr;
  const float* red2 = nullptr;
  const uint16_t* y1 = nullptr;
  const float* save1 = nullptr;
  const uint16_t* w = nullptr;
  uint16_t* dx = nullptr;
  float* slots1 = nullptr;
  float* slab = nullptr;
  int N = 0, H = 0;
};
int conv3x3_bwd_fused_grid(int N, int H);
void conv3x3_bwd_fused(const Conv3BwdArgs& a, int nblocks, hipStream_t s);
// the shortcut BN's reduction in pw_slab_reduce's tail (C = 0: none): red = [red3's sum g' | sum q]
struct PwSecReduce {
  float* slots = nullptr;
  const float* red3 = nullptr;
  const float* save = nullptr;  // the shortcut BN's [mu | istd | ...]
  float* red = nullptr;
  float* dgamma = nullptr;
  float* dbeta = nullptr;
  int C = 0;
};
bool pw_bwd_expand_ok(int CN, int64_t M);
int pw_bwd_expand_grid(int CN, int64_t M);
void pw_bwd_expand(const PwExpandArgs& args, int nblocks, hipStream_t s);
// dw[CW][CN] += sum of nslab slabs; + optional BN slot reduction (bn_slot_reduce's math) in tail blocks
// map: 0 = pw_bwd_expand's slab (dW3), 1 = pw_bwd_squeeze's (dW1, CO = CN, CI = 4 CN)
void pw_slab_reduce(const float* slab, int nslab, int CN, float* dw, float* sr_slots, int sr_C, float* sr_red,
                    float* sr_dgamma, float* sr_dbeta, const PwSecReduce& sec, hipStream_t s, int map = 0);
// Fused backward of an identity bottleneck's squeezing 1x1 conv1 with BN1's backward apply
// (pw_bwd.hip F1): dx = T1 . W1 + addend * amask, the previous tail BN's partials into pslots, the
// weight gradient into per-block slabs (pw_slab_reduce map 1).
struct PwSqueezeBwdArgs {
  const uint16_t* g1 = nullptr;    // [M][CO] BN1 output gradient
  const uint16_t* y1 = nullptr;    // [M][CO] BN1 input
  const float* save1 = nullptr;    // [4][CO]
  const float* red1 = nullptr;     // [2][CO] BN1 backward reduction
  const uint16_t* x = nullptr;     // [M][CI] conv1 input
  const uint16_t* w = nullptr;     // [CO][CI]
  const uint16_t* addend = nullptr;  // [M][CI] residual branch gradient (unmasked)
  const uint8_t* amask = nullptr;  // its ReLU mask bits
  const uint16_t* px = nullptr;    // [M][CI] previous tail BN input
  const float* psave = nullptr;    // [4][CI]
  const uint8_t* pmask = nullptr;  // previous tail ReLU mask bits
  float* pslots = nullptr;         // [NSLOT][2][CI]
  uint16_t* dx = nullptr;          // [M][CI]
  float* slab = nullptr;           // [grid][CO * CI]
  int M = 0, CI = 0, CO = 0;
};
bool pw_bwd_squeeze_ok(int CI, int CO, int64_t M);
int pw_bwd_squeeze_grid(int CI, int CO, int64_t M);                  // blocks (a multiple of the column split)
int64_t pw_bwd_squeeze_slab_floats(int CI, int CO, int nblocks);     // wgrad slab workspace
void pw_bwd_squeeze(const PwSqueezeBwdArgs& args, int nblocks, hipStream_t s);

// ---------------------------------------------------------------- f32 GEMM (MFMA f32, exact)
// C[M][N] = act(alpha * op(A) op(B) + bias) (+ C if accumulate); op = transpose flags
// allow_split: split K over blocks with f32-atomic partials when the output has few tiles (act 0)
void sgemm_launch(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
                  int ldb, int ldc, bool transA, bool transB, int act, bool accumulate, hipStream_t s,
                  bool allow_split = false);

// ---------------------------------------------------------------- batch norm (NHWC)
// slots: persistent per-layer workspace [NSLOT][2][C] f32, zero between uses (consumers re-zero it)
void bn_stats(const uint16_t* x, int64_t M, int C, float* slots, hipStream_t s);
// Deterministic-reduction test mode (op set_deterministic): the reductions whose f32 atomic order varies
// from run to run take a fixed order instead -- forward BN statistics recomputed by bn_stats_det before
// each finalize, split-K weight gradients unsplit (one block per output tile), slab reductions in one
// group.  Slower; for tests that compare fused and layer-wise paths bit-for-bit-stable.
void set_det_mode(bool on);
bool det_mode();
void bn_stats_det(const uint16_t* x, int64_t M, int C, float* slots, hipStream_t s);
void bn_finalize(float* slots, int64_t M, int C, const float* gamma, const float* beta, float eps,
                 float momentum, float* run_mean, float* run_var, float* save, hipStream_t s);
// slots -> red = [sum g' | sum g' xhat] (+= into dbeta / dgamma when given), slots re-zeroed
void bn_slot_reduce(float* slots, int C, float* red, float* dgamma, float* dbeta, hipStream_t s);
void bn_eval_prep(int C, const float* gamma, const float* beta, float eps, const float* run_mean,
                  const float* run_var, float* save, hipStream_t s);
bool igemm_xt_enabled();  // TFX_IGEMM_XT (igemm.hip)
// mask (optional, residual + ReLU on the C % 8 == 0 path): 1 bit per element, the ReLU mask of y
void bn_apply(const uint16_t* x, const uint16_t* res, const float* save, int64_t M, int C, bool relu,
              uint16_t* y, uint8_t* mask, hipStream_t s);
// residual + ReLU: pass the forward's mask (vector path) or res (generic path) for the ReLU mask
// y = act(bn(x) + bn'(res_x)): the residual BN (res_save) applied on the fly (vector path, vec_ok(C))
void bn_apply_res_bn(const uint16_t* x, const uint16_t* res_x, const float* save, const float* res_save, int64_t M,
                     int C, bool relu, uint16_t* y, uint8_t* mask, hipStream_t s);
// every 3x3 filter W[Ko][3][3][C] of a flat bf16 buffer -> Wf[C][3][3][Ko] flipped (wflip.hip);
// desc: nlayers x {src_off, dst_off, Ko, C, first_tile} int64 on the device, Ko % 64 == C % 64 == 0
void wflip3x3(const uint16_t* src, uint16_t* dst, const int64_t* desc, int nlayers, int ntiles, hipStream_t s);
bool bn_backward_apply_sec_ok(int C);
void bn_backward_apply_sec(const uint16_t* g, const uint16_t* x, const uint8_t* mask, const float* save,
                           const float* red, int64_t M, int C, bool relu, uint16_t* dx, uint16_t* dres,
                           const uint16_t* x2, const float* save2, float* slots2, hipStream_t s);
void bn_backward_apply(const uint16_t* g, const uint16_t* x, const uint16_t* res, const uint8_t* mask,
                       const float* save, const float* red, int64_t M, int C, bool relu, uint16_t* dx,
                       uint16_t* dres, hipStream_t s);
// backward partials (sum g', sum g' xhat) of the vector path into slots (no slot reduce)
void bn_bwd_reduce(const uint16_t* g, const uint16_t* x, const uint8_t* mask, bool has_res, const float* save,
                   int64_t M, int C, bool relu, float* slots, hipStream_t s);
void bn_backward(const uint16_t* g, const uint16_t* x, const uint16_t* res, const uint8_t* mask, const float* save,
                 int64_t M, int C, bool relu, float* slots, float* red, float* dgamma, float* dbeta, uint16_t* dx,
                 uint16_t* dres, hipStream_t s);

// ---------------------------------------------------------------- loss / pooling
void softmax_xent(const void* z, bool z_bf16, int B, int C, const int64_t* lab_idx, const float* lab_dense,
                  bool naive, float gscale, float* loss_rows, float* dz, float* probs, hipStream_t s);
// single-block variant for small batches: batch-mean loss + dz (f32 or bf16) in one launch
void softmax_xent_mean(const void* z, bool z_bf16, int B, int C, const int64_t* lab_idx, const float* lab_dense,
                       bool naive, float gscale, float* loss_mean, void* dz, bool dz_bf16, hipStream_t s);
void accuracy_count(const void* z, bool z_bf16, int B, int C, const int64_t* lab_idx, const float* lab_dense,
                    float* count, hipStream_t s);
void gap_fwd(const uint16_t* x, int N, int HW, int C, uint16_t* y16, float* y32, hipStream_t s);
void gap_bwd(const void* dy, bool dy_bf16, int N, int HW, int C, uint16_t* dx, hipStream_t s);

// fused classifier head (head.hip): gap -> FC -> softmax xent -> unit-seed input gradient, one block per
// sample; feat [N][C] bf16 and dz [N][O] bf16 are kept for dW / db; state = 3 zeroed u64 (self-resetting)
struct HeadXentArgs {
  const uint16_t* x = nullptr;       // [N][HW][C] bf16
  const uint16_t* w = nullptr;       // [O][C] bf16
  const float* b = nullptr;          // [O] f32 or null
  const int64_t* labels = nullptr;   // [N]
  uint16_t* feat = nullptr;          // [N][C] pooled features (bf16)
  uint16_t* dz = nullptr;            // [N][O] (p - onehot) * gscale (bf16)
  uint16_t* dfeat = nullptr;         // [N][HW][C] input gradient (bf16)
  float* loss = nullptr;             // [1] batch mean
  unsigned long long* state = nullptr;
  // tail mode (y3 set): x is not read; the input is relu(y3 * scale + shift + res) of the last block's
  // tail BN (save3 = its [4][C] save), its mask bits are written to mask [N*HW][C/8] and its backward
  // partials written to bn_rows [N][2][C] (head_rows_reduce sums them)
  const uint16_t* y3 = nullptr;
  const uint16_t* res = nullptr;
  const float* save3 = nullptr;
  uint8_t* mask = nullptr;
  float* bn_rows = nullptr;
  int C = 0, HW = 0, O = 0;
  float gscale = 0.f;
};
bool head_xent_ok(int C, int O, int HW);
void head_rows_reduce(const float* rows, int N, int C, float* red, float* dgamma, float* dbeta, hipStream_t s);
void head_xent_fwd(const HeadXentArgs& args, int N, hipStream_t s);
// dW [O][C] += dz^T feat, db += colsum(dz) (plain read-modify-write: one block per 8 channels)
void head_wgrad(const uint16_t* dz, const uint16_t* feat, int N, int C, int O, float* dw, float* db, hipStream_t s);

// CIFAR stem weight gradient (stem.hip): 3x3 s1 p1 conv of 32x32 images with 8 (padded) input channels,
// Ko = 64: dw [Ko][3][3][8] +=, one block per image into copies of a zeroed workspace (re-zeroed)
bool stem_wgrad_ok(int N, int H, int W, int C, int Ko);
int stem_wgrad_ws_floats(int Ko);
void stem_wgrad(const uint16_t* x, const uint16_t* dy, int N, int Ko, float* ws, float* dw, hipStream_t s);
// ... and its forward: y [N][32][32][Ko] bf16, BN statistics of y into slots [NSLOT][2][Ko]
void stem_fwd(const uint16_t* x, const uint16_t* w, int N, int Ko, uint16_t* y, float* slots, hipStream_t s);

// ---------------------------------------------------------------- optimizers (flat buffers)
void optimizer_apply(int kind, float* p, const void* g, bool g_bf16, float* m, float* v, int64_t n,
                     const float* lr, float gscale, float wd, float b1, float b2, float eps, const float* step,
                     const float* sumsq, float max_norm, uint16_t* pbf, const int* skip, float* gz,
                     hipStream_t s);
void sumsq_flat(const void* g, bool g_bf16, int64_t n, float* out, hipStream_t s);
void cast_f32_bf16(const float* x, int64_t n, uint16_t* y, hipStream_t s);

// ---------------------------------------------------------------- small fused elementwise ops (elementwise.hip)
// y = w[c] * x + b[c] over [n/C][C]; backward dx = g * w (dx may be null), dw / db += column sums
void affine_fwd(const float* x, const float* w, const float* b, int64_t n, int C, float* y, hipStream_t s);
void affine_bwd(const float* g, const float* x, const float* w, int64_t n, int C, float* dx, float* dw, float* db,
                hipStream_t s);
// loss[0] = sum (p - y)^2 ; dp = 2 (p - y) * g[0]
void sse_fwd(const float* p, const float* y, int64_t n, float* loss, hipStream_t s);
void sse_bwd(const float* p, const float* y, const float* g, int64_t n, float* dp, hipStream_t s);
// dz = g * act'(y) (act 0 none, 1 relu, 2 sigmoid, y = the activation OUTPUT); dbias += column sums
void act_bwd_colsum(const float* g, const float* y, int act, int64_t M, int N, float* dz, float* dbias,
                    hipStream_t s);
void act_bwd_colsum_bf16(const uint16_t* g, const uint16_t* y, int act, int64_t M, int N, uint16_t* dz,
                         float* dbias, hipStream_t s);
// linear layer with O <= 64 outputs (classifier head), bf16 g [B][O], x [B][I], W [O][I]:
// dx = g W (bf16, skipped when null), dW += g^T x, db += colsum(g) (f32 atomics, skipped when null)
void linear_small_bwd(const uint16_t* g, const uint16_t* x, const uint16_t* w, int B, int I, int O, uint16_t* dx,
                      float* dw, float* db, hipStream_t s);
// y = x * scal[0] (f32 or bf16 output)
void scale_by_scalar(const float* x, const float* scal, int64_t n, float* y32, uint16_t* y16, hipStream_t s);

// ---------------------------------------------------------------- pooling (NHWC bf16)
void maxpool_fwd(const uint16_t* x, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, uint16_t* y,
                 uint8_t* arg, hipStream_t st);
void maxpool_bwd(const uint16_t* dy, const uint8_t* arg, int N, int H, int W, int C, int k, int s, int pad, int P,
                 int Q, uint16_t* dx, hipStream_t st);
void avgpool_fwd(const uint16_t* x, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, uint16_t* y,
                 hipStream_t st);
void avgpool_bwd(const uint16_t* dy, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, uint16_t* dx,
                 hipStream_t st);

// ---------------------------------------------------------------- sparse (word2vec) / recurrent (LSTM)
void embedding_gather(const float* table, int64_t V, int D, const int64_t* ids, int64_t n, void* out, bool out_bf16,
                      hipStream_t s);
void embedding_scatter_add(float* table, int64_t V, int D, const int64_t* ids, int64_t n, const float* rows,
                           float alpha, hipStream_t s);
void log_uniform_sample(int64_t n, int64_t range, uint64_t seed, const int64_t* seed_dev, const int64_t* ids_in,
                        int64_t* out, float* logq, int num_expected, hipStream_t s);
void skipgram_batch(const int32_t* corpus, int64_t N, int B, int window, uint64_t seed, const int64_t* seed_dev,
                    int64_t* centers, int64_t* labels, hipStream_t s);
void sampled_loss(bool softmax, const float* E, const float* Wt, const float* bt, const float* nl, int B, int S, int D,
                  const float* logq_t, const float* logq_n, const int64_t* tid, const int64_t* sid, float gscale,
                  float* loss, float* dn, float* dE, float* dWt, float* dbt, hipStream_t s);
void lstm_cell_fwd(const float* gx, const float* gh, const float* bias, const float* c_prev, int B, int H,
                   float* act, float* c, float* h, uint16_t* h16, hipStream_t s);
void lstm_cell_bwd(const float* act, const float* c, const float* c_prev, const float* dh, const float* dc_next,
                   int B, int H, float* dgates, uint16_t* dg16, float* dc_prev, hipStream_t s);
// persistent whole-sequence recurrence (lstm_seq.hip): one launch per layer and direction
int lstm_seq_sync_words(int B, int H);
bool lstm_seq_supported(int B, int H, int num_cus);
// resident workgroups (occupancy API x CUs) of the forward / backward kernels at hidden size H
void lstm_seq_residency(int B, int H, int num_cus, int* fwd, int* bwd);
// status: a sticky health word (set to 1 when a bounded hand-off wait expires; never cleared by the
// launch) -- null = the sync buffer's own status word; spin_limit 0 = the default bound (tests force 1)
void lstm_seq_fwd(const float* gx, const uint16_t* whh, int T, int B, int H, uint16_t* hbuf, float* cbuf, float* act,
                  float* hT, unsigned* sync, unsigned* status, unsigned spin_limit, hipStream_t s);
void lstm_seq_bwd(const float* act, const float* cbuf, const uint16_t* dH, const float* dhT, const float* dc_in,
                  const uint16_t* whh, int T, int B, int H, uint16_t* dg, float* dc_out, float* dbias, unsigned* sync,
                  unsigned* status, unsigned spin_limit, hipStream_t s);

// ---------------------------------------------------------------- input pipeline
// uint8 NHWC [npix][cin] (cin <= 4) -> bf16 NHWC [npix][cout] (cout 4 or 8): (x/255 - mean)/std, zero pad
// pad-P random crop + flip (per-image off[n] = {ox, oy, flip}) fused with image_normalize
void augment_normalize(const uint8_t* x, int N, int H, int W, int cin, int cout, int pad, const int32_t* off,
                       const float* mean, const float* stdv, uint16_t* y, hipStream_t s);
void image_normalize(const uint8_t* x, int64_t npix, int cin, int cout, const float* mean, const float* stdv,
                     uint16_t* y, hipStream_t s,
                     const int64_t* lab = nullptr, int64_t* lab_out = nullptr, int nlab = 0);

// ---------------------------------------------------------------- ps transport over xGMI peer memory
// p -= lr*g on a (peer-mapped) arena range (g zeroed as consumed if zero_g); then, if step != null,
// bump the 64-bit global step there (system-scope atomic, after the whole update) and write the new
// value to step_out (worker-local).  ps_peer_copy: arena -> store.  IPC helpers return 0 / -hipError.
void ps_peer_sgd(float* p, float* g, int64_t n, float lr, bool zero_g, void* step, int64_t* step_out,
                 hipStream_t s);
void ps_peer_copy(float* dst, const float* src, int64_t n, hipStream_t s);
int ipc_alloc(int device, int64_t nbytes, void** ptr);
int ipc_free(int device, void* ptr);
int ipc_get_handle(void* ptr, uint8_t* out64);
int ipc_open(int device, const uint8_t* handle64, void** ptr);
int ipc_close(void* ptr);

// ---------------------------------------------------------------- one-GPU stand-in for an 8-rank ring all-reduce
// nblocks workgroups stream buf (read + write back the same bytes) for duration_us (<= 10 ms), holding
// their CUs like RCCL's channel blocks (dp_sim.hip; scripts/dp_contention.py)
void dp_ring_sim(void* buf, int64_t nbytes, int nblocks, double duration_us, int passes, hipStream_t s);

// ---------------------------------------------------------------- Philox4x32-10 init (dist 0 uniform [a,b),
// 1 normal(a, b), 2 normal(a, b) truncated at 2 sigma)
void philox_fill(float* out, int64_t n, uint64_t seed, uint64_t subseq, int dist, float a, float b, hipStream_t s);

}  // namespace tfx
