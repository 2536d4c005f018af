// TORCH_LIBRARY(tfx) registrations: shape/dtype validation on the host, then the raw-pointer
// HIP launchers of csrc/kernels on the current HIP stream (so every op is capturable in a
// hipGraph and ordered with PyTorch's own work).  The Python autograd layer lives in
// tensorflow_examples_amd/ops.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdlib>
#include <tuple>
#include <vector>

#include "tfx_kernels.h"
#include "../kernels/igemm_entry.h"

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be f32")

const uint16_t* bf(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bfm(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const float* fp(const optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }
float* fpm(const optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

void check_aligned16(const Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

struct ConvGeom {
  int64_t N, H, W, C, Ko, R, S, P, Q;
};

ConvGeom geom(const std::vector<int64_t>& xs, const std::vector<int64_t>& ws, int64_t st, int64_t pad, int64_t dil) {
  TORCH_CHECK(xs.size() == 4 && ws.size() == 4, "conv expects NHWC input and [Ko,R,S,C] weight");
  ConvGeom g;
  g.N = xs[0]; g.H = xs[1]; g.W = xs[2]; g.C = xs[3];
  g.Ko = ws[0]; g.R = ws[1]; g.S = ws[2];
  TORCH_CHECK(ws[3] == g.C, "weight C mismatch");
  TORCH_CHECK(g.C % 8 == 0 && g.Ko % 8 == 0, "conv needs C%8==0 and Ko%8==0 (pad channels)");
  g.P = (g.H + 2 * pad - dil * (g.R - 1) - 1) / st + 1;
  g.Q = (g.W + 2 * pad - dil * (g.S - 1) - 1) / st + 1;
  TORCH_CHECK(g.P > 0 && g.Q > 0, "conv output is empty");
  TORCH_CHECK(g.N * std::max(g.H * g.W * g.C, g.P * g.Q * g.Ko) * 2 < (int64_t(1) << 31),
              "conv tensors must be < 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(g.N * g.H * g.W < (int64_t(1) << 24) && g.N * g.P * g.Q < (int64_t(1) << 24) &&
                  g.R * g.S * g.C < (int64_t(1) << 24),
              "conv pixel counts must be < 2^24 (24-bit address multiplies): split the batch");
  return g;
}

tfx::IgemmArgs conv_args(const ConvGeom& g, int64_t st, int64_t pad, int64_t dil) {
  tfx::IgemmArgs a;
  a.Nb = g.N; a.H = g.H; a.W = g.W; a.C = g.C; a.Ko = g.Ko; a.R = g.R; a.S = g.S; a.P = g.P; a.Q = g.Q;
  a.sh = a.sw = st; a.ph = a.pw = pad; a.dh = a.dw = dil;
  TORCH_CHECK(st > 0 && (st & (st - 1)) == 0, "conv stride must be a power of two");
  a.sh_log2 = a.sw_log2 = __builtin_ctzll(st);
  a.fd_C = tfx::FastDiv(g.C); a.fd_S = tfx::FastDiv(g.S); a.fd_Ko = tfx::FastDiv(g.Ko);
  a.fd_PQ = tfx::FastDiv(g.P * g.Q); a.fd_Q = tfx::FastDiv(g.Q);
  return a;
}

// ------------------------------------------------------------------ conv
Tensor conv_fwd_impl(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil, float* stats) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w);
  auto g = geom(x.sizes().vec(), w.sizes().vec(), stride, pad, dil);
  auto y = at::empty({g.N, g.P, g.Q, g.Ko}, x.options());
  auto a = conv_args(g, stride, pad, dil);
  a.A = bf(x); a.B = bf(w); a.Cp = y.data_ptr();
  a.a_bytes = x.nbytes(); a.b_bytes = w.nbytes();
  a.M = g.N * g.P * g.Q; a.N = g.Ko; a.K = g.R * g.S * g.C; a.ldb = a.K; a.ldc = g.Ko;
  a.out_mode = tfx::OUT_BF16;
  a.stats = stats;
  tfx::igemm_launch(a, tfx::MODE_FWD, cur_stream());
  return y;
}

Tensor conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil) {
  return conv_fwd_impl(x, w, stride, pad, dil, nullptr);
}

// conv forward + the per-channel BN statistics of its output, fused into the GEMM epilogue and
// accumulated into the BN layer's persistent slot workspace ([NSLOT][2][Ko], zero on entry).
Tensor conv_fwd_stats(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil, Tensor slots) {
  CHECK_F32(slots);
  TORCH_CHECK(slots.numel() >= tfx::NSLOT * 2 * w.size(0), "stat slots size");
  return conv_fwd_impl(x, w, stride, pad, dil, slots.data_ptr<float>());
}

// dX = dgrad(dy) (+ addend: the gradient of x's other consumer, summed in the epilogue; the
// result is written in place into addend's storage when given)
// addend_mask: 1-bit ReLU mask of the addend (uint8 per 8 channels): dX = dgrad + addend * mask,
// into a fresh buffer (the addend -- a residual BN's unmasked output gradient -- stays intact)
const uint8_t* addend_mask_ptr(const optional<Tensor>& addend, const optional<Tensor>& mask) {
  if (!(mask.has_value() && mask->defined())) return nullptr;
  TORCH_CHECK(addend.has_value() && addend->defined(), "addend_mask without addend");
  TORCH_CHECK(mask->scalar_type() == at::kByte && mask->is_contiguous() && mask->numel() * 8 == addend->numel(),
              "addend_mask: uint8, one byte per 8 addend elements");
  return mask->data_ptr<uint8_t>();
}

// addend_s2: the addend is the compact even-pixel gradient [N][ceil(H/2)][ceil(W/2)][C] of a 1x1
// stride-2 branch (its data gradient computed on the strided grid only); the epilogue adds it at the
// even (y, x) pixels and nothing elsewhere -- no zero-filled full-size tensor is ever written
void set_addend_s2(tfx::IgemmArgs& a, const Tensor& addend, int64_t N, int64_t H, int64_t W, int64_t C) {
  const int64_t P2 = (H + 1) / 2, Q2 = (W + 1) / 2;
  CHECK_BF16(addend); CHECK_CONTIG(addend);
  TORCH_CHECK(addend.sizes() == at::IntArrayRef({N, P2, Q2, C}), "stride-2 compact addend shape");
  a.addend = bf(addend);
  a.addend_s2 = 1; a.s2_P = (int)P2; a.s2_Q = (int)Q2;
  a.fd_s2HW = tfx::FastDiv((uint32_t)(H * W)); a.fd_s2W = tfx::FastDiv((uint32_t)W);
}

// Data-gradient GEMM setup.  With ``wflip`` (= W flipped and channel-transposed, [C][3][3][Ko]) a
// 3x3 stride-1 pad-1 data gradient is posed as the forward conv of dY with it (MODE_DGRAD_FLIP:
// K-major operands, igemm_dgrad_flip.hip); otherwise the gathered data-gradient GEMM (MODE_DGRAD).
int dgrad_setup(tfx::IgemmArgs& a, const ConvGeom& g, const Tensor& dy, const Tensor& w,
                const optional<Tensor>& wflip, int64_t stride, int64_t pad, int64_t dil) {
  if (wflip.has_value() && wflip->defined() && g.R == 3 && g.S == 3 && stride == 1 && pad == 1 && dil == 1) {
    CHECK_BF16(*wflip); CHECK_CONTIG(*wflip);
    TORCH_CHECK(wflip->sizes() == at::IntArrayRef({g.C, 3, 3, g.Ko}), "wflip shape");
    auto gf = geom({g.N, g.P, g.Q, g.Ko}, {g.C, 3, 3, g.Ko}, 1, 1, 1);
    a = conv_args(gf, 1, 1, 1);
    a.A = bf(dy); a.B = bf(*wflip);
    a.a_bytes = dy.nbytes(); a.b_bytes = wflip->nbytes();
    a.M = g.N * g.H * g.W; a.N = g.C; a.K = 9 * g.Ko; a.ldb = a.K; a.ldc = g.C;
    return tfx::MODE_DGRAD_FLIP;
  }
  a = conv_args(g, stride, pad, dil);
  a.A = bf(dy); a.B = bf(w);
  a.a_bytes = dy.nbytes(); a.b_bytes = w.nbytes();
  a.M = g.N * g.H * g.W; a.N = g.C; a.K = g.R * g.S * g.Ko; a.ldc = g.C;
  return tfx::MODE_DGRAD;
}

// output-parity class (cph, cpw) of a stride-2 data gradient as a dense stride-1 implicit GEMM over
// its own taps r = r0 + 2 ri, s = s0 + 2 si (see conv_dgrad); rows = the class's sub-grid pixels
void cls_setup(tfx::IgemmArgs& a, const ConvGeom& g, const Tensor& dy, const Tensor& w, int64_t pad, int cph,
               int cpw) {
  const int r0 = (cph + pad) % 2, s0 = (cpw + pad) % 2;
  const int Rc = (int)(g.R - r0 + 1) / 2, Sc = (int)(g.S - s0 + 1) / 2;
  const int Hc = (int)(g.H - cph + 1) / 2, Wc = (int)(g.W - cpw + 1) / 2;
  a.Nb = g.N; a.H = Hc; a.W = Wc; a.C = g.C; a.Ko = g.Ko; a.R = Rc; a.S = Sc; a.P = g.P; a.Q = g.Q;
  a.sh = a.sw = 1; a.sh_log2 = a.sw_log2 = 0; a.dh = a.dw = 1;
  a.ph = (cph + pad - r0) / 2; a.pw = (cpw + pad - s0) / 2;  // p = y + ph - ri
  a.fd_C = tfx::FastDiv(g.C); a.fd_S = tfx::FastDiv(Sc); a.fd_Ko = tfx::FastDiv(g.Ko);
  a.fd_PQ = tfx::FastDiv(g.P * g.Q); a.fd_Q = tfx::FastDiv(g.Q);
  a.cls = 1; a.cph = cph; a.cpw = cpw; a.cr0 = r0; a.cs0 = s0; a.wR = g.R; a.wS = g.S;
  a.out_H = g.H; a.out_W = g.W;
  a.fd_cHW = tfx::FastDiv(Hc * Wc); a.fd_cW = tfx::FastDiv(Wc);
  a.A = bf(dy); a.B = bf(w);
  a.a_bytes = dy.nbytes(); a.b_bytes = w.nbytes();
  a.M = g.N * Hc * Wc; a.N = g.C; a.K = Rc * Sc * g.Ko; a.ldc = g.C;
}

Tensor conv_dgrad(Tensor dy, Tensor w, std::vector<int64_t> xshape, int64_t stride, int64_t pad, int64_t dil,
                  optional<Tensor> addend, optional<Tensor> addend_mask, bool addend_s2,
                  optional<Tensor> wflip) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(w); CHECK_CONTIG(w);
  auto g = geom(xshape, w.sizes().vec(), stride, pad, dil);
  TORCH_CHECK(dy.size(0) == g.N && dy.size(1) == g.P && dy.size(2) == g.Q && dy.size(3) == g.Ko, "dy shape");
  const bool acc = addend.has_value() && addend->defined();
  if (addend_s2) {
    TORCH_CHECK(acc && stride == 1 && !(addend_mask.has_value() && addend_mask->defined()),
                "stride-2 compact addend: stride-1 data gradients, no mask");
    auto dx = at::empty({g.N, g.H, g.W, g.C}, dy.options());
    tfx::IgemmArgs a;
    const int mode = dgrad_setup(a, g, dy, w, wflip, stride, pad, dil);
    a.Cp = dx.data_ptr();
    a.out_mode = tfx::OUT_BF16;
    set_addend_s2(a, *addend, g.N, g.H, g.W, g.C);
    tfx::igemm_launch(a, mode, cur_stream());
    return dx;
  }
  if (acc) {
    CHECK_BF16(*addend); CHECK_CONTIG(*addend);
    TORCH_CHECK(addend->sizes() == at::IntArrayRef({g.N, g.H, g.W, g.C}), "addend shape");
  }
  const uint8_t* amask = addend_mask_ptr(addend, addend_mask);
  if (amask) {
    TORCH_CHECK(stride == 1 && g.C % 8 == 0, "masked addend: stride-1 data gradients with C % 8 == 0");
    auto dx = at::empty({g.N, g.H, g.W, g.C}, dy.options());
    tfx::IgemmArgs a;
    const int mode = dgrad_setup(a, g, dy, w, wflip, stride, pad, dil);
    a.Cp = dx.data_ptr();
    a.out_mode = tfx::OUT_BF16;
    a.addend = bf(*addend); a.addend_mask = amask;
    tfx::igemm_launch(a, mode, cur_stream());
    return dx;
  }
  if (stride == 2 && dil == 1) {
    // Stride-2 data gradient by output-parity class: pixel (h, w) only receives taps with
    // r = h + pad (mod 2), s = w + pad (mod 2), so each of the 4 classes is a dense stride-1
    // implicit GEMM over its own taps -- a quarter of the MACs of the zero-filled single GEMM.
    bool empty_class = false;
    for (int cph = 0; cph < 2; ++cph)
      for (int cpw = 0; cpw < 2; ++cpw)
        if ((g.R - (cph + pad) % 2 + 1) / 2 <= 0 || (g.S - (cpw + pad) % 2 + 1) / 2 <= 0) empty_class = true;
    auto dx = acc ? *addend : (empty_class ? at::zeros({g.N, g.H, g.W, g.C}, dy.options())
                                           : at::empty({g.N, g.H, g.W, g.C}, dy.options()));
    for (int cph = 0; cph < 2; ++cph) {
      for (int cpw = 0; cpw < 2; ++cpw) {
        const int r0 = (cph + pad) % 2, s0 = (cpw + pad) % 2;
        const int Rc = (int)(g.R - r0 + 1) / 2, Sc = (int)(g.S - s0 + 1) / 2;
        const int Hc = (int)(g.H - cph + 1) / 2, Wc = (int)(g.W - cpw + 1) / 2;
        if (Rc <= 0 || Sc <= 0 || Hc <= 0 || Wc <= 0) continue;  // dx keeps addend / zeros there
        tfx::IgemmArgs a;
        cls_setup(a, g, dy, w, pad, cph, cpw);
        a.Cp = dx.data_ptr();
        a.out_mode = tfx::OUT_BF16;
        if (acc) a.addend = bf(*addend);
        tfx::igemm_launch(a, tfx::MODE_DGRAD_CLS, cur_stream());
      }
    }
    return dx;
  }
  auto dx = acc ? *addend : at::empty({g.N, g.H, g.W, g.C}, dy.options());
  tfx::IgemmArgs a;
  const int mode = dgrad_setup(a, g, dy, w, wflip, stride, pad, dil);
  a.Cp = dx.data_ptr();
  a.out_mode = tfx::OUT_BF16;
  if (acc) a.addend = bf(*addend);
  tfx::igemm_launch(a, mode, cur_stream());
  return dx;
}

// ---- fused BN epilogues.  ws = the BN layer's workspace: [NSLOT][2][C] f32 slots (all zero
// between uses; the finalize / slot-reduce kernels that consume them restore that).
void check_bn_ws(const Tensor& ws, int64_t C) {
  CHECK_F32(ws); CHECK_CONTIG(ws);
  TORCH_CHECK(ws.numel() >= tfx::NSLOT * 2 * C, "BN workspace too small for the fused epilogue");
}

// deterministic mode: the producer's epilogue statistics replaced by a fixed-order recompute from y
void det_restat(const Tensor& y, float* slots, int64_t M, int64_t C) {
  if (tfx::det_mode()) tfx::bn_stats_det(bf(y), M, (int)C, slots, cur_stream());
}

bool set_deterministic(bool on) {
  const bool prev = tfx::det_mode();
  tfx::set_det_mode(on);
  return prev;
}

bool g_stem_fwd = true;  // conv_fwd_bn routes the CIFAR stem (8 channels, 32x32, 64 outputs) to stem.hip

// conv forward whose epilogue produces the following BN's batch statistics, then the finalize:
// returns (y, save = [mean | invstd | scale | shift]) and updates the running statistics -- the BN
// then only applies (bn_apply_train).
std::tuple<Tensor, Tensor> conv_fwd_bn(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil, Tensor ws,
                                       optional<Tensor> gamma, optional<Tensor> beta, optional<Tensor> run_mean,
                                       optional<Tensor> run_var, double momentum, double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w);
  auto g = geom(x.sizes().vec(), w.sizes().vec(), stride, pad, dil);
  auto y = at::empty({g.N, g.P, g.Q, g.Ko}, x.options());
  auto save = at::empty({4 * g.Ko}, x.options().dtype(at::kFloat));
  auto a = conv_args(g, stride, pad, dil);
  a.A = bf(x); a.B = bf(w); a.Cp = y.data_ptr();
  a.a_bytes = x.nbytes(); a.b_bytes = w.nbytes();
  a.M = g.N * g.P * g.Q; a.N = g.Ko; a.K = g.R * g.S * g.C; a.ldb = a.K; a.ldc = g.Ko;
  a.out_mode = tfx::OUT_BF16;
  check_bn_ws(ws, g.Ko);
  a.stats = ws.data_ptr<float>();
  if (g_stem_fwd && stride == 1 && pad == 1 && dil == 1 && g.R == 3 && g.S == 3 &&
      tfx::stem_wgrad_ok((int)g.N, (int)g.H, (int)g.W, (int)g.C, (int)g.Ko)) {
    check_aligned16(x, "x"); check_aligned16(w, "w");
    tfx::stem_fwd(bf(x), bf(w), (int)g.N, (int)g.Ko, bfm(y), a.stats, cur_stream());  // the CIFAR stem (stem.hip)
  } else {
    tfx::igemm_launch(a, tfx::MODE_FWD, cur_stream());
  }
  det_restat(y, a.stats, a.M, g.Ko);
  tfx::bn_finalize(a.stats, a.M, g.Ko, fp(gamma), fp(beta), (float)eps, (float)momentum, fpm(run_mean),
                   fpm(run_var), save.data_ptr<float>(), cur_stream());
  return {y, save};
}

// A/B hook for the stem forward kernel; returns the previous setting
bool conv_stem_fwd(bool on) {
  const bool prev = g_stem_fwd;
  g_stem_fwd = on;
  return prev;
}

// conv_fwd_bn of relu(x * in_save[2C..3C) + in_save[3C..4C)) -- a plain ReLU BN applied on load by this
// 1x1 stride-1 conv of C <= 64 input channels (one k-tile, register path), so the BN output is never
// written.  Returns (y, save).  (Wider forms were measured slower than the apply pass, profiles/r05_bna.)
bool conv_fwd_bn_in_supported(int64_t M, int64_t Ko, int64_t C) { return M > 0 && Ko > 0 && C <= 64 && C % 8 == 0; }

std::tuple<Tensor, Tensor> conv_fwd_bn_in(Tensor x, Tensor in_save, Tensor w, Tensor ws, optional<Tensor> gamma,
                                          optional<Tensor> beta, optional<Tensor> run_mean, optional<Tensor> run_var,
                                          double momentum, double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w);
  CHECK_F32(in_save); CHECK_CONTIG(in_save);
  auto g = geom(x.sizes().vec(), w.sizes().vec(), 1, 0, 1);
  TORCH_CHECK(g.R == 1 && g.S == 1 && in_save.numel() == 4 * g.C && g.C <= 64 && g.C % 8 == 0,
              "conv_fwd_bn_in: 1x1 conv with <= 64 input channels and the input BN's [4][C] save");
  auto y = at::empty({g.N, g.P, g.Q, g.Ko}, x.options());
  auto save = at::empty({4 * g.Ko}, x.options().dtype(at::kFloat));
  auto a = conv_args(g, 1, 0, 1);
  a.A = bf(x); a.B = bf(w); a.Cp = y.data_ptr();
  a.a_bytes = x.nbytes(); a.b_bytes = w.nbytes();
  a.M = g.N * g.P * g.Q; a.N = g.Ko; a.K = g.C; a.ldb = a.K; a.ldc = g.Ko;
  a.out_mode = tfx::OUT_BF16;
  check_bn_ws(ws, g.Ko);
  a.stats = ws.data_ptr<float>();
  a.a_scale = in_save.data_ptr<float>() + 2 * g.C;
  a.a_shift = in_save.data_ptr<float>() + 3 * g.C;
  tfx::igemm_launch(a, tfx::MODE_FWD, cur_stream());
  det_restat(y, a.stats, a.M, g.Ko);
  tfx::bn_finalize(a.stats, a.M, g.Ko, fp(gamma), fp(beta), (float)eps, (float)momentum, fpm(run_mean),
                   fpm(run_var), save.data_ptr<float>(), cur_stream());
  return {y, save};
}

// Block tail + the next block's conv1 (1x1, CI -> CO) forward in one launch (pw_fwd.hip): writes the
// tail's output `out` and ReLU mask bits into the given buffers (allocated by the tail BN, which
// deferred its apply), then finalizes BN1 from the epilogue statistics as conv_fwd_bn does.
// res_save set: the residual is a never-written shortcut BN output (res = its input).  Returns (y1, save1).
std::tuple<Tensor, Tensor> pw_fwd_squeeze(Tensor y3, Tensor save3, Tensor res, optional<Tensor> res_save, Tensor w,
                                          Tensor out, Tensor mask, Tensor ws, optional<Tensor> gamma,
                                          optional<Tensor> beta, optional<Tensor> run_mean,
                                          optional<Tensor> run_var, double momentum, double eps) {
  CHECK_DEV(y3); CHECK_BF16(y3); CHECK_CONTIG(y3); CHECK_BF16(res); CHECK_CONTIG(res); CHECK_BF16(w);
  CHECK_CONTIG(w); CHECK_BF16(out); CHECK_CONTIG(out); CHECK_F32(save3);
  const int64_t CI = y3.size(-1), CO = w.size(0), M = y3.numel() / CI;
  TORCH_CHECK(w.numel() == CO * CI && res.numel() == M * CI && out.numel() == M * CI && save3.numel() == 4 * CI,
              "pw_fwd_squeeze: shapes");
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.is_contiguous() && mask.numel() * 8 == M * CI, "pw_fwd_squeeze: mask");
  TORCH_CHECK(tfx::pw_fwd_squeeze_ok((int)CI, (int)CO, M), "pw_fwd_squeeze: unsupported widths / rows");
  check_bn_ws(ws, CO);
  std::vector<int64_t> ysh = y3.sizes().vec();
  ysh.back() = CO;
  auto y1 = at::empty(ysh, y3.options());
  auto save = at::empty({4 * CO}, y3.options().dtype(at::kFloat));
  tfx::PwSqueezeArgs a;
  a.y3 = bf(y3); a.save3 = save3.data_ptr<float>(); a.res = bf(res); a.w = bf(w); a.out = bfm(out);
  a.mask = mask.data_ptr<uint8_t>(); a.y1 = bfm(y1); a.slots1 = ws.data_ptr<float>();
  a.M = (int)M; a.CI = (int)CI; a.CO = (int)CO;
  if (res_save.has_value() && res_save->defined()) {
    CHECK_F32(*res_save);
    TORCH_CHECK(res_save->numel() == 4 * CI, "pw_fwd_squeeze: res_save");
    a.save_r = res_save->data_ptr<float>();
  }
  tfx::pw_fwd_squeeze(a, tfx::pw_fwd_squeeze_grid((int)CI, (int)CO, M), cur_stream());
  det_restat(y1, a.slots1, M, CO);
  tfx::bn_finalize(a.slots1, M, (int)CO, fp(gamma), fp(beta), (float)eps, (float)momentum, fpm(run_mean),
                   fpm(run_var), save.data_ptr<float>(), cur_stream());
  return {y1, save};
}

bool pw_fwd_squeeze_supported(int64_t CI, int64_t CO, int64_t M) { return tfx::pw_fwd_squeeze_ok((int)CI, (int)CO, M); }

// BN apply into caller-provided buffers (the fallback of a deferred apply whose consumer could not
// fuse it): out = relu(x sc + sh + res'), res' = res, res * rsc + rsh (res_save) or none; mask bits
// (residual + ReLU layers only)
void bn_apply_into(Tensor x, optional<Tensor> res, Tensor save, optional<Tensor> res_save, Tensor out,
                   optional<Tensor> mask) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(out); CHECK_CONTIG(out);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(out.numel() == x.numel() && C % 8 == 0, "bn_apply_into: shapes");
  const bool has_res = res.has_value() && res->defined();
  uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->numel() * 8 == x.numel(), "bn_apply_into: mask");
    mk = mask->data_ptr<uint8_t>();
  }
  if (has_res) {
    CHECK_BF16(*res); CHECK_CONTIG(*res);
    TORCH_CHECK(res->numel() == x.numel(), "bn_apply_into: residual");
  }
  if (has_res && res_save.has_value() && res_save->defined())
    tfx::bn_apply_res_bn(bf(x), bf(*res), save.data_ptr<float>(), res_save->data_ptr<float>(), M, (int)C, true,
                         bfm(out), mk, cur_stream());
  else
    tfx::bn_apply(bf(x), has_res ? bf(*res) : nullptr, save.data_ptr<float>(), M, (int)C, true, bfm(out), mk,
                  cur_stream());
}

// Stage-1 3x3 conv (64 -> 64, stride 1, pad 1, width 32) applying its input BN + ReLU on load
// (conv3x3_fused.hip): x = the input BN's input, save_in its stats; the output BN's statistics land in
// ws and are finalized as conv_fwd_bn does.  Returns (y, save).
std::tuple<Tensor, Tensor> conv3x3_fwd_fused(Tensor x, Tensor save_in, Tensor w, Tensor ws, optional<Tensor> gamma,
                                             optional<Tensor> beta, optional<Tensor> run_mean,
                                             optional<Tensor> run_var, double momentum, double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_F32(save_in);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(1) == 3 && w.size(2) == 3, "conv3x3_fwd_fused: shapes");
  const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3), K = (int)w.size(0);
  TORCH_CHECK(w.size(3) == C && save_in.numel() == 4 * C, "conv3x3_fwd_fused: shapes");
  TORCH_CHECK(tfx::conv3x3_fused_ok(N, H, W, C, K), "conv3x3_fwd_fused: unsupported geometry");
  check_bn_ws(ws, K);
  auto y = at::empty({N, H, W, K}, x.options());
  auto save = at::empty({4 * K}, x.options().dtype(at::kFloat));
  tfx::Conv3Args a;
  a.x = bf(x); a.save_in = save_in.data_ptr<float>(); a.w = bf(w); a.y = bfm(y); a.slots = ws.data_ptr<float>();
  a.N = N; a.H = H;
  tfx::conv3x3_fwd_fused(a, cur_stream());
  det_restat(y, a.slots, (int64_t)N * H * W, K);
  tfx::bn_finalize(a.slots, (int64_t)N * H * W, K, fp(gamma), fp(beta), (float)eps, (float)momentum, fpm(run_mean),
                   fpm(run_var), save.data_ptr<float>(), cur_stream());
  return {y, save};
}

// Backward of the stage-1 3x3 conv with both BN layers fused (conv3x3_fused.hip): g2 / y2 / save2 / red2
// = the output BN's gradient, input, stats and backward reduction (its apply formed on load); y1 / save1
// = the input BN's input and stats (its ReLU output formed on load for the weight gradient).  dw += dW;
// returns (dx = the input BN's output gradient, red1 = its backward reduction) with dgamma1 / dbeta1 +=.
std::tuple<Tensor, Tensor> conv3x3_bwd_fused(Tensor g2, Tensor y2, Tensor save2, Tensor red2, Tensor y1, Tensor save1,
                                             Tensor w, Tensor dw, Tensor slots1, optional<Tensor> dgamma1,
                                             optional<Tensor> dbeta1) {
  CHECK_DEV(g2); CHECK_BF16(g2); CHECK_CONTIG(g2); CHECK_BF16(y2); CHECK_CONTIG(y2); CHECK_BF16(y1); CHECK_CONTIG(y1);
  CHECK_BF16(w); CHECK_CONTIG(w); CHECK_F32(dw); CHECK_CONTIG(dw); CHECK_F32(save2); CHECK_F32(red2); CHECK_F32(save1);
  TORCH_CHECK(y1.dim() == 4 && g2.sizes() == y1.sizes() && y2.sizes() == y1.sizes(), "conv3x3_bwd_fused: shapes");
  const int N = (int)y1.size(0), H = (int)y1.size(1), W = (int)y1.size(2), C = (int)y1.size(3), K = (int)w.size(0);
  TORCH_CHECK(tfx::conv3x3_fused_ok(N, H, W, C, K) && w.numel() == (int64_t)K * 9 * C && dw.numel() == w.numel(),
              "conv3x3_bwd_fused: unsupported geometry");
  TORCH_CHECK(save2.numel() == 4 * K && red2.numel() == 2 * K && save1.numel() == 4 * C, "conv3x3_bwd_fused: stats");
  check_bn_ws(slots1, C);
  auto dx = at::empty_like(y1);
  auto red1 = at::empty({2 * C}, y1.options().dtype(at::kFloat));
  const int nb = tfx::conv3x3_bwd_fused_grid(N, H);
  auto slab = at::empty({(int64_t)nb * K * 9 * C}, y1.options().dtype(at::kFloat));
  tfx::Conv3BwdArgs a;
  a.g2 = bf(g2); a.y2 = bf(y2); a.save2 = save2.data_ptr<float>(); a.red2 = red2.data_ptr<float>(); a.y1 = bf(y1);
  a.save1 = save1.data_ptr<float>(); a.w = bf(w); a.dx = bfm(dx); a.slots1 = slots1.data_ptr<float>();
  a.slab = slab.data_ptr<float>(); a.N = N; a.H = H;
  tfx::conv3x3_bwd_fused(a, nb, cur_stream());
  tfx::pw_slab_reduce(a.slab, nb, 64, dw.data_ptr<float>(), a.slots1, C, red1.data_ptr<float>(), fpm(dgamma1),
                      fpm(dbeta1), tfx::PwSecReduce{}, cur_stream(), 2);
  return {dx, red1};
}

bool conv3x3_fused_supported(int64_t N, int64_t H, int64_t W, int64_t C, int64_t K) {
  return tfx::conv3x3_fused_ok((int)N, (int)H, (int)W, (int)C, (int)K);
}

// stride-1 conv data gradient whose epilogue also reduces the backward of the BN that produced
// the conv's input (the gradient written here is that BN's complete output gradient): returns
// (dx, red = [sum g' | sum g' xhat]) with dgamma / dbeta accumulated -- the BN then only applies
// (bn_bwd_apply).  bn_mask: the residual + ReLU layer's forward mask bits (else the ReLU mask is
// recomputed from bn_x).
std::tuple<Tensor, Tensor> conv_dgrad_bn(Tensor dy, Tensor w, std::vector<int64_t> xshape, int64_t stride,
                                         int64_t pad, int64_t dil, optional<Tensor> addend, Tensor bn_x,
                                         Tensor bn_save, optional<Tensor> bn_mask, bool relu, Tensor ws,
                                         optional<Tensor> dgamma, optional<Tensor> dbeta,
                                         optional<Tensor> addend_mask, bool reduce, bool addend_s2,
                                         optional<Tensor> wflip) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(w); CHECK_CONTIG(w);
  TORCH_CHECK(stride == 1, "conv_dgrad_bn: stride-1 convs");
  auto g = geom(xshape, w.sizes().vec(), stride, pad, dil);
  TORCH_CHECK(dy.size(0) == g.N && dy.size(1) == g.P && dy.size(2) == g.Q && dy.size(3) == g.Ko, "dy shape");
  CHECK_BF16(bn_x); CHECK_CONTIG(bn_x); CHECK_F32(bn_save);
  TORCH_CHECK(bn_x.sizes() == at::IntArrayRef({g.N, g.H, g.W, g.C}), "bn_x shape");
  TORCH_CHECK(bn_save.numel() == 4 * g.C, "bn_save size");
  const bool acc = addend.has_value() && addend->defined();
  if (acc && !addend_s2) {
    CHECK_BF16(*addend); CHECK_CONTIG(*addend);
    TORCH_CHECK(addend->sizes() == at::IntArrayRef({g.N, g.H, g.W, g.C}), "addend shape");
  }
  TORCH_CHECK(!addend_s2 || (acc && !(addend_mask.has_value() && addend_mask->defined())),
              "stride-2 compact addend: no mask");
  const uint8_t* amask = addend_s2 ? nullptr : addend_mask_ptr(addend, addend_mask);
  auto dx = (acc && !amask && !addend_s2) ? *addend : at::empty({g.N, g.H, g.W, g.C}, dy.options());
  // reduce = false: the partials stay in the slots for a later launch to reduce (conv_wgrad_sr2 tail
  // blocks, or bn_slots_reduce)
  auto red = reduce ? at::empty({2 * g.C}, dy.options().dtype(at::kFloat)) : Tensor();
  const uint8_t* bmask = nullptr;
  if (bn_mask.has_value() && bn_mask->defined()) {
    TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() * 8 == bn_x.numel(), "bn_mask size");
    bmask = bn_mask->data_ptr<uint8_t>();
  }
  tfx::IgemmArgs a;
  const int mode = dgrad_setup(a, g, dy, w, wflip, stride, pad, dil);
  a.Cp = dx.data_ptr();
  a.out_mode = tfx::OUT_BF16;
  if (acc) a.addend = bf(*addend);
  if (addend_s2) set_addend_s2(a, *addend, g.N, g.H, g.W, g.C);
  a.addend_mask = amask;
  a.bnb_x = bf(bn_x); a.bnb_save = bn_save.data_ptr<float>();
  a.bnb_mask = bmask;
  a.bnb_relu = relu ? 1 : 0;
  check_bn_ws(ws, g.C);
  a.bnb_slots = ws.data_ptr<float>();
  tfx::igemm_launch(a, mode, cur_stream());
  if (reduce) tfx::bn_slot_reduce(a.bnb_slots, g.C, red.data_ptr<float>(), fpm(dgamma), fpm(dbeta), cur_stream());
  return {dx, red};
}

// dW (f32, [Ko][R][S][C]) = or += conv weight gradient
void conv_wgrad_impl(Tensor dy, Tensor x, Tensor dw, int64_t stride, int64_t pad, int64_t dil, bool accumulate,
                     const tfx::IgemmArgs* sr) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(dw); CHECK_CONTIG(dw);
  auto g = geom(x.sizes().vec(), dw.sizes().vec(), stride, pad, dil);
  TORCH_CHECK(dy.size(0) == g.N && dy.size(1) == g.P && dy.size(2) == g.Q && dy.size(3) == g.Ko, "dy shape");
  auto a = conv_args(g, stride, pad, dil);
  if (sr) {
    a.sr_slots = sr->sr_slots; a.sr_red = sr->sr_red; a.sr_dgamma = sr->sr_dgamma; a.sr_dbeta = sr->sr_dbeta;
    a.sr_C = sr->sr_C;
    a.sr2_slots = sr->sr2_slots; a.sr2_red = sr->sr2_red; a.sr2_dgamma = sr->sr2_dgamma; a.sr2_dbeta = sr->sr2_dbeta;
    a.sr2_C = sr->sr2_C;
  }
  const int64_t RSC = g.R * g.S * g.C;
  a.K = g.N * g.P * g.Q;
  a.out_mode = tfx::OUT_F32_ATOMIC;
  a.zero_out = accumulate ? 0 : 1;
  a.Cp = dw.data_ptr();
  a.ldc = RSC;
  if (g.Ko < 128 && RSC > g.Ko) {
    // narrow Ko: compute dW^T = Xcol^T dY (M = R*S*C on the 256-row tile side), store transposed
    a.A = bf(x); a.B = bf(dy); a.a_bytes = x.nbytes(); a.b_bytes = dy.nbytes();
    a.M = RSC; a.N = g.Ko; a.ldb = g.Ko; a.trans_out = 1;
    tfx::igemm_launch(a, tfx::MODE_WGRAD_T, cur_stream());
  } else {
    a.A = bf(dy); a.B = bf(x); a.a_bytes = dy.nbytes(); a.b_bytes = x.nbytes();
    a.M = g.Ko; a.N = RSC; a.lda = g.Ko;
    tfx::igemm_launch(a, tfx::MODE_WGRAD, cur_stream());
  }
}

// CIFAR stem weight gradient (stem.hip): dw [64][3][3][8] += dY^T . im2col(x), 32x32 images, 8 channels
bool stem_wgrad_supported(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ko) {
  return tfx::stem_wgrad_ok((int)N, (int)H, (int)W, (int)C, (int)Ko);
}

int64_t stem_wgrad_ws_floats(int64_t Ko) { return tfx::stem_wgrad_ws_floats((int)Ko); }

// ws: a zeroed f32 workspace of stem_wgrad_ws_floats(Ko) (left zero)
void stem_wgrad(Tensor dy, Tensor x, Tensor dw, Tensor ws) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(dw); CHECK_CONTIG(dw);
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dy.size(0) == x.size(0) && dy.size(1) == x.size(1) &&
                  dy.size(2) == x.size(2), "stem_wgrad: NHWC x and dy of one image size");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), Ko = dy.size(3);
  TORCH_CHECK(tfx::stem_wgrad_ok((int)N, (int)H, (int)W, (int)C, (int)Ko) && dw.numel() == Ko * 9 * C,
              "stem_wgrad: unsupported shape");
  check_aligned16(x, "x"); check_aligned16(dy, "dy");
  CHECK_F32(ws); CHECK_CONTIG(ws);
  TORCH_CHECK(ws.numel() >= tfx::stem_wgrad_ws_floats((int)Ko), "stem_wgrad: workspace too small");
  tfx::stem_wgrad(bf(x), bf(dy), (int)N, (int)Ko, ws.data_ptr<float>(), dw.data_ptr<float>(), cur_stream());
}

void conv_wgrad(Tensor dy, Tensor x, Tensor dw, int64_t stride, int64_t pad, int64_t dil, bool accumulate) {
  conv_wgrad_impl(dy, x, dw, stride, pad, dil, accumulate, nullptr);
}

// conv_wgrad + the backward slot reduction of the BN that produced x (its partials left in `slots` by
// conv_dgrad_bn(reduce=False)), in ONE launch: the reduction runs as tail blocks of the weight-gradient
// grid (no separate bn_slot_reduce launch).  Returns red = [sum g' | sum g' xhat]; dgamma / dbeta +=.
Tensor conv_wgrad_sr(Tensor dy, Tensor x, Tensor dw, int64_t stride, int64_t pad, int64_t dil, bool accumulate,
                     Tensor slots, optional<Tensor> dgamma, optional<Tensor> dbeta) {
  CHECK_DEV(slots); CHECK_F32(slots); CHECK_CONTIG(slots);
  const int64_t C = x.size(-1);
  TORCH_CHECK(slots.numel() >= tfx::NSLOT * 2 * C, "conv_wgrad_sr: slot workspace too small");
  auto red = at::empty({2 * C}, slots.options());
  tfx::IgemmArgs sr;
  sr.sr_slots = slots.data_ptr<float>(); sr.sr_red = red.data_ptr<float>();
  sr.sr_dgamma = fpm(dgamma); sr.sr_dbeta = fpm(dbeta); sr.sr_C = (int)C;
  conv_wgrad_impl(dy, x, dw, stride, pad, dil, accumulate, &sr);
  return red;
}

// conv_wgrad with up to two pending BN-backward slot reductions in the tail (either may be absent:
// an undefined slots tensor).  Returns (red1, red2), empty where absent.
std::tuple<Tensor, Tensor> conv_wgrad_sr2(Tensor dy, Tensor x, Tensor dw, int64_t stride, int64_t pad, int64_t dil,
                                          bool accumulate, optional<Tensor> slots, optional<Tensor> dgamma,
                                          optional<Tensor> dbeta, optional<Tensor> slots2, int64_t C2,
                                          optional<Tensor> dgamma2, optional<Tensor> dbeta2) {
  tfx::IgemmArgs sr;
  auto opts = dy.options().dtype(at::kFloat);
  Tensor red1 = at::empty({0}, opts), red2 = at::empty({0}, opts);
  if (slots.has_value() && slots->defined()) {
    CHECK_DEV(*slots); CHECK_F32(*slots); CHECK_CONTIG(*slots);
    const int64_t C = x.size(-1);
    TORCH_CHECK(slots->numel() >= tfx::NSLOT * 2 * C, "conv_wgrad_sr2: slot workspace too small");
    red1 = at::empty({2 * C}, opts);
    sr.sr_slots = slots->data_ptr<float>(); sr.sr_red = red1.data_ptr<float>();
    sr.sr_dgamma = fpm(dgamma); sr.sr_dbeta = fpm(dbeta); sr.sr_C = (int)C;
  }
  if (slots2.has_value() && slots2->defined()) {
    CHECK_DEV(*slots2); CHECK_F32(*slots2); CHECK_CONTIG(*slots2);
    TORCH_CHECK(C2 > 0 && slots2->numel() >= tfx::NSLOT * 2 * C2, "conv_wgrad_sr2: second slot workspace");
    red2 = at::empty({2 * C2}, opts);
    sr.sr2_slots = slots2->data_ptr<float>(); sr.sr2_red = red2.data_ptr<float>();
    sr.sr2_dgamma = fpm(dgamma2); sr.sr2_dbeta = fpm(dbeta2); sr.sr2_C = (int)C2;
  }
  conv_wgrad_impl(dy, x, dw, stride, pad, dil, accumulate, &sr);
  return {red1, red2};
}

// the reduce half of a BN backward only (no residual): per-column partials [sum g' | sum g' xhat] of
// the output gradient g into the layer's zeroed slot workspace -- a later launch reduces the slots
// (conv_wgrad_sr2 tail blocks, or bn_slots_reduce)
void bn_bwd_reduce_into(Tensor g, Tensor x, Tensor save, bool relu, optional<Tensor> mask, Tensor slots) {
  CHECK_DEV(g); CHECK_BF16(g); CHECK_CONTIG(g); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(slots);
  TORCH_CHECK(g.sizes() == x.sizes(), "bn_bwd_reduce_into: grad shape");
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(slots.numel() >= tfx::NSLOT * 2 * C, "bn_bwd_reduce_into: slot workspace");
  const uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() * 8 == x.numel(), "relu mask size");
    mk = mask->data_ptr<uint8_t>();
  }
  tfx::bn_bwd_reduce(bf(g), bf(x), mk, false, save.data_ptr<float>(), M, C, relu, slots.data_ptr<float>(),
                     cur_stream());
}

// the slot reduction alone: red = [sum g' | sum g' xhat] from the slots (re-zeroed), dgamma/dbeta +=
Tensor bn_slots_reduce(Tensor slots, int64_t C, optional<Tensor> dgamma, optional<Tensor> dbeta) {
  CHECK_DEV(slots); CHECK_F32(slots); CHECK_CONTIG(slots);
  TORCH_CHECK(slots.numel() >= tfx::NSLOT * 2 * C, "bn_slots_reduce: slot workspace");
  auto red = at::empty({2 * C}, slots.options());
  tfx::bn_slot_reduce(slots.data_ptr<float>(), (int)C, red.data_ptr<float>(), fpm(dgamma), fpm(dbeta), cur_stream());
  return red;
}

// ------------------------------------------------------------------ fused pointwise-conv backward
// Backward of an expanding 1x1 conv (a ResNet bottleneck's conv3, w = [CW][1][1][CN], CW = 4 CN)
// fused with the tail BN's backward apply (pw_bwd.hip): g = the block's output gradient, y3 / mask3 /
// save3 / red3 = the tail BN's input, ReLU mask bits, [mean|invstd|scale|shift] and reduction
// [sum g'|sum g' xhat]; a2 = the conv's input.  dw += the weight gradient.  With y2 (the BN2 input that
// produced a2), its save2 / relu2 and slots2: the BN2 backward partials of dA2 are reduced too and
// returned as red2 = [sum g'|sum g' xhat] (dgamma2 / dbeta2 +=).  With ysc (a projection block: the
// residual was the shortcut BN's output, input ysc, stats save_sc, slots slots_sc) that BN's backward
// reduction rides along too: red_sc (dgamma_sc / dbeta_sc +=).  Returns (dA2, red2, red_sc).
std::tuple<Tensor, Tensor, Tensor> pw_bwd_expand(Tensor g, Tensor y3, Tensor mask3, Tensor save3, Tensor red3,
                                                 Tensor a2, Tensor w, Tensor dw, optional<Tensor> y2,
                                                 optional<Tensor> save2, bool relu2, optional<Tensor> slots2,
                                                 optional<Tensor> dgamma2, optional<Tensor> dbeta2,
                                                 optional<Tensor> ysc, optional<Tensor> save_sc,
                                                 optional<Tensor> slots_sc, optional<Tensor> dgamma_sc,
                                                 optional<Tensor> dbeta_sc, optional<Tensor> a2_save) {
  CHECK_DEV(g); CHECK_BF16(g); CHECK_CONTIG(g); CHECK_BF16(y3); CHECK_CONTIG(y3); CHECK_BF16(a2); CHECK_CONTIG(a2);
  CHECK_BF16(w); CHECK_CONTIG(w); CHECK_F32(dw); CHECK_CONTIG(dw); CHECK_F32(save3); CHECK_F32(red3);
  const int64_t CW = w.size(0), CN = w.size(-1), M = a2.numel() / CN;
  TORCH_CHECK(w.numel() == CW * CN && CW == 4 * CN && dw.numel() == CW * CN, "pw_bwd_expand: weight shape");
  TORCH_CHECK(a2.size(-1) == CN && g.numel() == M * CW && y3.numel() == M * CW && g.size(-1) == CW, "pw_bwd_expand: shapes");
  TORCH_CHECK(mask3.scalar_type() == at::kByte && mask3.numel() * 8 == M * CW && mask3.is_contiguous(), "mask3");
  TORCH_CHECK(save3.numel() == 4 * CW && red3.numel() == 2 * CW, "save3 / red3");
  TORCH_CHECK(tfx::pw_bwd_expand_ok((int)CN, M), "pw_bwd_expand: unsupported width / rows");
  auto dA2 = at::empty_like(a2);
  tfx::PwExpandArgs a;
  a.g = bf(g); a.y3 = bf(y3); a.mask3 = mask3.data_ptr<uint8_t>(); a.save3 = save3.data_ptr<float>();
  a.red3 = red3.data_ptr<float>(); a.a2 = bf(a2); a.w = bf(w); a.dA2 = bfm(dA2); a.M = (int)M; a.CN = (int)CN;
  if (a2_save.has_value() && a2_save->defined()) {  // a2 = BN2's input: conv3's input formed on load
    CHECK_F32(*a2_save); CHECK_CONTIG(*a2_save);
    TORCH_CHECK(a2_save->numel() == 4 * CN, "pw_bwd_expand: a2_save = BN2's [4][CN] save");
    a.a2_save = a2_save->data_ptr<float>();
  }
  Tensor red2 = at::empty({0}, g.options().dtype(at::kFloat));
  const bool bnb = y2.has_value() && y2->defined();
  if (bnb) {
    CHECK_BF16(*y2); CHECK_CONTIG(*y2);
    TORCH_CHECK(y2->numel() == M * CN && save2.has_value() && save2->numel() == 4 * CN && slots2.has_value(),
                "pw_bwd_expand: BN2 arguments");
    check_bn_ws(*slots2, CN);
    a.y2 = bf(*y2); a.save2 = save2->data_ptr<float>(); a.relu2 = relu2 ? 1 : 0; a.slots2 = slots2->data_ptr<float>();
    red2 = at::empty({2 * CN}, g.options().dtype(at::kFloat));
  }
  Tensor red_sc = at::empty({0}, g.options().dtype(at::kFloat));
  tfx::PwSecReduce sec;
  if (ysc.has_value() && ysc->defined()) {
    CHECK_BF16(*ysc); CHECK_CONTIG(*ysc);
    TORCH_CHECK(ysc->numel() == M * CW && save_sc.has_value() && save_sc->numel() == 4 * CW && slots_sc.has_value(),
                "pw_bwd_expand: shortcut BN arguments");
    check_bn_ws(*slots_sc, CW);
    a.ysc = bf(*ysc); a.slots_sc = slots_sc->data_ptr<float>();
    red_sc = at::empty({2 * CW}, g.options().dtype(at::kFloat));
    sec.slots = a.slots_sc; sec.red3 = a.red3; sec.save = save_sc->data_ptr<float>(); sec.red = red_sc.data_ptr<float>();
    sec.dgamma = fpm(dgamma_sc); sec.dbeta = fpm(dbeta_sc); sec.C = (int)CW;
  }
  const int nb = tfx::pw_bwd_expand_grid((int)CN, M);
  auto slab = at::empty({(int64_t)nb * CW * CN}, g.options().dtype(at::kFloat));
  a.slab = slab.data_ptr<float>();
  tfx::pw_bwd_expand(a, nb, cur_stream());
  tfx::pw_slab_reduce(a.slab, nb, (int)CN, dw.data_ptr<float>(), bnb ? a.slots2 : nullptr, (int)CN,
                      bnb ? red2.data_ptr<float>() : nullptr, bnb ? fpm(dgamma2) : nullptr,
                      bnb ? fpm(dbeta2) : nullptr, sec, cur_stream());
  return {dA2, red2, red_sc};
}

bool pw_bwd_expand_supported(int64_t CN, int64_t M) { return tfx::pw_bwd_expand_ok((int)CN, M); }

// Backward of an identity bottleneck's squeezing 1x1 conv1 (w = [CO][1][1][CI]) fused with BN1's backward
// apply (pw_bwd.hip F1): g1 / y1 / save1 / red1 = BN1's output gradient, input, stats and reduction;
// x = conv1's input; addend / amask = the residual branch's parked gradient and ReLU mask bits;
// px / psave / pmask / pslots = the previous tail BN (input, stats, mask bits, slot workspace) whose
// backward partials the dx epilogue reduces.  dw += dW1.  Returns (dx, pred = [sum g'|sum g' xhat]) with
// pdgamma / pdbeta +=.
std::tuple<Tensor, Tensor> pw_bwd_squeeze(Tensor g1, Tensor y1, Tensor save1, Tensor red1, Tensor x, Tensor w,
                                          Tensor dw, Tensor addend, Tensor amask, Tensor px, Tensor psave,
                                          Tensor pmask, Tensor pslots, optional<Tensor> pdgamma,
                                          optional<Tensor> pdbeta) {
  CHECK_DEV(g1); CHECK_BF16(g1); CHECK_CONTIG(g1); CHECK_BF16(y1); CHECK_CONTIG(y1); CHECK_BF16(x); CHECK_CONTIG(x);
  CHECK_BF16(w); CHECK_CONTIG(w); CHECK_F32(dw); CHECK_CONTIG(dw); CHECK_BF16(addend); CHECK_CONTIG(addend);
  CHECK_BF16(px); CHECK_CONTIG(px); CHECK_F32(save1); CHECK_F32(red1); CHECK_F32(psave);
  const int64_t CO = w.size(0), CI = w.size(-1), M = x.numel() / CI;
  TORCH_CHECK(w.numel() == CO * CI && dw.numel() == CO * CI && x.size(-1) == CI, "pw_bwd_squeeze: weight shape");
  TORCH_CHECK(g1.numel() == M * CO && y1.numel() == M * CO && addend.numel() == M * CI && px.numel() == M * CI,
              "pw_bwd_squeeze: shapes");
  TORCH_CHECK(save1.numel() == 4 * CO && red1.numel() == 2 * CO && psave.numel() == 4 * CI, "pw_bwd_squeeze: stats");
  for (const Tensor* m : {&amask, &pmask})
    TORCH_CHECK(m->scalar_type() == at::kByte && m->is_contiguous() && m->numel() * 8 == M * CI, "pw_bwd_squeeze: mask");
  TORCH_CHECK(tfx::pw_bwd_squeeze_ok((int)CI, (int)CO, M), "pw_bwd_squeeze: unsupported widths / rows");
  check_bn_ws(pslots, CI);
  auto dx = at::empty_like(x);
  auto pred = at::empty({2 * CI}, x.options().dtype(at::kFloat));
  tfx::PwSqueezeBwdArgs a;
  a.g1 = bf(g1); a.y1 = bf(y1); a.save1 = save1.data_ptr<float>(); a.red1 = red1.data_ptr<float>(); a.x = bf(x);
  a.w = bf(w); a.addend = bf(addend); a.amask = amask.data_ptr<uint8_t>(); a.px = bf(px);
  a.psave = psave.data_ptr<float>(); a.pmask = pmask.data_ptr<uint8_t>(); a.pslots = pslots.data_ptr<float>();
  a.dx = bfm(dx); a.M = (int)M; a.CI = (int)CI; a.CO = (int)CO;
  const int nb = tfx::pw_bwd_squeeze_grid((int)CI, (int)CO, M);
  auto slab = at::empty({tfx::pw_bwd_squeeze_slab_floats((int)CI, (int)CO, nb)}, x.options().dtype(at::kFloat));
  a.slab = slab.data_ptr<float>();
  tfx::pw_bwd_squeeze(a, nb, cur_stream());
  tfx::pw_slab_reduce(a.slab, nb, (int)CO, dw.data_ptr<float>(), a.pslots, (int)CI, pred.data_ptr<float>(),
                      fpm(pdgamma), fpm(pdbeta), tfx::PwSecReduce{}, cur_stream(), 1);
  return {dx, pred};
}

bool pw_bwd_squeeze_supported(int64_t CI, int64_t CO, int64_t M) { return tfx::pw_bwd_squeeze_ok((int)CI, (int)CO, M); }

// ------------------------------------------------------------------ dense bf16 GEMM
// out = op(a) @ op(b) (+bias)(relu); a: [M,K] (or [K,M] if trans_a); b: [K,N] (or [N,K] if trans_b)
void gemm_setup(tfx::IgemmArgs& g, const Tensor& a, const Tensor& b, bool ta, bool tb) {
  CHECK_DEV(a); CHECK_BF16(a); CHECK_BF16(b);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm expects 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "gemm operands need unit inner stride");
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t K2 = tb ? b.size(1) : b.size(0), N = tb ? b.size(0) : b.size(1);
  TORCH_CHECK(K == K2, "gemm inner dims differ: ", K, " vs ", K2);
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm leading dims must be multiples of 8");
  TORCH_CHECK((ta ? M : K) % 8 == 0 && (tb ? K : N) % 8 == 0, "gemm contiguous dims must be multiples of 8");
  check_aligned16(a, "a");
  check_aligned16(b, "b");
  g.A = bf(a); g.B = bf(b);
  // buffer-resource extents: from the view's start to the end of its storage
  g.a_bytes = (a.storage().nbytes() - a.storage_offset() * a.element_size());
  g.b_bytes = (b.storage().nbytes() - b.storage_offset() * b.element_size());
  g.M = M; g.N = N; g.K = K;
  g.lda = a.stride(0); g.ldb = b.stride(0);
  g.a_kmajor = ta ? 0 : 1;
  g.b_kmajor = tb ? 1 : 0;
}

Tensor gemm(Tensor a, Tensor b, bool ta, bool tb, optional<Tensor> bias, bool relu, bool out_f32) {
  tfx::IgemmArgs g;
  gemm_setup(g, a, b, ta, tb);
  auto out = at::empty({g.M, g.N}, a.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  g.Cp = out.data_ptr(); g.ldc = g.N; g.bias = fp(bias); g.relu = relu;
  g.out_mode = out_f32 ? tfx::OUT_F32 : tfx::OUT_BF16;
  if (bias.has_value() && bias->defined()) { CHECK_F32(*bias); TORCH_CHECK(bias->numel() == g.N, "bias size"); }
  tfx::igemm_launch(g, tfx::MODE_GEMM, cur_stream());
  return out;
}

// f32 out (+)= op(a) @ op(b); split-K with atomics when the grid would be small
void gemm_into(Tensor a, Tensor b, bool ta, bool tb, Tensor out, bool accumulate) {
  tfx::IgemmArgs g;
  gemm_setup(g, a, b, ta, tb);
  CHECK_F32(out);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == g.M && out.size(1) == g.N && out.stride(1) == 1, "out shape");
  g.Cp = out.data_ptr(); g.ldc = out.stride(0);
  g.out_mode = tfx::OUT_F32_ATOMIC;
  g.zero_out = accumulate ? 0 : 1;
  if (!accumulate && out.stride(0) != g.N) {  // zeroing assumes a dense block
    out.zero_();
    g.zero_out = 0;
  }
  tfx::igemm_launch(g, tfx::MODE_GEMM, cur_stream());
}

// ------------------------------------------------------------------ f32 GEMM (MFMA f32)
Tensor sgemm(Tensor a, Tensor b, bool ta, bool tb, optional<Tensor> bias, int64_t act, bool split) {
  CHECK_DEV(a); CHECK_F32(a); CHECK_F32(b);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1, "sgemm operands");
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t N = tb ? b.size(0) : b.size(1);
  TORCH_CHECK((tb ? b.size(1) : b.size(0)) == K, "sgemm inner dims");
  auto out = at::empty({M, N}, a.options());
  tfx::sgemm_launch(a.data_ptr<float>(), b.data_ptr<float>(), out.data_ptr<float>(), fp(bias), M, N, K,
                    a.stride(0), b.stride(0), N, ta, tb, act, false, cur_stream(), split);
  return out;
}

void sgemm_into(Tensor a, Tensor b, bool ta, bool tb, Tensor out, bool accumulate, bool split) {
  CHECK_DEV(a); CHECK_F32(a); CHECK_F32(b); CHECK_F32(out);
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t N = tb ? b.size(0) : b.size(1);
  TORCH_CHECK(out.size(0) == M && out.size(1) == N && out.stride(1) == 1, "sgemm_into out shape");
  tfx::sgemm_launch(a.data_ptr<float>(), b.data_ptr<float>(), out.data_ptr<float>(), nullptr, M, N, K,
                    a.stride(0), b.stride(0), out.stride(0), ta, tb, 0, accumulate, cur_stream(), split);
}

// ------------------------------------------------------------------ batch norm
// slots: the layer's persistent [NSLOT][2][C] workspace; have_stats = the producer (conv epilogue)
// already accumulated this batch's statistics into it.
// returns (y, save, mask): mask = 1-bit ReLU mask of y (uint8 per 8 channels) for residual + ReLU
// layers on the vector path (what the backward reads instead of the residual), else undefined.
std::tuple<Tensor, Tensor, Tensor> bn_fwd_train(Tensor x, optional<Tensor> gamma, optional<Tensor> beta,
                                                optional<Tensor> run_mean, optional<Tensor> run_var, double momentum,
                                                double eps, optional<Tensor> res, bool relu, Tensor slots,
                                                bool have_stats) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(slots.numel() >= tfx::NSLOT * 2 * C && slots.scalar_type() == at::kFloat, "stat slots");
  auto save = at::empty({4 * C}, x.options().dtype(at::kFloat));
  auto y = at::empty_like(x);
  const uint16_t* r = nullptr;
  if (res.has_value() && res->defined()) {
    CHECK_BF16(*res); CHECK_CONTIG(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
    r = bf(*res);
  }
  auto s = cur_stream();
  float* sl = slots.data_ptr<float>();
  if (tfx::det_mode()) tfx::bn_stats_det(bf(x), M, (int)C, sl, s);
  else if (!have_stats) tfx::bn_stats(bf(x), M, C, sl, s);
  tfx::bn_finalize(sl, M, C, fp(gamma), fp(beta), eps, momentum, fpm(run_mean), fpm(run_var),
                   save.data_ptr<float>(), s);
  Tensor mask;
  if (r && relu && C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0)
    mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  tfx::bn_apply(bf(x), r, save.data_ptr<float>(), M, C, relu, bfm(y),
                mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, s);
  return {y, save, mask};
}

// forward apply only, with save from conv_fwd_bn: returns (y, mask) (mask as in bn_fwd_train)
std::tuple<Tensor, Tensor> bn_apply_train(Tensor x, optional<Tensor> res, Tensor save, bool relu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(save);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(save.numel() == 4 * C, "save size");
  auto y = at::empty_like(x);
  const uint16_t* r = nullptr;
  if (res.has_value() && res->defined()) {
    CHECK_BF16(*res); CHECK_CONTIG(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
    r = bf(*res);
  }
  Tensor mask;
  if (r && relu && C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0)
    mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  tfx::bn_apply(bf(x), r, save.data_ptr<float>(), M, C, relu, bfm(y),
                mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {y, mask};
}

// flipped 3x3 filter copies for the flipped-weight data gradient (wflip.hip): src / dst = flat bf16
// buffers, desc = [nlayers][5] int64 {src_off, dst_off, Ko, C, first_tile}, ntiles = total tiles
void wflip3x3(Tensor src, Tensor dst, Tensor desc, int64_t ntiles) {
  CHECK_DEV(src); CHECK_BF16(src); CHECK_BF16(dst); CHECK_CONTIG(src); CHECK_CONTIG(dst); CHECK_DEV(desc);
  TORCH_CHECK(desc.scalar_type() == at::kLong && desc.dim() == 2 && desc.size(1) == 5 && desc.is_contiguous(),
              "wflip3x3 desc");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(src.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(dst.data_ptr()) & 15) == 0, "wflip3x3: 16-byte aligned buffers");
  tfx::wflip3x3(bf(src), bfm(dst), desc.data_ptr<int64_t>(), (int)desc.size(0), (int)ntiles, cur_stream());
}

// bn_apply_train whose residual is a BN that was never applied: y = act(bn(x) + bn'(res_x)), with
// res_save = that BN's [mean|invstd|scale|shift] (ResNet projection shortcut, ops/nn.py defer).
std::tuple<Tensor, Tensor> bn_apply_res_bn(Tensor x, Tensor res_x, Tensor save, Tensor res_save, bool relu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(save); CHECK_BF16(res_x); CHECK_CONTIG(res_x);
  CHECK_F32(res_save);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(save.numel() == 4 * C && res_save.numel() == 4 * C, "save size");
  TORCH_CHECK(res_x.sizes() == x.sizes(), "residual shape");
  TORCH_CHECK(tfx::bn_backward_apply_sec_ok((int)C), "bn_apply_res_bn: channel count needs the vector path");
  auto y = at::empty_like(x);
  Tensor mask;
  if (relu) mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  tfx::bn_apply_res_bn(bf(x), bf(res_x), save.data_ptr<float>(), res_save.data_ptr<float>(), M, (int)C, relu,
                       bfm(y), relu ? mask.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {y, mask};
}

std::tuple<Tensor, Tensor> bn_fwd_eval(Tensor x, optional<Tensor> gamma, optional<Tensor> beta, Tensor run_mean,
                                       Tensor run_var, double eps, optional<Tensor> res, bool relu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = x.numel() / C;
  auto save = at::empty({4 * C}, x.options().dtype(at::kFloat));
  auto y = at::empty_like(x);
  auto s = cur_stream();
  tfx::bn_eval_prep(C, fp(gamma), fp(beta), eps, run_mean.data_ptr<float>(), run_var.data_ptr<float>(),
                    save.data_ptr<float>(), s);
  const uint16_t* r = (res.has_value() && res->defined()) ? bf(*res) : nullptr;
  tfx::bn_apply(bf(x), r, save.data_ptr<float>(), M, C, relu, bfm(y), nullptr, s);
  return {y, save};
}

// returns dx, dres (undefined unless res given), red = [dbeta(C) | dgamma(C)]; when dgamma/dbeta
// are given the parameter gradients are accumulated in place by the reduce kernel.
// residual layers: pass the forward's ``mask`` (vector path; then ``res`` may be omitted) or ``res``.
// want_dres = false: no dres tensor is written (the residual's consumer reads g and the mask bits
// itself: conv_dgrad(..., addend=g, addend_mask=mask))
std::tuple<Tensor, Tensor, Tensor> bn_bwd(Tensor g, Tensor x, optional<Tensor> res, Tensor save, bool relu,
                                          Tensor slots, optional<Tensor> dgamma, optional<Tensor> dbeta,
                                          optional<Tensor> mask, bool want_dres) {
  CHECK_DEV(g); CHECK_BF16(g); CHECK_CONTIG(g); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(g.sizes() == x.sizes(), "bn_bwd grad shape");
  TORCH_CHECK(slots.numel() >= tfx::NSLOT * 2 * C && slots.scalar_type() == at::kFloat, "stat slots");
  auto red = at::empty({2 * C}, x.options().dtype(at::kFloat));
  auto dx = at::empty_like(x);
  Tensor dres;
  const uint16_t* r = nullptr;
  const uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() * 8 == x.numel(), "relu mask size");
    mk = mask->data_ptr<uint8_t>();
  }
  if (res.has_value() && res->defined()) {
    CHECK_CONTIG(*res);
    r = bf(*res);
  }
  if ((r || mk) && want_dres) dres = at::empty_like(x);
  tfx::bn_backward(bf(g), bf(x), r, mk, save.data_ptr<float>(), M, C, relu, slots.data_ptr<float>(),
                   red.data_ptr<float>(), fpm(dgamma), fpm(dbeta), bfm(dx), dres.defined() ? bfm(dres) : nullptr,
                   cur_stream());
  return {dx, dres, red};
}

// bn_bwd_apply for a residual layer whose residual is another BN's output used only here (ResNet
// projection shortcut): dres is written as usual AND that BN's backward is reduced in the same pass
// (x2 = its input, save2 = its [mean|invstd|scale|shift], slots2 = its zeroed slot workspace).
// Returns (dx, dres, red2); dgamma2 / dbeta2 (optional) accumulate its parameter gradients.
// want_dres = false: dres is not written -- that BN's apply then reads g and the mask bits itself
// (bn_bwd_apply(g, x2, None, save2, red2, relu=True, mask): g' = g * mask is exactly its gradient).
std::tuple<Tensor, Tensor, Tensor> bn_bwd_apply_sec(Tensor g, Tensor x, Tensor save, Tensor red, bool relu,
                                                    optional<Tensor> mask, Tensor x2, Tensor save2, Tensor slots2,
                                                    optional<Tensor> dgamma2, optional<Tensor> dbeta2,
                                                    bool want_dres, bool reduce2) {
  CHECK_DEV(g); CHECK_BF16(g); CHECK_CONTIG(g); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(red);
  CHECK_BF16(x2); CHECK_CONTIG(x2); CHECK_F32(save2); CHECK_F32(slots2);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(g.sizes() == x.sizes() && x2.sizes() == x.sizes(), "bn_bwd_apply_sec shapes");
  TORCH_CHECK(tfx::bn_backward_apply_sec_ok((int)C), "bn_bwd_apply_sec: channel count needs the vector path");
  TORCH_CHECK(red.numel() == 2 * C && save.numel() == 4 * C && save2.numel() == 4 * C, "red / save size");
  TORCH_CHECK(slots2.numel() >= tfx::NSLOT * 2 * C, "stat slots");
  const uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() * 8 == x.numel(), "relu mask size");
    mk = mask->data_ptr<uint8_t>();
  }
  TORCH_CHECK(!relu || mk, "bn_bwd_apply_sec: a residual ReLU needs the forward mask bits");
  auto dx = at::empty_like(x);
  Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  // reduce2 = false: the residual BN's partials stay in slots2 for a later launch to reduce
  // (conv_wgrad_sr2 tail blocks / bn_slots_reduce); red2 is then empty
  auto red2 = at::empty({reduce2 ? 2 * C : 0}, x.options().dtype(at::kFloat));
  tfx::bn_backward_apply_sec(bf(g), bf(x), mk, save.data_ptr<float>(), red.data_ptr<float>(), M, (int)C, relu,
                             bfm(dx), want_dres ? bfm(dres) : nullptr, bf(x2), save2.data_ptr<float>(), slots2.data_ptr<float>(),
                             cur_stream());
  if (reduce2)
    tfx::bn_slot_reduce(slots2.data_ptr<float>(), (int)C, red2.data_ptr<float>(), fpm(dgamma2), fpm(dbeta2),
                        cur_stream());
  return {dx, dres, red2};
}

// backward apply only, with red from conv_dgrad_bn: returns (dx, dres)
std::tuple<Tensor, Tensor> bn_bwd_apply(Tensor g, Tensor x, optional<Tensor> res, Tensor save, Tensor red,
                                        bool relu, optional<Tensor> mask, bool want_dres) {
  CHECK_DEV(g); CHECK_BF16(g); CHECK_CONTIG(g); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(red);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(g.sizes() == x.sizes(), "bn_bwd_apply grad shape");
  TORCH_CHECK(red.numel() == 2 * C && save.numel() == 4 * C, "red / save size");
  auto dx = at::empty_like(x);
  Tensor dres;
  const uint16_t* r = nullptr;
  const uint8_t* mk = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() * 8 == x.numel(), "relu mask size");
    mk = mask->data_ptr<uint8_t>();
  }
  if (res.has_value() && res->defined()) {
    CHECK_CONTIG(*res);
    r = bf(*res);
  }
  if ((r || mk) && want_dres) dres = at::empty_like(x);
  tfx::bn_backward_apply(bf(g), bf(x), r, mk, save.data_ptr<float>(), red.data_ptr<float>(), M, C, relu, bfm(dx),
                         dres.defined() ? bfm(dres) : nullptr, cur_stream());
  return {dx, dres};
}

int64_t bn_nslot() { return tfx::NSLOT; }

// ------------------------------------------------------------------ loss / metrics / pooling
std::tuple<Tensor, Tensor> softmax_xent(Tensor z, optional<Tensor> lab_idx, optional<Tensor> lab_dense, bool naive,
                                        double gscale, bool want_grad) {
  CHECK_DEV(z); CHECK_CONTIG(z);
  TORCH_CHECK(z.dim() == 2, "logits must be [B,C]");
  const bool zb = z.scalar_type() == at::kBFloat16;
  TORCH_CHECK(zb || z.scalar_type() == at::kFloat, "logits dtype");
  const int64_t B = z.size(0), C = z.size(1);
  const int64_t* li = nullptr;
  const float* ld = nullptr;
  if (lab_idx.has_value() && lab_idx->defined()) {
    TORCH_CHECK(lab_idx->scalar_type() == at::kLong && lab_idx->numel() == B, "labels");
    li = lab_idx->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(lab_dense.has_value() && lab_dense->defined(), "need labels");
    CHECK_F32(*lab_dense); CHECK_CONTIG(*lab_dense);
    TORCH_CHECK(lab_dense->size(0) == B && lab_dense->size(1) == C, "dense labels shape");
    ld = lab_dense->data_ptr<float>();
  }
  auto opts = z.options().dtype(at::kFloat);
  auto loss = at::empty({B}, opts);
  Tensor dz;
  if (want_grad) dz = at::empty({B, C}, opts);
  tfx::softmax_xent(z.data_ptr(), zb, B, C, li, ld, naive, gscale, loss.data_ptr<float>(),
                    want_grad ? dz.data_ptr<float>() : nullptr, nullptr, cur_stream());
  return {loss, dz};
}

// Batch-mean loss (0-dim f32) and dz = d(mean)/dz in one single-block launch, dz in the logits'
// dtype when dz_native (bf16 logits get a bf16 gradient: no scale/cast launch in backward).
std::tuple<Tensor, Tensor> softmax_xent_mean(Tensor z, optional<Tensor> lab_idx, optional<Tensor> lab_dense,
                                             bool naive, bool want_grad, bool dz_native) {
  CHECK_DEV(z); CHECK_CONTIG(z);
  TORCH_CHECK(z.dim() == 2, "logits must be [B,C]");
  const bool zb = z.scalar_type() == at::kBFloat16;
  TORCH_CHECK(zb || z.scalar_type() == at::kFloat, "logits dtype");
  const int64_t B = z.size(0), C = z.size(1);
  TORCH_CHECK(B >= 1 && B * ((C + 63) / 64) <= 1024, "softmax_xent_mean: batch too large for one block");
  const int64_t* li = nullptr;
  const float* ld = nullptr;
  if (lab_idx.has_value() && lab_idx->defined()) {
    CHECK_DEV(*lab_idx);
    TORCH_CHECK(lab_idx->scalar_type() == at::kLong && lab_idx->numel() == B && lab_idx->is_contiguous(), "labels");
    li = lab_idx->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(lab_dense.has_value() && lab_dense->defined(), "need labels");
    CHECK_F32(*lab_dense); CHECK_CONTIG(*lab_dense);
    TORCH_CHECK(lab_dense->size(0) == B && lab_dense->size(1) == C, "dense labels shape");
    ld = lab_dense->data_ptr<float>();
  }
  auto loss = at::empty({}, z.options().dtype(at::kFloat));
  const bool db = dz_native && zb;
  Tensor dz;
  if (want_grad) dz = at::empty({B, C}, z.options().dtype(db ? at::kBFloat16 : at::kFloat));
  tfx::softmax_xent_mean(z.data_ptr(), zb, (int)B, (int)C, li, ld, naive, 1.0f / (float)B, loss.data_ptr<float>(),
                         want_grad ? dz.data_ptr() : nullptr, db, cur_stream());
  return {loss, dz};
}

// Fused classifier head (head.hip): returns (mean loss, dfeat [N,H,W,C], feat [N,C], dz [N,O]); the
// input gradient is for a unit seed (the caller's promise), feat / dz feed linear_small_bwd's dW / db.
// state: int64 [3] zeros, owned by the caller across launches (the kernel leaves it zero).
bool head_xent_supported(int64_t C, int64_t O, int64_t HW) { return tfx::head_xent_ok((int)C, (int)O, (int)HW); }

// the fused head's tail-BN backward rows [N][2C] -> red [2C]; dbeta += red[:C], dgamma += red[C:]
Tensor head_rows_reduce(Tensor rows, int64_t C, optional<Tensor> dgamma, optional<Tensor> dbeta) {
  CHECK_DEV(rows); CHECK_F32(rows); CHECK_CONTIG(rows);
  TORCH_CHECK(C > 0 && rows.numel() % (2 * C) == 0, "head_rows_reduce: rows [N][2C]");
  for (const auto* o : {&dgamma, &dbeta})
    if (o->has_value() && (*o)->defined()) {
      CHECK_F32(**o); TORCH_CHECK((*o)->numel() == C && (*o)->is_contiguous(), "head_rows_reduce: dgamma/dbeta [C]");
    }
  auto red = at::empty({2 * C}, rows.options());
  tfx::head_rows_reduce(rows.data_ptr<float>(), (int)(rows.numel() / (2 * C)), (int)C, red.data_ptr<float>(),
                        fpm(dgamma), fpm(dbeta), cur_stream());
  return red;
}

std::tuple<Tensor, Tensor, Tensor, Tensor> head_xent(Tensor x, Tensor w, optional<Tensor> b, Tensor labels,
                                                     Tensor state, optional<Tensor> y3, optional<Tensor> res,
                                                     optional<Tensor> save3, optional<Tensor> mask,
                                                     optional<Tensor> bn_rows) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 4, "head_xent expects NHWC features");
  const int64_t N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3), O = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == C, "head_xent: W [O, C]");
  TORCH_CHECK(tfx::head_xent_ok((int)C, (int)O, (int)HW) && N >= 1 && N <= 4095 && N * HW * C < (int64_t(1) << 31),
              "head_xent: unsupported shape");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.numel() == N && labels.is_contiguous(),
              "head_xent: int64 labels [N]");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kLong && state.numel() >= 3 && state.is_contiguous(),
              "head_xent: int64 state [3]");
  if (b.has_value() && b->defined()) { CHECK_F32(*b); TORCH_CHECK(b->numel() == O, "head_xent bias"); }
  check_aligned16(x, "x"); check_aligned16(w, "w");
  auto loss = at::empty({}, x.options().dtype(at::kFloat));
  auto dfeat = at::empty_like(x);
  auto feat = at::empty({N, C}, x.options());
  auto dz = at::empty({N, O}, x.options());
  tfx::HeadXentArgs a;
  a.x = bf(x); a.w = bf(w); a.b = fp(b); a.labels = labels.data_ptr<int64_t>();
  a.feat = bfm(feat); a.dz = bfm(dz); a.dfeat = bfm(dfeat); a.loss = loss.data_ptr<float>();
  a.state = reinterpret_cast<unsigned long long*>(state.data_ptr<int64_t>());
  a.C = (int)C; a.HW = (int)HW; a.O = (int)O; a.gscale = 1.0f / (float)N;
  if (y3.has_value() && y3->defined()) {
    // tail mode: x (the unwritten tail output) only gives the shape
    TORCH_CHECK(res.has_value() && save3.has_value() && mask.has_value() && bn_rows.has_value(),
                "head_xent tail mode: y3, res, save3, mask, bn_rows");
    for (const Tensor* tt : {&*y3, &*res}) {
      CHECK_BF16(*tt); CHECK_CONTIG(*tt);
      TORCH_CHECK(tt->sizes() == x.sizes(), "head_xent tail: y3 / res shape");
      check_aligned16(*tt, "tail operand");
    }
    CHECK_F32(*save3); TORCH_CHECK(save3->numel() == 4 * C, "head_xent tail: save3");
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->is_contiguous() && mask->numel() * 8 == x.numel(),
                "head_xent tail: mask");
    CHECK_F32(*bn_rows); CHECK_CONTIG(*bn_rows);
    TORCH_CHECK(bn_rows->numel() == N * 2 * C, "head_xent tail: bn rows [N][2][C]");
    a.y3 = bf(*y3); a.res = bf(*res); a.save3 = save3->data_ptr<float>(); a.mask = mask->data_ptr<uint8_t>();
    a.bn_rows = bn_rows->data_ptr<float>();
  }
  tfx::head_xent_fwd(a, (int)N, cur_stream());
  return {loss, dfeat, feat, dz};
}

// the fused head's parameter gradients: dw [O, C] += dz^T feat, db [O] += colsum(dz) (f32, in place)
void head_wgrad(Tensor dz, Tensor feat, optional<Tensor> dw, optional<Tensor> db) {
  CHECK_DEV(dz); CHECK_BF16(dz); CHECK_CONTIG(dz); CHECK_BF16(feat); CHECK_CONTIG(feat);
  const int64_t N = dz.size(0), O = dz.size(1), C = feat.size(1);
  TORCH_CHECK(feat.size(0) == N && C % 8 == 0 && O >= 1 && O <= 16, "head_wgrad shapes");
  if (dw.has_value() && dw->defined()) { CHECK_F32(*dw); TORCH_CHECK(dw->numel() == O * C && dw->is_contiguous(), "dw"); }
  if (db.has_value() && db->defined()) { CHECK_F32(*db); TORCH_CHECK(db->numel() == O && db->is_contiguous(), "db"); }
  check_aligned16(feat, "feat");
  tfx::head_wgrad(bf(dz), bf(feat), (int)N, (int)C, (int)O, fpm(dw), fpm(db), cur_stream());
}

Tensor accuracy_count(Tensor z, optional<Tensor> lab_idx, optional<Tensor> lab_dense) {
  CHECK_DEV(z); CHECK_CONTIG(z);
  const bool zb = z.scalar_type() == at::kBFloat16;
  auto out = at::empty({1}, z.options().dtype(at::kFloat));
  const int64_t* li = (lab_idx.has_value() && lab_idx->defined()) ? lab_idx->data_ptr<int64_t>() : nullptr;
  const float* ld = (lab_dense.has_value() && lab_dense->defined()) ? lab_dense->data_ptr<float>() : nullptr;
  TORCH_CHECK(li || ld, "need labels");
  tfx::accuracy_count(z.data_ptr(), zb, z.size(0), z.size(1), li, ld, out.data_ptr<float>(), cur_stream());
  return out;
}

Tensor gap_fwd(Tensor x, bool out_f32) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4, "gap expects NHWC");
  const int64_t N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto y = at::empty({N, C}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  tfx::gap_fwd(bf(x), N, HW, C, out_f32 ? nullptr : bfm(y), out_f32 ? y.data_ptr<float>() : nullptr, cur_stream());
  return y;
}

Tensor gap_bwd(Tensor dy, int64_t H, int64_t W) {
  CHECK_DEV(dy); CHECK_CONTIG(dy);
  const bool b16 = dy.scalar_type() == at::kBFloat16;
  const int64_t N = dy.size(0), C = dy.size(1);
  auto dx = at::empty({N, H, W, C}, dy.options().dtype(at::kBFloat16));
  tfx::gap_bwd(dy.data_ptr(), b16, N, H * W, C, bfm(dx), cur_stream());
  return dx;
}

// ------------------------------------------------------------------ small fused elementwise ops
Tensor affine_fwd(Tensor x, Tensor w, optional<Tensor> b) {
  CHECK_DEV(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_F32(w); CHECK_CONTIG(w);
  const int64_t C = w.numel();
  TORCH_CHECK(C >= 1 && C <= 256 && x.numel() % C == 0 && (x.dim() == 0 ? C == 1 : x.size(-1) == C || C == 1),
              "affine: w broadcasts over the last dim (<= 256 channels)");
  if (b.has_value() && b->defined()) TORCH_CHECK(b->numel() == C && b->scalar_type() == at::kFloat, "affine bias");
  auto y = at::empty_like(x);
  tfx::affine_fwd(x.data_ptr<float>(), w.data_ptr<float>(), fp(b), x.numel(), (int)C, y.data_ptr<float>(),
                  cur_stream());
  return y;
}

// returns dx (if want_dx); dw / db accumulated in place
Tensor affine_bwd(Tensor g, Tensor x, Tensor w, optional<Tensor> dw, optional<Tensor> db, bool want_dx) {
  CHECK_DEV(g); CHECK_F32(g); CHECK_CONTIG(g); CHECK_F32(x); CHECK_CONTIG(x);
  TORCH_CHECK(g.numel() == x.numel(), "affine_bwd sizes");
  const int64_t C = w.numel();
  Tensor dx;
  if (want_dx) dx = at::empty_like(x);
  tfx::affine_bwd(g.data_ptr<float>(), x.data_ptr<float>(), w.data_ptr<float>(), x.numel(), (int)C,
                  want_dx ? dx.data_ptr<float>() : nullptr, fpm(dw), fpm(db), cur_stream());
  return dx;
}

Tensor sse_fwd(Tensor p, Tensor y) {
  CHECK_DEV(p); CHECK_F32(p); CHECK_CONTIG(p); CHECK_F32(y); CHECK_CONTIG(y);
  TORCH_CHECK(p.numel() == y.numel(), "sse sizes");
  auto loss = at::empty({}, p.options());
  tfx::sse_fwd(p.data_ptr<float>(), y.data_ptr<float>(), p.numel(), loss.data_ptr<float>(), cur_stream());
  return loss;
}

Tensor sse_bwd(Tensor p, Tensor y, Tensor g) {
  CHECK_DEV(p); CHECK_F32(p); CHECK_CONTIG(p); CHECK_F32(y); CHECK_CONTIG(y); CHECK_F32(g);
  TORCH_CHECK(g.numel() == 1, "sse_bwd: scalar upstream gradient");
  auto dp = at::empty_like(p);
  tfx::sse_bwd(p.data_ptr<float>(), y.data_ptr<float>(), g.data_ptr<float>(), p.numel(), dp.data_ptr<float>(),
               cur_stream());
  return dp;
}

// f32: returns dz = g * act'(y).  bf16 (g, y bf16): returns dz for act != 0, or an empty tensor when
// act == 0 (only the bias column sums are wanted: g itself is the GEMM operand).
// backward of y = x W^T + b with few outputs: returns dx (undefined unless want_dx); dW / db
// (f32, [O][I] / [O]) are accumulated in place when given
Tensor linear_small_bwd(Tensor g, Tensor x, Tensor w, bool want_dx, optional<Tensor> dw, optional<Tensor> db) {
  CHECK_DEV(g); CHECK_BF16(g); CHECK_CONTIG(g); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w);
  const int64_t B = g.size(0), O = g.size(1), I = x.size(1);
  TORCH_CHECK(x.size(0) == B && w.size(0) == O && w.size(1) == I, "linear_small_bwd shapes");
  TORCH_CHECK(O <= 64, "linear_small_bwd: O <= 64");
  Tensor dx;
  if (want_dx) dx = at::empty({B, I}, x.options());
  if (dw.has_value() && dw->defined()) { CHECK_F32(*dw); TORCH_CHECK(dw->numel() == O * I && dw->is_contiguous(), "dw"); }
  if (db.has_value() && db->defined()) { CHECK_F32(*db); TORCH_CHECK(db->numel() == O, "db"); }
  tfx::linear_small_bwd(bf(g), bf(x), bf(w), (int)B, (int)I, (int)O, want_dx ? bfm(dx) : nullptr, fpm(dw), fpm(db),
                        cur_stream());
  return dx;
}

Tensor act_bwd_colsum(Tensor g, Tensor y, int64_t act, optional<Tensor> dbias) {
  CHECK_DEV(g); CHECK_CONTIG(g); CHECK_CONTIG(y);
  TORCH_CHECK(g.dim() == 2 && g.sizes() == y.sizes() && g.scalar_type() == y.scalar_type(),
              "act_bwd_colsum: [M, N] gradient and activation of one dtype");
  if (dbias.has_value() && dbias->defined()) {
    CHECK_F32(*dbias);
    TORCH_CHECK(dbias->numel() == g.size(1) && dbias->is_contiguous(), "dbias size");
  }
  if (g.scalar_type() == at::kBFloat16) {
    Tensor dz = act != 0 ? at::empty_like(g) : at::Tensor();
    tfx::act_bwd_colsum_bf16(bf(g), bf(y), (int)act, g.size(0), (int)g.size(1), act != 0 ? bfm(dz) : nullptr,
                             fpm(dbias), cur_stream());
    return dz;
  }
  CHECK_F32(g); CHECK_F32(y);
  auto dz = at::empty_like(g);
  tfx::act_bwd_colsum(g.data_ptr<float>(), y.data_ptr<float>(), (int)act, g.size(0), (int)g.size(1),
                      dz.data_ptr<float>(), fpm(dbias), cur_stream());
  return dz;
}

Tensor scale_by_scalar(Tensor x, Tensor scal, bool out_bf16) {
  CHECK_DEV(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_F32(scal);
  TORCH_CHECK(scal.numel() == 1, "scale_by_scalar: scalar");
  auto y = at::empty_like(x, x.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  tfx::scale_by_scalar(x.data_ptr<float>(), scal.data_ptr<float>(), x.numel(),
                       out_bf16 ? nullptr : y.data_ptr<float>(), out_bf16 ? bfm(y) : nullptr, cur_stream());
  return y;
}

// ------------------------------------------------------------------ optimizers
void optimizer_apply(int64_t kind, Tensor p, Tensor g, optional<Tensor> m, optional<Tensor> v, Tensor lr,
                     double gscale, double wd, double b1, double b2, double eps, optional<Tensor> step,
                     optional<Tensor> sumsq, double max_norm, optional<Tensor> pbf, optional<Tensor> skip_if,
                     optional<Tensor> zero_grad) {
  CHECK_DEV(p); CHECK_F32(p); CHECK_CONTIG(p); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() % 4 == 0, "flat buffers must match and be padded to 4");
  const bool gb = g.scalar_type() == at::kBFloat16;
  TORCH_CHECK(gb || g.scalar_type() == at::kFloat, "grad dtype");
  if (kind >= 1) TORCH_CHECK(m.has_value() && m->numel() == p.numel(), "momentum buffer");
  if (kind >= 3) TORCH_CHECK(v.has_value() && v->numel() == p.numel() && step.has_value(), "adam buffers");
  uint16_t* pb = nullptr;
  if (pbf.has_value() && pbf->defined()) {
    CHECK_BF16(*pbf);
    TORCH_CHECK(pbf->numel() == p.numel(), "bf16 shadow size");
    pb = bfm(*pbf);
  }
  const int* skip = nullptr;  // a device int32 word: nonzero -> the update is skipped on the device
  if (skip_if.has_value() && skip_if->defined()) {
    TORCH_CHECK(skip_if->is_cuda() && skip_if->scalar_type() == at::kInt && skip_if->numel() >= 1, "skip_if word");
    skip = skip_if->data_ptr<int>();
  }
  float* gz = nullptr;  // the f32 gradient buffer cleared in the same pass (the next step accumulates into it)
  if (zero_grad.has_value() && zero_grad->defined()) {
    CHECK_F32(*zero_grad); CHECK_CONTIG(*zero_grad);
    TORCH_CHECK(zero_grad->is_cuda() && zero_grad->numel() == p.numel(), "zero_grad: the f32 flat gradient buffer");
    gz = zero_grad->data_ptr<float>();
  }
  tfx::optimizer_apply(kind, p.data_ptr<float>(), g.data_ptr(), gb, fpm(m), fpm(v), p.numel(), lr.data_ptr<float>(),
                       gscale, wd, b1, b2, eps, fp(step), fp(sumsq), max_norm, pb, skip, gz, cur_stream());
}

Tensor sumsq(Tensor g) {
  CHECK_DEV(g); CHECK_CONTIG(g);
  TORCH_CHECK(g.numel() % 4 == 0, "sumsq needs numel % 4 == 0");
  auto out = at::empty({1}, g.options().dtype(at::kFloat));
  tfx::sumsq_flat(g.data_ptr(), g.scalar_type() == at::kBFloat16, g.numel(), out.data_ptr<float>(), cur_stream());
  return out;
}

void cast_f32_bf16(Tensor x, Tensor y) {
  CHECK_DEV(x); CHECK_F32(x); CHECK_BF16(y);
  TORCH_CHECK(x.numel() == y.numel() && x.is_contiguous() && y.is_contiguous(), "cast sizes");
  tfx::cast_f32_bf16(x.data_ptr<float>(), x.numel(), bfm(y), cur_stream());
}

// ------------------------------------------------------------------ ps transport over xGMI peer memory
// The arena is a raw hipMalloc allocation (IPC needs an allocation base, which the caching
// allocator does not hand out); the returned uint8 tensor owns it and frees it on release.
Tensor ipc_arena_alloc(int64_t nbytes, int64_t device) {
  TORCH_CHECK(nbytes > 0 && nbytes % 256 == 0, "arena size must be a positive multiple of 256");
  void* p = nullptr;
  const int r = tfx::ipc_alloc((int)device, nbytes, &p);
  TORCH_CHECK(r == 0, "hipMalloc of the ps arena failed (", r, ")");
  const int dev = (int)device;
  return at::from_blob(p, {nbytes}, [dev](void* q) { tfx::ipc_free(dev, q); },
                       at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
}

Tensor ipc_handle(Tensor arena) {
  CHECK_DEV(arena);
  auto out = at::zeros({64}, at::TensorOptions().dtype(at::kByte));
  const int r = tfx::ipc_get_handle(arena.data_ptr(), out.data_ptr<uint8_t>());
  TORCH_CHECK(r > 0, "hipIpcGetMemHandle failed (", r, "): the arena must come from ipc_arena_alloc");
  return out;
}

Tensor ipc_open(Tensor handle, int64_t nbytes, int64_t device) {
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte && handle.numel() == 64, "64-byte host handle");
  auto h = handle.contiguous();
  void* p = nullptr;
  const int r = tfx::ipc_open((int)device, h.data_ptr<uint8_t>(), &p);
  TORCH_CHECK(r == 0, "hipIpcOpenMemHandle failed (", r, ")");
  return at::from_blob(p, {nbytes}, [](void* q) { tfx::ipc_close(q); },
                       at::TensorOptions().dtype(at::kByte).device(at::kCUDA, (int)device));
}

// p, g: f32 ranges of equal length (p may be peer-mapped); step: int64 [1] view in the arena
// header or None; step_out: int64 [1] worker-local, receives the new global step.
void ps_peer_sgd(Tensor p, Tensor g, double lr, optional<Tensor> step, Tensor step_out, bool zero_g) {
  CHECK_DEV(p); CHECK_DEV(g); CHECK_F32(p); CHECK_F32(g); CHECK_CONTIG(p); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel(), "ps_peer_sgd: range sizes differ");
  CHECK_DEV(step_out);
  TORCH_CHECK(step_out.scalar_type() == at::kLong && step_out.numel() >= 1, "step_out must be int64");
  void* sp = nullptr;
  if (step.has_value() && step->defined()) {
    CHECK_DEV(*step);
    TORCH_CHECK(step->scalar_type() == at::kLong && reinterpret_cast<uintptr_t>(step->data_ptr()) % 8 == 0,
                "step must be an aligned int64 view");
    sp = step->data_ptr();
  }
  tfx::ps_peer_sgd(p.data_ptr<float>(), g.data_ptr<float>(), p.numel(), (float)lr, zero_g, sp,
                   step_out.data_ptr<int64_t>(), cur_stream());
}

// dst (worker-local store range) <- src (peer arena range)
void ps_peer_copy(Tensor dst, Tensor src) {
  CHECK_DEV(dst); CHECK_DEV(src); CHECK_F32(dst); CHECK_F32(src); CHECK_CONTIG(dst); CHECK_CONTIG(src);
  TORCH_CHECK(dst.numel() == src.numel(), "ps_peer_copy: range sizes differ");
  tfx::ps_peer_copy(dst.data_ptr<float>(), src.data_ptr<float>(), dst.numel(), cur_stream());
}

// ------------------------------------------------------------------ pooling (NHWC bf16)
int64_t pool_out(int64_t H, int64_t k, int64_t s, int64_t pad) { return (H + 2 * pad - k) / s + 1; }

std::tuple<Tensor, Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t s, int64_t pad) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4 && k >= 1 && k <= 15 && s >= 1 && pad >= 0 && pad < k, "maxpool args");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t P = pool_out(H, k, s, pad), Q = pool_out(W, k, s, pad);
  TORCH_CHECK(P > 0 && Q > 0, "maxpool output is empty");
  auto y = at::empty({N, P, Q, C}, x.options());
  auto arg = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  tfx::maxpool_fwd(bf(x), N, H, W, C, k, s, pad, P, Q, bfm(y), arg.data_ptr<uint8_t>(), cur_stream());
  return {y, arg};
}

Tensor maxpool_bwd(Tensor dy, Tensor arg, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(arg);
  TORCH_CHECK(arg.scalar_type() == at::kByte && arg.sizes() == dy.sizes(), "argmax shape");
  const int64_t N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  TORCH_CHECK(P == pool_out(H, k, s, pad) && Q == pool_out(W, k, s, pad), "maxpool_bwd geometry");
  auto dx = at::empty({N, H, W, C}, dy.options());
  tfx::maxpool_bwd(bf(dy), arg.data_ptr<uint8_t>(), N, H, W, C, k, s, pad, P, Q, bfm(dx), cur_stream());
  return dx;
}

Tensor avgpool_fwd(Tensor x, int64_t k, int64_t s, int64_t pad) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4 && k >= 1 && s >= 1 && pad >= 0 && pad < k, "avgpool args");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t P = pool_out(H, k, s, pad), Q = pool_out(W, k, s, pad);
  TORCH_CHECK(P > 0 && Q > 0, "avgpool output is empty");
  auto y = at::empty({N, P, Q, C}, x.options());
  tfx::avgpool_fwd(bf(x), N, H, W, C, k, s, pad, P, Q, bfm(y), cur_stream());
  return y;
}

Tensor avgpool_bwd(Tensor dy, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONTIG(dy);
  const int64_t N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  TORCH_CHECK(P == pool_out(H, k, s, pad) && Q == pool_out(W, k, s, pad), "avgpool_bwd geometry");
  auto dx = at::empty({N, H, W, C}, dy.options());
  tfx::avgpool_bwd(bf(dy), N, H, W, C, k, s, pad, P, Q, bfm(dx), cur_stream());
  return dx;
}

// ------------------------------------------------------------------ sparse embedding / sampled loss
void check_table(const Tensor& table) {
  CHECK_DEV(table); CHECK_F32(table); CHECK_CONTIG(table);
  TORCH_CHECK(table.dim() == 2 && table.size(1) >= 1, "embedding table must be [V, D]");
}

Tensor embedding_gather(Tensor table, Tensor ids, bool out_bf16) {
  check_table(table);
  CHECK_DEV(ids); CHECK_CONTIG(ids);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids must be int64");
  const int64_t n = ids.numel(), D = table.size(1);
  auto out = at::empty({n, D}, table.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  if (n) tfx::embedding_gather(table.data_ptr<float>(), table.size(0), D, ids.data_ptr<int64_t>(), n, out.data_ptr(),
                               out_bf16, cur_stream());
  return out;
}

void embedding_scatter_add(Tensor table, Tensor ids, Tensor rows, double alpha) {
  check_table(table);
  CHECK_DEV(ids); CHECK_CONTIG(ids); CHECK_CONTIG(rows); CHECK_F32(rows);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids must be int64");
  const int64_t n = ids.numel(), D = table.size(1);
  TORCH_CHECK(rows.numel() == n * D, "rows must be [n, D]");
  if (n) tfx::embedding_scatter_add(table.data_ptr<float>(), table.size(0), D, ids.data_ptr<int64_t>(), n,
                                    rows.data_ptr<float>(), alpha, cur_stream());
}

std::tuple<Tensor, Tensor> log_uniform_sample(int64_t n, int64_t range, int64_t seed, int64_t num_expected,
                                              at::Device device, optional<Tensor> seed_t) {
  TORCH_CHECK(n > 0 && range > 0, "sampler args");
  const int64_t* sd = nullptr;
  if (seed_t.has_value() && seed_t->defined()) {
    TORCH_CHECK(seed_t->scalar_type() == at::kLong && seed_t->is_cuda() && seed_t->numel() >= 1, "seed tensor");
    sd = seed_t->data_ptr<int64_t>();
  }
  auto opts = at::TensorOptions().device(device);
  auto ids = at::empty({n}, opts.dtype(at::kLong));
  auto logq = at::empty({n}, opts.dtype(at::kFloat));
  tfx::log_uniform_sample(n, range, (uint64_t)seed, sd, nullptr, ids.data_ptr<int64_t>(), logq.data_ptr<float>(),
                          (int)num_expected, cur_stream());
  return {ids, logq};
}

Tensor log_uniform_logq(Tensor ids, int64_t range, int64_t num_expected) {
  CHECK_DEV(ids); CHECK_CONTIG(ids);
  TORCH_CHECK(ids.scalar_type() == at::kLong && range > 0, "log_uniform_logq args");
  auto logq = at::empty({ids.numel()}, ids.options().dtype(at::kFloat));
  if (ids.numel())
    tfx::log_uniform_sample(ids.numel(), range, 0, nullptr, ids.data_ptr<int64_t>(), nullptr, logq.data_ptr<float>(),
                            (int)num_expected, cur_stream());
  return logq;
}

std::tuple<Tensor, Tensor> skipgram_batch(Tensor corpus, int64_t B, int64_t window, int64_t seed,
                                          optional<Tensor> seed_t) {
  CHECK_DEV(corpus); CHECK_CONTIG(corpus);
  TORCH_CHECK(corpus.scalar_type() == at::kInt, "corpus must be int32");
  TORCH_CHECK(B > 0 && window >= 1 && corpus.numel() > 2 * window, "skipgram_batch args");
  const int64_t* sd = nullptr;
  if (seed_t.has_value() && seed_t->defined()) {
    TORCH_CHECK(seed_t->scalar_type() == at::kLong && seed_t->is_cuda(), "seed tensor");
    sd = seed_t->data_ptr<int64_t>();
  }
  auto c = at::empty({B}, corpus.options().dtype(at::kLong)), l = at::empty({B}, corpus.options().dtype(at::kLong));
  tfx::skipgram_batch(corpus.data_ptr<int32_t>(), corpus.numel(), B, window, (uint64_t)seed, sd, c.data_ptr<int64_t>(),
                      l.data_ptr<int64_t>(), cur_stream());
  return {c, l};
}

// E, Wt: [B, D] f32 (gathered input / true-class rows); bt: [B] true-class biases (optional);
// neg_logits: [B, S] = E Ws^T + bs.  Returns (loss_rows [B], dneg [B,S], dE [B,D], dWt [B,D], dbt [B]).
std::vector<Tensor> sampled_loss(Tensor E, Tensor Wt, optional<Tensor> bt, Tensor neg_logits, optional<Tensor> logq_t,
                                 optional<Tensor> logq_n, optional<Tensor> true_ids, optional<Tensor> sampled_ids,
                                 double gscale, bool softmax) {
  CHECK_DEV(E); CHECK_F32(E); CHECK_CONTIG(E); CHECK_F32(Wt); CHECK_CONTIG(Wt);
  CHECK_F32(neg_logits); CHECK_CONTIG(neg_logits);
  TORCH_CHECK(E.dim() == 2 && Wt.sizes() == E.sizes() && neg_logits.dim() == 2, "sampled_loss shapes");
  const int64_t B = E.size(0), D = E.size(1), S = neg_logits.size(1);
  TORCH_CHECK(neg_logits.size(0) == B, "neg_logits must be [B, S]");
  if (fp(bt)) TORCH_CHECK(bt->numel() == B && bt->is_contiguous(), "bt");
  if (fp(logq_t)) TORCH_CHECK(logq_t->numel() == B, "logq_true");
  if (fp(logq_n)) TORCH_CHECK(logq_n->numel() == S, "logq_sampled");
  const bool hits = true_ids.has_value() && true_ids->defined() && sampled_ids.has_value() && sampled_ids->defined();
  if (hits) TORCH_CHECK(true_ids->numel() == B && sampled_ids->numel() == S && true_ids->scalar_type() == at::kLong &&
                        sampled_ids->scalar_type() == at::kLong, "accidental-hit ids");
  auto opts = E.options();
  auto loss = at::empty({B}, opts), dn = at::empty({B, S}, opts), dE = at::empty({B, D}, opts),
       dWt = at::empty({B, D}, opts), dbt = at::empty({B}, opts);
  tfx::sampled_loss(softmax, E.data_ptr<float>(), Wt.data_ptr<float>(), fp(bt), neg_logits.data_ptr<float>(), B, S, D,
                    fp(logq_t), fp(logq_n), hits ? true_ids->data_ptr<int64_t>() : nullptr,
                    hits ? sampled_ids->data_ptr<int64_t>() : nullptr, gscale, loss.data_ptr<float>(),
                    dn.data_ptr<float>(), dE.data_ptr<float>(), dWt.data_ptr<float>(), dbt.data_ptr<float>(),
                    cur_stream());
  return {loss, dn, dE, dWt, dbt};
}

// ------------------------------------------------------------------ LSTM cell
// gx, gh: [B, 4H] f32 (gh optional); bias [4H] optional; c_prev [B, H] optional
// outputs written into act [B, 4H], c [B, H], h [B, H] (+ optional bf16 copy of h)
void lstm_cell_fwd(Tensor gx, optional<Tensor> gh, optional<Tensor> bias, optional<Tensor> c_prev, Tensor act,
                   Tensor c, Tensor h, optional<Tensor> h16) {
  CHECK_DEV(gx); CHECK_F32(gx); CHECK_CONTIG(gx); CHECK_CONTIG(act); CHECK_CONTIG(c); CHECK_CONTIG(h);
  const int64_t B = c.size(0), H = c.size(1);
  TORCH_CHECK(gx.numel() == B * 4 * H && act.numel() == B * 4 * H && h.numel() == B * H, "lstm shapes");
  if (fp(gh)) TORCH_CHECK(gh->numel() == B * 4 * H && gh->is_contiguous(), "gh shape");
  if (fp(bias)) TORCH_CHECK(bias->numel() == 4 * H, "bias shape");
  if (fp(c_prev)) TORCH_CHECK(c_prev->numel() == B * H && c_prev->is_contiguous(), "c_prev shape");
  uint16_t* hb = nullptr;
  if (h16.has_value() && h16->defined()) {
    CHECK_BF16(*h16);
    TORCH_CHECK(h16->numel() == B * H && h16->is_contiguous(), "h16 shape");
    hb = bfm(*h16);
  }
  tfx::lstm_cell_fwd(gx.data_ptr<float>(), fp(gh), fp(bias), fp(c_prev), B, H, act.data_ptr<float>(),
                     c.data_ptr<float>(), h.data_ptr<float>(), hb, cur_stream());
}

// dgates (f32) and/or dg16 (bf16 copy for the MFMA GEMMs); dc_prev may alias dc_next (in place)
void lstm_cell_bwd(Tensor act, Tensor c, optional<Tensor> c_prev, optional<Tensor> dh, optional<Tensor> dc_next,
                   optional<Tensor> dgates, optional<Tensor> dg16, optional<Tensor> dc_prev) {
  CHECK_DEV(act); CHECK_F32(act); CHECK_CONTIG(act); CHECK_CONTIG(c);
  const int64_t B = c.size(0), H = c.size(1);
  TORCH_CHECK(act.numel() == B * 4 * H, "lstm bwd shapes");
  if (fp(dgates)) TORCH_CHECK(dgates->numel() == B * 4 * H && dgates->is_contiguous(), "dgates shape");
  uint16_t* d16 = nullptr;
  if (dg16.has_value() && dg16->defined()) {
    CHECK_BF16(*dg16);
    TORCH_CHECK(dg16->numel() == B * 4 * H && dg16->is_contiguous(), "dg16 shape");
    d16 = bfm(*dg16);
  }
  TORCH_CHECK(fp(dgates) || d16, "lstm_cell_bwd needs an output");
  for (const auto* t : {&c_prev, &dh, &dc_next, &dc_prev})
    if (fp(*t)) TORCH_CHECK((*t)->numel() == B * H && (*t)->is_contiguous(), "lstm bwd state shape");
  tfx::lstm_cell_bwd(act.data_ptr<float>(), c.data_ptr<float>(), fp(c_prev), fp(dh), fp(dc_next), B, H,
                     fpm(dgates), d16, fpm(dc_prev), cur_stream());
}

// Whole-sequence persistent LSTM (lstm_seq.hip).  gx [T,B,4H] f32 (input projection + bias),
// whh [4H,H] bf16; hbuf [T+1,B,H] bf16 and cbuf [T+1,B,H] f32 with h0 / c0 in slot 0; act [T,B,4H]
// f32 and hT [B,H] f32 are written.  status (optional): a persistent int32 [1] health word the
// launch sets to 1 if a hand-off wait exceeds its bound (results invalid); it is never cleared by a
// launch, so the host checks it at its own sync points (ops/rnn.py check_lstm_health).  Without it
// the launch's own status word is set instead.  Returns the launch's own word.  spin_limit 0 =
// the default bound.
bool lstm_seq_supported(int64_t B, int64_t H) {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return tfx::lstm_seq_supported((int)B, (int)H, cus);
}

// (resident workgroups the occupancy API allows for the forward / backward kernel, grid size)
std::tuple<int64_t, int64_t, int64_t> lstm_seq_residency(int64_t B, int64_t H) {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int f = 0, b = 0;
  tfx::lstm_seq_residency((int)B, (int)H, cus, &f, &b);
  return {f, b, (B / 16) * (H / 16)};
}

unsigned* lstm_status_ptr(const optional<Tensor>& status) {
  if (!(status.has_value() && status->defined())) return nullptr;
  TORCH_CHECK(status->is_cuda() && status->scalar_type() == at::kInt && status->numel() >= 1, "lstm status word");
  return reinterpret_cast<unsigned*>(status->data_ptr());
}

Tensor lstm_seq_fwd(Tensor gx, Tensor whh, Tensor hbuf, Tensor cbuf, Tensor act, Tensor hT, optional<Tensor> status,
                    int64_t spin_limit) {
  CHECK_DEV(gx); CHECK_F32(gx); CHECK_CONTIG(gx); CHECK_BF16(whh); CHECK_CONTIG(whh);
  CHECK_BF16(hbuf); CHECK_CONTIG(hbuf); CHECK_F32(cbuf); CHECK_CONTIG(cbuf); CHECK_F32(act); CHECK_CONTIG(act);
  CHECK_F32(hT); CHECK_CONTIG(hT);
  TORCH_CHECK(hbuf.dim() == 3, "hbuf must be [T+1,B,H]");
  const int64_t T = hbuf.size(0) - 1, B = hbuf.size(1), H = hbuf.size(2);
  TORCH_CHECK(T >= 1 && lstm_seq_supported(B, H), "lstm_seq: unsupported shape (B%16, H in 128..1024, grid <= CUs)");
  TORCH_CHECK(gx.numel() == T * B * 4 * H && act.numel() == T * B * 4 * H && cbuf.numel() == (T + 1) * B * H &&
                  whh.numel() == 4 * H * H && hT.numel() == B * H, "lstm_seq_fwd shapes");
  TORCH_CHECK(T * B * 4 * H * 4 < (int64_t(1) << 31), "lstm_seq: tensors must be < 2 GiB");
  for (const Tensor* t : {&gx, &whh, &hbuf}) check_aligned16(*t, "lstm_seq operand");
  Tensor sync = at::empty({tfx::lstm_seq_sync_words((int)B, (int)H)}, gx.options().dtype(at::kInt));
  unsigned* st = lstm_status_ptr(status);
  tfx::lstm_seq_fwd(gx.data_ptr<float>(), bf(whh), (int)T, (int)B, (int)H, bfm(hbuf), cbuf.data_ptr<float>(),
                    act.data_ptr<float>(), hT.data_ptr<float>(), reinterpret_cast<unsigned*>(sync.data_ptr()), st,
                    (unsigned)spin_limit, cur_stream());
  return sync.narrow(0, sync.numel() - 32, 1);  // this launch's own word (stays 0 when `status` is given)
}

// act, cbuf from the forward; dH [T,B,H] bf16 (optional) = gradient of every h_t from outside the
// recurrence; dhT / dc_in [B,H] f32 (optional) = gradients of h_T / c_T.  Writes dg [T,B,4H] bf16
// (gate pre-activation gradients), optionally dc_out [B,H] (gradient of c_0) and accumulates the
// bias gradient into dbias [4H] f32 (optional).
Tensor lstm_seq_bwd(Tensor act, Tensor cbuf, optional<Tensor> dH, optional<Tensor> dhT, optional<Tensor> dc_in,
                    Tensor whh, Tensor dg, optional<Tensor> dc_out, optional<Tensor> dbias, optional<Tensor> status,
                    int64_t spin_limit) {
  CHECK_DEV(act); CHECK_F32(act); CHECK_CONTIG(act); CHECK_F32(cbuf); CHECK_CONTIG(cbuf);
  CHECK_BF16(whh); CHECK_CONTIG(whh); CHECK_BF16(dg); CHECK_CONTIG(dg);
  TORCH_CHECK(cbuf.dim() == 3, "cbuf must be [T+1,B,H]");
  const int64_t T = cbuf.size(0) - 1, B = cbuf.size(1), H = cbuf.size(2);
  TORCH_CHECK(T >= 1 && lstm_seq_supported(B, H), "lstm_seq: unsupported shape");
  TORCH_CHECK(act.numel() == T * B * 4 * H && dg.numel() == T * B * 4 * H && whh.numel() == 4 * H * H,
              "lstm_seq_bwd shapes");
  const uint16_t* dh16 = nullptr;
  if (dH.has_value() && dH->defined()) {
    CHECK_BF16(*dH); CHECK_CONTIG(*dH);
    TORCH_CHECK(dH->numel() == T * B * H, "dH shape");
    dh16 = bf(*dH);
  }
  for (const auto* t : {&dhT, &dc_in, &dc_out})
    if (fp(*t)) TORCH_CHECK((*t)->numel() == B * H && (*t)->is_contiguous() && (*t)->scalar_type() == at::kFloat,
                            "lstm_seq_bwd state shape");
  if (fp(dbias)) TORCH_CHECK(dbias->numel() == 4 * H && dbias->is_contiguous() && dbias->scalar_type() == at::kFloat,
                             "dbias shape");
  check_aligned16(dg, "dg");
  Tensor sync = at::empty({tfx::lstm_seq_sync_words((int)B, (int)H)}, act.options().dtype(at::kInt));
  unsigned* st = lstm_status_ptr(status);
  tfx::lstm_seq_bwd(act.data_ptr<float>(), cbuf.data_ptr<float>(), dh16, fp(dhT), fp(dc_in), bf(whh), (int)T,
                    (int)B, (int)H, bfm(dg), fpm(dc_out), fpm(dbias), reinterpret_cast<unsigned*>(sync.data_ptr()), st,
                    (unsigned)spin_limit, cur_stream());
  return sync.narrow(0, sync.numel() - 32, 1);  // this launch's own word (stays 0 when `status` is given)
}

// ------------------------------------------------------------------ measured igemm launch configurations
void igemm_tune_set(int64_t fam, int64_t M, int64_t N, int64_t K, int64_t tile, int64_t ks, int64_t gls,
                    int64_t want) {
  TORCH_CHECK(fam >= 0 && fam < tfx::FAM_COUNT, "igemm_tune_set: family");
  tfx::igemm_tune_set((int)fam, (int)M, (int)N, (int)K, tfx::TuneCfg{(int)tile, (int)ks, (int)gls, (int)want});
}
void igemm_tune_clear() { tfx::igemm_tune_clear(); }
void igemm_tune_force(int64_t fam, int64_t tile, int64_t ks, int64_t gls, int64_t want) {
  tfx::igemm_tune_force((int)fam, tfx::TuneCfg{(int)tile, (int)ks, (int)gls, (int)want});
}
void igemm_tune_trace(bool on) { tfx::igemm_tune_trace(on); }
Tensor igemm_tune_traced() {
  std::vector<int> buf(4 * 4096);
  const int n = std::min(tfx::igemm_tune_traced(buf.data(), (int)buf.size()), 4096);
  auto out = at::empty({n, 4}, at::TensorOptions().dtype(at::kInt));
  std::copy(buf.begin(), buf.begin() + 4 * n, out.data_ptr<int>());
  return out;
}

void philox_fill(Tensor out, int64_t seed, int64_t subseq, int64_t dist, double a, double b) {
  CHECK_DEV(out); CHECK_F32(out); CHECK_CONTIG(out);
  TORCH_CHECK(dist >= 0 && dist <= 2, "philox dist");
  if (out.numel())
    tfx::philox_fill(out.data_ptr<float>(), out.numel(), (uint64_t)seed, (uint64_t)subseq, (int)dist, (float)a,
                     (float)b, cur_stream());
}

// uint8 NHWC images -> normalised bf16 NHWC with cout channels (the extra ones exactly zero)
Tensor image_normalize(Tensor x, std::vector<double> mean, std::vector<double> stdv, int64_t cout) {
  CHECK_DEV(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.scalar_type() == at::kByte, "image_normalize: uint8 images");
  const int64_t cin = x.size(-1);
  TORCH_CHECK(cin >= 1 && cin <= 4 && (int64_t)mean.size() == cin && (int64_t)stdv.size() == cin,
              "image_normalize: 1..4 channels with per-channel mean/std");
  TORCH_CHECK(cout == 4 || cout == 8, "image_normalize: cout 4 or 8");
  auto shape = x.sizes().vec();
  shape.back() = cout;
  auto y = at::empty(shape, x.options().dtype(at::kBFloat16));
  float m[4] = {0, 0, 0, 0}, s[4] = {1, 1, 1, 1};
  for (int64_t c = 0; c < cin; ++c) {
    m[c] = (float)mean[c];
    s[c] = (float)stdv[c];
  }
  tfx::image_normalize(x.data_ptr<uint8_t>(), x.numel() / cin, (int)cin, (int)cout, m, s, bfm(y), cur_stream());
  return y;
}

// Same kernel, written into a caller-owned device tensor.  `x` may be a GPU tensor or a PINNED host
// tensor: page-locked memory is mapped into the GPU's address space, so the kernel reads the batch
// straight over the host link (zero-copy input: no H2D staging copy, no copy stream, no device
// staging buffer).  The caller keeps the pinned buffer unmodified until the kernel has run
// (data/pipeline.py PinnedRing(zero_copy=True) orders that with an event per slot).
// Training augmentation (pad-`pad` random crop + flip; offsets [N][3] int32 = ox, oy, flip on the
// device) fused with the uint8 -> normalised bf16 conversion: returns [N][H][W][cout]
void augment_normalize_into(Tensor x, Tensor offsets, std::vector<double> mean, std::vector<double> stdv, int64_t pad,
                            Tensor y);

Tensor augment_normalize(Tensor x, Tensor offsets, std::vector<double> mean, std::vector<double> stdv, int64_t cout,
                         int64_t pad) {
  CHECK_DEV(x);
  auto y = at::empty({x.size(0), x.size(1), x.size(2), cout}, x.options().dtype(at::kBFloat16));
  augment_normalize_into(x, offsets, mean, stdv, pad, y);
  return y;
}

// the same into a preallocated bf16 NHWC tensor (e.g. a captured training graph's static input: the batch
// is written where the graph reads it, no copy)
void augment_normalize_into(Tensor x, Tensor offsets, std::vector<double> mean, std::vector<double> stdv, int64_t pad,
                            Tensor y) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_DEV(offsets); CHECK_CONTIG(offsets); CHECK_DEV(y); CHECK_CONTIG(y);
  CHECK_BF16(y);
  const int64_t cout = y.dim() == 4 ? y.size(3) : 0;
  TORCH_CHECK(y.dim() == 4 && x.dim() == 4 && y.size(0) == x.size(0) && y.size(1) == x.size(1) && y.size(2) == x.size(2),
              "augment_normalize: output [N][H][W][cout] of the image batch's size");
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4, "augment_normalize: uint8 NHWC images");
  TORCH_CHECK(offsets.scalar_type() == at::kInt && offsets.dim() == 2 && offsets.size(0) == x.size(0) &&
                  offsets.size(1) == 3, "augment_normalize: offsets [N][3] int32");
  const int64_t cin = x.size(3);
  TORCH_CHECK(cin >= 1 && cin <= 4 && (int64_t)mean.size() == cin && (int64_t)stdv.size() == cin,
              "augment_normalize: 1..4 channels with per-channel mean/std");
  TORCH_CHECK(cout == 4 || cout == 8, "augment_normalize: cout 4 or 8");
  TORCH_CHECK(pad >= 0 && pad < 64, "augment_normalize: pad");
  float m[4] = {0, 0, 0, 0}, sd[4] = {1, 1, 1, 1};
  for (int64_t c = 0; c < cin; ++c) {
    m[c] = (float)mean[c];
    sd[c] = (float)stdv[c];
  }
  tfx::augment_normalize(x.data_ptr<uint8_t>(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)cin, (int)cout,
                         (int)pad, offsets.data_ptr<int32_t>(), m, sd, bfm(y), cur_stream());
}

// End a capture left open on `stream` (a side stream forked into a HIP-graph capture that failed
// before the join): its partial graph is discarded.  Returns true if a capture was open.  While any
// stream of a thread stays capturing, that thread cannot run synchronous work at all.
bool end_stream_capture(int64_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st == hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return false;
  }
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(s, &g);
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return true;
}

// Host pointer of a pinned (page-locked) tensor as the GPU sees it (zero-copy reads over the host link).
static const void* pinned_device_ptr(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_pinned(), what, ": a host input must be pinned (page-locked)");
  void* dp = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&dp, const_cast<void*>(t.data_ptr()), 0) == hipSuccess && dp, what,
              ": pinned host buffer is not mapped into the GPU's address space");
  return dp;
}

// labels / labels_out (optional, int64 [N]): copied by the same launch (a pinned host source is read
// zero-copy), e.g. into a captured step's static label buffer.
void image_normalize_into(Tensor x, std::vector<double> mean, std::vector<double> stdv, Tensor out,
                          optional<Tensor> labels, optional<Tensor> labels_out) {
  CHECK_CONTIG(x); CHECK_DEV(out); CHECK_CONTIG(out); CHECK_BF16(out);
  TORCH_CHECK(x.scalar_type() == at::kByte, "image_normalize_into: uint8 images");
  const int64_t cin = x.size(-1), cout = out.size(-1);
  TORCH_CHECK(cin >= 1 && cin <= 4 && (int64_t)mean.size() == cin && (int64_t)stdv.size() == cin,
              "image_normalize_into: 1..4 channels with per-channel mean/std");
  TORCH_CHECK(cout == 4 || cout == 8, "image_normalize_into: cout 4 or 8");
  TORCH_CHECK(x.numel() / cin == out.numel() / cout && x.dim() == out.dim(),
              "image_normalize_into: pixel counts of x and out differ");
  const uint8_t* src = x.data_ptr<uint8_t>();
  if (!x.is_cuda()) src = static_cast<const uint8_t*>(pinned_device_ptr(x, "image_normalize_into"));
  float m[4] = {0, 0, 0, 0}, s[4] = {1, 1, 1, 1};
  for (int64_t c = 0; c < cin; ++c) {
    m[c] = (float)mean[c];
    s[c] = (float)stdv[c];
  }
  const int64_t* lab = nullptr;
  int64_t* lab_out = nullptr;
  int nlab = 0;
  if (labels.has_value() && labels->defined()) {
    TORCH_CHECK(labels_out.has_value() && labels_out->defined(), "image_normalize_into: labels need labels_out");
    const Tensor& l = *labels;
    const Tensor& lo = *labels_out;
    CHECK_DEV(lo); CHECK_CONTIG(lo); CHECK_CONTIG(l);
    TORCH_CHECK(l.scalar_type() == at::kLong && lo.scalar_type() == at::kLong && l.numel() == lo.numel() &&
                l.numel() < (1 << 30), "image_normalize_into: int64 labels of equal size");
    lab = l.is_cuda() ? l.data_ptr<int64_t>() : static_cast<const int64_t*>(pinned_device_ptr(l, "labels"));
    lab_out = lo.data_ptr<int64_t>();
    nlab = (int)l.numel();
  }
  tfx::image_normalize(src, x.numel() / cin, (int)cin, (int)cout, m, s, bfm(out), cur_stream(), lab, lab_out, nlab);
}

}  // namespace

// the CU / memory footprint of one bucket's 8-rank ring all-reduce on the current stream (dp_sim.hip)
void dp_ring_sim(Tensor buf, int64_t nblocks, double duration_us, int64_t passes) {
  CHECK_DEV(buf); CHECK_CONTIG(buf);
  tfx::dp_ring_sim(buf.data_ptr(), buf.nbytes(), (int)nblocks, duration_us, (int)passes, cur_stream());
}

int64_t igemm_persist_mode(int64_t mode) { return tfx::igemm_persist_set((int)mode); }

TORCH_LIBRARY(tfx, m) {
  m.def("image_normalize", &image_normalize);
  m.def("image_normalize_into", &image_normalize_into);
  m.def("augment_normalize", &augment_normalize);
  m.def("igemm_persist_mode", &igemm_persist_mode);
  m.def("dp_ring_sim(Tensor(a!) buf, int nblocks, float duration_us, int passes) -> ()", &dp_ring_sim);
  m.def("augment_normalize_into(Tensor x, Tensor offsets, float[] mean, float[] stdv, int pad, Tensor(a!) y) -> ()",
        &augment_normalize_into);
  m.def("end_stream_capture", &end_stream_capture);
  m.def("philox_fill", &philox_fill);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("embedding_gather", &embedding_gather);
  m.def("embedding_scatter_add", &embedding_scatter_add);
  m.def("log_uniform_sample", &log_uniform_sample);
  m.def("log_uniform_logq", &log_uniform_logq);
  m.def("sampled_loss", &sampled_loss);
  m.def("skipgram_batch", &skipgram_batch);
  m.def("lstm_cell_fwd", &lstm_cell_fwd);
  m.def("lstm_cell_bwd", &lstm_cell_bwd);
  m.def("lstm_seq_supported", &lstm_seq_supported);
  m.def("igemm_tune_set", &igemm_tune_set);
  m.def("igemm_tune_clear", &igemm_tune_clear);
  m.def("igemm_tune_force", &igemm_tune_force);
  m.def("igemm_tune_trace", &igemm_tune_trace);
  m.def("igemm_tune_traced", &igemm_tune_traced);
  m.def("lstm_seq_fwd(Tensor gx, Tensor whh, Tensor hbuf, Tensor cbuf, Tensor act, Tensor hT, "
        "Tensor? status=None, int spin_limit=0) -> Tensor", &lstm_seq_fwd);
  m.def("lstm_seq_bwd(Tensor act, Tensor cbuf, Tensor? dH, Tensor? dhT, Tensor? dc_in, Tensor whh, Tensor dg, "
        "Tensor? dc_out, Tensor? dbias, Tensor? status=None, int spin_limit=0) -> Tensor", &lstm_seq_bwd);
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_fwd_stats", &conv_fwd_stats);
  m.def("conv_dgrad(Tensor dy, Tensor w, int[] xshape, int stride, int pad, int dil, Tensor? addend, "
        "Tensor? addend_mask=None, bool addend_s2=False, Tensor? wflip=None) -> Tensor", &conv_dgrad);
  m.def("conv_wgrad", &conv_wgrad);
  m.def("conv_wgrad_sr", &conv_wgrad_sr);
  m.def("conv_wgrad_sr2", &conv_wgrad_sr2);
  m.def("bn_bwd_reduce_into", &bn_bwd_reduce_into);
  m.def("bn_slots_reduce", &bn_slots_reduce);
  m.def("gemm", &gemm);
  m.def("gemm_into", &gemm_into);
  m.def("sgemm(Tensor a, Tensor b, bool ta, bool tb, Tensor? bias, int act, bool split=False) -> Tensor", &sgemm);
  m.def("sgemm_into(Tensor a, Tensor b, bool ta, bool tb, Tensor(a!) out, bool accumulate, bool split=False) -> ()",
        &sgemm_into);
  m.def("bn_fwd_train", &bn_fwd_train);
  m.def("bn_apply_train", &bn_apply_train);
  m.def("wflip3x3(Tensor src, Tensor(a!) dst, Tensor desc, int ntiles) -> ()", &wflip3x3);
  m.def("bn_apply_res_bn(Tensor x, Tensor res_x, Tensor save, Tensor res_save, bool relu) -> (Tensor, Tensor)",
        &bn_apply_res_bn);
  m.def("bn_bwd_apply_sec(Tensor g, Tensor x, Tensor save, Tensor red, bool relu, Tensor? mask, Tensor x2, "
        "Tensor save2, Tensor slots2, Tensor? dgamma2=None, Tensor? dbeta2=None, bool want_dres=True, "
        "bool reduce2=True) -> (Tensor, Tensor, Tensor)",
        &bn_bwd_apply_sec);
  m.def("bn_bwd_apply(Tensor g, Tensor x, Tensor? res, Tensor save, Tensor red, bool relu, Tensor? mask, "
        "bool want_dres=True) -> (Tensor, Tensor)", &bn_bwd_apply);
  m.def("conv_fwd_bn", &conv_fwd_bn);
  m.def("conv_fwd_bn_in", &conv_fwd_bn_in);
  m.def("conv_fwd_bn_in_supported", &conv_fwd_bn_in_supported);
  m.def("stem_wgrad", &stem_wgrad);
  m.def("conv_stem_fwd", &conv_stem_fwd);
  m.def("set_deterministic", &set_deterministic);
  m.def("stem_wgrad_ws_floats", &stem_wgrad_ws_floats);
  m.def("stem_wgrad_supported", &stem_wgrad_supported);
  m.def("conv_dgrad_bn(Tensor dy, Tensor w, int[] xshape, int stride, int pad, int dil, Tensor? addend, "
        "Tensor bn_x, Tensor bn_save, Tensor? bn_mask, bool relu, Tensor ws, Tensor? dgamma, Tensor? dbeta, "
        "Tensor? addend_mask=None, bool reduce=True, bool addend_s2=False, Tensor? wflip=None) -> (Tensor, Tensor)",
        &conv_dgrad_bn);
  m.def("bn_nslot", &bn_nslot);
  m.def("pw_bwd_expand", &pw_bwd_expand);
  m.def("pw_bwd_expand_supported", &pw_bwd_expand_supported);
  m.def("pw_fwd_squeeze", &pw_fwd_squeeze);
  m.def("pw_bwd_squeeze", &pw_bwd_squeeze);
  m.def("pw_bwd_squeeze_supported", &pw_bwd_squeeze_supported);
  m.def("pw_fwd_squeeze_supported", &pw_fwd_squeeze_supported);
  m.def("bn_apply_into", &bn_apply_into);
  m.def("conv3x3_fwd_fused", &conv3x3_fwd_fused);
  m.def("conv3x3_fused_supported", &conv3x3_fused_supported);
  m.def("conv3x3_bwd_fused", &conv3x3_bwd_fused);
  m.def("bn_fwd_eval", &bn_fwd_eval);
  m.def("bn_bwd(Tensor g, Tensor x, Tensor? res, Tensor save, bool relu, Tensor slots, Tensor? dgamma, "
        "Tensor? dbeta, Tensor? mask, bool want_dres=True) -> (Tensor, Tensor, Tensor)", &bn_bwd);
  m.def("softmax_xent", &softmax_xent);
  m.def("softmax_xent_mean", &softmax_xent_mean);
  m.def("head_xent(Tensor x, Tensor w, Tensor? b, Tensor labels, Tensor state, Tensor? y3=None, Tensor? res=None, "
        "Tensor? save3=None, Tensor? mask=None, Tensor? bn_rows=None) -> (Tensor, Tensor, Tensor, Tensor)",
        &head_xent);
  m.def("head_rows_reduce", &head_rows_reduce);
  m.def("head_wgrad", &head_wgrad);
  m.def("head_xent_supported", &head_xent_supported);
  m.def("accuracy_count", &accuracy_count);
  m.def("gap_fwd", &gap_fwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("optimizer_apply", &optimizer_apply);
  m.def("lstm_seq_residency", &lstm_seq_residency);
  m.def("affine_fwd", &affine_fwd);
  m.def("affine_bwd", &affine_bwd);
  m.def("sse_fwd", &sse_fwd);
  m.def("sse_bwd", &sse_bwd);
  m.def("act_bwd_colsum", &act_bwd_colsum);
  m.def("linear_small_bwd", &linear_small_bwd);
  m.def("scale_by_scalar", &scale_by_scalar);
  m.def("sumsq", &sumsq);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("ipc_arena_alloc", &ipc_arena_alloc);
  m.def("ipc_handle", &ipc_handle);
  m.def("ipc_open", &ipc_open);
  m.def("ps_peer_sgd", &ps_peer_sgd);
  m.def("ps_peer_copy", &ps_peer_copy);
}
