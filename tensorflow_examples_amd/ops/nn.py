"""Differentiable ops of the framework.

Every op has two implementations behind one ``torch.autograd.Function``:

* GPU tensors  -> the hand-written gfx950 HIP kernels (``torch.ops.tfx.*``), bf16
  activations in NHWC, f32 statistics/accumulation;
* CPU tensors  -> a PyTorch reference (the numerics oracle of tests/, and the CPU
  training path used by ``simple/``, the MNIST softmax config and the PS demo).

Trainable parameters are :class:`~tensorflow_examples_amd.variables.Variable` views into a
flat store; backward passes ACCUMULATE parameter gradients straight into ``var.grad``
(the flat grad buffer) and fire ``store.grad_ready_hook`` so the data-parallel layer can
launch a bucket's all-reduce as soon as its last gradient lands.
"""
from __future__ import annotations

import os
import weakref
from typing import List, Optional

import torch
import torch.nn.functional as F

from . import _native, fusion
from ..variables import Variable


def _grad_ready(*vs: Optional[Variable]) -> None:
    for v in vs:
        if v is not None and v.store is not None and getattr(v.store, "grad_ready_hook", None) is not None:
            v.store.grad_ready_hook(v)


def _ref_param_grads(fn, x, params, grad_out, x_needs_grad, **kw):
    """CPU reference backward: re-run the reference forward under autograd."""
    with torch.enable_grad():
        xs = x.detach().requires_grad_(x_needs_grad) if x is not None else None
        ps = [p.master.detach().clone().requires_grad_(True) if p is not None else None for p in params]
        out = fn(xs, *ps, **kw)
        if isinstance(out, tuple):
            out = out[0]
        leaves = ([xs] if x_needs_grad else []) + [p for p in ps if p is not None]
        grads = torch.autograd.grad(out, leaves, grad_out, allow_unused=True)
    gx = grads[0] if x_needs_grad else None
    gp = list(grads[1:] if x_needs_grad else grads)
    it = iter(gp)
    for p in params:
        if p is not None:
            g = next(it)
            if g is not None:
                p.grad.add_(g.to(p.grad.dtype))
    _grad_ready(*params)
    return gx


# ====================================================================== conv2d (NHWC, KRSC)
def _conv_ref(x, w, stride=1, pad=0, dil=1):
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2).to(x.dtype), stride=stride, padding=pad, dilation=dil)
    return y.permute(0, 2, 3, 1).contiguous()


# Largest BN input (bytes) whose backward reduction runs in the consumer conv's dgrad epilogue:
# every ResNet-50 layer (since the identity blocks pass (gradient, mask bits) instead of a
# materialised residual gradient, fusing the 128 MB stage-1 inputs too is faster end to end:
# 9.46 -> 9.43 ms/step, profiles/r01_v9).
_BNB_MAX_BYTES = 256 << 20

# The BN-backward slot reduction of a fused data gradient runs as tail blocks of the same conv's
# weight-gradient launch (conv_wgrad_sr) instead of its own bn_slot_reduce launch; so do the
# reductions of a stride-2 conv2's input BN and of the projection-shortcut BN (deferred to the next
# weight-gradient launch's tail).  (Measured: profiles/r02_srfuse.  Rejected and removed: the same
# reduction in the stride-2 parity-class data gradients' epilogues, a wash -- profiles/r02_s2bnb.)
# Knobs (ops/fusion.py, group deferred_slot_reduce): sr_take off leaves every deferred reduction to
# its own BN's backward (the fallback path); sr_defer off never defers them (each BN reduces its own)


def _flip_ok(w, stride, pad, dil):
    """Stride-1 3x3 data gradients run as the forward conv of dY with flipped, transposed filters
    (igemm_dgrad_flip.hip); every layer's copy is refreshed by one launch per step."""
    sh = w.shape
    return stride == 1 and pad == 1 and dil == 1 and len(sh) == 4 and sh[1] == 3 and sh[2] == 3 \
        and getattr(w.store, "shadow", None) is not None and w.store.flip_index(w) is not None


def _wflip(w, stride, pad, dil):
    """The flipped copy of a 3x3 filter (refreshing every layer's copy first if the weights may
    have changed since the last refresh), or None where the data gradient stays gathered."""
    if not _flip_ok(w, stride, pad, dil):
        return None
    return w.store.flipped3x3(w)


# knob lazy_bn_bwd off keeps every tail BN backward materialised (the layer-wise path)
PW_EXPAND_CALLS = [0]  # fused expanding-1x1 backward launches (tests)


class LazyBNGrad:
    """The input gradient of a residual + ReLU batch norm (a ResNet bottleneck's tail), NOT
    materialised: dy = A (g * mask) + B x + D per channel, with g the BN's output gradient, x its
    input, mask the forward's ReLU mask bits and (A, B, D) folded from ``save`` and ``red``.  The BN's
    backward returns a zero-stride placeholder carrying this (fusion carrier "lazy_bnbwd"); its producer conv
    (the expanding 1x1 conv3) then forms dy on load inside its fused backward (pw_bwd.hip) -- or
    calls :meth:`materialize` (bn_bwd_apply, the layer-wise path) when it cannot.

    ``sec`` (a projection block's tail): the residual was the shortcut BN's output, whose gradient is
    the same g * mask; that BN's backward reduction is still owed (``sec.red`` is None until the fused
    kernel or :meth:`materialize` fills it -- whichever of conv3 / the shortcut BN runs first)."""
    __slots__ = ("g", "x", "save", "red", "relu", "mask", "sec", "dy")

    def __init__(self, g, x, save, red, relu, mask, sec=None):
        self.g, self.x, self.save, self.red, self.relu, self.mask = g, x, save, red, relu, mask
        self.sec, self.dy = sec, None

    def materialize(self) -> torch.Tensor:
        if self.dy is None:
            rb = self.sec
            if rb is None:
                self.dy = torch.ops.tfx.bn_bwd_apply(self.g, self.x, None, self.save, self.red, self.relu, self.mask,
                                                     False)[0]
            else:
                p_t = rb.dgamma is not None
                self.dy, _, rb.red = torch.ops.tfx.bn_bwd_apply_sec(
                    self.g, self.x, self.save, self.red, self.relu, self.mask, rb.x, rb.save, rb.ws,
                    rb.dgamma if p_t else None, rb.dbeta if p_t else None, False, True)
                rb.sec_lazy = None
        return self.dy


# knobs defer_tail / defer_bn_in off keep every block tail / plain BN applied by its own pass (the
# layer-wise forward); fuse_conv3_bwd off runs the stage-1 3x3 conv's backward layer-wise
PW_SQUEEZE_CALLS = [0]  # fused tail + conv1 forward launches (tests)


class TailPending:
    """A ReLU batch norm's output whose apply pass was deferred to its consumer conv: ``out`` (and,
    for a residual tail, the ReLU ``mask`` bits the backward saved) are allocated but not yet written.
    A residual tail's consumer (the next bottleneck's conv1) forms them while it loads its input
    (pw_fwd_squeeze, one launch, ``done``); a plain BN's consumer (the stage-1 3x3 conv2) applies it
    on load WITHOUT writing it (conv3x3_fwd_fused) -- whatever reads ``out`` later (that conv's
    weight gradient) calls :meth:`materialize` (bn_apply_into), as does any consumer that cannot fuse.
    Everything that reads ``out`` runs after that conv in the block's forward order."""
    __slots__ = ("x", "save", "res", "res_save", "_out", "mask", "done")

    def __init__(self, x, save, res, res_save, out, mask):
        # ``out`` carries this object (fusion carrier "tail"): held weakly, or the pair is a reference cycle
        # that only Python's full (rare) garbage collection frees -- with every step's tail activations
        # in it (an eager training loop ran out of HBM at ~280 steps of ResNet-50 at batch 128)
        self.x, self.save, self.res, self.res_save, self.mask = x, save, res, res_save, mask
        self._out = weakref.ref(out)
        self.done = False

    @property
    def out(self):
        return self._out()

    def materialize(self) -> None:
        if not self.done:
            torch.ops.tfx.bn_apply_into(self.x, self.res, self.save, self.res_save, self.out, self.mask)
            self.done = True


def _settle(t):
    """Write a deferred block-tail output before anything but its fused consumer reads it."""
    tp = fusion.carried(t, "tail") if t is not None else None
    if tp is not None and not tp.done:
        tp.materialize()
    return t


# Negative-control hook of the convergence-parity check (tests/test_convergence_gpu.py,
# scripts/convergence_parity.py): {fusion group: factor} -- the named fused backward group's input AND
# weight gradients are scaled by the factor after its kernel, i.e. a deliberately wrong fused gradient
# the check must catch.  Empty (the default) everywhere else; set from TFX_NEGCTL=group:factor.
NEG_CONTROL = {}
_neg = os.environ.get("TFX_NEGCTL", "")
if _neg:
    NEG_CONTROL[_neg.split(":")[0]] = float(_neg.split(":")[1])


def _negctl(group, dx, *ws):
    f = NEG_CONTROL.get(group)
    if f is None:
        return dx
    for w in ws:
        w.grad.mul_(f)
    return dx * f if dx is not None else None


CONV3_FWD_CALLS = [0]  # fused stage-1 3x3 forward launches (tests)
CONV3_BWD_CALLS = [0]  # ... and backward launches


def _conv3_bwd_fused_ok(w, lazy, bnb, tp) -> bool:
    """The stage-1 3x3 conv's fused backward (conv3x3_fused.hip) applies: its output gradient is a plain
    ReLU BN's lazy input gradient, its input the deferred output of the plain ReLU BN ``bnb`` (the
    forward ran conv3x3_fwd_fused), whose backward partials nobody reduced yet."""
    if not fusion.knob("fuse_conv3_bwd") or lazy.mask is not None or lazy.sec is not None or lazy.dy is not None \
            or not w.trainable:
        return False
    if bnb is None or bnb.mask is not None or not bnb.relu or bnb.deferred or bnb.red is not None or bnb.sr_pending:
        return False
    return bnb.x is tp.x and lazy.g.shape == tp.x.shape


def _std_geometry(x, w, stride, pad, dil) -> bool:
    """A square-kernel, same-padding, undilated NHWC conv over ``x``'s channels (the planner's layers)."""
    sh = w.shape
    return (x.dim() == 4 and len(sh) == 4 and sh[1] == sh[2] and pad == sh[1] // 2 and dil == 1
            and sh[3] == x.shape[-1])


_FUSED_INPUT = ("conv3x3_fwd_fused", "igemm_fwd_a_scale", "pw_fwd_squeeze")


def _fwd_choice_unplanned(x, w, stride, pad, dil, stats_into, tp) -> str:
    """The consumer of the deferred input ``tp`` for a conv no plan covers: the planner's rule
    (fusion.fwd_rule) on this call's shapes -- one of _FUSED_INPUT, or "materialize"."""
    if not (_std_geometry(x, w, stride, pad, dil) and x.is_contiguous() and isinstance(stats_into, BNWorkspace)):
        return "materialize"
    kind = "plain" if tp.res is None else ("tail" if tp.mask is not None else "other")
    if kind == "other":
        return "materialize"
    n, h, wd, c = x.shape
    pre, fwd = fusion.fwd_rule(kind, c, w.shape[0], w.shape[1], stride, n, (h, wd), ws="obj")
    return fwd if pre is None and fwd in _FUSED_INPUT else "materialize"


STEM_WGRAD_CALLS = [0]  # stem weight gradients by stem.hip (tests)


def _model_state(store) -> dict:
    """Per-model runtime state of the fused ops (the model's VariableStore ``fused_state``): two models in
    one process -- a train and an eval model, interleaved runs -- never share a workspace or a pending
    deferred reduction.  A conv / BN used outside a store (tests of single ops) gets a process-wide dict."""
    return store.fused_state if store is not None else _NO_STORE_STATE


_NO_STORE_STATE: dict = {}


def _cached_buffer(store, key, make) -> torch.Tensor:
    """A persistent per-model device buffer, allocated once OUTSIDE any graph capture when possible: a
    tensor allocated during a capture lives in that graph's private pool and is never cached (its
    allocation -- and zero fill -- are then recorded in the graph, so each replay still starts clean)."""
    st = _model_state(store)
    t = st.get(key)
    if t is None:
        t = make()
        if not torch.cuda.is_current_stream_capturing():
            st[key] = t
    return t


def _stem_ws(store, device, ko) -> torch.Tensor:
    """stem.hip's zeroed dW workspace copies (left zero by every launch), one per model and device."""
    return _cached_buffer(store, ("stem_ws", str(device), int(ko)), lambda: torch.zeros(
        int(torch.ops.tfx.stem_wgrad_ws_floats(ko)), dtype=torch.float32, device=device))


def _stem_ok(x, w, stride, pad, dil) -> bool:
    sh = w.shape
    if not (stride == 1 and pad == 1 and dil == 1 and x.dim() == 4 and len(sh) == 4 and sh[1] == 3 and sh[2] == 3
            and sh[3] == x.shape[-1]):
        return False
    n, h, wd, c = x.shape
    return bool(torch.ops.tfx.stem_wgrad_supported(n, h, wd, c, sh[0]))


PW_APPLY_CALLS = [0]  # 1x1 forwards that applied their input BN on load (tests)


def _pw_expand_ok(x, w, stride, pad, dil, lazy, sink) -> bool:
    """Can this conv's backward run as the fused expanding-1x1 kernel (pw_bwd.hip) on ``lazy``?"""
    sh = w.shape
    if not (stride == 1 and pad == 0 and dil == 1 and sink is None and w.trainable and len(sh) == 4
            and sh[1] == 1 and sh[2] == 1 and sh[0] == 4 * sh[3] and x.is_contiguous()):
        return False
    if lazy.mask is None or lazy.g.shape[-1] != sh[0] or x.shape[-1] != sh[3]:
        return False
    if lazy.dy is not None:  # already materialised (the shortcut BN's backward ran first)
        return False
    return bool(torch.ops.tfx.pw_bwd_expand_supported(sh[3], x.numel() // sh[3]))


PW_SQUEEZE_BWD_CALLS = [0]  # fused conv1 backward launches (tests)


def _pw_squeeze_bwd_ok(x, w, stride, pad, dil, lazy, sink, bnb) -> bool:
    """Can this conv's backward run as the fused squeezing-1x1 kernel (pw_bwd.hip F1) on ``lazy``
    (a plain ReLU BN's unmaterialised input gradient), with the residual branch's masked gradient
    parked in ``sink`` and the previous tail BN (``bnb``, with its ReLU mask bits) to reduce?"""
    sh = w.shape
    if not (stride == 1 and pad == 0 and dil == 1 and w.trainable and len(sh) == 4 and sh[1] == 1 and sh[2] == 1
            and x.is_contiguous() and lazy.mask is None and lazy.sec is None and lazy.dy is None):
        return False
    if sink is None or sink.mode != "consume" or not isinstance(sink.buf, tuple) or isinstance(sink.buf[0], str):
        return False
    if bnb is None or bnb.mask is None or not bnb.relu or bnb.deferred or bnb.red is not None or bnb.sr_pending:
        return False
    if lazy.g.shape[-1] != sh[0] or x.shape[-1] != sh[3] or bnb.x.shape != x.shape:
        return False
    return bool(torch.ops.tfx.pw_bwd_squeeze_supported(sh[3], sh[0], x.numel() // sh[3]))


def _conv_rows(x, w, stride, pad, dil) -> int:
    """Output pixels N*P*Q of an NHWC conv (the GEMM's M)."""
    n, h, wd = x.shape[0], x.shape[1], x.shape[2]
    r, s_ = w.shape[1], w.shape[2]
    p = (h + 2 * pad - dil * (r - 1) - 1) // stride + 1
    q = (wd + 2 * pad - dil * (s_ - 1) - 1) // stride + 1
    return n * p * q


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, w: Variable, stride, pad, dil, stats_into, sink, bnb):
        ctx.w, ctx.cfg, ctx.sink, ctx.bnb = w, (stride, pad, dil), sink, bnb
        ctx.native = _native.use_native(x)
        ctx.save_for_backward(x)
        # the layer's entry of its model's fusion plan (training steps only: eval passes no statistics
        # workspace); None = no plan covers this conv -- the same rules decide at call time
        lp = ctx.lp = fusion.layer_plan(w) if (ctx.native and stats_into is not None) else None
        if ctx.native:
            if _flip_ok(w, stride, pad, dil):
                w.store.flip_stale = True  # the weights may have changed since the last refresh
            tp = fusion.carried(x, "tail")
            if tp is not None and not tp.done:
                if lp is not None:
                    want = lp.fwd if (lp.pre is None and lp.fwd in _FUSED_INPUT) else "materialize"
                else:
                    want = _fwd_choice_unplanned(x, w, stride, pad, dil, stats_into, tp)
                ok_ws = isinstance(stats_into, BNWorkspace) and x.is_contiguous()
                if want == "conv3x3_fwd_fused":
                    if ok_ws and tp.res is None:
                        # BN + ReLU of the input applied on load, 3x3 conv from a halo tile, the output
                        # BN's statistics (conv3x3_fused.hip); x stays unwritten until something reads it
                        ws = stats_into
                        y, ws.pending_save = torch.ops.tfx.conv3x3_fwd_fused(tp.x, tp.save, w.value,
                                                                             ws.get(x.device), *ws.finalize_args)
                        ctx.pending_in = tp
                        CONV3_FWD_CALLS[0] += 1
                        fusion.note("bn_on_load", w.name, "conv3x3_fwd_fused")
                        return y
                    fusion.miss(w.name, want, "input is not a deferred plain BN")
                elif want == "igemm_fwd_a_scale":
                    if ok_ws and tp.res is None:
                        # a plain ReLU BN applied on load by this single-k-tile 1x1 conv (igemm a_scale):
                        # x stays unwritten (the fused backward forms it on load too)
                        ws = stats_into
                        y, ws.pending_save = torch.ops.tfx.conv_fwd_bn_in(tp.x, tp.save, w.value, ws.get(x.device),
                                                                          *ws.finalize_args)
                        ctx.pending_in = tp
                        PW_APPLY_CALLS[0] += 1
                        fusion.note("bn_on_load", w.name, "igemm_fwd_a_scale")
                        return y
                    fusion.miss(w.name, want, "input is not a deferred plain BN")
                elif want == "pw_fwd_squeeze":
                    if ok_ws and tp.res is not None and tp.mask is not None:
                        # the previous block's tail apply + this conv + its BN statistics in one launch:
                        # x (and the tail's mask bits) are written here (pw_fwd.hip)
                        ws = stats_into
                        y, ws.pending_save = torch.ops.tfx.pw_fwd_squeeze(
                            tp.x, tp.save, tp.res, tp.res_save, w.value, x, tp.mask, ws.get(x.device),
                            *ws.finalize_args)
                        tp.done = True
                        PW_SQUEEZE_CALLS[0] += 1
                        fusion.note("block_boundary_fwd", w.name, "pw_fwd_squeeze")
                        return y
                    fusion.miss(w.name, want, "input is not a deferred residual tail")
                fusion.note("layerwise", w.name, "bn_apply_into")
                tp.materialize()
            elif lp is not None and lp.fwd in _FUSED_INPUT:
                fusion.miss(w.name, lp.fwd, "input already written")
            if isinstance(stats_into, BNWorkspace):
                ws = stats_into
                if lp is not None:
                    stem = lp.fwd == "stem_fwd"
                else:
                    stem = fusion.knob("stem_wgrad") and _stem_ok(x, w, stride, pad, dil)
                # epilogue statistics, then the finalize: the BN only applies
                y, ws.pending_save = torch.ops.tfx.conv_fwd_bn(x.contiguous(), w.value, stride, pad, dil,
                                                               ws.get(x.device), *ws.finalize_args)
                fusion.note("bn_epilogue", w.name, "stem_fwd" if stem else "igemm_fwd_stats")
                return y
            if stats_into is not None:
                fusion.note("bn_epilogue", w.name, "igemm_fwd_stats_only")
                return torch.ops.tfx.conv_fwd_stats(x.contiguous(), w.value, stride, pad, dil, stats_into)
            fusion.note("conv", w.name, "igemm_fwd")
            return torch.ops.tfx.conv_fwd(x.contiguous(), w.value, stride, pad, dil)
        return _conv_ref(x, w.value.to(x.dtype), stride, pad, dil)

    @staticmethod
    def backward(ctx, gy, *unused):
        (x,) = ctx.saved_tensors
        w = ctx.w
        stride, pad, dil = ctx.cfg
        need_dx = ctx.needs_input_grad[0]
        tp = getattr(ctx, "pending_in", None)
        lazy = fusion.carried(gy, "lazy_bnbwd") if ctx.native else None
        lp = ctx.lp
        planned = lp.bwd if lp is not None else None

        def allowed(kernel):  # the plan's fused backward for this layer (no plan: every rule may fire)
            return lp is None or planned == kernel

        if tp is not None and not tp.done and lazy is not None and need_dx and allowed("conv3x3_bwd_fused") \
                and _conv3_bwd_fused_ok(w, lazy, ctx.bnb, tp):
            # the stage-1 3x3 conv's whole backward: the output BN's backward apply and the input BN's ReLU
            # output formed on load, data + weight gradient, the input BN's backward partials
            # (conv3x3_fused.hip) -- neither dy nor x is ever written
            bnb = ctx.bnb
            dx, bnb.red = torch.ops.tfx.conv3x3_bwd_fused(lazy.g.contiguous(), lazy.x, lazy.save, lazy.red, tp.x,
                                                          tp.save, w.value, w.grad, bnb.ws, bnb.dgamma, bnb.dbeta)
            CONV3_BWD_CALLS[0] += 1
            fusion.note("conv3_fused_bwd", w.name, "conv3x3_bwd_fused")
            dx = _negctl("conv3_fused_bwd", dx, w)
            _grad_ready(w)
            return dx, None, None, None, None, None, None, None, None
        if planned == "conv3x3_bwd_fused":
            fusion.miss(w.name, planned, "no fusible lazy gradient / pending input")
        expand = (ctx.native and lazy is not None and need_dx and allowed("pw_bwd_expand")
                  and _pw_expand_ok(x, w, stride, pad, dil, lazy, ctx.sink))
        if tp is not None and not (tp.res is None and expand):
            tp.materialize()  # the forward applied the input BN on load only
        if ctx.native:
            if lazy is not None:
                if need_dx and allowed("pw_bwd_squeeze") and _pw_squeeze_bwd_ok(x, w, stride, pad, dil, lazy, ctx.sink,
                                                                                ctx.bnb):
                    # BN1's backward apply + this conv's data AND weight gradient in one launch, the
                    # residual branch's masked gradient added and the previous tail BN's backward
                    # partials reduced in the dx epilogue (pw_bwd.hip F1)
                    add, amask, _ = _unpack_sink(ctx.sink.take())
                    bnb = ctx.bnb
                    dx, bnb.red = torch.ops.tfx.pw_bwd_squeeze(
                        lazy.g.contiguous(), lazy.x, lazy.save, lazy.red, x, w.value, w.grad, add.contiguous(), amask,
                        bnb.x, bnb.save, bnb.mask, bnb.ws, bnb.dgamma, bnb.dbeta)
                    PW_SQUEEZE_BWD_CALLS[0] += 1
                    fusion.note("lazy_bn_bwd", w.name, "pw_bwd_squeeze")
                    dx = _negctl("lazy_bn_bwd", dx, w)
                    _grad_ready(w)
                    return dx, None, None, None, None, None, None, None, None
                if expand:
                    # the tail BN's backward apply + this conv's data AND weight gradient in one
                    # launch; dy never written (pw_bwd.hip).  The BN2 backward partials of dx ride along.
                    # a2_lazy: the forward applied BN2 on load (x never written) -- formed on load here too
                    a2_lazy = tp is not None and not tp.done and tp.res is None
                    bnb = ctx.bnb
                    use_bnb = bnb is not None and bnb.mask is None and not bnb.deferred and bnb.red is None \
                        and x.numel() * x.element_size() <= _BNB_MAX_BYTES
                    # projection block: the shortcut BN's backward reduction too (F3-SEC)
                    rb = lazy.sec if lazy.dy is None else None
                    dx, red2, red_sc = torch.ops.tfx.pw_bwd_expand(
                        lazy.g.contiguous(), lazy.x, lazy.mask, lazy.save, lazy.red, tp.x if a2_lazy else x,
                        w.value, w.grad,
                        bnb.x if use_bnb else None, bnb.save if use_bnb else None, bool(use_bnb and bnb.relu),
                        bnb.ws if use_bnb else None, bnb.dgamma if use_bnb else None,
                        bnb.dbeta if use_bnb else None, rb.x if rb else None, rb.save if rb else None,
                        rb.ws if rb else None, rb.dgamma if rb else None, rb.dbeta if rb else None,
                        tp.save if a2_lazy else None)
                    if use_bnb:
                        bnb.red = red2
                    if rb is not None:
                        rb.red, rb.sec_lazy = red_sc, None
                    PW_EXPAND_CALLS[0] += 1
                    fusion.note("lazy_bn_bwd", w.name, "pw_bwd_expand")
                    dx = _negctl("lazy_bn_bwd", dx, w)
                    _grad_ready(w)
                    return dx, None, None, None, None, None, None, None, None
                if planned in ("pw_bwd_squeeze", "pw_bwd_expand"):
                    fusion.miss(w.name, planned, "the lazy gradient / sink state does not fit")
                fusion.note("layerwise", w.name, "bn_bwd_apply")
                gy = lazy.materialize()
            elif planned in ("pw_bwd_squeeze", "pw_bwd_expand"):
                fusion.miss(w.name, planned, "the output gradient arrived materialised")
            gy = gy.contiguous()
            sink = ctx.sink
            stem_w = (planned == "stem_wgrad") if lp is not None else (fusion.knob("stem_wgrad") and
                                                                        _stem_ok(x, w, stride, pad, dil))
            if not need_dx and w.trainable and stem_w and not _pending_sr(w.store):
                # the CIFAR stem (8 padded input channels, no input gradient): one block per image (stem.hip)
                torch.ops.tfx.stem_wgrad(gy, x.contiguous(), w.grad, _stem_ws(w.store, gy.device, w.shape[0]))
                STEM_WGRAD_CALLS[0] += 1
                fusion.note("stem_kernels", w.name, "stem_wgrad")
                _grad_ready(w)
                return None, None, None, None, None, None, None, None, None
            dx = None
            sr_bnb = None
            if need_dx:
                bnb = ctx.bnb
                if bnb is not None and stride == 1 and (sink is None or sink.mode == "consume") \
                        and x.numel() * x.element_size() <= _BNB_MAX_BYTES:
                    # dx is the complete gradient of the BN output x: the epilogue also reduces
                    # that BN's backward (sum g', sum g' xhat, dgamma, dbeta) -- see BNBackwardFusion
                    add, amask, s2 = _unpack_sink(sink.take()) if sink is not None else (None, None, False)
                    fusion.note("bn_epilogue", w.name, "igemm_dgrad_bnb" + ("+addend" if add is not None else ""))
                    if w.trainable:
                        # partials stay in the slots; the weight-gradient launch below reduces them in
                        # tail blocks of its grid (conv_wgrad_sr): no bn_slot_reduce launch
                        dx, _ = torch.ops.tfx.conv_dgrad_bn(
                            gy, w.value, list(x.shape), stride, pad, dil, add, bnb.x, bnb.save, bnb.mask, bnb.relu,
                            bnb.ws, None, None, amask, False, s2, _wflip(w, stride, pad, dil))
                        sr_bnb = bnb
                    else:
                        dx, bnb.red = torch.ops.tfx.conv_dgrad_bn(
                            gy, w.value, list(x.shape), stride, pad, dil, add, bnb.x, bnb.save, bnb.mask, bnb.relu,
                            bnb.ws, bnb.dgamma, bnb.dbeta, amask, True, s2, _wflip(w, stride, pad, dil))
                elif sink is not None and sink.mode == "consume":
                    # last consumer of x in backward order: fold the other branch's gradient in
                    add, amask, s2 = _unpack_sink(sink.take())
                    fusion.note("grad_sink", w.name, "igemm_dgrad_addend")
                    dx = torch.ops.tfx.conv_dgrad(gy, w.value, list(x.shape), stride, pad, dil, add, amask, s2,
                                                  _wflip(w, stride, pad, dil))
                elif sink is not None and sink.accept_s2 and stride == 2 and pad == 0 and w.shape[1] == 1 \
                        and w.shape[2] == 1 and x.shape[-1] % 8 == 0:
                    # 1x1 stride-2 branch: its input gradient is nonzero only at the even pixels --
                    # compute it on the strided grid (a 1x1 stride-1 data gradient) and park it compact
                    n, h, wd, c = x.shape
                    dxc = torch.ops.tfx.conv_dgrad(gy, w.value, [n, gy.shape[1], gy.shape[2], c], 1, 0, dil, None)
                    sink.put(("s2", dxc))
                    fusion.note("s2_addend", w.name, "igemm_dgrad_compact")
                    dx = None
                else:
                    dx = torch.ops.tfx.conv_dgrad(gy, w.value, list(x.shape), stride, pad, dil, None, None, False,
                                                  _wflip(w, stride, pad, dil))
                    if sink is not None:  # mode "produce": park it for the last consumer
                        sink.put(dx)
                        dx = None
                    elif bnb is not None and stride == 2 and fusion.knob("sr_defer") and w.trainable and bnb.mask is None \
                            and not bnb.deferred and bnb.red is None:
                        # dx is the complete output gradient of the BN that produced x: its backward
                        # partials go into the BN's slots now, their reduction rides in the tail of the
                        # weight-gradient launch below (no bn_bwd reduce + slot-reduce pair later)
                        torch.ops.tfx.bn_bwd_reduce_into(dx, bnb.x, bnb.save, bnb.relu, None, bnb.ws)
                        sr_bnb = bnb
            if w.trainable:
                pend = _pending_sr(w.store)
                if sr_bnb is not None or (fusion.knob("sr_take") and pend and pend[0].ws.device == gy.device):
                    take = fusion.knob("sr_take") and pend and pend[0].ws.device == gy.device
                    t2 = pend.pop(0) if take else None
                    t1 = sr_bnb
                    r1, r2 = torch.ops.tfx.conv_wgrad_sr2(
                        gy, x, w.grad, stride, pad, dil, True, t1.ws if t1 is not None else None,
                        t1.dgamma if t1 is not None else None, t1.dbeta if t1 is not None else None,
                        t2.ws if t2 is not None else None, t2.x.shape[-1] if t2 is not None else 0,
                        t2.dgamma if t2 is not None else None, t2.dbeta if t2 is not None else None)
                    if t1 is not None:
                        t1.red = r1
                    if t2 is not None:
                        t2.red, t2.sr_pending = r2, False
                    fusion.note("deferred_slot_reduce", w.name, "igemm_wgrad_sr%d" % ((t1 is not None) + (t2 is not None)))
                    _grad_ready(w)
                else:
                    torch.ops.tfx.conv_wgrad(gy, x, w.grad, stride, pad, dil, True)
                    fusion.note("conv", w.name, "igemm_wgrad")
                    _grad_ready(w)
            return dx, None, None, None, None, None, None, None, None
        dx = _ref_param_grads(lambda xx, ww: _conv_ref(xx, ww, stride, pad, dil), x, [w], gy, need_dx)
        return dx, None, None, None, None, None, None, None, None


def conv2d(x: torch.Tensor, w: Variable, stride: int = 1, pad: int = 0, dil: int = 1,
           bn_stats_into=None, grad_sink: Optional["GradSink"] = None, fuse_input_bn_backward: bool = False):
    """NHWC conv, weight stored [Ko, R, S, C]. GPU: implicit-GEMM MFMA kernels (igemm.hip).

    ``bn_stats_into`` = the following BN layer's workspace: a raw slot tensor (the epilogue
    produces the per-channel sum / sum-of-squares of ``y``; the BN finalizes) or a
    :class:`BNWorkspace` with ``finalize_args`` set (the finalize runs right after the conv; the BN
    only applies).  ``fuse_input_bn_backward``: the caller guarantees this conv's
    data gradient is the COMPLETE gradient of ``x`` (sole consumer, or the GradSink consumer); if
    ``x`` came from :func:`batch_norm` its backward reduction then runs in the dgrad epilogue.
    Ignored on CPU."""
    gpu = x.device.type == "cuda"
    ws = bn_stats_into if (bn_stats_into is not None and gpu) else None
    bnb = fusion.carried(x, "bnb") if (gpu and fuse_input_bn_backward) else None
    return _Conv2d.apply(x, w.store.anchor, w, stride, pad, dil, ws, grad_sink if gpu else None, bnb)


def _unpack_sink(item):
    """A parked gradient is a tensor, ``(g, mask)``: a residual BN's output gradient whose ReLU
    mask the consumer applies in its epilogue (the masked copy is never written), or
    ``("s2", g)``: a 1x1 stride-2 branch's gradient at the even pixels only (compact grid; the
    consumer adds it there and nothing elsewhere -- no zero-filled full-size tensor).
    Returns (addend, mask, compact_stride2)."""
    if isinstance(item, tuple):
        if isinstance(item[0], str):
            assert item[0] == "s2"
            return item[1], None, True
        return item[0], item[1], False
    return item, None, False


class GradSink:
    """Fuses the gradient sum of a tensor with two consumers (a ResNet block input feeds conv1 and
    the residual / projection branch).  The branch that runs FIRST in backward ("produce") parks
    its input-gradient here instead of returning it to autograd; the consumer that runs LAST
    ("consume", conv1's data-gradient) adds it in its GEMM epilogue -- no separate add kernel.
    Backward order is fixed by autograd's sequence numbers: conv1 is created first in the block,
    so it runs last (the ``take`` assertion guards this).

    ``accept_masked`` (set on the producer by a block whose consumer is a stride-1 conv): the
    residual BN may park ``(g, relu_mask)`` instead of writing the masked gradient tensor.
    ``accept_s2`` (same condition): a 1x1 stride-2 projection may park its gradient compact on the
    strided grid, ``("s2", g)``."""

    def __init__(self, mode: str):
        assert mode in ("produce", "consume")
        self.mode = mode
        self.buf = None
        self.peer: Optional["GradSink"] = None
        self.accept_masked = False
        self.accept_s2 = False

    @staticmethod
    def pair():
        prod, cons = GradSink("produce"), GradSink("consume")
        prod.peer = cons
        cons.peer = prod
        return prod, cons

    def put(self, g):
        tgt = self.peer if self.peer is not None else self
        assert tgt.buf is None, "gradient sink already holds a gradient"
        tgt.buf = g

    def take(self):
        g, self.buf = self.buf, None
        assert g is not None, "gradient sink consumed before its producer ran"
        return g


class BNWorkspace:
    """Per-BN-layer persistent f32 workspace: [NSLOT][2][C] statistics slots, zero between uses.
    The producing conv's epilogue adds the forward statistics into them and the finalize that
    follows re-zeroes them; in backward the consuming conv's data-gradient epilogue adds the BN
    backward partials and the slot reduction (a weight-gradient launch's tail blocks, or
    bn_slots_reduce) re-zeroes them.  With ``finalize_args`` set the producing conv finalizes the
    statistics and leaves [mean | invstd | scale | shift] in ``pending_save``."""
    NSLOT = 64  # = tfx::NSLOT (csrc/include/tfx_kernels.h), checked on first GPU use

    def __init__(self, channels: int, store=None):
        self.c = channels
        self.buf = None
        self.finalize_args = None
        self.pending_save = None
        self.store = store

    def get(self, device) -> torch.Tensor:
        if self.buf is None or self.buf.device != device:
            if device.type == "cuda" and _native.use_native_device(device):
                assert int(torch.ops.tfx.bn_nslot()) == self.NSLOT, "BNWorkspace.NSLOT != tfx::NSLOT"
            self.buf = torch.zeros(self.NSLOT * 2 * self.c, dtype=torch.float32, device=device)
        return self.buf


class BNBackwardFusion:
    """What a consumer conv's data-gradient epilogue needs to reduce a BN's backward (attached to
    the BN output as fusion carrier "bnb"): the BN input, its [mean|invstd|scale|shift], the residual
    layer's ReLU mask bits, the slot workspace and the parameter-gradient views.  The conv fills
    ``red`` ([sum g' | sum g' xhat]) (or a later weight-gradient launch does, from the slots); the BN
    backward then runs only its apply pass."""
    __slots__ = ("x", "save", "mask", "relu", "ws", "dgamma", "dbeta", "red", "in_mask", "deferred",
                 "sr_pending", "sec_lazy", "store")

    def __init__(self, x, save, mask, relu, ws, dgamma, dbeta, store=None):
        self.x, self.save, self.mask, self.relu, self.ws = x, save, mask, relu, ws
        self.store = store  # the model's VariableStore: its pending-reduction list (_pending_sr)
        self.dgamma, self.dbeta, self.red = dgamma, dbeta, None
        # set by a residual consumer (bn_bwd_apply_sec): the incoming gradient arrives unmasked,
        # the true gradient is g * in_mask (the consumer's ReLU mask bits)
        self.in_mask = None
        # the BN's output was never written (batch_norm(defer_output=True)): its only consumer, a
        # residual BN, normalizes ``x`` with ``save`` on the fly
        self.deferred = False
        # backward partials sit in ``ws`` waiting for a later launch to reduce them (_pending_sr)
        self.sr_pending = False
        # a projection tail's LazyBNGrad that still owes this (shortcut) BN's reduction
        self.sec_lazy = None


# ====================================================================== batch norm (+res, +relu)
def _bn_ref(x, gamma, beta, rm, rv, momentum, eps, res, relu, training, update=True):
    xf = x.float()
    dims = tuple(range(x.dim() - 1))
    if training:
        mean = xf.mean(dims)
        var = xf.var(dims, unbiased=False)
        if update and rm is not None:
            n = xf.numel() // xf.shape[-1]
            with torch.no_grad():
                rm.mul_(1 - momentum).add_(mean.detach() * momentum)
                rv.mul_(1 - momentum).add_(var.detach() * (n / max(n - 1, 1)) * momentum)
    else:
        mean, var = rm, rv
    y = (xf - mean) * torch.rsqrt(var + eps)
    if gamma is not None:
        y = y * gamma + beta
    if res is not None:
        y = y + res.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def _pending_sr(store) -> List["BNBackwardFusion"]:
    """The model's BN layers whose backward partials wait in their slot workspace for the next
    weight-gradient launch OF THE SAME MODEL to reduce them in its tail blocks (conv_wgrad_sr2) -- or for
    their own backward to reduce them (bn_slots_reduce) if no such launch came first."""
    st = _model_state(store)
    lst = st.get("pending_sr")
    if lst is None:
        lst = st["pending_sr"] = []
    return lst


def pending_slot_reductions(store=None) -> List["BNBackwardFusion"]:
    """The deferred BN-backward reductions still pending for ``store``'s model (tests: empty after a step)."""
    return list(_pending_sr(store))


# single-launch mean loss for small batches (else: per-row kernel + mean + scale launches)
_XENT_MEAN_MAX = 1024


def reset_pending_slot_reductions(store=None) -> None:
    """Forget ``store``'s deferred reductions of an abandoned step (an exception part-way through)."""
    pend = _pending_sr(store)
    for b in pend:
        b.sr_pending = False
    pend.clear()


def _resolve_pending(b: "BNBackwardFusion") -> None:
    if b.sr_pending:
        pend = _pending_sr(b.store)
        if b in pend:
            pend.remove(b)
        b.red = torch.ops.tfx.bn_slots_reduce(b.ws, b.x.shape[-1], b.dgamma, b.dbeta)
        b.sr_pending = False


_ZERO = {}


def _zero_scalar(dtype, device) -> torch.Tensor:
    """A persistent 0-d zero (the never-read placeholder of a BN output that is not written): no fill
    launch per step, and safe inside a captured graph (allocated once, outside any capture)."""
    key = (dtype, str(device))
    t = _ZERO.get(key)
    if t is None:
        t = torch.zeros((), dtype=dtype, device=device)
        if not (t.is_cuda and torch.cuda.is_current_stream_capturing()):  # never cache a graph-pool tensor
            _ZERO[key] = t
    return t


def _vec_ok(C):
    return C % 8 == 0 and C // 8 <= 256 and 256 % (C // 8) == 0


def _res_bn_sec_ok(ctx, gy, mask, relu, masked):
    """Can this residual BN's backward apply also reduce its residual's BN (bn_bwd_apply_sec)?"""
    rb = ctx.res_bnb
    if rb is None or not ctx.has_res or masked or ctx.res_sink is not None or rb.red is not None:
        return False
    if rb.relu or rb.mask is not None or rb.ws is None:
        return False
    if relu and mask is None:
        return False
    return rb.x.shape == gy.shape and rb.x.is_contiguous() and _vec_ok(gy.shape[-1])


class _BatchNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, anchor, gamma: Optional[Variable], beta: Optional[Variable], rm, rv, momentum, eps, relu,
                training, ws, stats_ready, res_sink, wsobj, bnb_out, res_bnb, defer, lazy_bwd, defer_apply):
        # res_bnb: (BNBackwardFusion of the residual, fuse its backward here); defer: the output is
        # only ever this layer's consumer's residual -- never written (see batch_norm); lazy_bwd: the
        # input gradient may be returned unmaterialised (LazyBNGrad) -- the producer is a conv
        ctx.lazy_bwd = bool(lazy_bwd)
        ctx.gamma, ctx.beta, ctx.cfg = gamma, beta, (rm, rv, momentum, eps, relu, training)
        ctx.res_sink = res_sink
        res_bnb, res_sec = res_bnb if res_bnb is not None else (None, False)
        ctx.res_bnb = res_bnb if res_sec else None
        ctx.native = _native.use_native(x)
        ctx.has_res = res is not None
        ctx.bnb = None
        g_t = gamma.master if gamma is not None else None
        b_t = beta.master if beta is not None else None
        if ctx.native:
            x = x.contiguous()
            if ws is None:
                ws = torch.zeros(BNWorkspace.NSLOT * 2 * x.shape[-1], dtype=torch.float32,
                                 device=x.device)
                stats_ready = False
            ctx.ws = ws
            mask = None
            pending = training and wsobj is not None and wsobj.pending_save is not None
            # residual = a BN output that was never written: normalize its input on the fly here
            # (bn_apply_res_bn), or materialize it for the other paths (autograd still routes its
            # gradient to that BN: the lazy tensor stays this Function's input)
            _settle(res)
            res_lazy = res is not None and res_bnb is not None and res_bnb.deferred
            fuse_res = res_lazy and pending and relu
            # residual + ReLU tail whose only first reader is the next block's conv1: leave the apply
            # to that conv (TailPending) -- it forms out / mask while loading its input
            defer_tail = defer_apply and fusion.knob("defer_tail") and pending and relu and res is not None and \
                x.shape[-1] % 8 == 0 and (fuse_res or not res_lazy)
            # plain ReLU BN whose only reader is a 3x3 conv that applies it on load
            defer_plain = defer_apply and fusion.knob("defer_bn_in") and pending and relu and res is None and x.shape[-1] % 8 == 0
            if res_lazy and not fuse_res:
                res = torch.ops.tfx.bn_apply_train(res_bnb.x, None, res_bnb.save, False)[0]
            defer_out = defer and pending and res is None and bnb_out is not None and _vec_ok(x.shape[-1])
            if pending:
                # the producing conv's epilogue already finalized the statistics (conv_fwd_bn)
                save, wsobj.pending_save = wsobj.pending_save, None
                if defer_plain:
                    y = torch.empty_like(x)
                    fusion.carry(y, "tail", TailPending(x, save, None, None, y, None))
                elif defer_tail:
                    y = torch.empty_like(x)
                    mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)
                    fusion.carry(y, "tail", TailPending(x, save, res_bnb.x if fuse_res else res.contiguous(),
                                                        res_bnb.save if fuse_res else None, y, mask))
                elif fuse_res:
                    y, mask = torch.ops.tfx.bn_apply_res_bn(x, res_bnb.x, save, res_bnb.save, relu)
                elif defer_out:
                    y = _zero_scalar(x.dtype, x.device).expand(x.shape)
                else:
                    y, mask = torch.ops.tfx.bn_apply_train(x, res, save, relu)
            elif training:
                y, save, mask = torch.ops.tfx.bn_fwd_train(x, g_t, b_t, rm, rv, momentum, eps, res, relu, ws,
                                                           bool(stats_ready))
            else:
                y, save = torch.ops.tfx.bn_fwd_eval(x, g_t, b_t, rm, rv, eps, res, relu)
            if mask is not None and mask.numel() == 0:
                mask = None
            # residual + ReLU: the backward needs only the 1-bit ReLU mask, not the residual tensor
            assert not fuse_res or mask is not None
            ctx.save_for_backward(x, None if mask is not None else res, save, mask)
            ctx.tp = fusion.carried(y, "tail") if (defer_plain or defer_tail) and pending else None
            if training and bnb_out is not None and (res is None or not relu or mask is not None) \
                    and x.shape[-1] % 8 == 0:
                train_p = gamma is not None and gamma.trainable
                ctx.bnb = BNBackwardFusion(x, save, mask, relu, ws, gamma.grad if train_p else None,
                                           beta.grad if train_p else None, gamma.store if gamma is not None else None)
                ctx.bnb.deferred = defer_out
                bnb_out.append(ctx.bnb)
            return y
        ctx.save_for_backward(x, res)
        with torch.no_grad():
            return _bn_ref(x, g_t, b_t, rm, rv, momentum, eps, res, relu, training)

    @staticmethod
    def backward(ctx, gy):
        rm, rv, momentum, eps, relu, training = ctx.cfg
        gamma, beta = ctx.gamma, ctx.beta
        if ctx.native:
            x, res, save, mask = ctx.saved_tensors
            if not training:
                raise RuntimeError("backward through eval-mode batch norm is not supported on the GPU path")
            if ctx.bnb is not None:
                if ctx.bnb.sec_lazy is not None:  # the tail's conv3 has not run yet: reduce here
                    ctx.bnb.sec_lazy.materialize()
                _resolve_pending(ctx.bnb)  # no weight-gradient launch took its deferred reduction
            train_p = gamma is not None and gamma.trainable
            gy = gy.contiguous()
            # residual gradient g' = gy * relu_mask: when the sink's consumer applies the mask itself
            # (stride-1 conv epilogue), park (gy, mask) and skip writing g' -- one full-size
            # tensor write less per identity block
            masked = ctx.has_res and ctx.res_sink is not None and mask is not None and \
                getattr(ctx.res_sink, "accept_masked", False) and relu
            if ctx.bnb is not None and ctx.bnb.red is not None and ctx.lazy_bwd and fusion.knob("lazy_bn_bwd") and relu \
                    and mask is not None and res is None and _res_bn_sec_ok(ctx, gy, mask, relu, masked) \
                    and x.shape[-1] % 4 == 0 \
                    and torch.ops.tfx.pw_bwd_expand_supported(x.shape[-1] // 4, x.numel() // x.shape[-1]):
                # projection tail: dx stays lazy and the shortcut BN's reduction is owed by it -- conv3's
                # fused backward forms both (pw_bwd.hip); the shortcut BN gets gy unmasked + the mask bits
                rb = ctx.res_bnb
                dx = _zero_scalar(x.dtype, x.device).expand(x.shape)
                lz = LazyBNGrad(gy, x, save, ctx.bnb.red, relu, mask, sec=rb)
                fusion.carry(dx, "lazy_bnbwd", lz)
                rb.sec_lazy = lz
                rb.in_mask, dres = mask, gy
                ctx.bnb.red = None
            elif ctx.bnb is not None and ctx.bnb.red is not None and _res_bn_sec_ok(ctx, gy, mask, relu, masked):
                # ... and the residual's own BN backward is reduced in the same pass
                rb = ctx.res_bnb
                p_t = rb.dgamma is not None
                # with a ReLU the residual gradient is gy * mask: hand the residual BN gy itself and
                # the mask bits instead of writing the masked copy
                pass_mask = relu
                # the residual BN's slot reduction is deferred to the tail of the next weight-gradient
                # launch (this block's conv3, which autograd runs before the residual BN)
                defer = fusion.knob("sr_defer")
                dx, dres, red2 = torch.ops.tfx.bn_bwd_apply_sec(gy, x, save, ctx.bnb.red, relu, mask, rb.x, rb.save,
                                                                 rb.ws, rb.dgamma if p_t else None,
                                                                 rb.dbeta if p_t else None, not pass_mask, not defer)
                if defer:
                    rb.red, rb.sr_pending = None, True
                    _pending_sr(rb.store).append(rb)
                else:
                    rb.red = red2
                if pass_mask:
                    rb.in_mask, dres = mask, gy
                ctx.bnb.red = None
            elif ctx.bnb is not None and ctx.bnb.red is not None and ctx.bnb.in_mask is not None:
                # gy arrived unmasked from a residual consumer: the apply's ReLU-mask path is g * mask
                assert not relu and not ctx.has_res
                dx, dres = torch.ops.tfx.bn_bwd_apply(gy, x, None, save, ctx.bnb.red, True, ctx.bnb.in_mask, False)
                ctx.bnb.red = ctx.bnb.in_mask = None
            elif ctx.bnb is not None and ctx.bnb.red is not None and ctx.lazy_bwd and fusion.knob("lazy_bn_bwd") and masked \
                    and res is None and relu and mask is not None:
                # residual + ReLU tail whose residual gradient is parked as (gy, mask): dx stays lazy --
                # the producing conv forms it on load (LazyBNGrad)
                dx = _zero_scalar(x.dtype, x.device).expand(x.shape)
                fusion.carry(dx, "lazy_bnbwd", LazyBNGrad(gy, x, save, ctx.bnb.red, relu, mask))
                dres = None
                ctx.bnb.red = None
            elif ctx.bnb is not None and ctx.bnb.red is not None and ctx.lazy_bwd and fusion.knob("lazy_bn_bwd") and relu \
                    and not ctx.has_res and mask is None and ctx.bnb.in_mask is None:
                # plain ReLU BN fed by a conv: dx stays lazy (LazyBNGrad, ReLU mask recomputed from x) --
                # a squeezing 1x1 producer forms it on load (pw_bwd.hip F1), any other materialises it
                dx = _zero_scalar(x.dtype, x.device).expand(x.shape)
                fusion.carry(dx, "lazy_bnbwd", LazyBNGrad(gy, x, save, ctx.bnb.red, relu, None))
                dres = None
                ctx.bnb.red = None
            elif ctx.bnb is not None and ctx.bnb.red is not None:
                # the consumer conv's dgrad epilogue reduced this backward (and dgamma / dbeta)
                dx, dres = torch.ops.tfx.bn_bwd_apply(gy, x, res, save, ctx.bnb.red, relu, mask, not masked)
                ctx.bnb.red = None
            else:
                dx, dres, red = torch.ops.tfx.bn_bwd(gy, x, res, save, relu, ctx.ws,
                                                     gamma.grad if train_p else None,
                                                     beta.grad if train_p else None, mask, not masked)
            if train_p:
                _grad_ready(gamma, beta)
            if ctx.has_res and ctx.res_sink is not None:
                ctx.res_sink.put((gy, mask) if masked else dres)
                dres = None
            return dx, (dres if ctx.has_res else None), None, None, None, None, None, None, None, None, None, None, None, \
                None, None, None, None, None, None, None
        x, res = ctx.saved_tensors
        with torch.enable_grad():
            xs = x.detach().requires_grad_(True)
            rs = res.detach().requires_grad_(True) if res is not None else None
            ps = [v.master.detach().clone().requires_grad_(True) if v is not None else None for v in (gamma, beta)]
            y = _bn_ref(xs, ps[0], ps[1], rm, rv, momentum, eps, rs, relu, training, update=False)
            leaves = [xs] + ([rs] if rs is not None else []) + [p for p in ps if p is not None]
            grads = list(torch.autograd.grad(y, leaves, gy))
        dx = grads.pop(0)
        dres = grads.pop(0) if rs is not None else None
        if gamma is not None:
            gamma.grad.add_(grads[0])
            beta.grad.add_(grads[1])
            _grad_ready(gamma, beta)
        return dx, dres, None, None, None, None, None, None, None, None, None, None, None, None, None, None, None, None, None, \
            None


def batch_norm(x, gamma: Optional[Variable], beta: Optional[Variable], running_mean, running_var, training=True,
               momentum=0.1, eps=1e-5, residual: Optional[torch.Tensor] = None, relu=False,
               workspace=None, stats_ready: bool = False,
               residual_grad_sink: Optional[GradSink] = None, fuse_residual_bn_backward: bool = False,
               defer_output: bool = False, lazy_backward: bool = False, defer_apply: bool = False):
    """Channels-last batch norm over all leading dims, with optional fused residual add + ReLU:
    ``y = relu(bn(x) + residual)`` (the ResNet bottleneck tail in one pass).

    ``workspace``: the layer's slot tensor or :class:`BNWorkspace` (then a statistics finalize
    done by the producing conv is picked up).  On the GPU in training mode the output carries a
    :class:`BNBackwardFusion` (fusion carrier "bnb") for a consumer conv that opts into reducing this
    BN's backward in its data-gradient epilogue.

    ``fuse_residual_bn_backward``: ``residual`` is another BN's output used ONLY here (a ResNet
    projection shortcut), so its gradient is exactly this layer's residual gradient -- reduce that
    BN's backward inside this layer's backward apply (one full pass over two tensors less).

    ``defer_output``: the caller promises the output is used ONLY as the ``residual`` of one
    later batch_norm (with ``fuse_residual_bn_backward``).  On the fused GPU path the output is then
    never written (a zero-stride placeholder that keeps the autograd edge); the consumer
    normalizes this BN's input on the fly.

    ``lazy_backward``: the caller promises ``x`` is the output of :func:`conv2d` (used nowhere else),
    so the input gradient may reach it unmaterialised (:class:`LazyBNGrad`).

    ``defer_apply`` (a residual + ReLU tail): the caller promises the output's FIRST reader is a
    1x1 :func:`conv2d` with a BN workspace (the next bottleneck's conv1); on the fused GPU path the
    apply pass is left to that conv (:class:`TailPending`), which writes the output while loading it."""
    anchor = gamma.store.anchor if gamma is not None else None
    wsobj = workspace if isinstance(workspace, BNWorkspace) else None
    if wsobj is not None:
        workspace = wsobj.get(x.device) if x.device.type == "cuda" else None
    if x.device.type != "cuda":
        workspace = None
    sink = residual_grad_sink if (x.device.type == "cuda" and residual is not None) else None
    bnb_out = [] if (x.device.type == "cuda" and training) else None
    rb = fusion.carried(residual, "bnb") if residual is not None else None
    res_bnb = None
    if rb is not None and (rb.deferred or fuse_residual_bn_backward):
        res_bnb = (rb, bool(fuse_residual_bn_backward))
    y = _BatchNorm.apply(x, residual, anchor, gamma, beta, running_mean, running_var, momentum, eps, relu, training,
                         workspace, stats_ready and training and workspace is not None, sink, wsobj, bnb_out, res_bnb,
                         bool(defer_output), bool(lazy_backward), bool(defer_apply))
    if bnb_out:
        fusion.carry(y, "bnb", bnb_out[0])
    return y


# ====================================================================== dense
def _pad_to(t: torch.Tensor, dim: int, mult: int) -> torch.Tensor:
    n = t.shape[dim]
    r = (-n) % mult
    if r == 0:
        return t
    pad = [0, 0] * (t.dim() - 1 - dim) + [0, r]
    return F.pad(t, pad)


def _linear_ref(x, w, b=None, relu=False):
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


class _Linear(torch.autograd.Function):
    """y = act(x @ W^T + b) with W stored [out, in] (bf16 MFMA GEMM on GPU)."""

    @staticmethod
    def forward(ctx, x, anchor, w: Variable, b: Optional[Variable], relu: bool):
        ctx.w, ctx.b, ctx.relu = w, b, relu
        ctx.native = _native.use_native(x) and x.dtype == torch.bfloat16
        if ctx.native:
            out_f = w.shape[0]
            xp = _pad_to(x.contiguous(), 1, 8)
            # W is the K-major B operand: rows past out_f are zero-filled by the loader's bounds, so
            # only its K (input) dim needs the 8-multiple -- no padded copy of W or the bias
            wp = _pad_to(w.value, 1, 8)
            bias = b.master if b is not None else None
            y = torch.ops.tfx.gemm(xp, wp, False, True, bias, relu, False)
            if y.shape[1] != out_f:
                y = y[:, :out_f].contiguous()
            ctx.save_for_backward(x, y if relu else None)
            return y
        ctx.save_for_backward(x, None)
        with torch.no_grad():
            return _linear_ref(x, w.value.to(x.dtype) if x.dtype != torch.float32 else w.master,
                               b.master if b is not None else None, relu)

    @staticmethod
    def backward(ctx, gy):
        x, y = ctx.saved_tensors
        w, b, relu = ctx.w, ctx.b, ctx.relu
        need_dx = ctx.needs_input_grad[0]
        if ctx.native and not relu and w.shape[0] <= 64 and x.dim() == 2 and w.value.is_contiguous():
            # few outputs (classifier head): dx, dW, db in one launch (elementwise.hip linear_small_bwd)
            g = gy.to(torch.bfloat16).contiguous()
            bias_grad = b.grad if (b is not None and b.trainable) else None
            dx = torch.ops.tfx.linear_small_bwd(g, x.contiguous(), w.value, need_dx,
                                                w.grad if w.trainable else None, bias_grad)
            _grad_ready(w if w.trainable else None, b if bias_grad is not None else None)
            return (dx if need_dx else None), None, None, None, None
        if ctx.native:
            g = gy.to(torch.bfloat16).contiguous()
            bias_grad = b.grad if (b is not None and b.trainable) else None
            if relu or bias_grad is not None:
                # one pass: ReLU mask (g' = g * [y > 0]) and the bias column sums
                yy = y.to(torch.bfloat16).contiguous() if relu else g
                gm = torch.ops.tfx.act_bwd_colsum(g, yy, 1 if relu else 0, bias_grad)
                if relu:
                    g = gm
            out_f, in_f = w.shape
            gp = _pad_to(g, 1, 8)
            dx = None
            if need_dx:
                wp = _pad_to(_pad_to(w.value, 1, 8), 0, 8)
                dx = torch.ops.tfx.gemm(gp, wp, False, False, None, False, False)
                if dx.shape[1] != in_f:
                    dx = dx[:, :in_f].contiguous()
            if w.trainable:
                xp = _pad_to(x.contiguous(), 1, 8)
                if gp.shape[1] == out_f and xp.shape[1] == in_f:
                    torch.ops.tfx.gemm_into(gp, xp, True, False, w.grad, True)
                else:
                    tmp = torch.zeros(gp.shape[1], xp.shape[1], device=x.device, dtype=torch.float32)
                    torch.ops.tfx.gemm_into(gp, xp, True, False, tmp, True)
                    w.grad.add_(tmp[:out_f, :in_f])
            _grad_ready(w if w.trainable else None, b if bias_grad is not None else None)
            return dx, None, None, None, None
        params = [w] + ([b] if b is not None else [])
        fn = (lambda xx, ww, bb: _linear_ref(xx, ww, bb, relu)) if b is not None else \
            (lambda xx, ww: _linear_ref(xx, ww, None, relu))
        dx = _ref_param_grads(fn, x, params, gy, need_dx)
        return dx, None, None, None, None


def linear(x, w: Variable, b: Optional[Variable] = None, relu: bool = False):
    return _Linear.apply(x, w.store.anchor, w, b, relu)


# ====================================================================== pooling
class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        ctx.native = _native.use_native(x)
        if ctx.native:
            return torch.ops.tfx.gap_fwd(_settle(x).contiguous(), False)
        return x.mean(dim=(1, 2))

    @staticmethod
    def backward(ctx, gy):
        N, H, W, C = ctx.shape
        if ctx.native:
            return torch.ops.tfx.gap_bwd(gy.contiguous(), H, W)
        return (gy[:, None, None, :] / (H * W)).expand(N, H, W, C).contiguous()


def global_avg_pool(x):
    """NHWC [N,H,W,C] -> [N,C]."""
    return _GlobalAvgPool.apply(x)


def _pool_ref(x, k, s, pad, kind):
    xc = x.permute(0, 3, 1, 2)
    if kind == "max":
        y = F.max_pool2d(xc, k, s, pad)
    else:
        y = F.avg_pool2d(xc, k, s, pad, count_include_pad=False)
    return y.permute(0, 2, 3, 1).contiguous()


class _Pool2d(torch.autograd.Function):
    """NHWC k x k pooling (pool.hip). Max pool keeps a uint8 in-window argmax so the backward is a
    deterministic gather (no atomics); avg pool divides by the in-bounds window size."""

    @staticmethod
    def forward(ctx, x, k, s, pad, kind):
        ctx.cfg, ctx.shape = (k, s, pad, kind), x.shape
        ctx.native = _native.use_native(x) and x.dtype == torch.bfloat16
        if ctx.native:
            xc = x.contiguous()
            if kind == "max":
                y, arg = torch.ops.tfx.maxpool_fwd(xc, k, s, pad)
                ctx.save_for_backward(arg)
                return y
            ctx.save_for_backward()
            return torch.ops.tfx.avgpool_fwd(xc, k, s, pad)
        ctx.save_for_backward(x)
        return _pool_ref(x, k, s, pad, kind)

    @staticmethod
    def backward(ctx, gy):
        k, s, pad, kind = ctx.cfg
        _, H, W, _ = ctx.shape
        if ctx.native:
            g = gy.to(torch.bfloat16).contiguous()
            if kind == "max":
                (arg,) = ctx.saved_tensors
                return torch.ops.tfx.maxpool_bwd(g, arg, H, W, k, s, pad), None, None, None, None
            return torch.ops.tfx.avgpool_bwd(g, H, W, k, s, pad), None, None, None, None
        (x,) = ctx.saved_tensors
        with torch.enable_grad():
            xx = x.detach().requires_grad_(True)
            (dx,) = torch.autograd.grad(_pool_ref(xx, k, s, pad, kind), [xx], gy)
        return dx, None, None, None, None


def max_pool2d(x, ksize: int = 2, stride: Optional[int] = None, pad: int = 0):
    """tf.nn.max_pool on NHWC (``pad`` explicit; SAME for k=2,s=2 on even sizes is pad=0)."""
    return _Pool2d.apply(x, ksize, stride or ksize, pad, "max")


def avg_pool2d(x, ksize: int = 2, stride: Optional[int] = None, pad: int = 0):
    """tf.nn.avg_pool on NHWC; padded taps are excluded from the mean (TF semantics)."""
    return _Pool2d.apply(x, ksize, stride or ksize, pad, "avg")


# ====================================================================== losses / metrics
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, naive, unit_seed=False):
        ctx.native = _native.use_native(logits)
        ctx.unit_seed = False
        B, C = logits.shape
        if ctx.native:
            idx = labels.contiguous() if labels.dtype == torch.long else None
            dense = labels.float().contiguous() if labels.dtype != torch.long else None
            ctx.dtype = logits.dtype
            if B * ((C + 63) // 64) <= _XENT_MEAN_MAX:
                # one launch: the mean loss and dz (already in the logits' dtype when the caller
                # promises a unit seed gradient, so backward launches nothing)
                loss, dz = torch.ops.tfx.softmax_xent_mean(logits.contiguous(), idx, dense, naive,
                                                           bool(ctx.needs_input_grad[0]), bool(unit_seed))
                ctx.unit_seed = bool(unit_seed) and dz is not None and dz.dtype == logits.dtype
                ctx.save_for_backward(dz)
                return loss
            loss_rows, dz = torch.ops.tfx.softmax_xent(logits.contiguous(), idx, dense, naive, 1.0 / B,
                                                       bool(ctx.needs_input_grad[0]))
            ctx.save_for_backward(dz)
            return loss_rows.mean()
        ctx.save_for_backward(logits, labels)
        ctx.naive = naive
        return _xent_ref(logits, labels, naive)

    @staticmethod
    def backward(ctx, g):
        if ctx.native:
            (dz,) = ctx.saved_tensors
            if ctx.unit_seed:
                return dz, None, None, None
            # upstream scale (1.0 for loss.backward()) + cast in one HIP launch
            gs = g.reshape(1).float().contiguous()
            return torch.ops.tfx.scale_by_scalar(dz, gs, ctx.dtype == torch.bfloat16), None, None, None
        logits, labels = ctx.saved_tensors
        with torch.enable_grad():
            z = logits.detach().requires_grad_(True)
            loss = _xent_ref(z, labels, ctx.naive)
            (dz,) = torch.autograd.grad(loss, [z], g)
        return dz, None, None, None


def _xent_ref(logits, labels, naive):
    z = logits.float()
    if labels.dtype == torch.long:
        y = F.one_hot(labels, z.shape[1]).float()
    else:
        y = labels.float()
    if naive:  # reference parity: -sum(y * log(softmax(z))) (R/distributed/distributed.py:99,102)
        p = torch.softmax(z, dim=1)
        return (-(y * torch.log(p)).sum(1)).mean()
    return (-(y * torch.log_softmax(z, dim=1)).sum(1)).mean()


def softmax_cross_entropy(logits, labels, naive: bool = False, unit_seed: bool = False):
    """Mean softmax cross-entropy. ``labels``: int64 class ids or dense [B,C] targets.
    ``naive=True`` reproduces TF1's ``reduce_mean(-reduce_sum(y_*log(softmax(z))))``.
    ``unit_seed=True`` is the caller's promise that backward is seeded with exactly 1 (the loss is
    the root, ``loss.backward()``): the gradient then leaves the forward launch ready to use."""
    return _SoftmaxXent.apply(logits, labels, naive, unit_seed)


# ---- fused classifier head (training step): gap -> linear -> mean softmax xent, one launch (head.hip)
HEAD_FUSED_CALLS = [0]
HEAD_TAIL_CALLS = [0]
_CHECK_SEED = os.environ.get("TFX_CHECK_SEED", "0") == "1"
def _head_state(store, device) -> torch.Tensor:
    """The fused head's self-resetting loss accumulator (3 zeroed int64 per model and device, left zero by
    every launch): allocated once, outside any graph capture's private pool when possible."""
    return _cached_buffer(store, ("head_state", str(device)), lambda: torch.zeros(3, dtype=torch.int64, device=device))


class _HeadXent(torch.autograd.Function):
    """Mean softmax cross-entropy of ``linear(global_avg_pool(feat))`` for a unit-seeded backward: the
    forward launch also produces the input gradient (the loss is the graph's root), so backward only
    accumulates dW += dz^T f and db += colsum(dz) (head_wgrad, one small launch)."""

    @staticmethod
    def forward(ctx, feat, anchor, w: Variable, b: Optional[Variable], labels, tail):
        # tail = (TailPending, BNBackwardFusion) of the last block's unwritten tail BN output: the kernel
        # forms it while pooling, writes its mask bits and that BN's backward partials (head.hip TAIL)
        ctx.w, ctx.b, ctx.tail_bnb = w, b, None
        bias = b.master if b is not None else None
        if tail is not None:
            tp, bnb = tail
            rows = torch.empty(2 * feat.numel() // (feat.shape[1] * feat.shape[2]), dtype=torch.float32,
                               device=feat.device)
            loss, dfeat, f, dz = torch.ops.tfx.head_xent(feat, w.value, bias, labels, _head_state(w.store, feat.device), tp.x,
                                                         tp.res, tp.save, tp.mask, rows)
            ctx.tail_bnb, ctx.tail_rows = bnb, rows
            HEAD_TAIL_CALLS[0] += 1
            fusion.note("head_tail", w.name, "head_xent_tail")
        else:
            loss, dfeat, f, dz = torch.ops.tfx.head_xent(feat, w.value, bias, labels, _head_state(w.store, feat.device), None,
                                                         None, None, None, None)
        ctx.save_for_backward(dfeat, f, dz)
        HEAD_FUSED_CALLS[0] += 1
        fusion.note("fused_head", w.name, "head_xent")
        return loss

    @staticmethod
    def backward(ctx, g):
        # unit-seed contract (classifier_head_xent): dfeat, dW, db and the tail BN's dgamma / dbeta were
        # formed in the forward for a seed of exactly 1 -- a scaled seed is NOT applied.  Callers that
        # scale the loss use unit_seed=False (the composed ops).  TFX_CHECK_SEED=1 verifies it (syncs).
        if _CHECK_SEED and float(g) != 1.0:
            raise RuntimeError("fused classifier head: backward seed %r != 1 (use unit_seed=False)" % float(g))
        dfeat, f, dz = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        bnb = ctx.tail_bnb
        if bnb is not None:  # the tail BN's backward reduction: the forward wrote its per-sample partials
            bnb.red = torch.ops.tfx.head_rows_reduce(ctx.tail_rows, bnb.x.shape[-1], bnb.dgamma, bnb.dbeta)
            ctx.tail_rows = None
        bias_grad = b.grad if (b is not None and b.trainable) else None
        if w.trainable or bias_grad is not None:
            torch.ops.tfx.head_wgrad(dz, f, w.grad if w.trainable else None, bias_grad)
        _grad_ready(w if w.trainable else None, b if bias_grad is not None else None)
        return dfeat, None, None, None, None, None


def _head_tail(feat):
    """(TailPending, BNBackwardFusion) when ``feat`` is a ReLU + identity-residual tail BN's output that
    was never written and whose backward reduction nobody owes yet: the fused head takes both over."""
    tp = fusion.carried(feat, "tail")
    bnb = fusion.carried(feat, "bnb")
    if not fusion.knob("head_tail") or tp is None or tp.done or bnb is None:
        return None
    if tp.res is None or tp.res_save is not None or tp.mask is None or bnb.mask is not tp.mask or not bnb.relu:
        return None
    if bnb.deferred or bnb.red is not None or bnb.sr_pending or bnb.x is not tp.x:
        return None
    return tp, bnb


def classifier_head_xent(feat, w: Variable, b: Optional[Variable], labels, naive: bool = False,
                         unit_seed: bool = False) -> torch.Tensor:
    """``softmax_cross_entropy(linear(global_avg_pool(feat), w, b), labels)`` -- the training head of an
    image classifier (NHWC ``feat``, int64 ``labels``).  With ``unit_seed`` (the loss is the root of
    ``loss.backward()``) on the GPU it runs as ONE launch that also forms the input gradient
    (csrc/kernels/head.hip); otherwise, and for TF1's naive loss, the three ops compose.  On the fused
    path the gradients are formed for a backward seed of exactly 1: a scaled seed (loss scaling,
    ``(loss * k).backward()``) is not applied -- such callers pass ``unit_seed=False``."""
    fused = (fusion.knob("fuse_head") and unit_seed and not naive and feat.is_cuda and feat.dim() == 4
             and feat.dtype == torch.bfloat16 and labels.dtype == torch.long and labels.is_cuda
             and w.value.dtype == torch.bfloat16 and w.value.dim() == 2 and w.value.is_contiguous()
             and _native.use_native(feat))
    if fused:
        n, h, wd, c = feat.shape
        fused = bool(torch.ops.tfx.head_xent_supported(c, w.shape[0], h * wd)) and labels.numel() == n <= 4095
    if fused:
        tail = _head_tail(feat)
        return _HeadXent.apply(feat if tail is not None else _settle(feat).contiguous(), w.store.anchor, w, b,
                               labels.contiguous(), tail)
    logits = linear(global_avg_pool(feat), w, b)
    return softmax_cross_entropy(logits, labels, naive=naive, unit_seed=unit_seed)


def accuracy(logits, labels) -> torch.Tensor:
    """Fraction of rows with argmax(logits) == label (tf.equal(argmax, argmax) + mean)."""
    if _native.use_native(logits):
        idx = labels if labels.dtype == torch.long else None
        dense = labels.float().contiguous() if labels.dtype != torch.long else None
        return torch.ops.tfx.accuracy_count(logits.contiguous(), idx, dense)[0] / logits.shape[0]
    tgt = labels if labels.dtype == torch.long else labels.argmax(1)
    return (logits.argmax(1) == tgt).float().mean()


# ====================================================================== f32 dense (parity models)
_ACT = {None: 0, "none": 0, "relu": 1, "sigmoid": 2}


def _dense_ref(x, w, b=None, act=0):
    y = x @ w
    if b is not None:
        y = y + b
    if act == 1:
        y = torch.relu(y)
    elif act == 2:
        y = torch.sigmoid(y)
    return y


class _DenseF32(torch.autograd.Function):
    """y = act(x @ W + b), W stored [in, out] like tf.matmul(x, W) (R/distributed/distributed.py:96-98).
    GPU: exact-f32 MFMA GEMM (sgemm.hip) with the bias + activation fused into its epilogue."""

    @staticmethod
    def forward(ctx, x, anchor, w: Variable, b: Optional[Variable], act: int):
        ctx.w, ctx.b, ctx.act = w, b, act
        ctx.native = _native.use_native(x)
        if ctx.native:
            y = torch.ops.tfx.sgemm(x.contiguous(), w.master, False, False, b.master if b is not None else None, act)
        else:
            y = _dense_ref(x, w.master, b.master if b is not None else None, act)
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y = ctx.saved_tensors
        w, b, act = ctx.w, ctx.b, ctx.act
        bias_done = False
        if ctx.native:
            # SigmoidGrad / ReluGrad x upstream and the bias column sum in ONE HIP launch
            db = b.grad if (b is not None and b.trainable) else None
            g = torch.ops.tfx.act_bwd_colsum(gy.float().contiguous(), y, act, db)
            bias_done = True
        else:
            g = gy
            if act == 1:
                g = g * (y > 0)
            elif act == 2:
                g = g * y * (1 - y)  # TF1 SigmoidGrad: dy * y * (1 - y)
        g = g.contiguous()
        dx = None
        if ctx.native:
            if ctx.needs_input_grad[0]:
                dx = torch.ops.tfx.sgemm(g, w.master, False, True, None, 0)
            if w.trainable:
                torch.ops.tfx.sgemm_into(x.contiguous(), g, True, False, w.grad, True)
        else:
            if ctx.needs_input_grad[0]:
                dx = g @ w.master.t()
            if w.trainable:
                w.grad.add_(x.t() @ g)
        if b is not None and b.trainable and not bias_done:
            b.grad.add_(g.sum(0))
        _grad_ready(w, b)
        return dx, None, None, None, None


def dense(x, w: Variable, b: Optional[Variable] = None, activation=None):
    """f32 fully-connected layer: ``activation(x @ W + b)``, W is [in, out]."""
    return _DenseF32.apply(x, w.store.anchor, w, b, _ACT[activation])


# ====================================================================== scalar / per-channel affine + SSE
class _Affine(torch.autograd.Function):
    """y = W * x + b with W, b per-channel (broadcast over the last dim; shape [1] for the scalar
    linear model of R/simple/simple.py:16).  GPU: elementwise.hip affine_fwd / affine_bwd."""

    @staticmethod
    def forward(ctx, x, anchor, w: Variable, b: Optional[Variable]):
        ctx.w, ctx.b = w, b
        ctx.native = _native.use_native(x)
        ctx.save_for_backward(x)
        if ctx.native:
            return torch.ops.tfx.affine_fwd(x.contiguous().float(), w.master, b.master if b is not None else None)
        y = w.master * x
        return y + b.master if b is not None else y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        need_dx = ctx.needs_input_grad[0]
        dw = w.grad if w.trainable else None
        db = b.grad if (b is not None and b.trainable) else None
        if ctx.native:
            dx = torch.ops.tfx.affine_bwd(g.contiguous().float(), x.contiguous().float(), w.master, dw, db, need_dx)
        else:
            # TF1 Mul/Add gradients reduced back to the parameter shape: dW = sum g*x, db = sum g
            C = w.numel
            gx = (g * x).reshape(-1, C)
            if dw is not None:
                dw.add_(torch.sum(gx, 0) if C > 1 else torch.sum(g * x).reshape(1))
            if db is not None:
                db.add_(torch.sum(g.reshape(-1, C), 0) if C > 1 else torch.sum(g).reshape(1))
            dx = g * w.master if need_dx else None
        _grad_ready(w, b)
        return dx, None, None, None


def scale_shift(x: torch.Tensor, w: Variable, b: Optional[Variable] = None) -> torch.Tensor:
    """``W * x + b`` (R/simple/simple.py:16: ``linear_model = W * x + b``)."""
    return _Affine.apply(x, w.store.anchor, w, b)


class _SSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, y):
        ctx.native = _native.use_native(pred)
        ctx.save_for_backward(pred, y)
        if ctx.native:
            return torch.ops.tfx.sse_fwd(pred.contiguous().float(), y.contiguous().float())
        return ((pred - y) ** 2).sum()

    @staticmethod
    def backward(ctx, g):
        pred, y = ctx.saved_tensors
        if ctx.native:
            return torch.ops.tfx.sse_bwd(pred.contiguous().float(), y.contiguous().float(),
                                         g.reshape(1).float().contiguous()), None
        return 2.0 * (pred - y) * g, None


def sum_squared_error(pred: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``reduce_sum(square(pred - y))`` (R/simple/simple.py:20), a scalar."""
    return _SSE.apply(pred, y)
