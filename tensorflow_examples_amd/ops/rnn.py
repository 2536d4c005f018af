"""GEMM-stacked LSTM layer (char-LSTM, BASELINE.json config 5).

TF1 equivalent: ``tf.contrib.rnn.BasicLSTMCell`` / ``LSTMBlockCell`` unrolled by
``tf.nn.dynamic_rnn`` -- one [B, In+H] x [In+H, 4H] MatMul per step followed by the gate
nonlinearities.  MI355X design (one autograd node for the whole sequence):

forward, T steps, batch B, hidden H:
    GX  = X[T*B, In] @ W_ih^T + b           ONE bf16 MFMA GEMM for all time steps (f32 out)
    for t:  GX[t] += h16[t-1] @ W_hh^T       bf16 MFMA GEMM accumulating in place (4 gates stacked)
            act[t], c[t], h16[t] = cell(GX[t], c[t-1])   fused pointwise kernel, f32 cell state
backward:
    for t = T-1 .. 0:
            dg16[t], dc = cell_bwd(act[t], c[t], c[t-1], dH[t], dc)   fused, dc carried in place
            dH[t-1] += dg16[t] @ W_hh                                 GEMM accumulating in place
    dW_hh += dG^T @ H_prev,  dW_ih += dG^T @ X,  dX = dG @ W_ih     three GEMMs over ALL steps
so only the inherently sequential part (one small GEMM + one pointwise kernel per step and
direction) runs T times; the weight gradients are batched over time into large GEMMs.

Persistent recurrence (default where it fits: B % 16 == 0, H in {128, 256, 512, 1024},
(B/16)*(H/16) <= CUs): the whole time loop of each direction is ONE kernel
(csrc/kernels/lstm_seq.hip) -- W_hh stays in VGPRs, h_t / dg_t move between workgroups through
write-through stores and per-row-block counters -- so the 2T dependent launches per direction
become one.  ``TFX_LSTM_PERSISTENT=0`` selects the per-step kernels above.
Gate order: i, f, g, o (f gets ``forget_bias`` added in the pointwise kernel through ``b``).
The whole step is HIP-graph capturable (no host syncs), which removes the per-step launch cost.

Co-residency of the persistent grid: :func:`_persistent` accepts a shape only when the occupancy API
(x CUs) admits every workgroup of both kernels at once, and an eager launch is cooperative (the
runtime refuses a grid that cannot be co-resident); a captured launch relies on that check.

Failure handling of the persistent kernels: their inter-workgroup waits are still bounded (a
workgroup kept off the device -- CUs taken by another stream or process, e.g. RCCL kernels under DP
-- would otherwise hang the grid).  On expiry a launch sets a per-device STICKY health word and
drains; its results are invalid.  The training step never synchronises on it, but it cannot
corrupt the weights either: the fused optimizer takes the word as its ``skip_if`` and skips the
update ON THE DEVICE while it is set (LMTrainer), so a bad step -- and any step until the host
looks -- leaves parameters and moments unchanged.  At the caller's own sync points
:func:`recover_persistent_failure` (LMTrainer.check) clears the word and switches this process to the
per-step kernels for the rest of the run; :func:`check_lstm_health` instead raises
:class:`LSTMHandoffError` for callers that want to stop.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from . import _native
from .nn import _grad_ready
from ..variables import Variable


def _lstm_ref(x, w_ih, w_hh, b, h0, c0):
    """PyTorch reference (f32): x [T,B,In] -> (out [T,B,H], h_T, c_T)."""
    T = x.shape[0]
    H = w_hh.shape[1]
    h, c = h0, c0
    outs = []
    gx = x.float() @ w_ih.t() + b
    for t in range(T):
        z = gx[t] + h @ w_hh.t()
        i, f, g, o = z.split(H, dim=1)
        i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
        c = f * c + i * g
        h = o * torch.tanh(c)
        outs.append(h)
    return torch.stack(outs), h, c


_SEQ_OK: Dict[Tuple[int, int, int], bool] = {}
_HEALTH: Dict[int, torch.Tensor] = {}
# test hook: a spin bound for the persistent kernels' hand-off waits (None = the kernel default)
_SPIN_LIMIT: Optional[int] = None


class LSTMHandoffError(RuntimeError):
    """A persistent LSTM launch gave up on an inter-workgroup hand-off: its outputs are invalid."""


def _health(dev: torch.device) -> torch.Tensor:
    h = _HEALTH.get(dev.index or 0)
    if h is None:
        assert not torch.cuda.is_current_stream_capturing(), "allocate the LSTM health word before capture"
        h = _HEALTH[dev.index or 0] = torch.zeros(1, dtype=torch.int32, device=dev)
    return h


def health_word(device) -> torch.Tensor:
    """The device's sticky persistent-LSTM health word (int32, 0 = healthy): pass it as the optimizer's
    ``skip_if`` so a step whose recurrence gave up on a hand-off is not applied."""
    return _health(torch.device(device))


# set once a persistent launch failed in this process: every later layer runs the per-step kernels
_PERSISTENT_OFF = False
PERSISTENT_LAUNCHES = [0]  # persistent fwd + bwd launches (tests)


def recover_persistent_failure(device=None) -> bool:
    """If a persistent launch on ``device`` (default: every device) timed out a hand-off since the last
    look: clear the health word, switch this process to the per-step kernels, return True.  The steps
    in between were skipped by the guarded optimizer (their updates are lost, never applied wrong)."""
    global _PERSISTENT_OFF
    devs = [torch.device(device).index or 0] if device is not None else list(_HEALTH)
    failed = False
    for d in devs:
        h = _HEALTH.get(d)
        if h is not None and int(h.item()) != 0:
            h.zero_()
            failed = True
    if failed:
        _PERSISTENT_OFF = True
    return failed


def check_lstm_health(device=None, reset: bool = True) -> None:
    """Raise :class:`LSTMHandoffError` if any persistent LSTM launch on ``device`` (default: all)
    timed out a hand-off since the last check.  Reads the device health word: call it where the host
    synchronises anyway (a logged loss), not inside the step."""
    devs = [torch.device(device).index or 0] if device is not None else list(_HEALTH)
    for d in devs:
        h = _HEALTH.get(d)
        if h is not None and int(h.item()) != 0:
            if reset:
                h.zero_()
            raise LSTMHandoffError("persistent LSTM recurrence on cuda:%d: an inter-workgroup hand-off exceeded "
                                   "its wait bound (not every workgroup resident?); the step's results are "
                                   "invalid -- rerun with TFX_LSTM_PERSISTENT=0" % d)


def _persistent(B: int, H: int, dev: torch.device) -> bool:
    if _PERSISTENT_OFF or os.environ.get("TFX_LSTM_PERSISTENT", "1") == "0" or not _native.use_native_device(dev):
        return False
    key = (B, H, dev.index or 0)
    if key not in _SEQ_OK:
        _SEQ_OK[key] = bool(torch.ops.tfx.lstm_seq_supported(B, H))
    return _SEQ_OK[key]


class _LSTMLayer(torch.autograd.Function):
    # per-launch status words of the last persistent launches (they stay 0: a timed-out wait sets the
    # device's sticky health word instead, which check_lstm_health reads at the caller's sync points)
    last_status: Dict[str, torch.Tensor] = {}

    @staticmethod
    def forward(ctx, x, anchor, w_ih: Variable, w_hh: Variable, b: Variable, h0, c0):
        T, B, In = x.shape
        H = w_hh.shape[1]
        ctx.vars = (w_ih, w_hh, b)
        ctx.native = _native.use_native(x) and x.dtype == torch.bfloat16
        if not ctx.native:
            ctx.save_for_backward(x, h0, c0)
            with torch.no_grad():
                out, hT, cT = _lstm_ref(x, w_ih.master, w_hh.master, b.master, h0, c0)
            return out.to(x.dtype), hT, cT
        dev = x.device
        xf = x.reshape(T * B, In).contiguous()
        gx = torch.ops.tfx.gemm(xf, w_ih.value, False, True, b.master, False, True)  # [T*B, 4H] f32
        hbuf = torch.empty(T + 1, B, H, dtype=torch.bfloat16, device=dev)
        cbuf = torch.empty(T + 1, B, H, dtype=torch.float32, device=dev)
        hbuf[0].copy_(h0)
        cbuf[0].copy_(c0)
        act = torch.empty(T, B, 4 * H, dtype=torch.float32, device=dev)
        hT = torch.empty(B, H, dtype=torch.float32, device=dev)
        gx = gx.view(T, B, 4 * H)
        ctx.persistent = _persistent(B, H, dev)
        if ctx.persistent:
            PERSISTENT_LAUNCHES[0] += 1
            _LSTMLayer.last_status["fwd"] = torch.ops.tfx.lstm_seq_fwd(gx, w_hh.value, hbuf, cbuf, act, hT,
                                                                       _health(dev), int(_SPIN_LIMIT or 0))
        else:
            for t in range(T):
                torch.ops.tfx.gemm_into(hbuf[t], w_hh.value, False, True, gx[t], True)
                torch.ops.tfx.lstm_cell_fwd(gx[t], None, None, cbuf[t], act[t], cbuf[t + 1], hT, hbuf[t + 1])
        ctx.save_for_backward(xf, hbuf, cbuf, act)
        return hbuf[1:], hT, cbuf[T].clone()

    @staticmethod
    def backward(ctx, gout, g_hT, g_cT):
        w_ih, w_hh, b = ctx.vars
        if not ctx.native:
            x, h0, c0 = ctx.saved_tensors
            with torch.enable_grad():
                xs = x.detach().float().requires_grad_(True)
                ps = [v.master.detach().clone().requires_grad_(True) for v in (w_ih, w_hh, b)]
                out, hT, cT = _lstm_ref(xs, *ps, h0, c0)
                outs, grads_in = [out], [gout.float()]
                if g_hT is not None:
                    outs.append(hT)
                    grads_in.append(g_hT)
                if g_cT is not None:
                    outs.append(cT)
                    grads_in.append(g_cT)
                gr = torch.autograd.grad(outs, [xs] + ps, grads_in, allow_unused=True)
            for v, g in zip((w_ih, w_hh, b), gr[1:]):
                if v.trainable and g is not None:
                    v.grad.add_(g)
            _grad_ready(w_ih, w_hh, b)
            return gr[0].to(x.dtype), None, None, None, None, None, None
        xf, hbuf, cbuf, act = ctx.saved_tensors
        T = act.shape[0]
        B, H = cbuf.shape[1], cbuf.shape[2]
        dg = torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=xf.device)
        bias_done = False
        if ctx.persistent:
            # the kernel reads the bf16 output gradient as is, folds in dh_T / dc_T, and accumulates
            # the bias gradient (sum over t and rows of the f32 gate gradients)
            dH16 = gout.to(torch.bfloat16).contiguous() if gout is not None else None
            dhT = g_hT.float().contiguous() if g_hT is not None else None
            dc_in = g_cT.float().contiguous() if g_cT is not None else None
            PERSISTENT_LAUNCHES[0] += 1
            _LSTMLayer.last_status["bwd"] = torch.ops.tfx.lstm_seq_bwd(
                act, cbuf, dH16, dhT, dc_in, w_hh.value, dg, None, b.grad if b.trainable else None,
                _health(xf.device), int(_SPIN_LIMIT or 0))
            bias_done = True
        else:
            dH = gout.float().contiguous().clone() if gout is not None else \
                torch.zeros(T, B, H, dtype=torch.float32, device=xf.device)
            if g_hT is not None:
                dH[T - 1].add_(g_hT)
            dc = g_cT.float().contiguous().clone() if g_cT is not None else \
                torch.zeros(B, H, dtype=torch.float32, device=xf.device)
            for t in range(T - 1, -1, -1):
                torch.ops.tfx.lstm_cell_bwd(act[t], cbuf[t + 1], cbuf[t], dH[t], dc, None, dg[t], dc)
                if t > 0:
                    torch.ops.tfx.gemm_into(dg[t], w_hh.value, False, False, dH[t - 1], True)
        dgf = dg.view(T * B, 4 * H)
        if w_hh.trainable:
            torch.ops.tfx.gemm_into(dgf, hbuf[:T].reshape(T * B, H), True, False, w_hh.grad, True)
        if w_ih.trainable:
            torch.ops.tfx.gemm_into(dgf, xf, True, False, w_ih.grad, True)
        if b.trainable and not bias_done:
            b.grad.add_(dgf.float().sum(0))
        _grad_ready(w_ih, w_hh, b)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.tfx.gemm(dgf, w_ih.value, False, False, None, False, False).view(T, B, -1)
        return dx, None, None, None, None, None, None


def lstm_layer(x: torch.Tensor, w_ih: Variable, w_hh: Variable, b: Variable,
               state: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    """Run one LSTM layer over a whole sequence. ``x`` [T,B,In] (bf16 on GPU), weights
    ``w_ih`` [4H,In], ``w_hh`` [4H,H], ``b`` [4H].  ``state`` = (h0, c0) f32 [B,H] (zeros if None);
    it is treated as a constant (truncated BPTT).  Returns (out [T,B,H], (h_T, c_T))."""
    T, B, _ = x.shape
    H = w_hh.shape[1]
    if state is None:
        h0 = torch.zeros(B, H, dtype=torch.float32, device=x.device)
        c0 = torch.zeros(B, H, dtype=torch.float32, device=x.device)
    else:
        h0, c0 = (s.detach().float().contiguous() for s in state)
    out, hT, cT = _LSTMLayer.apply(x, w_ih.store.anchor, w_ih, w_hh, b, h0, c0)
    return out, (hT.detach(), cT.detach())


__all__ = ["lstm_layer", "check_lstm_health", "LSTMHandoffError", "health_word", "recover_persistent_failure"]
