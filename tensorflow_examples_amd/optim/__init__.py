"""Fused optimizers over the flat variable store (one launch per step for the whole model).

GPU: ``tfx::optimizer_apply`` (csrc/kernels/optim.hip) updates the f32 master buffer and
rewrites the bf16 compute shadow in the same pass.  CPU: the same math in PyTorch.
Reference: ``tf.train.GradientDescentOptimizer(lr).minimize`` (R/simple/simple.py:22-23,
R/distributed/distributed.py:105-108); Momentum / Adam are the north-star fused optimizers.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import _native
from ..variables import VariableStore

SGD, MOMENTUM, NESTEROV, ADAM, ADAMW = 0, 1, 2, 3, 4


class Optimizer:
    kind = SGD

    def __init__(self, store: VariableStore, learning_rate: float, weight_decay: float = 0.0,
                 beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
        self.store = store
        self.wd, self.b1, self.b2, self.eps = float(weight_decay), float(beta1), float(beta2), float(eps)
        dev = store.device
        self.lr_t = torch.tensor([float(learning_rate)], dtype=torch.float32, device=dev)
        self._lr = float(learning_rate)  # host copy for the sparse (IndexedSlices) updates
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.m = torch.zeros_like(store.master) if self.kind >= MOMENTUM else None
        self.v = torch.zeros_like(store.master) if self.kind >= ADAM else None
        self.iterations = 0

    @property
    def learning_rate(self) -> float:
        return self._lr

    def set_learning_rate(self, lr: float) -> None:
        self._lr = float(lr)
        self.lr_t.fill_(float(lr))

    def apply_sparse(self, grad_scale: float = 1.0) -> None:
        """Apply and clear the pending IndexedSlices gradients of every :class:`SparseVariable`:
        ``table[ids] -= lr * grad_scale * rows`` (scatter-add kernel, duplicates summed, TF sparse
        ``ApplyGradientDescent`` semantics).  Only plain SGD has a sparse form here."""
        for sv in self.store.sparse:
            if not sv.pending:
                continue
            if self.kind != SGD:
                raise NotImplementedError("sparse (embedding) variables need GradientDescentOptimizer")
            alpha = -self._lr * grad_scale
            for ids, rows in sv.pending:
                if _native.use_native(sv.table):
                    torch.ops.tfx.embedding_scatter_add(sv.table, ids, rows, alpha)
                else:
                    sv.table.index_add_(0, ids, rows, alpha=alpha)
            sv.clear()

    def apply_gradients(self, grad_scale: float = 1.0, sumsq: Optional[torch.Tensor] = None,
                        max_norm: float = 0.0, skip_if: Optional[torch.Tensor] = None,
                        grad: Optional[torch.Tensor] = None, zero_grad: bool = False) -> None:
        """p <- update(p, grad_scale * g); refreshes the bf16 shadow. ``sumsq`` (device scalar
        ||g||^2) enables clip-by-global-norm at ``max_norm``.  ``skip_if`` (a device int32 word, GPU):
        when it is nonzero at execution time the update is skipped ON THE DEVICE -- parameters,
        moments, shadow and Adam's bias-correction step unchanged (the persistent LSTM's health word guards
        its steps this way); only the native dense path has that guard, so ``skip_if`` with sparse
        variables or a CPU store raises.  ``iterations`` (host count of calls) still advances.
        ``grad``: the flat gradient buffer to apply instead of the store's f32 one (same layout; f32 or
        bf16 -- the DP bf16 wire format hands its all-reduced bf16 buffer straight to the kernel).
        ``zero_grad``: the native kernel also clears the store's f32 gradient buffer in the same pass (the
        next ``VariableStore.zero_grad`` is then a no-op): the training step needs no separate gradient
        fill.  The gradients read zero after the call -- callers that inspect them leave it off."""
        st = self.store
        if skip_if is not None and (st.sparse or not _native.use_native(st.master)):
            # the device-side skip is honoured only by the native dense kernel: refuse rather than apply
            # an update the caller asked to be skipped (sparse tables / the CPU path have no such guard)
            raise ValueError("skip_if needs the native dense optimizer (no sparse variables, GPU store)")
        self.iterations += 1
        if self.kind >= ADAM:  # only the bias corrections read the device step counter (one launch less)
            if skip_if is not None:
                # a skipped step must not advance the bias-correction step either: += (skip == 0)
                self.step_t.add_((skip_if.reshape(-1)[:1] == 0).to(self.step_t.dtype))
            else:
                self.step_t.add_(1.0)
        if st.sparse:
            self.apply_sparse(grad_scale)
        if not st.vars:
            return
        if _native.use_native(st.master):
            gz = st.grad if zero_grad else None
            torch.ops.tfx.optimizer_apply(self.kind, st.master, st.grad if grad is None else grad, self.m, self.v,
                                          self.lr_t, grad_scale,
                                          self.wd, self.b1, self.b2, self.eps, self.step_t, sumsq, max_norm,
                                          st.shadow, skip_if, gz)
            if gz is not None:
                st.grads_clean = True
            return
        with torch.no_grad():
            g = (st.grad if grad is None else grad.float()) * grad_scale
            if sumsq is not None:
                nrm = float(sumsq.sqrt())
                if nrm > max_norm:
                    g = g * (max_norm / nrm)
            p, lr = st.master, self.lr_t
            if self.kind == SGD:
                p.sub_(lr * (g + self.wd * p))
            elif self.kind in (MOMENTUM, NESTEROV):
                d = g + self.wd * p
                self.m.mul_(self.b1).add_(d)
                p.sub_(lr * ((self.b1 * self.m + d) if self.kind == NESTEROV else self.m))
            else:
                d = g + self.wd * p if self.kind == ADAM else g
                self.m.mul_(self.b1).add_((1 - self.b1) * d)
                self.v.mul_(self.b2).add_((1 - self.b2) * d * d)
                t = float(self.step_t)
                upd = (self.m / (1 - self.b1 ** t)) / ((self.v / (1 - self.b2 ** t)).sqrt() + self.eps)
                if self.kind == ADAMW:
                    upd = upd + self.wd * p
                p.sub_(lr * upd)
            st.refresh_shadow()

    def global_norm_sq(self, grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        g = self.store.grad if grad is None else grad
        if _native.use_native(g):
            return torch.ops.tfx.sumsq(g)
        return (g.double() ** 2).sum().float().reshape(1)


class GradientDescentOptimizer(Optimizer):
    kind = SGD


class MomentumOptimizer(Optimizer):
    kind = MOMENTUM

    def __init__(self, store, learning_rate, momentum=0.9, use_nesterov=False, weight_decay=0.0):
        if use_nesterov:
            self.kind = NESTEROV
        super().__init__(store, learning_rate, weight_decay=weight_decay, beta1=momentum)


class AdamOptimizer(Optimizer):
    kind = ADAM

    def __init__(self, store, learning_rate=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-8, weight_decay=0.0,
                 decoupled=False):
        if decoupled:
            self.kind = ADAMW
        super().__init__(store, learning_rate, weight_decay, beta1, beta2, epsilon)


__all__ = ["Optimizer", "GradientDescentOptimizer", "MomentumOptimizer", "AdamOptimizer",
           "SGD", "MOMENTUM", "NESTEROV", "ADAM", "ADAMW"]
