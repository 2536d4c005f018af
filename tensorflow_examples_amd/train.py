"""Training-step drivers shared by bench.py, the examples and the smoke test.

``ClassifierTrainer`` runs one synchronous step of an image classifier on the flat
variable store: zero grads -> forward -> softmax-xent -> backward (bucketed RCCL
all-reduce overlapped) -> fused optimizer (+bf16 shadow refresh; with ``fuse_zero_grad`` it also
clears the gradients for the next step, so no fill launch remains).  Optionally the whole
step is captured once into a HIP graph and replayed (launch-bound small models).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from . import ops
from .ops.nn import reset_pending_slot_reductions
from .optim import Optimizer
from .parallel.allreduce import GradAllReduce
from .utils import trace
from .variables import VariableStore


class ClassifierTrainer:
    def __init__(self, store: VariableStore, model: Callable, optimizer: Optimizer,
                 dp: Optional[GradAllReduce] = None, naive_xent: bool = False, fuse_zero_grad: bool = False):
        self.store, self.model, self.opt, self.dp = store, model, optimizer, dp
        # fuse_zero_grad: the optimizer kernel clears the gradients in its pass (no fill launch per step);
        # the store's gradients then read zero after each step
        self.fuse_zero_grad = fuse_zero_grad
        self.naive = naive_xent
        self.graph = None
        self._static = None
        self._one = None
        self.plan = None  # ops.fusion.record of the first step: which fusion group ran which layer

    def _step(self, x, y):
        if self.plan is None and not (x.is_cuda and torch.cuda.is_current_stream_capturing()):
            from .ops import fusion
            with fusion.record() as rec:
                loss = self._step_impl(x, y)
            self.plan = rec
            return loss
        return self._step_impl(x, y)

    def _step_impl(self, x, y):
        # roctx ranges (TFX_ROCTX=1) label the phases on a rocprofv3 --marker-trace timeline
        reset_pending_slot_reductions(self.store)  # nothing deferred survives an abandoned step
        self.store.zero_grad()
        with trace.range("forward"):
            head = getattr(self.model, "training_loss", None)
            if head is not None:  # the model fuses its classifier head with the loss (seeded by _one)
                loss = head(x, y, naive=self.naive, unit_seed=True)
            else:
                logits = self.model(x, training=True)
                loss = ops.softmax_cross_entropy(logits, y, naive=self.naive, unit_seed=True)  # seeded by _one
        with trace.range("backward"):
            # a persistent unit seed gradient: no ones-fill launch per step (graph-safe: never written)
            one = self._one
            if one is None or one.device != loss.device or one.dtype != loss.dtype:
                one = torch.ones((), dtype=loss.dtype, device=loss.device)
                if not (one.is_cuda and torch.cuda.is_current_stream_capturing()):  # not from a graph pool
                    self._one = one
            loss.backward(one)
        scale, grad = 1.0, None
        if self.dp is not None:
            with trace.range("allreduce_wait"):
                self.dp.finish()
            scale, grad = self.dp.grad_scale, self.dp.reduced_grad
        with trace.range("optimizer"):
            self.opt.apply_gradients(grad_scale=scale, grad=grad, zero_grad=self.fuse_zero_grad)
        return loss.detach()

    def input_buffer(self):
        """The captured graph's static input tensor (None when eager): a producer may write the next
        batch into it directly, and :meth:`step` then skips the copy."""
        return self._static[0] if self.graph is not None else None

    def label_buffer(self):
        """The captured graph's static label tensor (None when eager), see :meth:`input_buffer`."""
        return self._static[1] if self.graph is not None else None

    def step(self, x, y):
        if self.graph is not None:
            if x is not self._static[0]:
                self._static[0].copy_(x, non_blocking=True)
            if y is not self._static[1]:
                self._static[1].copy_(y, non_blocking=True)
            self.graph.replay()
            return self._static[2]
        return self._step(x, y)

    def capture(self, x, y, warmup: int = 3):
        """Capture one training step into a HIP graph.

        With a ``GradAllReduce`` the bucketed RCCL all-reduces are captured too: the grad-ready
        hooks fire during the captured backward, so every bucket becomes a collective node on
        RCCL's stream that forks from the compute stream where its last gradient is written and
        joins before the optimizer -- the same overlap as eager, replayed without Python or
        per-kernel launches.  Capture runs in thread-local mode so the process group's watchdog
        thread (which polls events of earlier eager collectives) cannot invalidate it.  All ranks
        must capture: the collectives are recorded, not executed, and run at replay time."""
        sx, sy = x.clone(), y.clone()
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    self._step(sx, sy)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            mode = "thread_local" if self.dp is not None else "global"
            with torch.cuda.graph(g, capture_error_mode=mode):
                loss = self._step(sx, sy)
        except BaseException:
            # a failure part-way through the (captured) backward leaves the bucket bookkeeping
            # mid-step: some buckets marked launched, captured never-executed Work objects queued.
            # Reset it so the eager fallback reduces every bucket exactly once.
            self.graph, self._static = None, None
            if self.dp is not None:
                self.dp.reset()
            raise
        self.graph = g
        self._static = (sx, sy, loss)
        return g
