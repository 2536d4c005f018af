"""Character-level LSTM language model (BASELINE.json config 5: "PTB-shaped char-LSTM language
model DP on 4xMI355X (MFMA GEMM-stacked LSTM cell)").

PTB ``ptb_word_lm``-style model, per character: embedding [V,E] -> L stacked LSTM layers of
width H (4 gates stacked into one GEMM, ops/rnn.py) -> softmax projection [V,H] -> mean
softmax cross-entropy over ``num_steps x batch`` positions; truncated BPTT with the final
(h, c) of each window carried into the next; SGD with clip_by_global_norm(max_grad_norm),
i.e. ``tf.clip_by_global_norm`` + ``GradientDescentOptimizer`` as in ptb_word_lm.

MI355X layout: time-major [T,B,*] activations, bf16 GEMM operands, f32 cell state and gate
math; weights live in the flat store so DP all-reduces them in large contiguous buckets and the
fused optimizer applies the global-norm clip on device (no host sync).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch

from .. import ops
from ..ops import rnn as rnn_ops
from ..variables import Uniform, VariableStore, Zeros, Constant

State = List[Tuple[torch.Tensor, torch.Tensor]]


class CharLSTM:
    def __init__(self, store: VariableStore, vocab_size: int = 65, embed: int = 128, hidden: int = 512,
                 layers: int = 2, init_scale: float = 0.1, forget_bias: float = 1.0):
        assert embed % 8 == 0 and hidden % 8 == 0, "embed / hidden must be multiples of 8 (MFMA GEMM operands)"
        self.V, self.E, self.H, self.L = vocab_size, embed, hidden, layers
        u = Uniform(-init_scale, init_scale)
        with store.scope("char_lstm"):
            self.embedding = store.variable([vocab_size, embed], u, name="embedding")
            self.cells = []
            for l in range(layers):
                with store.scope("cell_%d" % l):
                    din = embed if l == 0 else hidden
                    w_ih = store.variable([4 * hidden, din], u, name="w_ih")
                    w_hh = store.variable([4 * hidden, hidden], u, name="w_hh")
                    # gate order i, f, g, o: the forget gate's bias starts at forget_bias
                    bias = store.variable([4 * hidden], _ForgetBias(hidden, forget_bias), name="bias")
                    self.cells.append((w_ih, w_hh, bias))
            with store.scope("softmax"):
                self.w_out = store.variable([vocab_size, hidden], u, name="softmax_w")
                self.b_out = store.variable([vocab_size], Zeros(), name="softmax_b")
        self.store = store

    def zero_state(self, batch: int, device) -> State:
        z = lambda: torch.zeros(batch, self.H, dtype=torch.float32, device=device)  # noqa: E731
        return [(z(), z()) for _ in range(self.L)]

    def __call__(self, ids: torch.Tensor, state: Optional[State] = None) -> Tuple[torch.Tensor, State]:
        """``ids`` [T,B] int64 -> (logits [T*B, V], new state)."""
        T, B = ids.shape
        bf16 = self.store.compute_dtype == torch.bfloat16 and ids.device.type == "cuda"
        x = ops.embedding_lookup(self.embedding, ids, bf16=bf16)  # [T,B,E]
        new_state: State = []
        for l, (w_ih, w_hh, b) in enumerate(self.cells):
            x, st = ops.lstm_layer(x, w_ih, w_hh, b, state[l] if state is not None else None)
            new_state.append(st)
        logits = ops.linear(x.reshape(T * B, self.H), self.w_out, self.b_out)
        return logits, new_state


class _ForgetBias(Constant):
    def __init__(self, hidden: int, value: float):
        super().__init__(0.0)
        self.hidden, self.fb = hidden, value

    def __call__(self, shape, gen):
        t = torch.zeros(shape, dtype=torch.float32)
        t[self.hidden:2 * self.hidden] = self.fb
        return t


class LMTrainer:
    """One truncated-BPTT SGD step: forward, mean xent, backward (bucketed all-reduce overlapped),
    global-norm clip + update fused in the optimizer kernel."""

    def __init__(self, model: CharLSTM, optimizer, dp=None, max_grad_norm: float = 5.0):
        self.model, self.opt, self.dp, self.max_norm = model, optimizer, dp, max_grad_norm
        self.store = model.store

    def step(self, x: torch.Tensor, y: torch.Tensor, state: Optional[State]):
        self.store.zero_grad()
        logits, new_state = self.model(x, state)
        loss = ops.softmax_cross_entropy(logits, y.reshape(-1))
        loss.backward()
        scale, grad = 1.0, None
        if self.dp is not None:
            self.dp.finish()
            scale, grad = self.dp.grad_scale, self.dp.reduced_grad
        sumsq = self.opt.global_norm_sq(grad) if self.max_norm > 0 else None
        # the kernel clips on ||raw grad||; the raw DP grad is the SUM over ranks -> scale the bound.
        # GPU: the persistent LSTM's sticky health word guards the update (skipped on the device
        # while it is set: a timed-out hand-off never reaches the weights)
        dev = self.store.master.device
        guard = rnn_ops.health_word(dev) if dev.type == "cuda" else None
        if guard is not None and self.dp is not None and getattr(self.dp, "world", 1) > 1:
            # every rank skips together: a failed rank's gradient is inside everyone's all-reduced sum
            # (a 4-byte MAX on the DP group, stream-ordered: no host sync)
            import torch.distributed as dist
            dist.all_reduce(guard, op=dist.ReduceOp.MAX, group=getattr(self.dp, "group", None))
        self.opt.apply_gradients(grad_scale=scale, sumsq=sumsq, max_norm=self.max_norm / scale, skip_if=guard,
                                 grad=grad)
        return loss.detach(), new_state

    def check(self) -> bool:
        """Look at the device health word (call it where the host synchronises anyway, e.g. when
        logging).  If a persistent LSTM launch timed out a hand-off since the last check, the guarded
        optimizer has skipped those steps; switch to the per-step kernels for the rest of the run,
        report it and return True."""
        dev = self.store.master.device if self.store.master.is_cuda else None
        if dev is None:
            return False
        # under DP the word was MAX-reduced before every update, so all ranks see the same value here
        failed = rnn_ops.recover_persistent_failure(dev)
        if failed:
            print("warning: persistent LSTM hand-off timed out; the affected steps were skipped on the device, "
                  "continuing on the per-step recurrence kernels", flush=True)
        return failed


def build_char_lstm(device="cuda", vocab_size=65, embed=128, hidden=512, layers=2, dtype=torch.bfloat16,
                    seed=0) -> Tuple[VariableStore, CharLSTM]:
    store = VariableStore(device=device, compute_dtype=dtype, seed=seed)
    model = CharLSTM(store, vocab_size, embed, hidden, layers)
    store.finalize()
    return store, model


def perplexity(mean_xent: float) -> float:
    return math.exp(min(mean_xent, 50.0))
