"""Op layer: autograd wrappers over the gfx950 HIP kernels (GPU) / PyTorch references (CPU)."""
import contextlib

from . import _native, fusion
from .nn import (BNWorkspace, GradSink, accuracy, avg_pool2d, batch_norm, classifier_head_xent, conv2d, dense,
                 global_avg_pool, linear,
                 max_pool2d, scale_shift, softmax_cross_entropy, sum_squared_error)
from .rnn import LSTMHandoffError, check_lstm_health, lstm_layer
from .sparse import (embedding_lookup, gather_rows, log_uniform_logq, log_uniform_sample, nce_loss,
                     sampled_loss_grads, sampled_softmax_loss, scatter_add_rows)

__all__ = ["_native", "BNWorkspace", "GradSink", "accuracy", "avg_pool2d", "batch_norm", "classifier_head_xent",
           "conv2d", "dense",
           "global_avg_pool", "linear", "max_pool2d", "scale_shift", "softmax_cross_entropy", "sum_squared_error", "lstm_layer", "check_lstm_health", "LSTMHandoffError", "embedding_lookup",
           "gather_rows", "log_uniform_logq", "log_uniform_sample", "nce_loss", "sampled_loss_grads",
           "sampled_softmax_loss", "scatter_add_rows", "deterministic"]


@contextlib.contextmanager
def deterministic(on: bool = True):
    """Deterministic-reduction test mode of the native library for the block (then restored).

    The step's f32 atomics add in arrival order, so two runs of one path differ in the last bits, and a
    random-init ResNet-50 amplifies a forward difference that small into 20-100 % of a gradient
    (profiles/r04_determinism).  In this mode the forward BN statistics are recomputed in a fixed order
    before every finalize (one adder per slot address: bn_stats_det), split-K weight gradients run
    unsplit and slab reductions in one group, so a path's forward is bit-stable and two paths can be
    compared at a fixed tolerance.  Slower: a test mode, not a training mode.  The BN-backward partial
    sums keep their slot atomics -- their order noise enters the backward linearly (f32-sized), it is
    not amplified like the forward's (tests/test_determinism_gpu.py measures both)."""
    import torch
    if not _native.load():
        raise RuntimeError("deterministic(): the native library is not loaded")
    prev = torch.ops.tfx.set_deterministic(bool(on))
    try:
        yield
    finally:
        torch.ops.tfx.set_deterministic(prev)
