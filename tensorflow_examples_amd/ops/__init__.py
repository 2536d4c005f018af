"""Op layer: autograd wrappers over the gfx950 HIP kernels (GPU) / PyTorch references (CPU)."""
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
           "sampled_softmax_loss", "scatter_add_rows"]
