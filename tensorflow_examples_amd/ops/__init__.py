"""Op layer: autograd wrappers over the gfx950 HIP kernels (GPU) / PyTorch references (CPU)."""
from . import _native
from .nn import (BNWorkspace, GradSink, accuracy, batch_norm, conv2d, dense, global_avg_pool, linear, softmax_cross_entropy)

__all__ = ["_native", "BNWorkspace", "GradSink", "accuracy", "batch_norm", "conv2d", "dense", "global_avg_pool", "linear", "softmax_cross_entropy"]
