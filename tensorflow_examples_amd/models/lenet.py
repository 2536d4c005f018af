"""LeNet-5 for MNIST (BASELINE.json config 2: "MNIST LeNet-5 CNN bf16 on one MI355X").

    [N,28,28,1] -> conv 5x5 SAME, 6 ch -> BN + ReLU -> max-pool 2x2
                -> conv 5x5 VALID, 16 ch -> BN + ReLU -> max-pool 2x2      [N,5,5,16]
                -> flatten 400 -> FC 120 + ReLU -> FC 84 + ReLU -> FC 10

(the classic 32x32 VALID first layer == 28x28 SAME; batch norm replaces the conv biases, as in
the north-star "conv2d/batchnorm HIP kernel bring-up").  61 728 trainable parameters.

MI355X layout: NHWC bf16 activations, [Ko,R,S,C] conv weights.  Channel counts 1 / 6 are
carried as 8 (the 16-byte granularity of the implicit-GEMM loaders); the padded weights and BN
parameters are zero-initialised (:class:`~tensorflow_examples_amd.variables.Padded`) and receive
exactly-zero gradients, so the padded net is the unpadded LeNet-5.  Conv -> BN statistics are
fused into the conv epilogue, BN + ReLU is one pass, max-pool keeps an argmax byte for an
atomic-free backward, the FC layers run on the bf16 MFMA GEMM.
"""
from __future__ import annotations

from typing import Tuple

import torch

from .. import ops
from ..ops.nn import BNWorkspace
from ..variables import Constant, GlorotUniform, HeNormal, Padded, VariableStore, Zeros

PAD = 8


def _pad8(c: int) -> int:
    return (c + PAD - 1) // PAD * PAD


class _ConvBN:
    def __init__(self, store: VariableStore, cin: int, cout: int, k: int, pad: int, name: str):
        ci, co = _pad8(cin), _pad8(cout)
        with store.scope(name):
            self.w = store.variable([co, k, k, ci], Padded(HeNormal(), (cout, k, k, cin)), name="weights")
            self.gamma = store.variable([co], Padded(Constant(1.0), (cout,)), name="gamma")
            self.beta = store.variable([co], Zeros(), name="beta")
            self.mean = store.add_state("moving_mean", torch.zeros(co))
            self.var = store.add_state("moving_variance", torch.ones(co))
        self.pad, self.ws = pad, BNWorkspace(co)
        self.real = cout

    def __call__(self, x, training: bool):
        fused = training and x.device.type == "cuda"
        ws = self.ws.get(x.device) if x.device.type == "cuda" else None
        y = ops.conv2d(x, self.w, 1, self.pad, bn_stats_into=ws if fused else None)
        return ops.batch_norm(y, self.gamma, self.beta, self.mean, self.var, training=training, momentum=0.1,
                              eps=1e-5, relu=True, workspace=ws, stats_ready=fused)


class LeNet5:
    def __init__(self, store: VariableStore, num_classes: int = 10):
        self.store = store
        with store.scope("lenet5"):
            self.c1 = _ConvBN(store, 1, 6, 5, 2, "conv1")
            self.c2 = _ConvBN(store, 6, 16, 5, 0, "conv2")
            with store.scope("fc1"):
                self.w3 = store.variable([120, 400], GlorotUniform(), name="kernel")
                self.b3 = store.variable([120], Zeros(), name="bias")
            with store.scope("fc2"):
                self.w4 = store.variable([84, 120], GlorotUniform(), name="kernel")
                self.b4 = store.variable([84], Zeros(), name="bias")
            with store.scope("fc3"):
                self.w5 = store.variable([num_classes, 84], GlorotUniform(), name="kernel")
                self.b5 = store.variable([num_classes], Zeros(), name="bias")
        self.num_classes = num_classes

    def effective_params(self) -> int:
        """Trainable parameters of the unpadded LeNet-5 (61 728)."""
        conv = 6 * 25 * 1 + 2 * 6 + 16 * 25 * 6 + 2 * 16
        fc = 400 * 120 + 120 + 120 * 84 + 84 + 84 * 10 + 10
        return conv + fc

    def __call__(self, x: torch.Tensor, training: bool = True) -> torch.Tensor:
        o = ops.max_pool2d(self.c1(x, training), 2)       # [N,14,14,8]
        o = ops.max_pool2d(self.c2(o, training), 2)       # [N,5,5,16]
        o = o.reshape(o.shape[0], -1)                     # 400 (NHWC flatten, like tf.reshape)
        o = ops.linear(o, self.w3, self.b3, relu=True)
        o = ops.linear(o, self.w4, self.b4, relu=True)
        return ops.linear(o, self.w5, self.b5)


def build_lenet5(device="cuda", dtype=torch.bfloat16, seed=0, num_classes=10) -> Tuple[VariableStore, LeNet5]:
    store = VariableStore(device=device, compute_dtype=dtype, seed=seed)
    model = LeNet5(store, num_classes)
    store.finalize()
    return store, model


def to_model_input(images: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """MNIST [N,784] (or [N,28,28]) floats in [0,1] -> [N,28,28,8] NHWC (channels 1..7 zero)."""
    x = images.reshape(images.shape[0], 28, 28, 1)
    if x.dtype == torch.uint8:
        x = x.float() / 255.0
    out = torch.zeros(x.shape[0], 28, 28, PAD, device=x.device, dtype=dtype)
    out[..., :1] = x.to(dtype)
    return out
