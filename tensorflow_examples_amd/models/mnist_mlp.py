"""The reference's MNIST model (R/distributed/distributed.py:83-102) and MNIST softmax regression
(BASELINE.json config 1).

MnistMLP: 784 -> 100 (sigmoid) -> 10 (softmax), W ~ N(0, 1) (tf.random_normal, :85-86), zero
biases (:90-91), TF variable names ``weights/Variable``, ``weights/Variable_1``,
``biases/Variable``, ``biases/Variable_1``; loss = reduce_mean(-reduce_sum(y_ * log(softmax(z3))))
(the NAIVE form of :102, reproduced by the fused HIP kernel's naive mode); f32 end to end
(exact-f32 MFMA GEMMs on the GPU).  Init values differ from TF1's Philox stream (no TF here);
the distribution and seeding-by-creation-order semantics are the same.
"""
from __future__ import annotations

import torch

from .. import ops
from ..variables import RandomNormal, VariableStore, Zeros


class MnistMLP:
    def __init__(self, store: VariableStore, hidden: int = 100, inputs: int = 784, classes: int = 10):
        with store.scope("weights"):
            self.W1 = store.variable([inputs, hidden], RandomNormal(0.0, 1.0))
            self.W2 = store.variable([hidden, classes], RandomNormal(0.0, 1.0))
        with store.scope("biases"):
            self.b1 = store.variable([hidden], Zeros())
            self.b2 = store.variable([classes], Zeros())
        self.store = store

    def logits(self, x: torch.Tensor) -> torch.Tensor:
        a2 = ops.dense(x, self.W1, self.b1, activation="sigmoid")  # z2 = x W1 + b1; a2 = sigmoid(z2)
        return ops.dense(a2, self.W2, self.b2)                    # z3 = a2 W2 + b2

    def loss(self, x, y_, naive: bool = True):
        return ops.softmax_cross_entropy(self.logits(x), y_, naive=naive)

    def graph_nodes(self, device_of=lambda name: ""):
        """GraphDef nodes for the TensorBoard graph (names as TF1 would create them)."""
        n = lambda name, op, inputs=(), dev="": {"name": name, "op": op, "inputs": list(inputs),  # noqa: E731
                                                 "device": dev}
        return [
            n("global_step", "VariableV2", dev=device_of("global_step")),
            n("input/x-input", "Placeholder"), n("input/y-input", "Placeholder"),
            n("weights/Variable", "VariableV2", dev=device_of("weights/Variable")),
            n("weights/Variable_1", "VariableV2", dev=device_of("weights/Variable_1")),
            n("biases/Variable", "VariableV2", dev=device_of("biases/Variable")),
            n("biases/Variable_1", "VariableV2", dev=device_of("biases/Variable_1")),
            n("softmax/MatMul", "MatMul", ["input/x-input", "weights/Variable"]),
            n("softmax/Add", "Add", ["softmax/MatMul", "biases/Variable"]),
            n("softmax/Sigmoid", "Sigmoid", ["softmax/Add"]),
            n("softmax/MatMul_1", "MatMul", ["softmax/Sigmoid", "weights/Variable_1"]),
            n("softmax/Add_1", "Add", ["softmax/MatMul_1", "biases/Variable_1"]),
            n("softmax/Softmax", "Softmax", ["softmax/Add_1"]),
            n("cross_entropy/Log", "Log", ["softmax/Softmax"]),
            n("cross_entropy/mul", "Mul", ["input/y-input", "cross_entropy/Log"]),
            n("cross_entropy/Sum", "Sum", ["cross_entropy/mul"]),
            n("cross_entropy/Neg", "Neg", ["cross_entropy/Sum"]),
            n("cross_entropy/Mean", "Mean", ["cross_entropy/Neg"]),
            n("Accuracy/ArgMax", "ArgMax", ["softmax/Softmax"]),
            n("Accuracy/ArgMax_1", "ArgMax", ["input/y-input"]),
            n("Accuracy/Equal", "Equal", ["Accuracy/ArgMax", "Accuracy/ArgMax_1"]),
            n("Accuracy/Mean", "Mean", ["Accuracy/Equal"]),
            n("cost", "ScalarSummary", ["cross_entropy/Mean"]),
            n("accuracy", "ScalarSummary", ["Accuracy/Mean"]),
            n("train/GradientDescent", "ApplyGradientDescent", ["cross_entropy/Mean"]),
        ]


class MnistSoftmax:
    """784 -> 10 softmax regression (the classic TF MNIST-for-beginners model)."""

    def __init__(self, store: VariableStore, inputs: int = 784, classes: int = 10):
        self.W = store.variable([inputs, classes], Zeros(), name="W")
        self.b = store.variable([classes], Zeros(), name="b")

    def logits(self, x):
        return ops.dense(x, self.W, self.b)

    def loss(self, x, y_, naive: bool = False):
        return ops.softmax_cross_entropy(self.logits(x), y_, naive=naive)
