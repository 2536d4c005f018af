"""tensorflow_examples_amd -- an MI355X-native (gfx950 / CDNA4) example-model training framework
with the capabilities of manigoswami/tensorflow-examples.

Layers: flags / cluster / parallel (RCCL DP + async parameter server) /
models / ops (autograd over hand-written HIP kernels) / variables (flat store) /
optim (fused) / summary (tfevents) / ckpt (TF-style checkpoints) / data.
"""
__version__ = "0.1.0"
