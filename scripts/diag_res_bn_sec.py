"""Per-variable gradient differences: residual-BN fused backward on vs off vs off again (run-to-run)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd import ops  # noqa: E402
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.ops import nn  # noqa: E402


def run(fused, batch):
    nn._FUSE_RES_BN = fused
    g = torch.Generator().manual_seed(5)
    img = torch.randint(0, 256, (batch, 32, 32, 3), dtype=torch.uint8, generator=g).cuda()
    lab = torch.randint(0, 10, (batch,), generator=g).cuda()
    st, m = build_resnet_cifar(device="cuda", depth=50, dtype=torch.bfloat16, seed=9)
    st.zero_grad()
    loss = ops.softmax_cross_entropy(m(to_model_input(img), training=True), lab)
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), {v.name: v.grad.float().clone() for v in st.trainable()}


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


for batch in (64, 256):
    la, a = run(True, batch)
    lb, b = run(False, batch)
    lc, c = run(False, batch)
    print(f"batch {batch}: loss fused {la:.5f} unfused {lb:.5f} {lc:.5f}")
    for k in b:
        print(f"  {k:45s} fused-vs-off {rel(a[k], b[k]):.3e}   off-vs-off {rel(c[k], b[k]):.3e}")
