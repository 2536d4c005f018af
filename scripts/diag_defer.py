"""Block-by-block forward: deferred shortcut BN (TFX_DEFER_RES_BN) on vs off, and vs fp32 reference ops."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.ops import nn, _native  # noqa: E402


def outs(defer, batch, ref=False):
    nn._DEFER_RES_BN = defer
    g = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (batch, 32, 32, 3), dtype=torch.uint8, generator=g)
    st, m = build_resnet_cifar(device="cuda", depth=50, dtype=torch.float32 if ref else torch.bfloat16, seed=3)
    res = []
    ctxm = _native.reference_mode() if ref else torch.enable_grad()
    with ctxm:
        x = to_model_input(img.cuda(), dtype=torch.float32 if ref else torch.bfloat16)
        o = m.stem_bn.after_conv(m.stem, x, True, relu=True)
        res.append(o.float())
        for blk in m.blocks:
            o = blk(o, True)
            res.append(o.float())
    torch.cuda.synchronize()
    return res


for batch in (8, 64):
    a, b, r = outs(True, batch), outs(False, batch), outs(False, batch, ref=True)
    print("batch", batch)
    for i, (x, y, z) in enumerate(zip(a, b, r)):
        e1 = ((x - y).norm() / y.norm()).item()
        e2 = ((x - z).norm() / z.norm()).item()
        e3 = ((y - z).norm() / z.norm()).item()
        print(f"  block {i:2d}: on-vs-off {e1:.3e}  on-vs-ref {e2:.3e}  off-vs-ref {e3:.3e}")
