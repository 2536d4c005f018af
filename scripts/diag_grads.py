"""Diagnostic: per-variable gradient error of the GPU (bf16 HIP) path vs the CPU fp32 reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd import ops  # noqa: E402
from tensorflow_examples_amd.models import resnet  # noqa: E402


def run(depth, fused, batch=8):
    sg, mg = resnet.build_resnet_cifar(device="cuda", depth=depth, dtype=torch.bfloat16, seed=3)
    sc, mc = resnet.build_resnet_cifar(device="cpu", depth=depth, dtype=torch.float32, seed=3)
    sc.master.copy_(sg.master.cpu())
    sc.master.copy_(sc.master.bfloat16().float())  # same (bf16-representable) weights on both sides
    sg.master.copy_(sc.master.cuda()); sg.refresh_shadow()
    if not fused:
        orig = resnet._Conv.__call__
        resnet._Conv.__call__ = lambda self, x, ws=None: ops.conv2d(x, self.w, self.stride, self.pad)
    g = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (batch, 32, 32, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, 10, (batch,), generator=g)
    xin = resnet.to_model_input(img, dtype=torch.bfloat16)
    for st, m, dev, dt in ((sg, mg, "cuda", torch.bfloat16), (sc, mc, "cpu", torch.float32)):
        st.zero_grad()
        logits = m(xin.to(dev).to(dt), training=True)
        loss = ops.softmax_cross_entropy(logits, lab.to(dev))
        loss.backward()
        st._loss = loss.item(); st._logits = logits.detach().float().cpu()
    if not fused:
        resnet._Conv.__call__ = orig
    print(f"depth {depth} fused={fused} loss gpu {sg._loss:.5f} cpu {sc._loss:.5f}  logits rel "
          f"{((sg._logits - sc._logits).norm() / sc._logits.norm()).item():.4f}")
    for v in sc.trainable():
        gc, gg = v.grad, sg.by_name[v.name].grad.cpu()
        r = ((gg - gc).norm() / (gc.norm() + 1e-12)).item()
        print(f"  {r:8.4f}  |g|={gc.norm().item():10.4e}  {v.name}")


if __name__ == "__main__":
    from tensorflow_examples_amd.ops import _native
    assert _native.load()
    run(18, True)
    run(18, False)
