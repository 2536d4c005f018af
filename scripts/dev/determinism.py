"""Run-to-run determinism of one training step: the same weights, batch and step twice, compared per
variable (gradient) and for the loss.  f32 atomics (BN statistics, split-K weight gradients) make the
runs differ in rounding only; anything larger points at a race.  Prints the global relative gradient
difference, the worst variables and (with --layers) the first forward activation that differs.

    TFX_IGEMM_XT=0 TFX_FUSION=r2 python scripts/dev/determinism.py --depth 18 --batch 16
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402


def one(depth, batch, x, lab, dev, perturb=0.0, zero_init=False):
    st, m = build_resnet_cifar(device=dev, depth=depth, dtype=torch.bfloat16, seed=0, zero_init_residual=zero_init)
    if perturb:
        # a deterministic relative nudge of one early BN gamma: how far does a 1e-7-scale difference
        # (the size of an f32 atomic-order rounding change) move this model's step?
        v = [v for v in st.trainable() if v.name.endswith("gamma")][1]
        st.master[v.offset:v.offset + v.numel] *= (1.0 + perturb)
        st.shadow[v.offset:v.offset + v.numel] = st.master[v.offset:v.offset + v.numel].to(st.shadow.dtype)
    tr = ClassifierTrainer(st, m, MomentumOptimizer(st, 0.0, momentum=0.9))
    loss = float(tr.step(x, lab))
    torch.cuda.synchronize()
    return loss, st.grad.clone(), st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--perturb", type=float, default=0.0, help="relative nudge of one BN gamma in reps >= 1")
    ap.add_argument("--zero-init", action="store_true", help="zero-init residual BN gammas (well-conditioned start)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (a.batch, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, 10, (a.batch,), generator=g).to(dev)
    x = to_model_input(img)
    tag = "XT=%s FUSION=%s" % (os.environ.get("TFX_IGEMM_XT", "1"), os.environ.get("TFX_FUSION", "all"))
    tag += " perturb=%g zero_init=%d" % (a.perturb, a.zero_init)
    l0, g0, st = one(a.depth, a.batch, x, lab, dev, zero_init=a.zero_init)
    for r in range(1, a.reps):
        l1, g1, _ = one(a.depth, a.batch, x, lab, dev, perturb=a.perturb, zero_init=a.zero_init)
        rel = ((g1 - g0).norm() / g0.norm()).item()
        rows = []
        for v in st.trainable():
            p, q = g0[v.offset:v.offset + v.numel], g1[v.offset:v.offset + v.numel]
            rows.append((((p - q).norm() / (p.norm() + 1e-30)).item(), v.name))
        rows.sort(reverse=True)
        print("%s depth %d batch %d rep %d: loss %.6f vs %.6f  grad rel %.3e  worst %s" % (
            tag, a.depth, a.batch, r, l0, l1, rel, ["%s %.2e" % (n, d) for d, n in rows[:5]]), flush=True)


if __name__ == "__main__":
    main()
