#!/usr/bin/env python3
"""One-step parity of the HIP-graph-replayed training step against the eager step, with chaos removed:
before every step the graph trainer's store (master, bf16 shadow, momentum, BN running statistics)
is set to the eager trainer's, then both take the same batch.  Reports the loss pair and the largest
per-variable relative difference of the updated weights (bf16 / f32-atomic noise is ~1e-3).

usage: python scripts/diag_graph_step.py [depth=18] [steps=30] [batch=64]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_examples_amd.data.cifar import synthetic_cifar  # noqa: E402
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402


def make(dev, depth):
    store, model = build_resnet_cifar(device=dev, depth=depth, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32,
                                      seed=0)
    opt = MomentumOptimizer(store, 0.1, momentum=0.9, weight_decay=5e-4)
    return ClassifierTrainer(store, model, opt)


def sync_state(dst, src):
    dst.store.master.copy_(src.store.master)
    dst.store.refresh_shadow()
    dst.opt.m.copy_(src.opt.m)
    for k, t in src.store.state.items():
        dst.store.state[k].copy_(t)


def per_var(store, ga, gb):
    out = []
    for v in store.trainable():
        a = ga[v.offset:v.offset + v.numel].float().cpu()
        b = gb[v.offset:v.offset + v.numel].float().cpu()
        out.append(((a - b).norm().item() / (a.norm().item() + 1e-12), a.norm().item(), v.name))
    return sorted(out, reverse=True)


def main():
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    xtr, ytr = synthetic_cifar(bs * steps, 0)
    dev = torch.device("cuda")
    batches = [(to_model_input(torch.as_tensor(xtr[i * bs:(i + 1) * bs], device=dev)),
                torch.as_tensor(ytr[i * bs:(i + 1) * bs], device=dev).long()) for i in range(steps)]
    ea, gb = make(dev, depth), make(dev, depth)
    cc = make(torch.device("cpu"), depth) if os.environ.get("DIAG_CPU", "1") == "1" else None
    gb.capture(*batches[0])
    worst_all = 0.0
    for i, (x, y) in enumerate(batches):
        sync_state(gb, ea)
        m0 = ea.opt.m.clone()
        p0 = ea.store.master.clone()
        s0 = {k: t.clone() for k, t in ea.store.state.items()}
        la = float(ea.step(x, y))
        lb = float(gb.step(x, y))
        torch.cuda.synchronize()
        # momentum-buffer increments = this step's (weight-decayed) gradients of each trainer
        ga, gg = ea.opt.m - 0.9 * m0, gb.opt.m - 0.9 * m0
        rel = []
        for v in ea.store.trainable():
            a = ga[v.offset:v.offset + v.numel]
            b = gg[v.offset:v.offset + v.numel]
            a0 = a.norm().item() + 1e-12
            rel.append(((a - b).norm().item() / a0, v.name))
        rs = []
        for k, t in ea.store.state.items():
            u = gb.store.state[k]
            rs.append(((t.float() - u.float()).norm().item() / (t.float().norm().item() + 1e-12), k))
        rel.sort(reverse=True)
        rs.sort(reverse=True)
        worst_all = max(worst_all, rel[0][0])
        print("%3d loss eager %.4f graph %.4f | worst grad rel %.2e %s | worst state rel %.2e %s" % (
            i, la, lb, rel[0][0], rel[0][1], rs[0][0], rs[0][1]), flush=True)
        if cc is not None and i < 4:
            cc.store.master.copy_(p0.cpu())
            cc.store.refresh_shadow()
            cc.opt.m.copy_(m0.cpu())
            for k, t in s0.items():
                cc.store.state[k].copy_(t.cpu())
            lc = float(cc.step(x.float().cpu(), y.cpu()))
            gc = cc.opt.m - 0.9 * m0.cpu()
            for tag, g in (("eager", ga), ("graph", gg)):
                w = per_var(cc.store, gc, g)
                print("    vs cpu fp32 (loss %.4f): %s worst %s" % (lc, tag, "; ".join(
                    "%s rel %.2e |g| %.3g" % (n.split("/", 1)[1], r, nrm) for r, nrm, n in w[:4])), flush=True)
    print("worst per-variable relative difference over all steps: %.3e" % worst_all)


if __name__ == "__main__":
    main()
