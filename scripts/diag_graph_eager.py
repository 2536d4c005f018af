#!/usr/bin/env python3
"""Eager vs HIP-graph-replayed training of the same ResNet from the same init on the same batches:
per-step loss side by side (and an fp32 CPU reference for the first steps), then eval accuracy.

usage: python scripts/diag_graph_eager.py [depth=18] [steps=40] [batch=64]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_examples_amd import ops  # noqa: E402
from tensorflow_examples_amd.data.cifar import synthetic_cifar  # noqa: E402
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402


def make(dev, depth, dtype):
    store, model = build_resnet_cifar(device=dev, depth=depth, dtype=dtype, seed=0)
    opt = MomentumOptimizer(store, 0.1, momentum=0.9, weight_decay=5e-4)
    return ClassifierTrainer(store, model, opt), model


def evaluate(model, xte, yte, dev, dtype):
    with torch.no_grad():
        x = to_model_input(torch.as_tensor(xte, device=dev), dtype)
        return float(ops.accuracy(model(x, training=False), torch.as_tensor(yte, device=dev)))


def main():
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    ncpu = int(os.environ.get("DIAG_CPU_STEPS", "6"))
    xtr, ytr = synthetic_cifar(bs * steps, 0)
    xte, yte = synthetic_cifar(1000, 1)
    dev = torch.device("cuda")
    batches = [(torch.as_tensor(xtr[i * bs:(i + 1) * bs]), torch.as_tensor(ytr[i * bs:(i + 1) * bs]).long())
               for i in range(steps)]
    ea, ma = make(dev, depth, torch.bfloat16)
    gb, mb = make(dev, depth, torch.bfloat16)
    cc, mc = make(torch.device("cpu"), depth, torch.float32)
    x0, y0 = batches[0]
    # the capture warms up on batch 0 three times: the eager and CPU runs take those steps too
    gb.capture(to_model_input(x0.to(dev)), y0.to(dev))
    for _ in range(3):
        ea.step(to_model_input(x0.to(dev)), y0.to(dev))
        if ncpu:
            cc.step(to_model_input(x0, dtype=torch.float32), y0)
    print("step  eager_loss  graph_loss  cpu_fp32_loss")
    for i, (x, y) in enumerate(batches):
        la = float(ea.step(to_model_input(x.to(dev)), y.to(dev)))
        lb = float(gb.step(to_model_input(x.to(dev)), y.to(dev)))
        lc = float(cc.step(to_model_input(x, dtype=torch.float32), y)) if i < ncpu else float("nan")
        print("%4d  %10.4f  %10.4f  %10.4f" % (i, la, lb, lc), flush=True)
    torch.cuda.synchronize()
    print("eval accuracy (running stats) eager %.3f graph %.3f" % (evaluate(ma, xte, yte, dev, torch.bfloat16),
                                                                   evaluate(mb, xte, yte, dev, torch.bfloat16)))

    def batch_stat_acc(model):
        with torch.no_grad():
            x = to_model_input(torch.as_tensor(xte[:500], device=dev))
            return float(ops.accuracy(model(x, training=True), torch.as_tensor(yte[:500], device=dev)))

    print("eval accuracy (batch stats) eager %.3f graph %.3f" % (batch_stat_acc(ma), batch_stat_acc(mb)))
    # refresh the running statistics with forward passes over training batches (no weight update)
    for m in (ma, mb):
        with torch.no_grad():
            for x, _ in batches[:30]:
                m(to_model_input(x.to(dev)), training=True)
    print("eval accuracy (running stats after 30 refresh passes) eager %.3f graph %.3f" % (
        evaluate(ma, xte, yte, dev, torch.bfloat16), evaluate(mb, xte, yte, dev, torch.bfloat16)))
    da = (ea.store.master - gb.store.master).abs().max().item()
    print("max |master_eager - master_graph| %.4g" % da)


if __name__ == "__main__":
    main()
