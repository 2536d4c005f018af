#!/usr/bin/env python3
"""Probe: does the graph-replayed ResNet-50 step speed up over a process's life, and why?

scripts/tune_step.py saw the step go from 7.10 to 6.93 ms over a 330 s run with unchanged
configurations (profiles/r06_tune_step).  Phase A replays ONE captured graph for --secs seconds
(clock / thermal drift); phase B re-captures before every measurement (allocation drift); phase C
replays the last capture again.  Prints one line per measurement: phase, elapsed s, us/step.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflow_examples_amd.ops import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=60.0)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_batch
    from tensorflow_examples_amd.optim import MomentumOptimizer
    from tensorflow_examples_amd.train import ClassifierTrainer
    assert _native.load()
    dev = torch.device("cuda")
    store, model = build_resnet_cifar(device=dev, depth=50, dtype=torch.bfloat16, seed=0)
    opt = MomentumOptimizer(store, 0.1, momentum=0.9, weight_decay=5e-4)
    tr = ClassifierTrainer(store, model, opt, None, fuse_zero_grad=True)
    img = torch.randint(0, 256, (256, 32, 32, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (256,), device=dev)
    x, y = to_model_batch(img, lab, dtype=torch.bfloat16, device=dev)

    def capture():
        tr.graph, tr._static = None, None
        torch.cuda.synchronize()
        tr.capture(x, y, warmup=1)
        torch.cuda.synchronize()

    def timed(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            tr.graph.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n * 1e3

    t0 = time.time()
    capture()
    for phase, recap in (("A", False), ("B", True), ("C", False)):
        t1 = time.time()
        while time.time() - t1 < (a.secs if phase != "C" else a.secs / 3):
            if recap:
                capture()
            print("%s %6.1f %8.1f" % (phase, time.time() - t0, timed(a.steps)), flush=True)
            time.sleep(0.2 if not recap else 0.0)


if __name__ == "__main__":
    main()
