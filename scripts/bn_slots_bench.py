#!/usr/bin/env python3
"""BN pass microbenchmark over the ResNet-50/CIFAR batch-256 BN shapes: the slot-consuming passes
(bn_fwd_slots / bn_bwd_slots with the producer's slots already filled) against the older
finalize + apply (bn_fwd_train with stats ready) and apply-only backward (bn_bwd_apply with red).
Each case is captured as a HIP graph of ITER launches, so the numbers include the kernel
boundaries the training-step graph pays."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402
from scripts.bn_bench import shapes  # noqa: E402

ITER = 20


def graph_us(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(ITER):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * ITER) * 1e3


def main():
    assert _native.load()
    ns = int(torch.ops.tfx.bn_nslot())
    tot = [0.0] * 4
    for M, C, res, cnt in shapes():
        x = torch.randn(M, C, device="cuda").bfloat16()
        g = torch.randn(M, C, device="cuda").bfloat16()
        r = torch.randn(M, C, device="cuda").bfloat16() if res else None
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        ws = torch.zeros(64 * 2 * C + 64, device="cuda")
        sf = torch.rand(ns * 2 * C + 64, device="cuda")
        sb = torch.rand(ns * 2 * C + 64, device="cuda")
        y, save, mask = torch.ops.tfx.bn_fwd_train(x, gam, bet, None, None, 0.1, 1e-5, r, True, ws, False)
        mask = mask if (mask is not None and mask.numel()) else None
        red = torch.rand(2 * C, device="cuda")
        of = graph_us(lambda: torch.ops.tfx.bn_fwd_train(x, gam, bet, None, None, 0.1, 1e-5, r, True, ws, True))
        nf = graph_us(lambda: torch.ops.tfx.bn_fwd_slots(x, gam, bet, None, None, 0.1, 1e-5, r, True, sf, sb, True))
        ob = graph_us(lambda: torch.ops.tfx.bn_bwd_apply(g, x, None, save, red, True, mask, True))
        nb = graph_us(lambda: torch.ops.tfx.bn_bwd_slots(g, x, res, save, True, mask, sb, sf, None, None, True,
                                                         True))
        print(f"M={M:7d} C={C:5d} res={int(res)} x{cnt:2d}: fwd finalize+apply {of:6.1f} us | slots {nf:6.1f} us"
              f"   bwd apply {ob:6.1f} us | slots {nb:6.1f} us", flush=True)
        for i, v in enumerate((of, nf, ob, nb)):
            tot[i] += cnt * v
    print(f"TOTAL per step (us): fwd old {tot[0]:.0f} new {tot[1]:.0f}   bwd old(apply only) {tot[2]:.0f} "
          f"new {tot[3]:.0f}")


if __name__ == "__main__":
    main()
