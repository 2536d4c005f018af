#!/usr/bin/env python3
"""BN microbenchmark over the ResNet-50/CIFAR BN shapes (batch 256): forward apply and backward
(reduce + apply) with and without the fused residual; reports effective HBM bandwidth."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402


def shapes(B=256):
    out = []  # (M, C, res, count)
    hw = 32
    for si, n in enumerate([3, 4, 6, 3]):
        w = 64 * 2 ** si
        st = 2 if si > 0 else 1
        out.append((B * hw * hw, w, False, 1))            # bn1 of first block (input res)
        hw2 = hw // st
        out.append((B * hw2 * hw2, w, False, 1 + 2 * (n - 1) + (n - 1)))  # bn2s and later bn1s
        out.append((B * hw2 * hw2, 4 * w, True, n))       # bn3 with residual
        hw = hw2
    return out


def t(fn, it=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    assert _native.load()
    tot_f = tot_b = 0.0
    for M, C, res, cnt in shapes():
        x = torch.randn(M, C, device="cuda").bfloat16()
        g = torch.randn(M, C, device="cuda").bfloat16()
        r = torch.randn(M, C, device="cuda").bfloat16() if res else None
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        ws = torch.zeros(64 * 2 * C, device="cuda")
        y, save, mask = torch.ops.tfx.bn_fwd_train(x, gam, bet, None, None, 0.1, 1e-5, r, True, ws, False)
        mask = mask if (mask is not None and mask.numel()) else None
        tf = t(lambda: torch.ops.tfx.bn_fwd_train(x, gam, bet, None, None, 0.1, 1e-5, r, True, ws, False))
        tb = t(lambda: torch.ops.tfx.bn_bwd(g, x, None if mask is not None else r, save, True, ws, None, None, mask))
        nb = M * C * 2
        bf, bb = nb * (4 if res else 3) + (nb // 16 if res else 0), nb * (6 if res else 4) + (nb // 8 if res else 0)
        print(f"M={M:7d} C={C:5d} res={int(res)} x{cnt}: fwd {tf:7.1f}us ({bf / tf / 1e3:5.2f} GB/s)  "
              f"bwd {tb:7.1f}us ({bb / tb / 1e3:5.2f} GB/s)")
        tot_f += cnt * tf
        tot_b += cnt * tb
    print(f"TOTAL per step: fwd {tot_f / 1e3:.3f} ms, bwd {tot_b / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
