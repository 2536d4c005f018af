#!/usr/bin/env python3
"""Run one conv pass under a forced igemm launch configuration (a target for rocprofv3 --pmc):
conv_cfg.py N,H,W,C,K,R,st pass(fwd|dgrad|wgrad) tile,ks,gls,want [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402

N, H, W, C, K, R, st = [int(v) for v in sys.argv[1].split(",")]
ps = sys.argv[2]
cfg = [int(v) for v in sys.argv[3].split(",")]
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
assert _native.load()
pad = R // 2
FAM = {"fwd": 0 if R == 1 and st == 1 else 1, "dgrad": 2 if R == 1 and st == 1 else 3,
       "wgrad": 6 if R == 1 else (7 if K >= 128 else 8)}[ps]
torch.ops.tfx.igemm_tune_force(FAM, *cfg)
x = torch.randn(N, H, W, C, device="cuda").bfloat16()
w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
slots = torch.zeros(64 * 2 * K + 64, device="cuda")
y = torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots)
gy = torch.randn_like(y)
dw = torch.zeros(K, R, R, C, device="cuda")
for _ in range(iters):
    if ps == "fwd":
        torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots)
    elif ps == "dgrad":
        torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None)
    else:
        torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, True)
torch.cuda.synchronize()
print("done")
