#!/usr/bin/env python3
"""Run one 1x1 conv data gradient N times (for rocprofv3 --pmc passes): usage
dgrad_one.py <bn 0|1> [N H W C Ko] [iters]  -- bn=1: conv_dgrad_bn (fused BN-backward epilogue)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402

assert _native.load()
bn = int(sys.argv[1])
B, H, W, C, Ko = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else "256,32,32,256,64".split(","))]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ns = int(torch.ops.tfx.bn_nslot())
dy = torch.randn(B, H, W, Ko, device="cuda").bfloat16()
w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.05).bfloat16()
xb = torch.randn(B, H, W, C, device="cuda").bfloat16()
ws = torch.zeros(ns * 2 * C + 64, device="cuda")
save = torch.rand(4 * C, device="cuda")
for _ in range(iters):
    if bn:
        torch.ops.tfx.conv_dgrad_bn(dy, w, [B, H, W, C], 1, 0, 1, None, xb, save, None, True, ws, None, None, None,
                                    True)
    else:
        torch.ops.tfx.conv_dgrad(dy, w, [B, H, W, C], 1, 0, 1, None, None)
torch.cuda.synchronize()
print("ok")
