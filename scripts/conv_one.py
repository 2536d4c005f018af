"""Run one conv shape (fwd, dgrad, wgrad) N times -- a small target for rocprofv3 --pmc."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native, tuning  # noqa: E402

N, H, W, C, K, R, st = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "256,16,16,128,128,3,1").split(",")]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
assert _native.load()
tuning.load()  # the measured launch table, as in the training step
pad = R // 2
x = torch.randn(N, H, W, C, device="cuda").bfloat16()
w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
slots = torch.zeros(64 * 2 * K, device="cuda")
y = torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots)
gy = torch.randn_like(y)
dw = torch.zeros(K, R, R, C, device="cuda")
for _ in range(iters):
    torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots)
    torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None)
    torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, True)
torch.cuda.synchronize()
print("done")
