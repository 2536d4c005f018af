"""What the BN slot-reduction tail blocks cost a weight-gradient launch: conv_wgrad alone vs
conv_wgrad_sr2 with one / two pending reductions, at the stage 2-4 1x1 and 3x3 shapes (batch 256),
HIP-graph replayed.  The tail blocks need a CU the GEMM blocks free (the kernel's static LDS allows one
block per CU), so they can only run after the GEMM wave.

    python scripts/dev/wgrad_sr_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from tensorflow_examples_amd.ops import _native, tuning  # noqa: E402
from operand_major_bench import graph_us  # noqa: E402

assert _native.load()
tuning.load()
dev = torch.device("cuda")
# (N, H, W, C, K, R): x [N,H,W,C], dy [N,H,W,K]
for (N, H, W, C, K, R) in [(256, 8, 8, 1024, 256, 1), (256, 8, 8, 256, 1024, 1), (256, 8, 8, 256, 256, 3),
                           (256, 16, 16, 512, 128, 1), (256, 4, 4, 2048, 512, 1)]:
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    dy = torch.randn(N, H, W, K, device=dev).bfloat16()
    dw = torch.zeros(K, R, R, C, device=dev)
    s1 = torch.zeros(64 * 2 * C, device=dev)
    s2 = torch.zeros(64 * 2 * 1024, device=dev)
    pad = R // 2
    t0 = graph_us(lambda: torch.ops.tfx.conv_wgrad(dy, x, dw, 1, pad, 1, True))
    t1 = graph_us(lambda: torch.ops.tfx.conv_wgrad_sr2(dy, x, dw, 1, pad, 1, True, s1, None, None, None, 0, None, None))
    t2 = graph_us(lambda: torch.ops.tfx.conv_wgrad_sr2(dy, x, dw, 1, pad, 1, True, s1, None, None, s2, 1024, None,
                                                      None))
    print(f"wgrad x={N}x{H}x{W}x{C} dy K={K} R={R}: plain {t0:6.1f} us  +sr(C={C}) {t1:6.1f}  +sr+sr2(1024) {t2:6.1f}",
          flush=True)
