"""Time the fused-BN 1x1 data gradient (conv_dgrad_bn with a masked residual addend, reduce=False -- the
training step's form for every block-input conv1 of stages 2-4) at the batch-256 shapes, HIP-graph
replayed; prints us and effective HBM TB/s (dY + addend + x + masks read, dX written)."""
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
for (N, H, W, C, K) in [(256, 32, 32, 256, 64), (256, 16, 16, 512, 128), (256, 8, 8, 1024, 256), (256, 4, 4, 2048, 512)]:
    M = N * H * W
    gy = torch.randn(N, H, W, K, device=dev).bfloat16()
    w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).bfloat16()
    add = torch.randn(N, H, W, C, device=dev).bfloat16()
    amask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev)
    bx = torch.randn(N, H, W, C, device=dev).bfloat16()
    bmask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev)
    save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
    ws = torch.zeros(64 * 2 * C, device=dev)

    def run():
        torch.ops.tfx.conv_dgrad_bn(gy, w, [N, H, W, C], 1, 0, 1, add, bx, save, bmask, True, ws, None, None, amask,
                                    False, False, None)

    t = graph_us(run)
    by = 2 * M * K + 3 * 2 * M * C + 2 * M * C // 8
    print(f"dgrad_bn M={M} C={C} K={K}: {t:7.1f} us  {by / t / 1e6:5.2f} TB/s", flush=True)
