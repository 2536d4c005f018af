"""Isolated timing of the fused-BN 1x1 data gradient (conv_dgrad_bn with the masked residual addend,
as a bottleneck conv1's backward) with the persistent kernel off / on, at the ResNet-50 batch-256
shapes the persistent routing takes.  HIP-graph replay of 20 calls, best of 3."""
import sys
import torch

sys.path.insert(0, ".")
from tensorflow_examples_amd.ops import _native  # noqa: E402

_native.load()
dev = torch.device("cuda")
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
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / ITER * 1e3)
    return best


# (N, H, W, C = dX channels, Ko = dY channels, with addend)
shapes = [(256, 32, 32, 256, 128, True), (256, 16, 16, 512, 128, True), (256, 16, 16, 128, 512, False),
          (256, 8, 8, 1024, 256, True), (256, 4, 4, 2048, 512, True)]
for (N, H, W, C, Ko, use_add) in shapes:
    M = N * H * W
    gy = torch.randn(N, H, W, Ko, device=dev).bfloat16()
    w = (torch.randn(Ko, 1, 1, C, device=dev) * 0.05).bfloat16()
    add = torch.randn(N, H, W, C, device=dev).bfloat16() if use_add else None
    amask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev) if use_add else None
    bx = torch.randn(N, H, W, C, device=dev).bfloat16()
    bmask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev) if use_add else None
    save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
    ws = torch.zeros(64 * 2 * C + 64, device=dev)
    row = []
    for m in (0, 1):
        prev = torch.ops.tfx.igemm_persist_dgrad(m)
        us = graph_us(lambda: torch.ops.tfx.conv_dgrad_bn(gy, w, [N, H, W, C], 1, 0, 1, add, bx, save, bmask, True,
                                                           ws, None, None, amask, False, False, None))
        torch.ops.tfx.igemm_persist_dgrad(prev)
        row.append(us)
    mb = (M * Ko + M * C * (3 if use_add else 2)) * 2 / 1e6  # dY + x (+ addend) read, dX written
    print("M %6d C %4d Ko %4d addend %d: per-tile %7.2f us | persistent %7.2f us  (%.2f / %.2f TB/s)" % (
        M, C, Ko, use_add, row[0], row[1], mb / row[0], mb / row[1]), flush=True)  # MB / us = TB/s
