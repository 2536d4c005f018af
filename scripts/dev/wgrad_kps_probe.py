"""Per-block fixed cost vs per-k-tile cost of the split-K 1x1 weight gradient (family 6, the 0.71 ms/step
`igemm_kernel<10,10,128,64,..,2,3>` family): the launch configuration is forced (tile 128x64, in-block
split-K KS, LDS-DMA ring depth 3, `want` blocks), the grid stays the same, and the pixel count (the GEMM's
reduction dimension) is scaled with the batch -- so the k-tiles each block streams scale 1:1 with the batch.
A linear fit  t = fixed + kps * per_ktile  separates the per-block fixed costs (launch, ring fill, KS=2
hand-off, split-K f32 atomic epilogue, grid tail) from the cost of one ring step.

    python scripts/dev/wgrad_kps_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from tensorflow_examples_amd.ops import _native  # noqa: E402
from operand_major_bench import graph_us  # noqa: E402

FAM_WGRAD_1X1 = 6
BKT = 64

assert _native.load()
dev = torch.device("cuda")


def kps_of(tiles, nkt, want, ks):
    # launch_t / pick_splits (csrc/kernels/igemm_impl.h) for OUT_F32_ATOMIC
    s = want // tiles if tiles < want else 1
    if tiles < want and s * tiles < want * 3 // 4:
        s = (want + tiles - 1) // tiles
    s = max(1, min(s, max(1, nkt // 4)))
    kps = (nkt + s - 1) // s
    if ks == 2:
        kps = (kps + 3) & ~3
    elif s > 1:
        kps += kps & 1
    return kps, (nkt + kps - 1) // kps


cfgs = [("ks2 ring3 want256 (production)", 2, 2, 3, 256), ("ks1 ring3 want512 (2 blocks/CU)", 2, 1, 3, 512)]
for (H, W, C, K) in [(8, 8, 1024, 256), (16, 16, 128, 512), (16, 16, 512, 128)]:
    tiles = (K // 128) * (C // 64)
    for name, tile, ks, gls, want in cfgs:
        torch.ops.tfx.igemm_tune_force(FAM_WGRAD_1X1, tile, ks, gls, want)
        pts = []
        for nb in (32, 64, 128, 256, 512):
            x = torch.randn(nb, H, W, C, device=dev).bfloat16()
            dy = torch.randn(nb, H, W, K, device=dev).bfloat16()
            dw = torch.zeros(K, 1, 1, C, device=dev)
            us = graph_us(lambda: torch.ops.tfx.conv_wgrad(dy, x, dw, 1, 0, 1, True))
            nkt = (nb * H * W + BKT - 1) // BKT
            kps, splits = kps_of(tiles, nkt, want, ks)
            pts.append((kps, us))
            print(f"x={nb}x{H}x{W}x{C} K={K} [{name}] tiles {tiles} x splits {splits} = {tiles * splits} blocks, "
                  f"{kps} k-tiles/block: {us:7.2f} us", flush=True)
        n = len(pts)
        mx = sum(p[0] for p in pts) / n
        my = sum(p[1] for p in pts) / n
        b = sum((p[0] - mx) * (p[1] - my) for p in pts) / sum((p[0] - mx) ** 2 for p in pts)
        a = my - b * mx
        kb = (128 + 64) * BKT * 2 / 1024  # KB of operand per k-tile per block
        print(f"  fit [{name}] {H}x{W} C={C} K={K}: fixed {a:6.2f} us + {b * 1e3:6.1f} ns per k-tile "
              f"({kb:.0f} KB/k-tile per block -> {kb * 1024 / (b * 1e-6) / 1e9 / 2.4:5.1f} B/clk per CU in the loop)",
              flush=True)
torch.ops.tfx.igemm_tune_force(-1, 0, 0, 0, 0)
