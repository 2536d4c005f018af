"""Bytes and time of the 1x1 data gradients with the fused BN-backward epilogue (conv_dgrad_bn, the
model's form: residual addend + its ReLU mask bits) against the plain data gradient and a streaming
calibration (torch.add of two tensors of dX's size: 2 reads + 1 write), at the ResNet-50/CIFAR
batch-256 shapes whose per-step launches run longest.  Each op runs REPS times eagerly; the counters
come from rocprofv3 --pmc passes over this script (scripts/dev/pmc_by_dispatch.py groups them by kernel
and grid).  Prints each call's logical bytes, so FETCH_SIZE (x2 for wide reads, MI355X_MICROARCH.md)
and WRITE_SIZE can be set against them.
usage: python scripts/dev/dgrad_bytes_probe.py [--time]   (--time: graph-replayed us per call)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflow_examples_amd.ops import _native  # noqa: E402

NSLOT = 64
REPS = 3
# (N, H, W, C = dX channels, Ko = dY channels): stage-2 conv1, stage-3 conv1, stage-2 first block conv1
SHAPES = [(256, 16, 16, 512, 128), (256, 8, 8, 1024, 256), (256, 32, 32, 256, 128)]


def graph_us(fn, it=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / it * 1e3)
    return best


def main():
    timing = "--time" in sys.argv
    assert _native.load()
    dev = torch.device("cuda")
    for N, H, W, C, K in SHAPES:
        M = N * H * W
        torch.manual_seed(5)
        dy = torch.randn(N, H, W, K, device=dev).bfloat16()
        w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).bfloat16()
        xb = (torch.randn(N, H, W, C, device=dev) + 0.2).bfloat16()
        add = torch.randn(N, H, W, C, device=dev).bfloat16()
        amask = torch.randint(0, 256, (M * C // 8,), device=dev, dtype=torch.uint8)
        save = torch.cat([torch.full((C,), 0.2), torch.ones(C), torch.full((C,), 1.3), torch.full((C,), -0.1)]).to(dev)
        ws = torch.zeros(NSLOT * 2 * C + 64, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        out = torch.empty_like(xb)
        ops = {
            "plain": lambda: torch.ops.tfx.conv_dgrad(dy, w, [N, H, W, C], 1, 0, 1, None),
            "bn_add": lambda: torch.ops.tfx.conv_dgrad_bn(dy, w, [N, H, W, C], 1, 0, 1, add, xb, save, None, True,
                                                          ws, dg, db, amask),
            "bn": lambda: torch.ops.tfx.conv_dgrad_bn(dy, w, [N, H, W, C], 1, 0, 1, None, xb, save, None, True,
                                                      ws, dg, db),
            "calib_add": lambda: torch.add(xb, add, out=out),
        }
        mb = lambda n: n * 2 / 1e6  # bf16 elements -> MB
        logical = {"plain": (mb(M * K), mb(M * C)), "bn_add": (mb(M * K) + 2 * mb(M * C) + M * C / 8e6, mb(M * C)),
                   "bn": (mb(M * K) + mb(M * C), mb(M * C)), "calib_add": (2 * mb(M * C), mb(M * C))}
        for name, fn in ops.items():
            rd, wr = logical[name]
            line = "M=%d C=%d Ko=%d %-9s logical read %7.1f MB write %6.1f MB" % (M, C, K, name, rd, wr)
            if timing:
                us = graph_us(fn)
                line += "  %7.1f us  %5.2f TB/s logical" % (us, (rd + wr) / us)
            else:
                for _ in range(REPS):
                    fn()
                    torch.cuda.synchronize()
            print(line, flush=True)


if __name__ == "__main__":
    main()
