#!/usr/bin/env python3
"""3x3 stride-1 data gradient: gathered data-gradient GEMM vs the forward conv of dY with the
flipped, transposed filter (wflip), both with the fused BN-backward epilogue as the model runs it
(conv_dgrad_bn), at the ResNet-50/CIFAR batch-256 shapes.  HIP-graph timed; checks agreement."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402

ITER = 20
SWEEP = "--sweep" in sys.argv
FAM_DGRAD_X, FAM_FLIP = 3, 9


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
    tot0 = tot1 = 0.0
    for (B, H, W, C, cnt) in [(256, 32, 32, 64, 3), (256, 16, 16, 128, 3), (256, 8, 8, 256, 5), (256, 4, 4, 512, 2)]:
        Ko = C
        dy = torch.randn(B, H, W, Ko, device="cuda").bfloat16()
        w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).bfloat16()
        wf = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
        xb = (torch.randn(B, H, W, C, device="cuda") + 0.2).bfloat16()
        save = torch.cat([torch.full((C,), 0.2), torch.ones(C), torch.full((C,), 1.3),
                          torch.full((C,), -0.1)]).cuda()
        ws = torch.zeros(ns * 2 * C + 64, device="cuda")
        dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")

        def run(flip):
            return torch.ops.tfx.conv_dgrad_bn(dy, w, [B, H, W, C], 1, 1, 1, None, xb, save, None, True, ws, dg, db,
                                               None, True, False, wf if flip else None)
        dx0, r0 = run(False)
        dx1, r1 = run(True)
        torch.cuda.synchronize()
        e_dx = ((dx1.float() - dx0.float()).norm() / dx0.float().norm()).item()
        e_r = ((r1 - r0).norm() / r0.norm()).item()
        t0, t1 = graph_us(lambda: run(False)), graph_us(lambda: run(True))
        t_tr = graph_us(lambda: w.flip(1, 2).permute(3, 1, 2, 0).contiguous())
        tot0 += cnt * t0
        tot1 += cnt * t1
        print(f"3x3 {B}x{H}x{W}x{C} (x{cnt}): dgrad_bn gathered {t0:6.1f} us | flipped-fwd {t1:6.1f} us "
              f"(torch flip {t_tr:5.1f} us)  rel dx {e_dx:.1e} red {e_r:.1e}", flush=True)
        if SWEEP:
            res = []
            for cand in [(t, 0, g, 0) for t in (1, 2, 3) for g in (0, 2, 3)] + \
                    [(t, 2, g, 0) for t in (1, 2) for g in (0, 2)]:
                torch.ops.tfx.igemm_tune_force(FAM_FLIP, *cand)
                res.append((graph_us(lambda: run(True)), cand))
                torch.ops.tfx.igemm_tune_force(FAM_DGRAD_X, *cand)
                res.append((graph_us(lambda: run(False)), ("gathered",) + cand))
                torch.ops.tfx.igemm_tune_force(-1, 0, 0, -1, 0)
            res.sort()
            print("    best:", ", ".join(f"{c} {t:.1f}" for t, c in res[:6]), flush=True)
    print(f"per step (13 convs): gathered {tot0:.0f} us, flipped {tot1:.0f} us, saving {tot0 - tot1:.0f} us")


if __name__ == "__main__":
    main()
