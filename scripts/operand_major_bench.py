#!/usr/bin/env python3
"""Does the B operand's staging (K-major ds_read_b128 image vs MN-major ds_read_b64_tr image) set
the speed of the conv data gradients?  Times the plain bf16 igemm GEMM on the 1x1 data-gradient
shapes of ResNet-50/CIFAR (batch 256) with W stored both ways, next to the real conv_dgrad_bn and
the forward conv of the same GEMM dims.  HIP-graph timed (20 launches per replay)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402

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
    # (N, H, W, C_in, Ko): data gradient dX[M, C] = dY[M, Ko] @ W[Ko, C]
    for (B, H, W, C, Ko) in [(256, 8, 8, 256, 1024), (256, 16, 16, 128, 512), (256, 32, 32, 64, 256),
                             (256, 4, 4, 512, 2048), (256, 8, 8, 1024, 256), (256, 32, 32, 256, 64)]:
        M = B * H * W
        dy = torch.randn(M, Ko, device="cuda").bfloat16()
        w = (torch.randn(Ko, C, device="cuda") * 0.05).bfloat16()
        wt = w.t().contiguous()
        t_mn = graph_us(lambda: torch.ops.tfx.gemm(dy, w, False, False, None, False, False))
        t_km = graph_us(lambda: torch.ops.tfx.gemm(dy, wt, False, True, None, False, False))
        xb = torch.randn(B, H, W, C, device="cuda").bfloat16()
        sf = torch.zeros(ns * 2 * C, device="cuda")
        sb = torch.zeros_like(sf)
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        _, save, _ = torch.ops.tfx.bn_fwd_train(xb, gam, bet, None, None, 0.1, 1e-5, None, True, sf, False)
        w4 = w.reshape(Ko, 1, 1, C)
        dy4 = dy.reshape(B, H, W, Ko)
        t_dg = graph_us(lambda: torch.ops.tfx.conv_dgrad_bn(dy4, w4, [B, H, W, C], 1, 0, 1, None, xb, save, None,
                                                            True, sb, None, None, None, False))
        t_dgp = graph_us(lambda: torch.ops.tfx.conv_dgrad(dy4, w4, [B, H, W, C], 1, 0, 1, None, None))
        wf = wt.reshape(C, 1, 1, Ko)
        t_fw = graph_us(lambda: torch.ops.tfx.conv_fwd_stats(dy4, wf, 1, 0, 1, sf))
        fl = 2.0 * M * C * Ko
        print(f"M={M:6d} N=C={C:5d} K=Ko={Ko:5d}: gemm B MN-major {t_mn:6.1f} us ({fl / t_mn / 1e6:5.0f} TF/s) | "
              f"B K-major {t_km:6.1f} us ({fl / t_km / 1e6:5.0f})   conv_dgrad {t_dgp:6.1f}  conv_dgrad_bn {t_dg:6.1f}"
              f"  conv_fwd_stats(same dims) {t_fw:6.1f}", flush=True)


def bench_3x3():
    """Stride-1 3x3 data gradient as the forward conv of dY with the flipped, transposed filter
    (Wf[c][r][s][ko] = W[ko][R-1-r][S-1-s][c]) vs the gathered data-gradient kernel."""
    for (B, H, W, C) in [(256, 32, 32, 64), (256, 16, 16, 128), (256, 8, 8, 256), (256, 4, 4, 512)]:
        Ko = C
        dy = torch.randn(B, H, W, Ko, device="cuda").bfloat16()
        w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).bfloat16()
        wf = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
        t_dg = graph_us(lambda: torch.ops.tfx.conv_dgrad(dy, w, [B, H, W, C], 1, 1, 1, None, None))
        t_fw = graph_us(lambda: torch.ops.tfx.conv_fwd(dy, wf, 1, 1, 1))
        t_tr = graph_us(lambda: w.flip(1, 2).permute(3, 1, 2, 0).contiguous())
        a = torch.ops.tfx.conv_dgrad(dy, w, [B, H, W, C], 1, 1, 1, None, None)
        b = torch.ops.tfx.conv_fwd(dy, wf, 1, 1, 1)
        err = ((a.float() - b.float()).norm() / a.float().norm()).item()
        print(f"3x3 {B}x{H}x{W}x{C}: conv_dgrad {t_dg:6.1f} us | conv_fwd(dY, Wf) {t_fw:6.1f} us  "
              f"(torch flip-transpose {t_tr:5.1f} us, rel diff {err:.2e})", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "3x3":
        assert _native.load()
        bench_3x3()
        sys.exit(0)
    main()
