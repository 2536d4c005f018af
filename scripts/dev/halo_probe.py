#!/usr/bin/env python3
"""Round-6 cost probe: how much of the stride-1 3x3 implicit GEMMs' time is the A (im2col) operand
stream?  Times the model's forward (conv_fwd_bn) and flipped data gradient (conv_dgrad_bn) at the
stage 2-4 shapes, batch 256, normally and with the A (or B) loads returning zeros without a memory
access (igemm_probe bit 0 / 1).  HIP-graph-free, interleaved rounds in one process."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflow_examples_amd.ops import _native  # noqa: E402

assert _native.load()
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256


def timeit(fn, iters=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


rows = []
for hw, c in ((16, 128), (8, 256), (4, 512)):
    x = (torch.randn(B, hw, hw, c, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(c, 3, 3, c, device=dev) * 0.05).to(torch.bfloat16)
    wf = w.permute(3, 1, 2, 0).flip(1, 2).contiguous()
    ws = torch.zeros(64 * 2 * c + 64, device=dev)
    ws2 = torch.zeros(64 * 2 * c + 64, device=dev)
    gam, bet = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    save = torch.cat([torch.zeros(c, device=dev), torch.ones(c, device=dev), gam, bet]).contiguous()
    fwd = lambda: torch.ops.tfx.conv_fwd_bn(x, w, 1, 1, 1, ws, gam, bet, None, None, 0.1, 1e-5)
    dgr = lambda: torch.ops.tfx.conv_dgrad_bn(x, w, [B, hw, hw, c], 1, 1, 1, None, x, save, None, True, ws2,
                                              None, None, None, True, False, wf)
    for name, fn in (("fwd", fwd), ("dgrad_flip", dgr)):
        res = {}
        for rnd in range(3):
            for mode in (0, 1, 2):
                prev = torch.ops.tfx.igemm_probe(mode)
                try:
                    t = timeit(fn)
                finally:
                    torch.ops.tfx.igemm_probe(prev)
                res.setdefault(mode, []).append(t)
        med = {m: sorted(v)[1] for m, v in res.items()}
        print("%-10s %2dx%-2d c%-4d  normal %7.1f us   A-free %7.1f us (%.2fx)   B-free %7.1f us (%.2fx)" % (
            name, hw, hw, c, med[0], med[1], med[0] / med[1], med[2], med[0] / med[2]), flush=True)
