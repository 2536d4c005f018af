"""How much of a layer's weight-gradient launch could hide under its data-gradient launch if the two ran
as parallel branches of the HIP graph (a side stream forked and joined inside capture) instead of one after
the other on the capture stream.  The split-K weight gradient spends ~10 us of a ~21 us launch in per-launch
fixed costs (profiles/r04_kps: ring fill, KS=2 hand-off, f32 atomic epilogue, grid tail) that another
kernel's blocks could fill.

    python scripts/dev/wgrad_overlap_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tensorflow_examples_amd.ops import _native, tuning  # noqa: E402

assert _native.load()
tuning.load()
dev = torch.device("cuda")
ITER = 20


def replay_us(g):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * ITER) * 1e3


def capture(body):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(ITER):
            body()
    return g


side = torch.cuda.Stream()
# (N, H, W, C, K, R): x [N,H,W,C] -> y [N,H,W,K]
for (N, H, W, C, K, R) in [(256, 8, 8, 256, 1024, 1), (256, 8, 8, 1024, 256, 1), (256, 16, 16, 128, 512, 1),
                           (256, 16, 16, 512, 128, 1), (256, 4, 4, 512, 2048, 1), (256, 8, 8, 256, 256, 3)]:
    pad = R // 2
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    gy = torch.randn(N, H, W, K, device=dev).bfloat16()
    w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
    dw = torch.zeros(K, R, R, C, device=dev)
    shape = list(x.shape)

    def dgrad():
        return torch.ops.tfx.conv_dgrad(gy, w, shape, 1, pad, 1, None, None, False, None)

    def wgrad():
        torch.ops.tfx.conv_wgrad(gy, x, dw, 1, pad, 1, True)

    def serial():
        dgrad()
        wgrad()

    def parallel():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            wgrad()
        dgrad()
        cur.wait_stream(side)

    t_d = replay_us(capture(dgrad))
    t_w = replay_us(capture(wgrad))
    t_s = replay_us(capture(serial))
    t_p = replay_us(capture(parallel))
    print(f"x={N}x{H}x{W}x{C} K={K} R={R}: dgrad {t_d:6.1f}  wgrad {t_w:6.1f}  serial pair {t_s:6.1f}  "
          f"parallel branches {t_p:6.1f} us  ({t_s - t_p:+5.1f} us, {100 * (t_s - t_p) / t_s:4.1f} %)", flush=True)
