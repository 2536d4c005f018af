"""Isolated timing of the 1x1 forward (conv_fwd_bn) with the persistent kernel off / ring 2 / ring 3
(TFX igemm_persist_mode), at the ResNet-50 batch-256 1x1 shapes.  HIP-graph replayed, best of 3."""
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


# (batch, H, W, C_in, C_out): the 1x1 forward shapes of the CIFAR ResNet-50 at batch 256 (32x32 input)
shapes = [(256, 32, 32, 64, 64), (256, 32, 32, 64, 256), (256, 32, 32, 256, 64), (256, 32, 32, 256, 128),
          (256, 16, 16, 128, 512), (256, 16, 16, 256, 512), (256, 16, 16, 512, 128), (256, 16, 16, 512, 256),
          (256, 8, 8, 256, 1024), (256, 8, 8, 512, 1024), (256, 8, 8, 1024, 256), (256, 8, 8, 1024, 512),
          (256, 4, 4, 512, 2048), (256, 4, 4, 1024, 2048), (256, 4, 4, 2048, 512)]
modes = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "2", "3"])]
for (N, H, W, C, K) in shapes:
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(K, 1, 1, C, device=dev) / C ** 0.5).bfloat16()
    gamma, beta = torch.ones(K, device=dev), torch.zeros(K, device=dev)
    ws = torch.zeros(64 * 2 * K + 64, device=dev)
    row = []
    for m in modes:
        prev = torch.ops.tfx.igemm_persist_mode(m)
        us = graph_us(lambda: torch.ops.tfx.conv_fwd_bn(x, w, 1, 0, 1, ws, gamma, beta, None, None, 0.1, 1e-5))
        torch.ops.tfx.igemm_persist_mode(prev)
        row.append("mode %d %7.2f us" % (m, us))
    print("M %6d N %5d K %5d: %s" % (N * H * W, K, C, " | ".join(row)), flush=True)
