"""A/B of the A-operand BN transform (verdict item 2): the stage 2-4 conv3 forward as (a) the plain BN
apply pass + the conv with fused statistics, (b) the persistent kernel applying the BN on load
(conv_fwd_bn_in), (c) the conv alone on an already-written input -- HIP-graph replay, best of 3."""
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


EAGER = "--eager" in sys.argv  # PMC passes: plain launches, no graph replay / timing

for (N, H, W, C) in [(256, 16, 16, 128), (256, 8, 8, 256), (256, 4, 4, 512)]:
    K = 4 * C
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(K, 1, 1, C, device=dev) / C ** 0.5).bfloat16()
    in_save = torch.cat([torch.zeros(C), torch.ones(C), torch.rand(C) + 0.5, torch.randn(C) * 0.5]).to(dev)
    gamma, beta = torch.ones(K, device=dev), torch.zeros(K, device=dev)
    ws = torch.zeros(64 * 2 * K + 64, device=dev)
    a_buf = torch.empty_like(x)

    def apply_then_conv():
        torch.ops.tfx.bn_apply_into(x, None, in_save, None, a_buf, None)
        torch.ops.tfx.conv_fwd_bn(a_buf, w, 1, 0, 1, ws, gamma, beta, None, None, 0.1, 1e-5)

    if EAGER:
        for _ in range(5):
            apply_then_conv()
            for form in (1, 2):
                prev = torch.ops.tfx.igemm_bna_mode(form)
                torch.ops.tfx.conv_fwd_bn_in(x, in_save, w, ws, gamma, beta, None, None, 0.1, 1e-5)
                torch.ops.tfx.igemm_bna_mode(prev)
        torch.cuda.synchronize()
        continue
    t_apply = graph_us(lambda: torch.ops.tfx.bn_apply_into(x, None, in_save, None, a_buf, None))
    t_conv = graph_us(lambda: torch.ops.tfx.conv_fwd_bn(a_buf, w, 1, 0, 1, ws, gamma, beta, None, None, 0.1, 1e-5))
    t_ab = graph_us(apply_then_conv)
    t_in = {}
    for form in (1, 2):
        prev = torch.ops.tfx.igemm_bna_mode(form)
        t_in[form] = graph_us(lambda: torch.ops.tfx.conv_fwd_bn_in(x, in_save, w, ws, gamma, beta, None, None, 0.1,
                                                                    1e-5))
        torch.ops.tfx.igemm_bna_mode(prev)
    print("M %6d C %4d K %5d: apply %6.2f + conv %6.2f = seq %6.2f us | BN on load: registers %6.2f (saves %+.2f), "
          "in-LDS %6.2f (saves %+.2f)" % (N * H * W, C, K, t_apply, t_conv, t_ab, t_in[1], t_ab - t_in[1], t_in[2],
                                           t_ab - t_in[2]), flush=True)
