import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native
from scripts.operand_major_bench import graph_us
assert _native.load()
for (N, H, W, C, K, R, st) in [(256, 32, 32, 64, 64, 3, 1), (256, 16, 16, 128, 128, 3, 1), (256, 8, 8, 256, 256, 3, 1),
                               (256, 4, 4, 512, 512, 3, 1), (256, 32, 32, 64, 256, 1, 1), (256, 8, 8, 256, 1024, 1, 1),
                               (256, 8, 8, 1024, 256, 1, 1), (256, 16, 16, 128, 512, 1, 1)]:
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    gy = torch.randn(N, (H - 1) // st + 1, (W - 1) // st + 1, K, device="cuda").bfloat16()
    dw = torch.zeros(K, R, R, C, device="cuda")
    t = graph_us(lambda: torch.ops.tfx.conv_wgrad(gy, x, dw, st, R // 2, 1, True))
    print(f"wgrad {[N, H, W, C, K, R, st]}: {t:6.1f} us ({2.0 * N * H * W * C * K * R * R / st / st / t / 1e6:5.0f} TF/s)",
          flush=True)
