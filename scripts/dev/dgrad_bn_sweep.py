"""Every igemm launch configuration of the fused-BN 1x1 data gradient in its TRAINING-STEP form (masked
residual addend + BN-backward partials, reduce=False: the block-input conv1 of stages 2-4), at the
batch-256 shapes, HIP-graph replayed.  scripts/tune_convs.py tunes this pass without the addend; this
sweep checks whether the launch table's choice still wins with it.  Prints us and effective TB/s.

    python scripts/dev/dgrad_bn_sweep.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from tensorflow_examples_amd.ops import _native, tuning  # noqa: E402
from operand_major_bench import graph_us  # noqa: E402
from tune_convs import BF16_CANDS, force, traced  # noqa: E402

assert _native.load()
tuning.load()
dev = torch.device("cuda")
for (N, H, W, C, K) in [(256, 32, 32, 256, 128), (256, 16, 16, 512, 128), (256, 8, 8, 1024, 256),
                        (256, 4, 4, 2048, 512), (256, 16, 16, 128, 512), (256, 8, 8, 256, 1024)]:
    M = N * H * W
    gy = torch.randn(N, H, W, K, device=dev).bfloat16()
    w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).bfloat16()
    add = torch.randn(N, H, W, C, device=dev).bfloat16()
    amask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev)
    bx = torch.randn(N, H, W, C, device=dev).bfloat16()
    bmask = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev)
    save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
    ws = torch.zeros(64 * 2 * C, device=dev)
    use_add = C >= 4 * K  # conv1 (squeeze) carries the residual addend; conv3's dgrad (expand) does not

    def run():
        torch.ops.tfx.conv_dgrad_bn(gy, w, [N, H, W, C], 1, 0, 1, add if use_add else None, bx, save,
                                    bmask if use_add else None, True, ws, None, None, amask if use_add else None,
                                    False, False, None)

    fams = sorted({r[0] for r in traced(run)})
    by = 2 * M * K + (3 if use_add else 2) * 2 * M * C + (2 if use_add else 0) * M * C // 8
    force(fams, None)
    t0 = graph_us(run)
    res = []
    for c in BF16_CANDS:
        try:
            force(fams, c)
            res.append((graph_us(run), c))
        except Exception as e:  # an unsupported combination for this shape
            res.append((float("inf"), c))
    force(fams, None)
    res.sort()
    best = ", ".join("%s %.1f" % ("/".join(map(str, c)), t) for t, c in res[:4])
    print(f"M={M} C={C} K={K} addend={int(use_add)} fams={fams}: table {t0:6.1f} us ({by / t0 / 1e6:4.2f} TB/s)  "
          f"best: {best}", flush=True)
