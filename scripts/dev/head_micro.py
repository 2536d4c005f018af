"""Micro-benchmark of the fused head kernels at the bench shape (256 x 4 x 4 x 2048, 10 classes):
tail mode vs plain mode vs the apply pass it replaces.  Run under rocprofv3 --kernel-trace --stats."""
import torch
from tensorflow_examples_amd.ops import _native

assert _native.load()

dev = torch.device("cuda:0")
N, H, W, C, O = 256, 4, 4, 2048, 10
y3 = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
res = torch.randn(N, H, W, C, device=dev).clamp_min(0).to(torch.bfloat16)
save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
w = (torch.randn(O, C, device=dev) * 0.05).to(torch.bfloat16)
b = torch.zeros(O, device=dev)
lab = torch.randint(0, O, (N,), device=dev)
state = torch.zeros(3, dtype=torch.long, device=dev)
out = torch.empty_like(y3)
mask = torch.empty(y3.numel() // 8, dtype=torch.uint8, device=dev)
rows = torch.empty(N * 2 * C, device=dev)
for _ in range(30):
    torch.ops.tfx.head_xent(out, w, b, lab, state, y3, res, save, mask, rows)
for _ in range(30):
    torch.ops.tfx.bn_apply_into(y3, res, save, None, out, mask)
    torch.ops.tfx.head_xent(out, w, b, lab, state)
for _ in range(30):
    torch.ops.tfx.head_rows_reduce(rows, C, None, None)
torch.cuda.synchronize()
print("done")
