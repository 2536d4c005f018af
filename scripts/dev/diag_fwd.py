"""Diagnostic: pw_fwd_squeeze vs the layer-wise pair (y1 bit agreement), and ResNet-50 first-step
losses with the deferred tails on / off over repeated runs."""
import torch
from tensorflow_examples_amd import ops
from tensorflow_examples_amd.ops import fusion, nn as nnops  # noqa: F401
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input

dev = torch.device("cuda")
from tensorflow_examples_amd.ops import _native
assert _native.load()
torch.manual_seed(11)
N, H, W, CI, co = 256, 32, 32, 256, 64
M = N * H * W
bf = lambda t: t.to(torch.bfloat16)
y3 = bf(torch.randn(N, H, W, CI, device=dev) * 1.2 + 0.1)
res = bf(torch.randn(N, H, W, CI, device=dev) * 0.8 - 0.2)
ws3 = torch.zeros(64 * 2 * CI, device=dev)
_, save3, _ = torch.ops.tfx.bn_fwd_train(y3, torch.rand(CI, device=dev) + .5, torch.randn(CI, device=dev) * .3,
                                         None, None, 0.1, 1e-5, None, False, ws3, False)
w1 = bf(torch.randn(co, 1, 1, CI, device=dev) * 0.06)
out_ref, _ = torch.ops.tfx.bn_apply_train(y3, res, save3, True)
ws = torch.zeros(64 * 2 * co, device=dev)
y1_ref, s_ref = torch.ops.tfx.conv_fwd_bn(out_ref, w1, 1, 0, 1, ws, None, None, None, None, 0.1, 1e-5)
out = torch.empty_like(y3)
mask = torch.empty(M * CI // 8, dtype=torch.uint8, device=dev)
y1, s1 = torch.ops.tfx.pw_fwd_squeeze(y3, save3, res, None, w1, out, mask, ws, None, None, None, None, 0.1, 1e-5)
f32 = out.float().reshape(M, CI) @ w1.float().reshape(co, CI).t()
d = (y1.float().reshape(M, co) - y1_ref.float().reshape(M, co)).abs()
print("out equal", torch.equal(out, out_ref), "y1 max abs diff", d.max().item(), "frac differing", (d > 0).float().mean().item())
print("y1 vs f32 rel", ((y1.float().reshape(M, co) - f32).norm() / f32.norm()).item(),
      "ref vs f32 rel", ((y1_ref.float().reshape(M, co) - f32).norm() / f32.norm()).item())
print("save diff", (s1 - s_ref).abs().max().item())

g = torch.Generator().manual_seed(9)
img = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, generator=g)
lab = torch.randint(0, 10, (32,), generator=g).to(dev)
xin = to_model_input(img.to(dev))


def run():
    st, m = build_resnet_cifar(device=dev, depth=50, dtype=torch.bfloat16, seed=4)
    loss = ops.softmax_cross_entropy(m(xin, training=True), lab)
    torch.cuda.synchronize()
    return float(loss)


for flag in (True, True, False, False, True):
    fusion.CONFIG.set("defer_tail", flag)
    print("defer", flag, "loss", run())
