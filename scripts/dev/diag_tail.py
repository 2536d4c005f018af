"""Diagnostic: ResNet-50/CIFAR training_loss repeatability with / without the head's tail takeover."""
import torch
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input
from tensorflow_examples_amd.ops import fusion, nn as opsnn  # noqa: F401

gpu = torch.device("cuda:0")
torch.manual_seed(0)
img = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device=gpu)
lab = torch.randint(0, 10, (32,), device=gpu)
st, m = build_resnet_cifar(device=gpu, depth=50, dtype=torch.bfloat16, seed=7)
base = None
for tail in (False, False, True, True, False):
    fusion.CONFIG.set("head_tail", tail)
    st.zero_grad()
    loss = m.training_loss(to_model_input(img), lab, unit_seed=True)
    loss.backward()
    torch.cuda.synchronize()
    g = st.grad.clone()
    if base is None:
        base = g
    rel = ((g - base).norm() / base.norm()).item()
    print(f"tail={tail} loss={loss.item():.6f} grad_rel_vs_first={rel:.3e}", flush=True)
