"""End-to-end ResNet training steps on the GPU through the HIP kernels."""
import pytest
import torch

from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input
from tensorflow_examples_amd.optim import MomentumOptimizer
from tensorflow_examples_amd.train import ClassifierTrainer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("depth", [18, 50])
def test_resnet_gpu_matches_cpu_reference_first_step(gpu, depth):
    """One forward/backward: GPU (bf16 HIP kernels, fused BN stats) vs CPU (fp32 torch reference)."""
    sg, mg = build_resnet_cifar(device=gpu, depth=depth, dtype=torch.bfloat16, seed=3)
    sc, mc = build_resnet_cifar(device="cpu", depth=depth, dtype=torch.float32, seed=3)
    sc.master.copy_(sg.master.cpu())
    g = torch.Generator().manual_seed(1)
    img = torch.randint(0, 256, (8, 32, 32, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, 10, (8,), generator=g)
    from tensorflow_examples_amd import ops
    for st, m, dev, dt in ((sg, mg, gpu, torch.bfloat16), (sc, mc, torch.device("cpu"), torch.float32)):
        st.zero_grad()
        x = to_model_input(img.to(dev), dtype=dt)
        loss = ops.softmax_cross_entropy(m(x, training=True), lab.to(dev))
        loss.backward()
        st._loss = loss.item()
    assert abs(sg._loss - sc._loss) < 0.05 * abs(sc._loss) + 0.05
    rel = ((sg.grad.cpu() - sc.grad).norm() / sc.grad.norm()).item()
    worst = []
    for v in sc.trainable():
        gc, gg = v.grad, sg.by_name[v.name].grad.cpu()
        r = ((gg - gc).norm() / (gc.norm() + 1e-8)).item()
        worst.append((r, v.name))
    worst.sort(reverse=True)
    print("worst per-variable grad rel err:", worst[:5])
    assert rel < 0.1, (rel, worst[:5])
    assert worst[0][0] < 0.25, worst[:5]


def test_graph_capture_step(gpu):
    store, model = build_resnet_cifar(device=gpu, depth=18, dtype=torch.bfloat16, seed=0)
    opt = MomentumOptimizer(store, 0.05, momentum=0.9)
    tr = ClassifierTrainer(store, model, opt)
    img = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, device=gpu)
    lab = torch.randint(0, 10, (16,), device=gpu)
    x = to_model_input(img)
    tr.capture(x, lab)
    l1 = tr.step(x, lab).item()
    l2 = tr.step(x, lab).item()
    assert l1 == l1 and l2 == l2


def test_resnet50_steps_reduce_loss(gpu):
    store, model = build_resnet_cifar(device=gpu, depth=50, dtype=torch.bfloat16, seed=0)
    assert 23_000_000 < store.num_params() < 24_000_000
    opt = MomentumOptimizer(store, 0.01, momentum=0.9)
    tr = ClassifierTrainer(store, model, opt)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, generator=g).to(gpu)
    lab = torch.randint(0, 10, (32,), generator=g).to(gpu)
    x = to_model_input(img)
    losses = [tr.step(x, lab).item() for _ in range(12)]
    assert all(l == l for l in losses), losses  # no NaN
    assert losses[-1] < losses[0], losses  # memorising one batch


