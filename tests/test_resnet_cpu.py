"""CPU reference path of the ResNet model + flat store + optimizer (no GPU needed)."""
import torch

from tensorflow_examples_amd import ops
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input
from tensorflow_examples_amd.optim import MomentumOptimizer
from tensorflow_examples_amd.train import ClassifierTrainer


def test_resnet18_cpu_trains():
    store, model = build_resnet_cifar(device="cpu", depth=18, dtype=torch.float32, seed=0)
    opt = MomentumOptimizer(store, 0.05, momentum=0.9)
    tr = ClassifierTrainer(store, model, opt)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (8, 32, 32, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, 10, (8,), generator=g)
    x = to_model_input(img, dtype=torch.float32)
    losses = [tr.step(x, lab).item() for _ in range(6)]
    assert losses[-1] < losses[0]
    # padded stem channels stay exactly zero
    assert store.by_name["resnet18/conv0"].master[..., 3:].abs().max().item() == 0.0


def test_resnet50_param_count_cpu():
    store, model = build_resnet_cifar(device="cpu", depth=50, dtype=torch.float32, seed=0)
    # 23.52M for the CIFAR ResNet-50 (+ 5*3*3*64 zero weights of the padded stem channels)
    assert abs(store.num_params() - 23_520_842 - 5 * 9 * 64) < 1000, store.num_params()


def test_to_model_batch_cpu_fallback():
    """Without static buffers or a GPU, to_model_batch is to_model_input plus the labels as given."""
    from tensorflow_examples_amd.models.resnet import to_model_batch
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, 10, (4,), generator=g)
    x, y = to_model_batch(img, lab, dtype=torch.float32, device="cpu")
    assert torch.equal(x, to_model_input(img, dtype=torch.float32)) and y is lab


def test_softmax_xent_unit_seed_cpu_same_gradient():
    """unit_seed is a promise about the backward seed; on the reference path it changes nothing."""
    torch.manual_seed(0)
    z = torch.randn(8, 10)
    y = torch.randint(0, 10, (8,))
    grads = []
    for unit in (False, True):
        zz = z.clone().requires_grad_(True)
        loss = ops.softmax_cross_entropy(zz, y, unit_seed=unit)
        loss.backward()
        grads.append(zz.grad)
    assert torch.allclose(grads[0], grads[1])
    ref = torch.nn.functional.cross_entropy(z, y)
    assert abs(float(ops.softmax_cross_entropy(z, y, unit_seed=True)) - float(ref)) < 1e-5
