"""CIFAR augmentation offsets (tensorflow_examples_amd/data/cifar.py): crop origins in [0, 2 pad] and a
fair flip coin (a horizontal flip with probability 1/2)."""
import torch

from tensorflow_examples_amd.data.cifar import augment_offsets


def test_augment_offsets_ranges_and_fair_flip():
    g = torch.Generator().manual_seed(0)
    r = augment_offsets(200000, "cpu", g, pad=4)
    assert r.dtype == torch.int32 and r.shape == (200000, 3)
    assert int(r[:, :2].min()) == 0 and int(r[:, :2].max()) == 8
    assert set(r[:, 2].unique().tolist()) == {0, 1}
    p = r[:, 2].float().mean().item()
    assert abs(p - 0.5) < 0.005, p  # randint(0, 9) % 2 would give 4/9 = 0.444
