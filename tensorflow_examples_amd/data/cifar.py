"""CIFAR-10 input: the binary distribution (``data_batch_{1..5}.bin``, ``test_batch.bin``: records
of 1 label byte + 3072 image bytes in CHW order) read with numpy only -- no pickle -- and a
deterministic synthetic fallback of the same shape (there is no dataset download on the box).

Images are returned NHWC uint8 [N,32,32,3]; :func:`augment` does the standard CIFAR training
augmentation (4-pixel pad + random 32x32 crop + horizontal flip) on the device, batched.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch

RECORD = 1 + 3 * 32 * 32
TRAIN_FILES = ["data_batch_%d.bin" % i for i in range(1, 6)]
TEST_FILE = "test_batch.bin"


def read_cifar_bin(path: str) -> Tuple[np.ndarray, np.ndarray]:
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size % RECORD:
        raise ValueError(f"{path}: size {raw.size} is not a multiple of {RECORD}")
    rec = raw.reshape(-1, RECORD)
    labels = rec[:, 0].astype(np.int64)
    images = rec[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy()
    return images, labels


def synthetic_cifar(n: int, seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Learnable CIFAR-shaped data: per-class random colour/texture prototypes plus noise."""
    rng = np.random.RandomState(seed)
    protos = np.random.RandomState(4321).randint(0, 256, size=(10, 8, 8, 3)).astype(np.float32)
    labels = rng.randint(0, 10, size=n).astype(np.int64)
    base = np.repeat(np.repeat(protos[labels], 4, axis=1), 4, axis=2)
    imgs = np.clip(base + rng.normal(0, 40, size=base.shape), 0, 255).astype(np.uint8)
    return imgs, labels


def hard_synthetic_cifar(n: int, seed: int = 0, label_noise: float = 0.15) -> Tuple[np.ndarray, np.ndarray]:
    """A CIFAR-shaped task a ResNet does NOT solve perfectly: every image mixes its class's texture with
    a random other class's (weight 0..0.9 of its own), at a random circular shift of up to 4 pixels,
    under heavy pixel noise, and ``label_noise`` of the labels are replaced by uniform random classes
    (the same for train and test, so test accuracy is capped near 1 - 0.9 label_noise).  Used by the
    convergence-parity check (tests/test_convergence_gpu.py), where the perfect accuracy every path
    reaches on :func:`synthetic_cifar` could not expose a wrong gradient."""
    cls = np.random.RandomState(97531)
    protos = cls.randint(0, 256, size=(10, 8, 8, 3)).astype(np.float32) - 127.5  # centred class textures
    protos += 0.5 * np.repeat(np.repeat(cls.randint(0, 256, size=(10, 4, 4, 3)).astype(np.float32) - 127.5,
                                        2, axis=1), 2, axis=2)  # + coarser structure
    rng = np.random.RandomState(seed + 1000)
    labels = rng.randint(0, 10, size=n).astype(np.int64)
    other = (labels + rng.randint(1, 10, size=n)) % 10
    w_own = rng.uniform(0.6, 1.0, size=(n, 1, 1, 1)).astype(np.float32)
    w_oth = (w_own * rng.uniform(0.0, 0.9, size=(n, 1, 1, 1))).astype(np.float32)
    base = w_own * protos[labels] + w_oth * protos[other]
    base = np.repeat(np.repeat(base, 4, axis=1), 4, axis=2)
    out = np.empty((n, 32, 32, 3), dtype=np.uint8)
    sy, sx = rng.randint(-4, 5, size=n), rng.randint(-4, 5, size=n)
    for i in range(0, n, 2048):  # bounded temporaries
        j = min(n, i + 2048)
        img = base[i:j] * 0.45 + 127.5 + rng.normal(0, 55, size=(j - i, 32, 32, 3)).astype(np.float32)
        for k in range(i, j):
            img[k - i] = np.roll(img[k - i], (sy[k], sx[k]), axis=(0, 1))
        out[i:j] = np.clip(img, 0, 255).astype(np.uint8)
    flip = rng.uniform(size=n) < label_noise
    labels = np.where(flip, rng.randint(0, 10, size=n), labels).astype(np.int64)
    return out, labels


def load_cifar10(data_dir: Optional[str], synthetic_train: int = 50000, synthetic_test: int = 10000):
    """(train_images, train_labels, test_images, test_labels, is_synthetic)."""
    if data_dir:
        for sub in ("", "cifar-10-batches-bin"):
            d = os.path.join(data_dir, sub)
            if all(os.path.exists(os.path.join(d, f)) for f in TRAIN_FILES + [TEST_FILE]):
                parts = [read_cifar_bin(os.path.join(d, f)) for f in TRAIN_FILES]
                xtr = np.concatenate([p[0] for p in parts])
                ytr = np.concatenate([p[1] for p in parts])
                xte, yte = read_cifar_bin(os.path.join(d, TEST_FILE))
                return xtr, ytr, xte, yte, False
    xtr, ytr = synthetic_cifar(synthetic_train, 0)
    xte, yte = synthetic_cifar(synthetic_test, 1)
    return xtr, ytr, xte, yte, True


def augment_offsets(n: int, device, generator: Optional[torch.Generator] = None, pad: int = 4) -> torch.Tensor:
    """Per-image crop origin in the padded image and flip bit: int32 [n, 3] = (ox, oy, flip)."""
    r = torch.randint(0, 2 * pad + 1, (n, 3), device=device, generator=generator, dtype=torch.int32)
    # the flip bit is its own fair coin (randint(0, 2 pad + 1) % 2 would favour 0: 5 of 9)
    r[:, 2] = torch.randint(0, 2, (n,), device=device, generator=generator, dtype=torch.int32)
    return r


def augment(images: torch.Tensor, generator: Optional[torch.Generator] = None,
            offsets: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Random 4-pixel-padded crop + horizontal flip of an NHWC uint8 batch (on its device).
    ``offsets``: explicit :func:`augment_offsets` (else drawn from ``generator``)."""
    n = images.shape[0]
    dev = images.device
    padded = torch.nn.functional.pad(images.permute(0, 3, 1, 2), (4, 4, 4, 4)).permute(0, 2, 3, 1)
    if offsets is None:
        offsets = augment_offsets(n, dev, generator)
    ox, oy, flip = offsets[:, 0].long(), offsets[:, 1].long(), offsets[:, 2].bool()
    ar = torch.arange(32, device=dev)
    rows = (oy[:, None] + ar[None, :])                                  # [n,32]
    cols = ox[:, None] + torch.where(flip[:, None], 31 - ar[None, :], ar[None, :])
    bidx = torch.arange(n, device=dev)[:, None, None]
    return padded[bidx, rows[:, :, None], cols[:, None, :]]


def augment_model_input(images: torch.Tensor, dtype=torch.bfloat16, generator: Optional[torch.Generator] = None,
                        offsets: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """:func:`augment` + ``models.resnet.to_model_input`` -- on the GPU one fused HIP kernel
    (csrc/kernels/image.hip ``augment_norm_kernel``: crop, flip, normalise, pad to 8 channels) after
    one offsets draw, instead of ~10 elementwise/gather launches; elsewhere the two-step path.
    ``out``: write the batch there (a captured training graph's static input,
    ``ClassifierTrainer.input_buffer``) instead of a new tensor; returns it."""
    from ..models.resnet import IN_CH_PAD, _MEAN, _STD, to_model_input
    from ..ops import _native
    if offsets is None:
        offsets = augment_offsets(images.shape[0], images.device, generator)
    if images.is_cuda and images.dtype == torch.uint8 and dtype == torch.bfloat16 and images.shape[1:] == (32, 32, 3) \
            and _native.use_native(images):
        if out is not None and out.shape == (images.shape[0], 32, 32, IN_CH_PAD) and out.dtype == dtype:
            torch.ops.tfx.augment_normalize_into(images.contiguous(), offsets.contiguous(), list(_MEAN), list(_STD), 4,
                                                 out)
            return out
        return torch.ops.tfx.augment_normalize(images.contiguous(), offsets.contiguous(), list(_MEAN), list(_STD),
                                               IN_CH_PAD, 4)
    x = to_model_input(augment(images, offsets=offsets), dtype)
    if out is not None and out.shape == x.shape:
        out.copy_(x)
        return out
    return x
