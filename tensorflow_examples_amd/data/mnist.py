"""MNIST input with the semantics of TF1's ``input_data.read_data_sets`` / ``DataSet.next_batch``
(used at R/distributed/distributed.py:52-55,142,146,164).

* ``read_data_sets(train_dir, one_hot=True)`` -> ``Datasets(train, validation, test)`` with
  train = 55 000, validation = 5 000 (the first 5 000 of the 60 000 training images),
  test = 10 000; images float32 [N, 784] in [0, 1]; labels one-hot float32 [N, 10] (or int64).
* IDX files (``train-images-idx3-ubyte[.gz]`` ...) are read from ``train_dir`` when present.
  There is no network on the MI355X boxes, so nothing is downloaded: when the files are
  absent a deterministic, LEARNABLE synthetic MNIST of the same shapes is generated
  (class prototypes of random strokes + translation / intensity / noise) and a notice is
  printed.  ``fake_data=True`` mirrors TF1's all-ones fake data.
* ``next_batch`` reproduces TF1 exactly: shuffle at the first call, carry the remainder
  of an epoch into the next batch, reshuffle at each epoch boundary.
"""
from __future__ import annotations

import gzip
import os
import struct
import sys
from typing import NamedTuple, Optional

import numpy as np

NUM_CLASSES = 10
FILES = {
    "train_images": "train-images-idx3-ubyte",
    "train_labels": "train-labels-idx1-ubyte",
    "test_images": "t10k-images-idx3-ubyte",
    "test_labels": "t10k-labels-idx1-ubyte",
}


# ---------------------------------------------------------------- IDX format
def _open(path):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    with _open(path) as f:
        data = f.read()
    zero, dtype_code, ndim = struct.unpack_from(">HBB", data, 0)
    if zero != 0 or dtype_code != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    dims = struct.unpack_from(">" + "I" * ndim, data, 4)
    off = 4 + 4 * ndim
    arr = np.frombuffer(data, dtype=np.uint8, count=int(np.prod(dims)), offset=off)
    return arr.reshape(dims)


def write_idx(path: str, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    hdr = struct.pack(">HBB", 0, 0x08, arr.ndim) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
        f.write(hdr + arr.tobytes())


def _find(train_dir: str, base: str) -> Optional[str]:
    for cand in (base, base + ".gz"):
        p = os.path.join(train_dir, cand)
        if os.path.exists(p):
            return p
    return None


# ---------------------------------------------------------------- synthetic MNIST
def _prototypes(seed: int) -> np.ndarray:
    rng = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    protos = np.zeros((NUM_CLASSES, 28, 28), np.float32)
    for c in range(NUM_CLASSES):
        img = np.zeros((28, 28), np.float32)
        for _ in range(3 + c % 3):  # a few strokes per digit
            x0, y0, x1, y1 = rng.uniform(6, 22, size=4)
            for t in np.linspace(0, 1, 12):
                cx, cy = x0 + (x1 - x0) * t, y0 + (y1 - y0) * t
                img += np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / 3.0)
        protos[c] = img / img.max()
    return protos


def synthetic_mnist(n: int, seed: int) -> tuple:
    """Deterministic learnable MNIST-shaped data: (images uint8 [n,28,28], labels uint8 [n])."""
    protos = _prototypes(1234)
    rng = np.random.RandomState(seed)
    labels = rng.randint(0, NUM_CLASSES, size=n).astype(np.uint8)
    imgs = np.empty((n, 28, 28), np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = protos[labels[s:e]]
        dx, dy = rng.randint(-2, 3, size=(2, e - s))
        out = np.empty_like(base)
        for i in range(e - s):
            out[i] = np.roll(np.roll(base[i], dy[i], axis=0), dx[i], axis=1)
        out *= rng.uniform(0.7, 1.0, size=(e - s, 1, 1)).astype(np.float32)
        out += rng.normal(0, 0.08, size=out.shape).astype(np.float32)
        imgs[s:e] = (np.clip(out, 0, 1) * 255).astype(np.uint8)
    return imgs, labels


# ---------------------------------------------------------------- DataSet
def dense_to_one_hot(labels: np.ndarray, num_classes: int = NUM_CLASSES) -> np.ndarray:
    out = np.zeros((labels.shape[0], num_classes), np.float32)
    out[np.arange(labels.shape[0]), labels.astype(np.int64)] = 1.0
    return out


class DataSet:
    def __init__(self, images: np.ndarray, labels: np.ndarray, fake_data: bool = False, one_hot: bool = False,
                 dtype=np.float32, reshape: bool = True, seed: Optional[int] = None):
        self._rng = np.random.RandomState(seed)
        if fake_data:
            self._num_examples = 10000
            self.one_hot = one_hot
        else:
            assert images.shape[0] == labels.shape[0], (images.shape, labels.shape)
            self._num_examples = images.shape[0]
            if reshape:
                images = images.reshape(images.shape[0], -1)
            if dtype == np.float32:
                images = images.astype(np.float32) * (1.0 / 255.0)
        self._images = images
        self._labels = labels
        self._epochs_completed = 0
        self._index_in_epoch = 0
        self._fake = fake_data

    images = property(lambda self: self._images)
    labels = property(lambda self: self._labels)
    num_examples = property(lambda self: self._num_examples)
    epochs_completed = property(lambda self: self._epochs_completed)

    def next_batch(self, batch_size: int, fake_data: bool = False, shuffle: bool = True):
        if fake_data or self._fake:
            fake_image = [1.0] * 784
            fake_label = [1] + [0] * 9 if self.one_hot else 0
            return ([fake_image for _ in range(batch_size)], [fake_label for _ in range(batch_size)])
        start = self._index_in_epoch
        if self._epochs_completed == 0 and start == 0 and shuffle:
            perm0 = np.arange(self._num_examples)
            self._rng.shuffle(perm0)
            self._images = self._images[perm0]
            self._labels = self._labels[perm0]
        if start + batch_size > self._num_examples:
            self._epochs_completed += 1
            rest = self._num_examples - start
            images_rest = self._images[start:self._num_examples]
            labels_rest = self._labels[start:self._num_examples]
            if shuffle:
                perm = np.arange(self._num_examples)
                self._rng.shuffle(perm)
                self._images = self._images[perm]
                self._labels = self._labels[perm]
            start = 0
            self._index_in_epoch = batch_size - rest
            end = self._index_in_epoch
            return (np.concatenate((images_rest, self._images[start:end]), axis=0),
                    np.concatenate((labels_rest, self._labels[start:end]), axis=0))
        self._index_in_epoch += batch_size
        end = self._index_in_epoch
        return self._images[start:end], self._labels[start:end]


class Datasets(NamedTuple):
    train: DataSet
    validation: DataSet
    test: DataSet


def read_data_sets(train_dir: str, fake_data: bool = False, one_hot: bool = False, dtype=np.float32,
                   reshape: bool = True, validation_size: int = 5000, seed: Optional[int] = None,
                   synthetic: Optional[bool] = None, verbose: bool = True) -> Datasets:
    if fake_data:
        mk = lambda: DataSet([], [], fake_data=True, one_hot=one_hot, dtype=dtype, seed=seed)  # noqa: E731
        return Datasets(mk(), mk(), mk())
    paths = {k: _find(train_dir, v) for k, v in FILES.items()}
    have = all(paths.values())
    if synthetic is None:
        synthetic = not have
    if synthetic:
        if verbose:
            print(f"MNIST IDX files not found in {train_dir!r} (no network: nothing is downloaded); "
                  "using deterministic synthetic MNIST of the same shapes.", file=sys.stderr)
        tr_img, tr_lab = synthetic_mnist(60000, seed=1)
        te_img, te_lab = synthetic_mnist(10000, seed=2)
    else:
        tr_img, tr_lab = read_idx(paths["train_images"]), read_idx(paths["train_labels"])
        te_img, te_lab = read_idx(paths["test_images"]), read_idx(paths["test_labels"])
    if one_hot:
        tr_lab, te_lab = dense_to_one_hot(tr_lab), dense_to_one_hot(te_lab)
    else:
        tr_lab, te_lab = tr_lab.astype(np.int64), te_lab.astype(np.int64)
    if not 0 <= validation_size <= len(tr_img):
        raise ValueError(f"validation_size should be between 0 and {len(tr_img)}")
    val = DataSet(tr_img[:validation_size], tr_lab[:validation_size], dtype=dtype, reshape=reshape, seed=seed)
    train = DataSet(tr_img[validation_size:], tr_lab[validation_size:], dtype=dtype, reshape=reshape, seed=seed)
    test = DataSet(te_img, te_lab, dtype=dtype, reshape=reshape, seed=seed)
    return Datasets(train, val, test)
