"""Loader for the in-tree HIP kernel library (``_lib/libtfx_ops.so``).

GPU tensors ALWAYS go through the hand-written gfx950 kernels.  If the library is
missing on a machine with a GPU the first op raises -- there is no silent eager
fallback (set ``TFX_ALLOW_TORCH_FALLBACK=1`` only for debugging; it is never used by
tests marked ``gpu`` or by ``bench.py``).  CPU tensors use the PyTorch reference
implementations in :mod:`tensorflow_examples_amd.ops.nn`, which are also the numerics
oracle for the kernel tests.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")
# TFX_OPS_LIB: another build of the kernel library (same-box A/B runs of two builds)
OPS_LIB = os.environ.get("TFX_OPS_LIB") or os.path.join(_LIB_DIR, "libtfx_ops.so")
RT_LIB = os.path.join(_LIB_DIR, "libtfx_rt.so")

_lock = threading.Lock()
_loaded = False
_load_error: Exception | None = None


def load() -> bool:
    """Load libtfx_ops.so once; returns True on success."""
    global _loaded, _load_error
    with _lock:
        if _loaded:
            return True
        if _load_error is not None:
            return False
        try:
            if not os.path.exists(OPS_LIB):
                raise FileNotFoundError(f"{OPS_LIB} not built (run `python build.py`)")
            torch.ops.load_library(OPS_LIB)
            from . import tuning
            tuning.load()
            _loaded = True
        except Exception as e:  # pragma: no cover - depends on build state
            _load_error = e
        return _loaded


def available() -> bool:
    return load()


def fallback_allowed() -> bool:
    return os.environ.get("TFX_ALLOW_TORCH_FALLBACK", "0") == "1"


_ref = threading.local()


class reference_mode:
    """Context manager: run the PyTorch reference implementation of every op even on GPU tensors.
    Tests only -- it builds an fp32 (or bf16) PyTorch oracle of the SAME model on the GPU, for
    shapes too large for the CPU (the batch-256 ResNet-50 gradient check)."""

    def __enter__(self):
        self._prev = getattr(_ref, "on", False)
        _ref.on = True
        return self

    def __exit__(self, *exc):
        _ref.on = self._prev


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU: then the HIP kernel path is mandatory."""
    if t.device.type != "cuda" or getattr(_ref, "on", False):
        return False
    if load():
        return True
    if fallback_allowed():
        return False
    raise RuntimeError(f"tensorflow_examples_amd: HIP kernel library unavailable on a GPU run: {_load_error}")


def use_native_device(device: torch.device) -> bool:
    """use_native for a device instead of a tensor."""
    if device.type != "cuda" or getattr(_ref, "on", False):
        return False
    if load():
        return True
    if fallback_allowed():
        return False
    raise RuntimeError(f"tensorflow_examples_amd: HIP kernel library unavailable on a GPU run: {_load_error}")


def ops():
    if not load():
        raise RuntimeError(f"HIP kernel library unavailable: {_load_error}")
    return torch.ops.tfx
