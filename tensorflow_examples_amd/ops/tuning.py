"""Measured igemm launch configurations (csrc/kernels/igemm.hip ``igemm_tune_*``).

The implicit-GEMM dispatcher picks a tile shape, in-block split-K groups, LDS-DMA ring depth and a
split-K block target per launch from built-in heuristics.  ``scripts/tune_convs.py`` times every
candidate configuration of every ResNet-50/CIFAR conv (forward with its fused BN-statistics epilogue,
data gradient with its fused BN-backward epilogue, weight gradient) on an MI355X and writes the
winners -- keyed by (kernel family, M, N, K) -- to ``tune/igemm_gfx950.json``.  The table is loaded
into the dispatcher when the kernel library loads; ``TFX_TUNE=0`` ignores it (A/B), ``TFX_TUNE_FILE``
points at another table.  ``scripts/tune_step.py`` then re-checks each row inside the graph-replayed
training step (rows marked ``step-tuned``; profiles/r06_tune_step).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tune", "igemm_gfx950.json")

FAMILIES = ["fwd_pointwise", "fwd_im2col", "dgrad_pointwise", "dgrad_general", "dgrad_cls_dense", "dgrad_cls",
            "wgrad_dense", "wgrad_x", "wgrad_t_x", "dgrad_flip"]
ATOMIC_FAMILIES = {6, 7, 8}


def load(path: Optional[str] = None) -> int:
    """Install the table into the dispatcher; returns the number of entries (0 when disabled)."""
    if os.environ.get("TFX_TUNE", "1") == "0":
        return 0
    path = path or os.environ.get("TFX_TUNE_FILE", TABLE)
    if not os.path.exists(path):
        return 0
    with open(path) as f:
        entries = json.load(f).get("entries", [])
    for e in entries:
        torch.ops.tfx.igemm_tune_set(int(e["fam"]), int(e["M"]), int(e["N"]), int(e["K"]), int(e["tile"]),
                                     int(e.get("ks", 0)), int(e.get("gls", -1)), int(e.get("want", 0)))
    return len(entries)


def clear() -> None:
    torch.ops.tfx.igemm_tune_clear()
