"""Process-group bring-up: one process per GPU, rendezvous over 127.0.0.1 by default.

Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun contract).
Backend: ``nccl`` (RCCL over xGMI) for GPU runs, ``gloo`` for CPU runs and CPU tests.
"""
from __future__ import annotations

import os
from datetime import timedelta

import torch
import torch.distributed as dist


def world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def rank() -> int:
    return int(os.environ.get("RANK", "0"))


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: str | None = None, device: str = "cuda", timeout_s: int = 600):
    """Initialise the default process group if WORLD_SIZE > 1. Returns the device to use."""
    ws = world_size()
    if device == "cuda":
        dev = torch.device("cuda", local_rank())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    # TFX_DP_FORCE_COLLECTIVE=1 under a launcher: a 1-rank process group, so a one-GPU box runs the
    # real RCCL path of the DP step (GradAllReduce issues its collectives at world size 1 too)
    force = os.environ.get("TFX_DP_FORCE_COLLECTIVE", "0") == "1" and "RANK" in os.environ
    if (ws > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = backend or ("nccl" if dev.type == "cuda" else "gloo")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend=backend, rank=rank(), world_size=ws, timeout=timedelta(seconds=timeout_s), **kw)
    return dev
