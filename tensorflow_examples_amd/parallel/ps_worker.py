"""One asynchronous parameter-server training step (between-graph replication).

Equivalent of the reference worker's
``sess.run([train_op, cross_entropy, summary_op, global_step], feed_dict=...)``
(R/distributed/distributed.py:148-150): pull every variable from its ps task -> forward ->
naive softmax cross-entropy + accuracy (summary values) -> backward -> push gradients; the ps
applies ApplyGradientDescent and AssignAdd(global_step).  On the GPU the model runs on the exact
f32 MFMA GEMM kernels with fused bias+sigmoid (sgemm.hip) and the fused naive-xent kernel.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from .. import ops
from ..cluster.ps import PSClient


class AsyncPSWorker:
    def __init__(self, model, client: PSClient, learning_rate: float, naive_xent: bool = True):
        self.model, self.client, self.lr, self.naive = model, client, float(learning_rate), naive_xent
        self.store = client.store
        self.device = self.store.device

    def _to_dev(self, a) -> torch.Tensor:
        t = torch.as_tensor(np.asarray(a, dtype=np.float32))
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t

    def step(self, batch_x, batch_y) -> Tuple[float, float, int]:
        """Returns (cost, accuracy, global_step before this update)."""
        x, y = self._to_dev(batch_x), self._to_dev(batch_y)
        self.client.pull()
        self.store.zero_grad()
        logits = self.model.logits(x)
        loss = ops.softmax_cross_entropy(logits, y, naive=self.naive)
        acc = ops.accuracy(logits.detach(), y)
        loss.backward()
        new_step = self.client.push(self.lr)
        return float(loss.item()), float(acc.item()), new_step - 1

    @torch.no_grad()
    def evaluate(self, images, labels, batch: int = 10000) -> float:
        self.client.pull()
        hits = 0.0
        for s in range(0, len(images), batch):
            x, y = self._to_dev(images[s:s + batch]), self._to_dev(labels[s:s + batch])
            hits += float(ops.accuracy(self.model.logits(x), y)) * x.shape[0]
        return hits / len(images)
