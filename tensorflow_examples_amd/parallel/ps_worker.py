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
from ..data.pipeline import PinnedRing


class AsyncPSWorker:
    def __init__(self, model, client: PSClient, learning_rate: float, naive_xent: bool = True):
        self.model, self.client, self.lr, self.naive = model, client, float(learning_rate), naive_xent
        self.store = client.store
        self.device = self.store.device
        # the feed (feed_dict of R/distributed/distributed.py:150) goes through a fixed pinned ring:
        # host batch -> pinned slot -> async H2D on the copy stream, no per-batch pinning
        self.ring = PinnedRing(self.device, depth=2) if self.device.type == "cuda" else None
        # an xGMI push clears the local gradient in its SGD kernel: no separate zero pass
        self._grad_clean = False

    def _feed(self, *arrays):
        hs = [np.ascontiguousarray(a, dtype=np.float32) for a in arrays]
        if self.ring is None:
            return tuple(torch.from_numpy(h) for h in hs)
        return self.ring.acquire(self.ring.stage(tuple(hs)))

    def _to_dev(self, a) -> torch.Tensor:
        t = torch.as_tensor(np.asarray(a, dtype=np.float32))
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t

    def _push(self) -> int:
        if getattr(self.client, "push_zeroes_grad", False):
            step = self.client.push(self.lr, zero_grad=True)
            self._grad_clean = True
            return step
        return self.client.push(self.lr)

    def step(self, batch_x, batch_y) -> Tuple[float, float, int]:
        """Returns (cost, accuracy, global_step before this update)."""
        x, y = self._feed(batch_x, batch_y)
        self.client.pull()
        if not self._grad_clean:
            self.store.zero_grad()
        logits = self.model.logits(x)
        loss = ops.softmax_cross_entropy(logits, y, naive=self.naive)
        acc = ops.accuracy(logits.detach(), y)
        loss.backward()
        new_step = self._push()
        return float(loss.item()), float(acc.item()), new_step - 1

    @torch.no_grad()
    def evaluate(self, images, labels, batch: int = 10000) -> float:
        self.client.pull()
        hits = 0.0
        for s in range(0, len(images), batch):
            x, y = self._to_dev(images[s:s + batch]), self._to_dev(labels[s:s + batch])
            hits += float(ops.accuracy(self.model.logits(x), y)) * x.shape[0]
        return hits / len(images)


class GraphedPSLoop:
    """The asynchronous xGMI worker step as ONE HIP graph (``--transport=xgmi``, async replicas).

    Per replay, all on the device: the feed -- the batch gathered from the training set resident
    on the GPU at a device-side cursor (the ``feed_dict`` of R/distributed/distributed.py:150
    without a host hop) -- the PULL of every variable out of the ps arenas (xGMI reads), forward,
    the reference's naive cross-entropy and accuracy, backward, the peer SGD into the ps arenas
    and the global-step bump behind it (R/distributed/distributed.py:107-108), and one row
    (cost, accuracy, global step) of a device-side history ring.  The host only enqueues replays;
    it reads the history back at the log cadence (``read``), where the per-step summaries are
    written.  ``dataset`` keeps TF1's ``next_batch`` order (the same RNG draws): the arrangement is
    permuted on the device at each epoch boundary, between replays.
    Requires ``num_examples % batch_size == 0`` (no batch straddles an epoch)."""

    EAGER_STEPS = 2  # run eagerly before the capture (allocator / autograd warm-up)

    def __init__(self, worker: AsyncPSWorker, dataset, batch_size: int, ring: int = 128):
        self.w, self.ds, self.B = worker, dataset, int(batch_size)
        self.dev = worker.device
        self.N = int(dataset.num_examples)
        if self.N % self.B:
            raise ValueError("GraphedPSLoop needs num_examples % batch_size == 0")
        self.X = torch.as_tensor(np.ascontiguousarray(dataset.images, dtype=np.float32)).to(self.dev)
        self.Y = torch.as_tensor(np.ascontiguousarray(dataset.labels, dtype=np.float32)).to(self.dev)
        self.ar = torch.arange(self.B, device=self.dev)
        self.cursor = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.ring = int(ring)
        self.hist = torch.zeros(self.ring, 3, dtype=torch.float64, device=self.dev)
        self.k = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.hist_host = torch.zeros(self.ring, 3, dtype=torch.float64, pin_memory=True)
        self.start = 0          # host mirror of the cursor (TF1 DataSet._index_in_epoch)
        self.pending = 0        # replays since the last read
        self.steps = 0
        self.graph = None

    # ---- feed order: TF1 DataSet.next_batch (R/.../input_data.py), index-only
    def _advance(self) -> None:
        ds = self.ds
        if ds._epochs_completed == 0 and self.start == 0 and ds._index_in_epoch == 0:
            self._permute()
        if self.start + self.B > self.N:
            ds._epochs_completed += 1
            self._permute()
            self.start = 0
            self.cursor.zero_()
        self.start += self.B
        ds._index_in_epoch = self.start

    def _permute(self) -> None:
        perm = np.arange(self.N)
        self.ds._rng.shuffle(perm)
        p = torch.as_tensor(perm, device=self.dev)
        self.X.copy_(self.X.index_select(0, p))
        self.Y.copy_(self.Y.index_select(0, p))

    def _body(self) -> None:
        w = self.w
        idx = self.cursor + self.ar
        x, y = self.X.index_select(0, idx), self.Y.index_select(0, idx)
        self.cursor.add_(self.B)
        w.client.pull()
        logits = w.model.logits(x)
        loss = ops.softmax_cross_entropy(logits, y, naive=w.naive)
        acc = ops.accuracy(logits.detach(), y)
        loss.backward()
        step = w.client.push_async(w.lr, zero_grad=True)
        row = torch.stack([loss.detach().double().reshape(()), acc.double().reshape(()),
                           (step.double() - 1).reshape(())])
        self.hist.index_copy_(0, self.k, row[None])
        self.k.add_(1)

    def step(self) -> None:
        """Enqueue one training step (no host sync)."""
        if self.pending >= self.ring:
            raise RuntimeError("GraphedPSLoop: read() the history at least every %d steps" % self.ring)
        self._advance()
        if self.graph is None and self.steps >= self.EAGER_STEPS:
            s = torch.cuda.Stream(self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(self.graph, stream=s):
                    self._body()
            torch.cuda.current_stream(self.dev).wait_stream(s)
            # the capture recorded the work without running it: replay it for this step
        if self.graph is not None:
            self.graph.replay()
        else:
            self.w.store.zero_grad()
            self._body()
        self.w._grad_clean = True
        self.pending += 1
        self.steps += 1

    def read(self):
        """(cost, accuracy, global step before the update) of every step since the last read."""
        n = self.pending
        self.hist_host[:n].copy_(self.hist[:n], non_blocking=True)
        torch.cuda.current_stream(self.dev).synchronize()
        self.k.zero_()
        self.pending = 0
        return [(float(c), float(a), int(st)) for c, a, st in self.hist_host[:n].tolist()]


class SyncReplicasPSWorker(AsyncPSWorker):
    """Synchronous replicas over the parameter server (``--sync_replicas``).

    The reference only carries a commented-out ``tf.train.SyncReplicasOptimizer`` with
    ``replicas_to_aggregate = total_num_replicas = len(workers)`` (R/distributed/distributed.py:
    109-112).  Its semantics realised here: every global step aggregates the gradients of ALL
    workers.  Each worker pulls the same parameters, computes its gradient, the gradients are
    averaged across workers with one all-reduce of the flat f32 grad buffer (a gloo process group
    over the worker hosts -- the payload is the 318 KB MLP gradient, host-resident anyway for the
    PS push), the chief pushes the average once (the ps applies SGD and bumps ``global_step`` once
    per aggregated step) and broadcasts the new step, which doubles as the barrier that keeps the
    next pull behind the update.
    """

    def __init__(self, model, client, learning_rate: float, group, is_chief: bool, naive_xent: bool = True):
        super().__init__(model, client, learning_rate, naive_xent)
        import torch.distributed as dist
        self.dist, self.group, self.is_chief = dist, group, is_chief
        self.world = dist.get_world_size(group)
        self._host = torch.zeros(self.store.total, dtype=torch.float32)
        self._step_t = torch.zeros(1, dtype=torch.float64)

    def step(self, batch_x, batch_y):
        x, y = self._feed(batch_x, batch_y)
        self.client.pull()
        self.store.zero_grad()
        logits = self.model.logits(x)
        loss = ops.softmax_cross_entropy(logits, y, naive=self.naive)
        acc = ops.accuracy(logits.detach(), y)
        loss.backward()
        self._host.copy_(self.store.grad)
        self.dist.all_reduce(self._host, group=self.group)
        self._host.mul_(1.0 / self.world)
        if self.is_chief:
            self.store.grad.copy_(self._host)
            self._step_t[0] = self.client.push(self.lr)
        self.dist.broadcast(self._step_t, src=0, group=self.group)
        return float(loss.item()), float(acc.item()), int(self._step_t[0]) - 1


def init_worker_group(worker_hosts, task_index: int, port_offset: int = 1000, timeout_s: float = 120.0):
    """gloo process group over the worker tasks: rank = task_index, rendezvous on worker 0's host at
    its port + ``port_offset`` (the worker's own port is the reference's server address)."""
    import datetime

    import torch.distributed as dist
    host, port = worker_hosts[0].rsplit(":", 1)
    dist.init_process_group("gloo", init_method=f"tcp://{host}:{int(port) + port_offset}",
                            rank=task_index, world_size=len(worker_hosts),
                            timeout=datetime.timedelta(seconds=timeout_s))
    return dist.group.WORLD
