"""Host -> HBM input pipeline: pinned host staging + async copies on a side HIP stream,
double-buffered (the tf.data ``prefetch_to_device`` of the north star).

    for x, y in DevicePrefetcher(batches, device, depth=2):
        ...  # x, y are already resident in HBM; the next batch is in flight

Each host batch (numpy or CPU tensors) is copied into a page-locked staging buffer, then a
non-blocking copy is enqueued on a dedicated copy stream; the consumer's compute stream waits
on that copy's event only when it takes the batch, so the DMA engine overlaps the H2D transfer
with the previous step's kernels.  Tensors handed out are recorded on the consumer stream so the
caching allocator never recycles them while a kernel still reads them.
"""
from __future__ import annotations

import collections
from typing import Iterable, Iterator, Sequence

import numpy as np
import torch


def _to_tensor(a):
    if isinstance(a, torch.Tensor):
        return a
    return torch.from_numpy(np.ascontiguousarray(a))


class DevicePrefetcher:
    def __init__(self, source: Iterable, device, depth: int = 2):
        self.source = source
        self.device = torch.device(device)
        self.depth = max(1, depth)
        self.gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.gpu else None

    def _stage(self, batch):
        items = batch if isinstance(batch, (tuple, list)) else (batch,)
        out = []
        for a in items:
            t = _to_tensor(a)
            if not self.gpu:
                out.append(t)
                continue
            pinned = t.pin_memory() if not t.is_pinned() else t
            with torch.cuda.stream(self.stream):
                out.append(pinned.to(self.device, non_blocking=True))
        ev = None
        if self.gpu:
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return out, ev, not isinstance(batch, (tuple, list))

    def __iter__(self) -> Iterator:
        it = iter(self.source)
        q = collections.deque()
        for _ in range(self.depth):
            try:
                q.append(self._stage(next(it)))
            except StopIteration:
                break
        while q:
            out, ev, single = q.popleft()
            if ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for t in out:
                    t.record_stream(cur)
            try:
                q.append(self._stage(next(it)))
            except StopIteration:
                pass
            yield out[0] if single else tuple(out)


def batches(arrays: Sequence[np.ndarray], batch_size: int, shuffle: bool = True, seed: int = 0,
            drop_last: bool = True) -> Iterator[tuple]:
    """One epoch of aligned mini-batches over ``arrays`` (first axis)."""
    n = len(arrays[0])
    idx = np.random.RandomState(seed).permutation(n) if shuffle else np.arange(n)
    stop = n - (n % batch_size) if drop_last else n
    for i in range(0, stop, batch_size):
        j = idx[i:i + batch_size]
        yield tuple(a[j] for a in arrays)
