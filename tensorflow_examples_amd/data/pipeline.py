"""Host -> HBM input pipeline: a fixed ring of pinned host staging slots + async H2D copies on a
side HIP stream (the north star's "pinned-host hipMemcpyAsync double-buffering"; it replaces
TF1's per-step ``feed_dict`` conversion, R/distributed/distributed.py:146-150).

    ring = PinnedRing(device, depth=2)
    slot = ring.stage((x_np, y_np))      # host copy into a pinned slot, async H2D on the copy stream
    x, y = ring.acquire(slot)            # compute stream waits on that copy's event only

    for x, y in DevicePrefetcher(batches, device, depth=2):
        ...  # x, y already resident in HBM; the next `depth` batches are in flight

Every slot owns, for each field, one page-locked host buffer and one device buffer, allocated once
(re-allocated only if a batch's shape changes, e.g. a ragged last batch) -- no per-batch
``pin_memory()`` or device allocation.  Two events per slot order the reuse:

* ``h2d``: recorded on the copy stream after the slot's async copy.  The compute stream waits on it
  in :meth:`acquire`; the host waits on it (normally long since complete) before it overwrites the
  slot's pinned buffer with a later batch.
* ``free``: recorded on the compute stream when the consumer asks for its NEXT batch (every kernel
  that read this slot's device tensors has been enqueued by then).  The copy stream waits on it
  before it overwrites the slot's device buffer -- a device-side dependency, no host sync.

So a tensor handed out by :meth:`acquire` stays valid until the consumer has acquired ``depth``
more batches.  On the CPU (no GPU) the ring degenerates to plain tensors.
"""
from __future__ import annotations

from typing import Iterable, Iterator, List, Optional, Sequence

import numpy as np
import torch


def _to_tensor(a):
    if isinstance(a, torch.Tensor):
        return a
    return torch.from_numpy(np.ascontiguousarray(a))


class _Slot:
    __slots__ = ("host", "dev", "h2d", "free", "h2d_pending", "free_pending")

    def __init__(self):
        self.host: List[torch.Tensor] = []
        self.dev: List[torch.Tensor] = []
        self.h2d = None
        self.free = None
        self.h2d_pending = False
        self.free_pending = False


class PinnedRing:
    """``zero_copy=True``: no device staging buffers and no copy stream -- :meth:`acquire` hands out
    the pinned host tensors themselves and the consumer's first kernel reads them over the host
    link (``torch.ops.tfx.image_normalize_into`` maps page-locked memory into the GPU's address
    space).  The host then waits on a slot's ``free`` event (the consumer's kernels that read it have
    run) before overwriting it; ``nslots`` = ``depth`` + 1 slots let the host run ``depth`` steps
    ahead of the GPU."""

    def __init__(self, device, depth: int = 2, zero_copy: bool = False):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.zero_copy = bool(zero_copy) and self.gpu
        # depth batches in flight + the one being consumed
        self.nslots = max(1, depth) + 1
        self.slots = [_Slot() for _ in range(self.nslots)]
        self.stream = torch.cuda.Stream(self.device) if self.gpu and not self.zero_copy else None
        self._next = 0
        self._held: Optional[int] = None
        if self.gpu:
            for s in self.slots:
                s.h2d = torch.cuda.Event()
                s.free = torch.cuda.Event()

    def _ensure(self, s: _Slot, items: Sequence[torch.Tensor]) -> None:
        same = len(s.host) == len(items) and all(
            h.shape == t.shape and h.dtype == t.dtype for h, t in zip(s.host, items))
        if same:
            return
        # (re)allocate once: every earlier use of the old buffers must have finished
        if s.h2d_pending:
            s.h2d.synchronize()
        if s.free_pending:
            s.free.synchronize()
        s.host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in items]
        s.dev = s.host if self.zero_copy else [torch.empty(t.shape, dtype=t.dtype, device=self.device) for t in items]

    def stage(self, batch) -> int:
        """Copy one host batch (tuple of arrays/CPU tensors) into the next slot and start its async
        H2D copy.  Returns the slot id to :meth:`acquire`."""
        items = [_to_tensor(a) for a in (batch if isinstance(batch, (tuple, list)) else (batch,))]
        k = self._next
        self._next = (k + 1) % self.nslots
        s = self.slots[k]
        if not self.gpu:
            s.dev = items
            return k
        if k == self._held:
            raise RuntimeError("PinnedRing: staging over the slot still held by the consumer (too many in flight)")
        self._ensure(s, items)
        if self.zero_copy:
            # the consumer's kernels read this pinned buffer directly: they must have run
            if s.free_pending:
                s.free.synchronize()
                s.free_pending = False
            for h, t in zip(s.host, items):
                h.copy_(t)
            return k
        if s.h2d_pending:  # the previous copy out of this pinned buffer must have been read
            s.h2d.synchronize()
        for h, t in zip(s.host, items):
            h.copy_(t)
        with torch.cuda.stream(self.stream):
            if s.free_pending:  # the consumer's kernels on the old device contents are enqueued first
                self.stream.wait_event(s.free)
            for d, h in zip(s.dev, s.host):
                d.copy_(h, non_blocking=True)
            s.h2d.record(self.stream)
        s.h2d_pending = True
        return k

    def acquire(self, k: int):
        """Device tensors of slot ``k``; the current stream waits for their copy.  The slot acquired
        before this one is released (its ``free`` event recorded on the current stream)."""
        s = self.slots[k]
        if self.gpu:
            cur = torch.cuda.current_stream(self.device)
            if self._held is not None and self._held != k:
                h = self.slots[self._held]
                h.free.record(cur)
                h.free_pending = True
            if not self.zero_copy:
                cur.wait_event(s.h2d)
        self._held = k
        return tuple(s.dev)

    @classmethod
    def for_batches(cls, host_batches: Sequence, device, depth: int = 2, zero_copy: bool = False) -> "CyclicFeeder":
        return CyclicFeeder(host_batches, cls(device, depth, zero_copy=zero_copy), depth)

    def close(self) -> None:
        if self.stream is not None:
            self.stream.synchronize()
        elif self.zero_copy:
            torch.cuda.synchronize(self.device)  # no kernel may still read a pinned slot
        self.slots = []


class CyclicFeeder:
    """Feeds a fixed list of host batches round-robin through a :class:`PinnedRing`, ``depth``
    batches ahead of the consumer (bench.py ``--host-input``): each :meth:`next` returns the next
    batch on the device, its H2D copy issued ``depth`` calls earlier."""

    def __init__(self, host_batches: Sequence, ring: PinnedRing, depth: int):
        self.host, self.ring, self.depth = list(host_batches), ring, max(1, depth)
        self._q: List[int] = []
        self._n = 0  # batches staged so far

    def _stage_one(self) -> None:
        self._q.append(self.ring.stage(self.host[self._n % len(self.host)]))
        self._n += 1

    def next(self):
        if self.ring.zero_copy:
            # nothing to prefetch (no copy): stage on demand into the slot used nslots batches ago,
            # whose free event is nslots - 1 steps old -- the host stays that far ahead of the GPU
            self._stage_one()
            return self.ring.acquire(self._q.pop(0))
        if not self._q:
            self._stage_one()
        out = self.ring.acquire(self._q.pop(0))
        while len(self._q) < self.depth:
            self._stage_one()
        return out

    def close(self) -> None:
        self.ring.close()


class DevicePrefetcher:
    """Iterate host batches as device tensors, ``depth`` batches ahead (tf.data prefetch_to_device).

    Lifetime: on a GPU the yielded tensors ARE the ring's device slot.  Work enqueued on the current
    stream before the iterator advances may read them; the slot is released at the next step and
    overwritten ``depth`` + 1 batches later, so a batch kept beyond its step (e.g. for evaluation at
    the end of an epoch) must be copied -- ``copy=True`` yields a private clone of every batch
    (one device-to-device copy per tensor, made on the current stream)."""

    def __init__(self, source: Iterable, device, depth: int = 2, copy: bool = False):
        self.source = source
        self.ring = PinnedRing(device, depth)
        self.depth = max(1, depth)
        self.copy = bool(copy)

    def __iter__(self) -> Iterator:
        it = iter(self.source)
        q: List[tuple] = []
        single = False
        for _ in range(self.depth):
            try:
                b = next(it)
            except StopIteration:
                break
            single = not isinstance(b, (tuple, list))
            q.append(self.ring.stage(b))
        while q:
            k = q.pop(0)
            out = self.ring.acquire(k)
            if self.copy:
                out = tuple(t.clone() for t in out)
            try:
                b = next(it)
                single = not isinstance(b, (tuple, list))
                q.append(self.ring.stage(b))
            except StopIteration:
                pass
            yield out[0] if single else out


def batches(arrays: Sequence[np.ndarray], batch_size: int, shuffle: bool = True, seed: int = 0,
            drop_last: bool = True) -> Iterator[tuple]:
    """One epoch of aligned mini-batches over ``arrays`` (first axis)."""
    n = len(arrays[0])
    idx = np.random.RandomState(seed).permutation(n) if shuffle else np.arange(n)
    stop = n - (n % batch_size) if drop_last else n
    for i in range(0, stop, batch_size):
        j = idx[i:i + batch_size]
        yield tuple(a[j] for a in arrays)
