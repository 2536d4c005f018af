"""Synchronous data parallelism: bucketed gradient all-reduce over the flat grad buffer,
overlapped with backward.

Design for one MI355X node (8 GPUs, 7 point-to-point xGMI links of ~153 GB/s per GPU):

* one process per GPU, ``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm);
* the gradient of every trainable variable lives in ONE flat f32 buffer laid out in
  creation (= forward) order, so backward produces gradients from the END of the buffer
  towards its start.  Buckets are contiguous slices of that buffer, cut in reverse order:
  a bucket is a single RCCL call on a contiguous view -- no flatten/unflatten copies;
* a bucket is launched the moment its last gradient has been written (the ops fire
  ``store.grad_ready_hook``), so RCCL's ring runs on its own stream beside the remaining
  backward kernels;
* default bucket size 32 MB: a ring over xGMI is bound by one link per hop
  (~2(N-1)/N * S / 153 GB/s ~ 0.37 ms for 32 MB at N = 8), large enough to amortise
  RCCL's launch/latency cost yet small enough that the first bucket starts early in
  backward (ResNet-50: 94 MB of f32 gradients -> 3 buckets);
* averaging is folded into the optimizer (``grad_scale = 1/world``), no extra pass;
* optional bf16 wire format (``compress_bf16``) halves the bytes on the wire: a persistent flat bf16
  twin of the grad buffer (same layout, allocated once -- no per-bucket allocation, graph-safe), each
  bucket cast into it by one vectorised launch right before its collective, reduced IN PLACE in bf16,
  and the fused optimizer reads the reduced bf16 gradients directly into the f32 master update
  (``reduced_grad``) -- no cast back, 47 MB less for the optimizer to read (ResNet-50).

The reference has no synchronous DP at all -- only a commented-out
``SyncReplicasOptimizer`` remnant (R/distributed/distributed.py:110-113); this is the
north-star RCCL path of BASELINE.json (configs 3 and 5).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..variables import ALIGN, Variable, VariableStore


def premul_scalar(factor: float, dtype: torch.dtype) -> float:
    """The Python float to hand ``dist._make_nccl_premul_sum`` so RCCL scales a ``dtype`` buffer by ``factor``.

    On this image (torch 2.10 + RCCL 2.26.6) the pre-multiplied sum of a bf16 buffer reads the LOW 16 bits
    of the 4-byte float scalar torch passes as the bf16 factor: 2.0f = 0x40000000 becomes bf16 0x0000, so
    the collective returned zeros (round 4); a float whose low half is bf16 0x4000 scales by exactly 2
    (measured, ``scripts/diag_premul_bf16.py`` -> ``profiles/r05_dp/diag_premul_bf16.txt``).  For bf16 the
    scalar is therefore built with the factor's bf16 bits in BOTH halves: read as a float it is the
    factor to within 2^-7, read as its low half it is exactly bf16(factor) -- right under either
    interpretation.  Other dtypes get the factor unchanged."""
    if dtype != torch.bfloat16:
        return float(factor)
    b = int(torch.tensor([factor], dtype=torch.bfloat16).view(torch.int16).item()) & 0xFFFF
    return float(torch.tensor([(b << 16) | b], dtype=torch.int64).to(torch.int32).view(torch.float32).item())


class GradAllReduce:
    def __init__(self, store: VariableStore, bucket_bytes: int = 32 << 20, group=None, overlap: bool = True,
                 compress_bf16: bool = False, tail_bytes: int = 2 << 20, force_collective: Optional[bool] = None,
                 premul: Optional[float] = None, simulate_ring: Optional[dict] = None):
        self.store = store
        # simulate_ring = {"blocks": B, "ranks": N, "link_gbps": G, "latency_us": L}: one-GPU contention
        # rehearsal of an N-rank node (scripts/dp_contention.py) -- each bucket's collective is replaced by
        # dp_ring_sim: B workgroups streaming the bucket on a side stream for the ring's modelled time
        # 2 (N-1)/N S / G + L, forked at the bucket's ready point and joined before the optimizer
        self.sim = dict(simulate_ring) if simulate_ring else None
        self._sim_stream = None
        self._sim_events = []
        self.group = group
        # premul: RCCL pre-multiplied sum (each rank's bucket scaled by `premul` inside the
        # collective).  Used by the GPU tests to make a 1-rank collective observable: a bucket whose
        # all-reduce was dropped, or ran before its gradient was written, then shows up as a wrong
        # (unscaled) gradient.  With the bf16 wire the scalar is encoded by premul_scalar (RCCL reads a
        # bf16 factor from the float's low half on this image).
        self.premul = premul
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # issue the collectives even at world size 1 (TFX_DP_FORCE_COLLECTIVE=1): lets a one-GPU box
        # exercise the RCCL launch / HIP-graph capture path of the DP step
        if force_collective is None:
            force_collective = os.environ.get("TFX_DP_FORCE_COLLECTIVE", "0") == "1"
        self.force = bool(force_collective) and dist.is_initialized()
        self.overlap = overlap
        self.compress = compress_bf16
        # the bf16 twin of the flat grad buffer (zeros outside the buckets: padding and frozen vars)
        self.grad16 = torch.zeros_like(store.grad, dtype=torch.bfloat16) if compress_bf16 else None
        self._used16 = False
        elem = store.grad.element_size()
        cap = max(1, bucket_bytes // elem)
        tail_cap = max(1, tail_bytes // elem)
        self.buckets: List[List[int]] = []  # [lo, hi) element ranges of the flat grad buffer
        self.members: List[List[Variable]] = []
        self.var_bucket: Dict[int, int] = {}
        groups: List[List[Variable]] = []
        cur: List[Variable] = []
        size = 0
        for v in reversed(store.trainable()):
            cur.append(v)
            size += v.numel
            if size >= cap:
                groups.append(cur)
                cur, size = [], 0
        if cur:
            groups.append(cur)
        # The LAST bucket holds the first layers' gradients, which are ready only when backward
        # ends: its all-reduce is the one part that cannot overlap compute.  Cut it down to a tail of
        # at most ``tail_bytes`` (ResNet-50: the stem + stage-1 grads, ~1 MB) so the exposed
        # collective is short; the rest of that group still overlaps the early layers' backward.
        if tail_bytes > 0 and groups and sum(v.numel for v in groups[-1]) > tail_cap:
            last = groups.pop()
            acc, k = 0, len(last)
            while k > 0 and acc + last[k - 1].numel <= tail_cap:
                k -= 1
                acc += last[k].numel
            if 0 < k < len(last):
                groups.extend([last[:k], last[k:]])
            else:
                groups.append(last)
        for g in groups:
            self._close(g)
        self._pending: List[int] = []
        self._launched: List[bool] = []
        self._works = []
        if overlap and (self.world > 1 or self.force or self.sim):
            store.grad_ready_hook = self._on_ready
        self.start_step()

    def _close(self, vs: List[Variable]) -> None:
        lo = min(v.offset for v in vs)
        # every bucket spans whole ALIGN-element (256-B) granules: the store pads each variable to
        # ALIGN, so the padding is zeros owned by nobody.  RCCL's pre-multiplied sum left the tail
        # of a bucket ending mid-granule unscaled (ResNet fc/bias, 10 floats: profiles/r02_dp/
        # diag_rccl_18.log) -- keep every collective on a 256-B multiple.
        hi = min(self.store.total, -(-max(v.offset + v.numel for v in vs) // ALIGN) * ALIGN)
        b = len(self.buckets)
        self.buckets.append([lo, hi])
        self.members.append(list(vs))
        for v in vs:
            self.var_bucket[v.index] = b

    @property
    def bucket_sizes_bytes(self) -> List[int]:
        e = self.store.grad.element_size()
        return [(hi - lo) * e for lo, hi in self.buckets]

    def reset(self) -> None:
        """Abandon a step that failed part-way through backward (e.g. a HIP-graph capture error):
        its queued Work objects may be captured, never-executed collectives, so they are dropped
        without waiting, and the next step starts with every bucket pending."""
        self.start_step()

    def _on_ready(self, v: Variable) -> None:
        b = self.var_bucket.get(v.index)
        if b is None:
            return
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def sim_ring_us(self, nbytes: int) -> float:
        n, g = self.sim.get("ranks", 8), self.sim.get("link_gbps", 153.0)
        return 2.0 * (n - 1) / n * nbytes / (g * 1e3) + self.sim.get("latency_us", 0.0)

    def _launch_sim(self, b: int) -> None:
        lo, hi = self.buckets[b]
        view = self.store.grad[lo:hi]
        if self.compress:  # the bf16 wire: the cast runs on the compute stream as in the real path
            g16 = self.grad16[lo:hi]
            torch.ops.tfx.cast_f32_bf16(view, g16)
            self._used16 = True
            view = g16
        if self._sim_stream is None:
            self._sim_stream = torch.cuda.Stream()
        cur = torch.cuda.current_stream()
        self._sim_stream.wait_stream(cur)
        with torch.cuda.stream(self._sim_stream):
            torch.ops.tfx.dp_ring_sim(view, int(self.sim.get("blocks", 16)),
                                      float(self.sim_ring_us(view.numel() * view.element_size())),
                                      int(self.sim.get("passes", 2)))
            e = torch.cuda.Event()
            e.record()
        self._sim_events.append(e)

    def _launch(self, b: int) -> None:
        if self.sim is not None and not self._launched[b]:
            self._launched[b] = True
            self._launch_sim(b)
            return
        if self._launched[b] or (self.world == 1 and not self.force):
            self._launched[b] = True
            return
        self._launched[b] = True
        lo, hi = self.buckets[b]
        view = self.store.grad[lo:hi]
        if view.is_cuda and torch.cuda.is_current_stream_capturing() and \
                dist.get_backend(self.group) != dist.Backend.NCCL:
            # only RCCL collectives are stream-ordered device work a HIP graph can record; refuse
            # before forking the launch stream (a forked, never-joined stream would stay capturing)
            raise RuntimeError("HIP graph capture of the DP step needs the nccl (RCCL) backend, not %s"
                               % dist.get_backend(self.group))
        op = dist.ReduceOp.SUM if self.premul is None else \
            dist._make_nccl_premul_sum(premul_scalar(self.premul, torch.bfloat16 if self.compress else view.dtype))
        # issued from the compute stream right after the bucket's last gradient kernel: RCCL runs it
        # on its own stream, ordered after that kernel, beside the rest of backward
        if self.compress:
            g16 = self.grad16[lo:hi]
            if view.is_cuda:
                torch.ops.tfx.cast_f32_bf16(view, g16)
            else:
                g16.copy_(view)
            self._used16 = True
            self._works.append((dist.all_reduce(g16, op=op, group=self.group, async_op=True), None, None))
        else:
            self._works.append((dist.all_reduce(view, op=op, group=self.group, async_op=True), None, None))

    def finish(self) -> None:
        """Launch buckets not yet started (in order) and make the current stream wait for all."""
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        for work, view, tmp in self._works:
            work.wait()
            if view is not None:
                view.copy_(tmp)
        for e in self._sim_events:
            torch.cuda.current_stream().wait_event(e)
        self._sim_events = []
        self._pending = [len(m) for m in self.members]
        self._launched = [False] * len(self.buckets)
        self._works = []

    def start_step(self) -> None:
        self._pending = [len(m) for m in self.members]
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._sim_events = []
        self._used16 = False

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    @property
    def reduced_grad(self) -> Optional[torch.Tensor]:
        """The flat buffer holding the all-reduced gradients for the optimizer: the bf16 twin when the
        bf16 wire format ran collectives this step, else None (the f32 grad buffer itself)."""
        return self.grad16 if (self.compress and self._used16) else None


def broadcast_variables(store: VariableStore, src: int = 0, group=None) -> None:
    """Make every rank start from rank ``src``'s weights (one broadcast of the flat buffer)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.broadcast(store.master, src=src, group=group)
    for sv in store.sparse:
        dist.broadcast(sv.table, src=src, group=group)
    for t in store.state.values():
        dist.broadcast(t, src=src, group=group)
    store.refresh_shadow()
