"""Tracing: roctx ranges around the phases of a training step + device-event step timers.

The reference's only instrumentation is wall-clock deltas printed every 100 steps
(R/distributed/distributed.py:133,140,155-161).  This module adds what a
MI355X user profiles with:

* ``range(name)`` -- a roctx range (``roctxRangePushA`` / ``roctxRangePop`` from ROCm's
  ``librocprofiler-sdk-roctx`` or ``libroctx64``), so ``rocprofv3 --marker-trace`` shows the
  forward / backward / all-reduce / optimizer phases of each step on the timeline next to the
  kernels.  Enabled by ``TFX_ROCTX=1`` (or :func:`enable`); otherwise a no-op costing one
  attribute test.  Ranges are host-side: inside a captured HIP graph they mark the capture, not
  each replay.
* :class:`StepTimer` -- per-step device time from HIP events recorded on the current stream
  (no host synchronisation inside the loop), with a ``perf_counter`` fallback on the CPU.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import List, Optional

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


class _Roctx:
    def __init__(self):
        self.lib = None
        self.on = False

    def load(self) -> bool:
        if self.lib is not None:
            return True
        roots = [os.environ.get("ROCM_PATH", "/opt/rocm")]
        for name in _LIBS:
            for cand in [os.path.join(r, "lib", name) for r in roots] + [name]:
                try:
                    lib = ctypes.CDLL(cand)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    self.lib = lib
                    return True
                except (OSError, AttributeError):
                    continue
        return False


_R = _Roctx()


def enable(on: bool = True) -> bool:
    """Turn roctx ranges on (returns False if no roctx library could be loaded)."""
    _R.on = bool(on) and _R.load()
    return _R.on


def enabled() -> bool:
    return _R.on


@contextlib.contextmanager
def range(name: str):  # noqa: A001  (mirrors roctx's vocabulary)
    if not _R.on:
        yield
        return
    _R.lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _R.lib.roctxRangePop()


def mark(name: str) -> None:
    if _R.on:
        _R.lib.roctxMarkA(name.encode())


class StepTimer:
    """Device-side step timing: ``start()`` / ``stop()`` around each step record HIP events on the
    current stream; :meth:`summary` synchronises once and returns per-step milliseconds."""

    def __init__(self, device=None):
        import torch
        self.cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self._events: List = []
        self._t0: Optional[float] = None
        self._cpu: List[float] = []

    def start(self) -> None:
        if self.cuda:
            import torch
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append([e, None])
        else:
            self._t0 = time.perf_counter()

    def stop(self) -> None:
        if self.cuda:
            import torch
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events[-1][1] = e
        else:
            self._cpu.append((time.perf_counter() - self._t0) * 1e3)

    def times_ms(self) -> List[float]:
        if self.cuda:
            import torch
            torch.cuda.synchronize()
            return [a.elapsed_time(b) for a, b in self._events if b is not None]
        return list(self._cpu)

    def summary(self) -> dict:
        t = sorted(self.times_ms())
        if not t:
            return {"steps": 0}
        return {"steps": len(t), "mean_ms": sum(t) / len(t), "p50_ms": t[len(t) // 2], "min_ms": t[0],
                "max_ms": t[-1]}


if os.environ.get("TFX_ROCTX", "0") not in ("", "0"):
    enable(True)
