"""Pinned-ring input pipeline (data/pipeline.py) on the GPU: slot reuse must never overwrite a batch
that a queued kernel still reads, and the copies must arrive before the consumer's kernels run."""
import numpy as np
import pytest
import torch

from tensorflow_examples_amd.data.pipeline import DevicePrefetcher, PinnedRing

pytestmark = pytest.mark.gpu


def _host_batches(n, rows=4096, cols=256, ragged_last=False):
    out = []
    for i in range(n):
        r = rows if not (ragged_last and i == n - 1) else rows // 2
        out.append((np.full((r, cols), float(i), dtype=np.float32), np.full((r,), i, dtype=np.int64)))
    return out


def test_prefetcher_values_with_slow_consumer(gpu):
    batches = _host_batches(12, ragged_last=True)
    big = torch.randn(2048, 2048, device=gpu)
    seen = []
    for i, (x, y) in enumerate(DevicePrefetcher(batches, gpu, depth=2)):
        for _ in range(4):  # keep the compute stream busy so later copies queue behind it
            big = big @ big * 1e-3
        seen.append((x.sum(), y.float().sum(), x.shape[0]))
    torch.cuda.synchronize()
    assert len(seen) == 12
    for i, (sx, sy, rows) in enumerate(seen):
        assert float(sx) == float(i) * rows * 256, (i, float(sx))
        assert float(sy) == float(i) * rows, (i, float(sy))


def test_ring_reuses_fixed_buffers(gpu):
    ring = PinnedRing(gpu, depth=2)
    batches = _host_batches(9)
    ptrs = set()
    for i, b in enumerate(batches):
        k = ring.stage(b)
        x, _ = ring.acquire(k)
        ptrs.add(x.data_ptr())
        assert float(x[0, 0]) == float(i)
    assert len(ptrs) == ring.nslots  # one device buffer per slot, allocated once
    ring.close()


def test_bench_host_input_runs(gpu):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--depth", "18", "--batch", "32", "--steps", "4",
           "--warmup", "2", "--host-input"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["config"]["host_input"] is True and rec["value"] > 0
