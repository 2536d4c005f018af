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
    assert rec["config"]["host_input"] == "zerocopy" and rec["value"] > 0


def test_image_normalize_into_zero_copy_matches_reference(gpu):
    from tensorflow_examples_amd.models.resnet import _MEAN, _STD, to_model_input
    g = torch.Generator().manual_seed(3)
    img = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g)
    ref = to_model_input(img, dtype=torch.float32)  # CPU fp32 reference path
    dev_out = to_model_input(img.to(gpu))  # device-resident input
    pin_out = to_model_input(img.pin_memory(), device=gpu)  # zero-copy from pinned host memory
    torch.cuda.synchronize()
    assert pin_out.device.type == "cuda" and pin_out.shape == (16, 32, 32, 8)
    assert torch.equal(pin_out, dev_out)
    assert (pin_out.float().cpu() - ref).abs().max().item() < 2e-2
    assert float(pin_out[..., 3:].abs().max()) == 0.0
    with pytest.raises(RuntimeError):  # pageable host memory is refused, not silently copied
        torch.ops.tfx.image_normalize_into(img, list(_MEAN), list(_STD), torch.empty_like(dev_out), None, None)


def test_input_kernel_carries_labels(gpu):
    """The input kernel copies the batch's labels (pinned host or device) into a label buffer in the
    same launch; to_model_batch falls back to a plain copy without static buffers."""
    from tensorflow_examples_amd.models.resnet import _MEAN, _STD, to_model_batch, to_model_input
    g = torch.Generator().manual_seed(3)
    img = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, generator=g).pin_memory()
    lab = torch.randint(0, 10, (16,), dtype=torch.int64, generator=g).pin_memory()
    ref = to_model_input(img.to(gpu))
    xo = torch.empty_like(ref)
    yo = torch.full((16,), -1, dtype=torch.int64, device=gpu)
    x, y = to_model_batch(img, lab, device=gpu, out=xo, labels_out=yo)
    torch.cuda.synchronize()
    assert x is xo and y is yo and torch.equal(x, ref) and torch.equal(y.cpu(), lab)
    yo2 = torch.full((16,), -1, dtype=torch.int64, device=gpu)
    x2, y2 = to_model_batch(img.to(gpu), lab.to(gpu), device=gpu, out=torch.empty_like(ref), labels_out=yo2)
    assert torch.equal(x2, ref) and torch.equal(y2.cpu(), lab)
    x3, y3 = to_model_batch(img, lab, device=gpu)  # no static buffers: zero-copy image, copied labels
    assert torch.equal(x3, ref) and y3.is_cuda and torch.equal(y3.cpu(), lab)
    with pytest.raises(RuntimeError):  # pageable host labels are refused, not silently copied
        torch.ops.tfx.image_normalize_into(img, list(_MEAN), list(_STD), torch.empty_like(ref), lab.clone(), yo)


def test_zero_copy_ring_never_overwrites_a_queued_batch(gpu):
    """The host restages a slot only after the kernels that read it (queued behind slow work) ran."""
    from tensorflow_examples_amd.models.resnet import to_model_input
    host = [(torch.full((8, 32, 32, 3), 10 * i, dtype=torch.uint8), torch.full((8,), i, dtype=torch.long))
            for i in range(7)]
    feeder = PinnedRing.for_batches(host, gpu, depth=2, zero_copy=True)
    big = torch.randn(2048, 2048, device=gpu)
    outs = []
    for i in range(20):
        for _ in range(3):  # keep the stream busy so the host runs ahead of the GPU
            big = big @ big * 1e-3
        img, lab = feeder.next()
        assert img.device.type == "cpu" and img.is_pinned()
        outs.append((to_model_input(img, device=gpu), lab.to(gpu, non_blocking=True)))
    torch.cuda.synchronize()
    ref = [to_model_input(h[0].to(gpu)) for h in host]
    for i, (x, y) in enumerate(outs):
        assert torch.equal(x, ref[i % 7]), i
        assert int(y[0]) == i % 7
    feeder.close()


def test_bench_host_input_copy_mode_runs(gpu):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--depth", "18", "--batch", "32", "--steps", "4",
           "--warmup", "2", "--host-input", "copy"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["config"]["host_input"] == "copy" and rec["value"] > 0


def test_fused_augment_normalize_matches_two_step(gpu):
    """augment_model_input: crop + flip + normalise in one HIP kernel == augment() then
    to_model_input() with the same per-image offsets (bit-exact: same fma), incl. padding pixels."""
    from tensorflow_examples_amd.data.cifar import augment, augment_model_input, augment_offsets
    from tensorflow_examples_amd.models.resnet import to_model_input
    g = torch.Generator(device=gpu).manual_seed(11)
    img = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=gpu)
    off = augment_offsets(64, gpu, g)
    off[0] = torch.tensor([0, 0, 1], dtype=torch.int32, device=gpu)  # corner crop + flip: padding visible
    off[1] = torch.tensor([8, 8, 0], dtype=torch.int32, device=gpu)
    fused = augment_model_input(img, offsets=off)
    ref = to_model_input(augment(img, offsets=off))
    torch.cuda.synchronize()
    assert fused.shape == (64, 32, 32, 8) and fused.dtype == torch.bfloat16
    assert torch.equal(fused, ref)
    cpu = augment_model_input(img.cpu(), dtype=torch.float32, offsets=off.cpu())  # the CPU reference path
    assert (cpu - fused.float().cpu()).abs().max().item() < 2e-2


def test_prefetcher_copy_keeps_batches(gpu):
    """copy=True: batches held past their step keep their values (the ring slots are overwritten)."""
    batches = _host_batches(8)
    kept = [x for x, _ in DevicePrefetcher(batches, gpu, depth=2, copy=True)]
    torch.cuda.synchronize()
    for i, x in enumerate(kept):
        assert float(x.mean()) == float(i)
