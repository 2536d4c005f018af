"""Shared helpers of the fused-vs-layer-wise whole-step GPU tests (deterministic-reduction mode).

A random-init bf16 ResNet-50 is chaotic: two runs of the SAME path differ by 20-100 % in a first-step
gradient because the f32 atomics that accumulate the forward BN statistics add in arrival order and 50
layers amplify the last-bit differences (profiles/r04_determinism; `scripts/dev/det_probe.py`: median
per-variable distance 0.97 between two default runs).  Under ``ops.deterministic()`` the forward is
bit-stable -- the same loss bits on every path of these tests -- and the remaining differences are the
BN-backward partial sums' slot-atomic order (entering the backward linearly: <= 1.3e-2 on a few
near-zero-sum BN gradients, 0 on ~2/3 of the variables) plus each path's own rounding.  So every
comparison uses ONE fixed per-variable gate, DET_TOL, and each test proves the gate can fail: its fused
group's output scaled by 0.95 (negative control) must push variables past it.

Calibration (`profiles/r06_det/det_probe.txt`, batch 32): same path <= 1.24e-2, fused vs alternative
<= 1.93e-2 (the head's tail mode: f32 in-kernel tail vs the materialised bf16 tail), negative controls
put 8-160 of 161 variables past 3e-2.
"""
import contextlib

import torch

DET_TOL = 3e-2


def rel_dists(g_ref, g_other, store):
    """Per-variable relative distance ||g_other - g_ref|| / ||g_ref|| over the store's trainable variables."""
    out = {}
    for v in store.trainable():
        sl = slice(v.offset, v.offset + v.numel)
        n = g_ref[sl].norm().item() + 1e-12
        out[v.name] = (g_other[sl] - g_ref[sl]).norm().item() / n
    return out


def assert_within_gate(g_ref, g_other, store, tag=""):
    d = rel_dists(g_ref, g_other, store)
    bad = sorted(((e, k) for k, e in d.items() if e > DET_TOL), reverse=True)
    assert not bad, (tag, bad[:5])
    return max(d.values())


def assert_gate_catches(g_ref, g_bad, store, tag=""):
    """The negative control: the gate must reject a run whose fused group's output was scaled by 0.95."""
    d = rel_dists(g_ref, g_bad, store)
    n = sum(e > DET_TOL for e in d.values())
    assert n >= 1, (tag, "a x0.95 fused-group output slipped under the fixed gate", max(d.values()))
    return n


@contextlib.contextmanager
def scaled_output(opname, pick, factor=0.95):
    """Run with ``torch.ops.tfx.<opname>`` wrapped so that ``pick(args, out)`` (the tensors the fused group
    produces) are scaled in place by ``factor`` after each call -- the negative control's injected error.
    Scaled through ``.data`` so autograd's version counters do not see it."""
    ns = torch.ops.tfx
    orig = getattr(ns, opname)

    def wrap(*a):
        out = orig(*a)
        for t in pick(a, out):
            if t is not None and t.numel():
                t.data.mul_(factor)
        return out
    setattr(ns, opname, wrap)
    try:
        yield
    finally:
        setattr(ns, opname, orig)
