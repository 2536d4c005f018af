#!/usr/bin/env python3
"""Round-6 calibration of the deterministic-reduction test mode (ops.deterministic): ResNet-50 first-step
gradients (batch 32, random init) of the five fused-vs-layer-wise comparisons of the GPU suite, each
run twice on the fused path and once on the alternative path, with the mode off and on.  Prints, per
comparison and mode, the worst and median per-variable relative distance (same path / fused vs
alternative) and the loss gap."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflow_examples_amd import ops  # noqa: E402
from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.ops import fusion, nn as nnops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator().manual_seed(5)
img = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, generator=g)
lab = torch.randint(0, 10, (32,), generator=g).to(dev)
xin = to_model_input(img.to(dev))


def run(seed=3, head=False):
    st, m = build_resnet_cifar(device=dev, depth=50, dtype=torch.bfloat16, seed=seed)
    st.zero_grad()
    if head:
        loss = m.training_loss(xin, lab, unit_seed=True)
    else:
        loss = ops.softmax_cross_entropy(m(xin, training=True), lab)
    loss.backward()
    torch.cuda.synchronize()
    return float(loss.detach()), st.grad.clone(), st


def dist(ga, gb, st):
    out = []
    for v in st.trainable():
        sl = slice(v.offset, v.offset + v.numel)
        n = ga[sl].norm().item() + 1e-12
        out.append(((gb[sl] - ga[sl]).norm().item() / n, v.name))
    out.sort()
    return out


def alt_lazy():
    so, sq = nnops._pw_expand_ok, nnops._pw_squeeze_bwd_ok
    nnops._pw_expand_ok = lambda *a: False
    nnops._pw_squeeze_bwd_ok = lambda *a: False
    try:
        return run()
    finally:
        nnops._pw_expand_ok, nnops._pw_squeeze_bwd_ok = so, sq


def alt_override(**kv):
    def f(head=False):
        with fusion.override(**kv):
            return run(head=head)
    return f


TFX = torch.ops.tfx


def scaled(opname, pick):
    """A run with the fused group's output scaled by 0.95 (negative control): ``pick(args, out)`` returns
    the tensors to scale."""
    def f(head=False):
        orig = getattr(TFX, opname)

        def wrap(*a):
            out = orig(*a)
            for t in pick(a, out):
                if t is not None and t.numel():
                    t.data.mul_(0.95)
            return out
        setattr(TFX, opname, wrap)
        try:
            return run(head=head)
        finally:
            setattr(TFX, opname, orig)
    return f


def neg_lazy(head=False):
    o1, o2 = TFX.pw_bwd_expand, TFX.pw_bwd_squeeze

    def w1(*a):
        out = o1(*a)
        out[0].data.mul_(0.95)
        return out

    def w2(*a):
        out = o2(*a)
        out[0].data.mul_(0.95)
        return out
    TFX.pw_bwd_expand, TFX.pw_bwd_squeeze = w1, w2
    try:
        return run()
    finally:
        TFX.pw_bwd_expand, TFX.pw_bwd_squeeze = o1, o2


# (name, alternative path, negative control, head loss)
CASES = [
    ("sr_take_off", alt_override(sr_take=False), scaled("conv_wgrad_sr2", lambda a, o: [o[1]] if a[10] is not None else []), False),
    ("sr_defer_off", alt_override(sr_defer=False), scaled("conv_wgrad_sr2", lambda a, o: [o[1]] if a[10] is not None else []), False),
    ("lazy_kernels_off", lambda: alt_lazy(), neg_lazy, False),
    ("lazy_bn_bwd_off", alt_override(lazy_bn_bwd=False), neg_lazy, False),
    ("defer_tail_off", alt_override(defer_tail=False), scaled("pw_fwd_squeeze", lambda a, o: [a[5]]), False),
    ("defer_bn_in_off", alt_override(defer_bn_in=False), scaled("conv3x3_bwd_fused", lambda a, o: [o[0]]), False),
    ("head_tail_off", alt_override(head_tail=False), scaled("head_xent", lambda a, o: [o[1]] if a[5] is not None else []), True),
]


def summ(d):
    e = [x[0] for x in d]
    return "max %.2e (%s) med %.2e n>1e-3 %d n>2e-2 %d n>3e-2 %d n>4e-2 %d" % (
        d[-1][0], d[-1][1].replace("resnet50/", ""), e[len(e) // 2], sum(x > 1e-3 for x in e), sum(x > 2e-2 for x in e),
        sum(x > 3e-2 for x in e), sum(x > 4e-2 for x in e))


with ops.deterministic(True):
    for name, alt, neg, head in CASES:
        l0, g0, st = run(head=head)
        l1, g1, _ = run(head=head)
        l2, g2, _ = alt(head) if head else alt()
        l3, g3, _ = neg(head)
        print("%-16s nvars %d loss %.6f %.6f alt %.6f neg %.6f" % (name, len(list(st.trainable())), l0, l1, l2, l3))
        print("   same: " + summ(dist(g0, g1, st)))
        print("   alt : " + summ(dist(g0, g2, st)))
        print("   neg : " + summ(dist(g0, g3, st)), flush=True)
