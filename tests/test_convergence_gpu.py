"""Convergence parity that can fail (verdict round 4, item 3): 300 steps of the fused bf16 ResNet-50 training
step against the same model in fp32 PyTorch reference ops, same init, same batches of the HARD synthetic
CIFAR task (overlapping class textures, shifts, 15 % label noise: ~73 % test accuracy after 300 steps, not
the 100 % every path reaches on the easy prototypes), same momentum-SGD recipe.

Tolerances come from the measured spread (profiles/r05_conv/): two fused runs stayed within 0.42 % of the
fp32 loss in every 50-step window and within 1.2 points of its accuracy, so the window-loss bound is 1 %
and the accuracy bound 2 points.  The negative control -- the stage-1 fused BN-backward group
(pw_bwd_expand / pw_bwd_squeeze) with its input and weight gradients scaled by 0.8 -- deviates by 2.3 %
and must FAIL the same comparison.  Reference: the final accuracy line, R/distributed/distributed.py:164."""
import importlib.util
import os
import types

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL_TOL, ACC_TOL = 0.01, 0.02


def _mod():
    spec = importlib.util.spec_from_file_location("convergence_parity", os.path.join(ROOT, "scripts",
                                                                                     "convergence_parity.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_resnet50_fused_bf16_converges_like_fp32_and_negative_control_fails(gpu):
    cp = _mod()
    from tensorflow_examples_amd.data.cifar import hard_synthetic_cifar
    from tensorflow_examples_amd.models.resnet import build_resnet_cifar
    a = types.SimpleNamespace(steps=300, batch=128, depth=50, lr=0.05, wd=5e-4, warmup=50, seed=0)
    xtr, ytr = hard_synthetic_cifar(a.steps * a.batch, 0)
    xte, yte = hard_synthetic_cifar(2000, 1)
    data = tuple(torch.as_tensor(t, device=gpu) for t in (xtr, ytr, xte, yte))
    st0, _ = build_resnet_cifar(device=gpu, depth=50, dtype=torch.bfloat16, seed=0, zero_init_residual=True)
    w0 = st0.master.bfloat16().float()
    del st0
    ref = cp.run("ref32", a, data, w0)
    fused = cp.run("fused", a, data, w0)
    neg = cp.run("fused", a, data, w0, negctl="lazy_bn_bwd:0.8")
    c_ok, c_neg = cp.compare(ref, fused, REL_TOL, ACC_TOL), cp.compare(ref, neg, REL_TOL, ACC_TOL)
    print("ref", ref["window_loss"], ref["test_accuracy"])
    print("fused", fused["window_loss"], fused["test_accuracy"], c_ok["max_rel_window_loss"], c_ok["accuracy_delta"])
    print("negctl", neg["window_loss"], neg["test_accuracy"], c_neg["max_rel_window_loss"], c_neg["accuracy_delta"])
    assert 0.5 < ref["test_accuracy"] < 0.9, ref  # the task is learnable and not solved perfectly
    assert c_ok["pass"], c_ok
    assert not c_neg["pass"], c_neg  # the check catches a fused gradient that is 20 % wrong


DP_WORKER = r"""
import importlib.util, json, os, sys, types, numpy as np, torch
sys.path.insert(0, os.environ["ROOT"])
spec = importlib.util.spec_from_file_location("cp", os.path.join(os.environ["ROOT"], "scripts", "convergence_parity.py"))
cp = importlib.util.module_from_spec(spec); spec.loader.exec_module(cp)
d = np.load(os.environ["DATA"])
data = tuple(torch.as_tensor(d[k]) for k in ("xtr", "ytr", "xte", "yte"))
w0 = torch.as_tensor(d["w0"])
a = types.SimpleNamespace(**json.loads(os.environ["ARGS"]))
r = cp.run_dp(a, data, w0, wire=os.environ["WIRE"])
if r["rank"] == 0:
    print("RESULT " + json.dumps(r), flush=True)
"""


def _dp_run(tmp_path, wire, args):
    import json
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, DATA=str(tmp_path / "data.npz"), ARGS=json.dumps(args), WIRE=wire,
                   RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="4")
        procs.append(subprocess.Popen([sys.executable, "-c", DP_WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=900) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    line = [ln for ln in outs[0][0].splitlines() if ln.startswith("RESULT ")]
    return json.loads(line[0][len("RESULT "):])


DP_REL_TOL = 0.025  # DP vs the single-process fp32 run: per-rank BN statistics over half the batch
# ... and its test accuracy: the f32-wire DP run measured 1.6 points (profiles/r06_dp_wire) and 2.25 points
# (round-6 HEAD suite) below the single-process run -- per-rank BN again, not the wire (that is gated at 2)
DP_ACC_TOL = 0.03


def test_dp_wire_formats_converge_like_fp32(gpu, tmp_path):
    """The N > 1 gradient wire decided with evidence (verdict round 5, item 2): the same 300-step parity as
    above, but the fused step runs through the data-parallel path -- 2 gloo ranks on one GPU, each on half of
    every batch, bucketed GradAllReduce -- once with the f32 wire and once with the bf16 wire (the gradients
    cast per bucket, reduced in bf16, read by the optimizer directly).

    The WIRE is judged against the f32 wire on the same DP path: the bf16 run must stay within the 1 %
    window-loss / 2-point accuracy gate of the f32 run (measured: <= 0.45 % / 0.8 points,
    profiles/r06_dp_wire).  Against the single-process fp32 reference both DP runs sit ~1-2 % higher in
    the late windows -- each rank's BN statistics cover 64 images instead of 128, a property of DP
    without synchronised BN, the same for both wires -- so that comparison uses a 2.5 % gate."""
    import json
    import numpy as np
    cp = _mod()
    from tensorflow_examples_amd.data.cifar import hard_synthetic_cifar
    from tensorflow_examples_amd.models.resnet import build_resnet_cifar
    args = dict(steps=300, batch=128, depth=50, lr=0.05, wd=5e-4, warmup=50, seed=0)
    a = types.SimpleNamespace(**args)
    xtr, ytr = hard_synthetic_cifar(a.steps * a.batch, 0)
    xte, yte = hard_synthetic_cifar(2000, 1)
    st0, _ = build_resnet_cifar(device=gpu, depth=50, dtype=torch.bfloat16, seed=0, zero_init_residual=True)
    w0 = st0.master.bfloat16().float()
    del st0
    np.savez(tmp_path / "data.npz", xtr=np.asarray(xtr), ytr=np.asarray(ytr), xte=np.asarray(xte),
             yte=np.asarray(yte), w0=w0.cpu().numpy())
    data = tuple(torch.as_tensor(t, device=gpu) for t in (xtr, ytr, xte, yte))
    ref = cp.run("ref32", a, data, w0)
    torch.cuda.empty_cache()
    res = {}
    for wire in ("f32", "bf16"):
        r = _dp_run(tmp_path, wire, args)
        res[wire] = (r, cp.compare(ref, r, REL_TOL, ACC_TOL))
        print(wire, r["window_loss"], r["test_accuracy"], res[wire][1]["max_rel_window_loss"],
              res[wire][1]["accuracy_delta"], r["seconds"])
        assert r["buckets"] >= 2 and r["wire_used_bf16"] == (wire == "bf16")
    print("ref", ref["window_loss"], ref["test_accuracy"])
    wire = cp.compare(res["f32"][0], res["bf16"][0], REL_TOL, ACC_TOL)
    print("bf16 vs f32 wire", wire["rel_window_loss"], wire["accuracy_delta"])
    assert wire["pass"], wire
    for w in ("f32", "bf16"):
        c = cp.compare(ref, res[w][0], DP_REL_TOL, DP_ACC_TOL)
        assert c["pass"], (w, c)
