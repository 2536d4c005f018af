#!/usr/bin/env python3
"""Per-launch achieved rate of every implicit-GEMM launch in one ResNet-50 training step.

Run under ``rocprofv3 --kernel-trace --output-format csv``: the script runs 3 eager steps, then a 4th
under the igemm launch trace and writes the traced (family, M, N, K) keys in launch order to
--keys.  ``--join <kernel_trace.csv>`` (no GPU) then pairs the 4th step's igemm kernels (between the
3rd and 4th optimizer kernels) with those keys and prints us, TF/s and the kernel name per launch,
slowest rate first -- the outliers are where a launch configuration or kernel is worth a look.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

FAMILIES = ["fwd_pointwise", "fwd_im2col", "dgrad_pointwise", "dgrad_general", "dgrad_cls_dense", "dgrad_cls",
            "wgrad_dense", "wgrad_x", "wgrad_t_x", "dgrad_flip"]


def run(keys_path):
    import torch
    from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_batch
    from tensorflow_examples_amd.ops import _native, tuning
    from tensorflow_examples_amd.optim import MomentumOptimizer
    from tensorflow_examples_amd.train import ClassifierTrainer
    assert _native.load()
    tuning.load()
    dev = torch.device("cuda")
    store, model = build_resnet_cifar(device=dev, depth=50, dtype=torch.bfloat16, seed=0)
    opt = MomentumOptimizer(store, 0.1, momentum=0.9, weight_decay=5e-4)
    tr = ClassifierTrainer(store, model, opt, None, fuse_zero_grad=True)
    img = torch.randint(0, 256, (256, 32, 32, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (256,), device=dev)
    x, y = to_model_batch(img, lab, dtype=torch.bfloat16, device=dev)
    for _ in range(3):
        tr.step(x, y)
    torch.cuda.synchronize()
    torch.ops.tfx.igemm_tune_trace(True)
    tr.step(x, y)
    torch.cuda.synchronize()
    torch.ops.tfx.igemm_tune_trace(False)
    rows = torch.ops.tfx.igemm_tune_traced().tolist()
    with open(keys_path, "w") as f:
        json.dump(rows, f)
    print("traced %d igemm launches" % len(rows))


def join(trace_csv, keys_path):
    with open(keys_path) as f:
        keys = [tuple(r) for r in json.load(f)]
    with open(trace_csv) as f:
        ks = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(ks) if "opt_kernel" in r["Kernel_Name"]]
    step = ks[opt[-2] + 1:opt[-1] + 1]
    # the persistent 1x1 forward (igemm_persist) is routed before the tuned lookup: no traced key
    gem = [r for r in step if "igemm_kernel" in r["Kernel_Name"]]
    if len(gem) != len(keys):
        print("warning: %d igemm kernels vs %d traced keys" % (len(gem), len(keys)))
    out = []
    for r, k in zip(gem, keys):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        fl = 2.0 * k[1] * k[2] * k[3]
        name = r["Kernel_Name"].replace("tfx::(anonymous namespace)::", "")
        out.append((fl / us / 1e6, us, k, name))
    tot = sum(o[1] for o in out)
    print("%d launches, %.1f us total" % (len(out), tot))
    for tf, us, k, name in sorted(out):
        print("%7.1f TF/s %7.1f us  %-15s M=%6d N=%5d K=%6d  %s" % (tf, us, FAMILIES[k[0]], k[1], k[2], k[3], name[:70]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", default="gpurun_out/rates/keys.json")
    ap.add_argument("--join", default=None, help="kernel_trace.csv to pair with --keys (no GPU)")
    a = ap.parse_args()
    if a.join:
        join(a.join, a.keys)
    else:
        os.makedirs(os.path.dirname(a.keys) or ".", exist_ok=True)
        run(a.keys)
