#!/usr/bin/env python3
"""Conv <-> BN fusion microbenchmark over the distinct convs of ResNet-50/CIFAR (batch B).

forward : unfused = conv_fwd_stats + bn_fwd_train(stats ready)   (finalize kernel + apply)
          fused   = conv_fwd_bn (epilogue finalize)  + bn_apply_train
backward: unfused = conv_dgrad + bn_bwd                           (reduce + slot-reduce + apply)
          fused   = conv_dgrad_bn (epilogue reduce)  + bn_bwd_apply   (stride-1 convs only)
The BN of the backward is the one that produced the conv's INPUT (C channels, ReLU; residual mask
for the block-input convs).  Times in us per pair, interleaved in one process."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402
from scripts.conv_bench import resnet50_convs, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/epi_bench.json")
    a = ap.parse_args()
    assert _native.load()
    dev = torch.device("cuda")
    uniq = {}
    for sh in resnet50_convs(a.batch):
        uniq[sh] = uniq.get(sh, 0) + 1
    T = {"fwd_unfused": 0.0, "fwd_fused": 0.0, "bwd_unfused": 0.0, "bwd_fused": 0.0}
    rows = []
    for (N, H, W, C, K, R, st), cnt in uniq.items():
        pad = R // 2
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        gk, bk = torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev)
        rmk, rvk = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        wsk = torch.zeros(64 * 2 * K + 64, device=dev)
        r = {"shape": [N, H, W, C, K, R, st], "count": cnt}

        def fwd_unfused():
            y = torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, wsk)
            torch.ops.tfx.bn_fwd_train(y, gk, bk, rmk, rvk, 0.1, 1e-5, None, True, wsk, True)

        def fwd_fused():
            y, save = torch.ops.tfx.conv_fwd_bn(x, w, st, pad, 1, wsk, gk, bk, rmk, rvk, 0.1, 1e-5)
            torch.ops.tfx.bn_apply_train(y, None, save, True)

        r["fwd_unfused"] = timeit(fwd_unfused, a.iters)
        r["fwd_fused"] = timeit(fwd_fused, a.iters)
        if st == 1 and C % 8 == 0 and C >= 64:
            # BN of the input: x = relu(bn(xb) [+ res]); block-input convs (C = 4*width) carry a residual
            xb = torch.randn(N, H, W, C, device=dev).bfloat16()
            gc, bc = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
            wsc = torch.zeros(64 * 2 * C + 64, device=dev)
            res = torch.randn(N, H, W, C, device=dev).bfloat16() if (R == 1 and C > K) else None
            xin, save, mask = torch.ops.tfx.bn_fwd_train(xb, gc, bc, None, None, 0.1, 1e-5, res, True, wsc, False)
            if mask is not None and mask.numel() == 0:
                mask = None
            y = torch.ops.tfx.conv_fwd(xin, w, st, pad, 1)
            gy = torch.randn_like(y)
            dgc, dbc = torch.zeros(C, device=dev), torch.zeros(C, device=dev)

            def bwd_unfused():
                dx = torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None)
                torch.ops.tfx.bn_bwd(dx, xb, None, save, True, wsc, dgc, dbc, mask)

            def bwd_fused():
                dx, red = torch.ops.tfx.conv_dgrad_bn(gy, w, list(x.shape), st, pad, 1, None, xb, save, mask, True,
                                                      wsc, dgc, dbc)
                torch.ops.tfx.bn_bwd_apply(dx, xb, None, save, red, True, mask)

            r["bwd_unfused"] = timeit(bwd_unfused, a.iters)
            r["bwd_fused"] = timeit(bwd_fused, a.iters)
            r["dgrad_only"] = timeit(lambda: torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None), a.iters)
        for k in T:
            if k in r:
                T[k] += cnt * r[k]
        rows.append(r)
        print(f"{str(r['shape']):34s} x{cnt} fwd {r['fwd_unfused']:6.1f} -> {r['fwd_fused']:6.1f} us"
              + (f" | bwd {r['bwd_unfused']:6.1f} -> {r['bwd_fused']:6.1f} us (dgrad alone {r['dgrad_only']:6.1f})"
                 if "bwd_fused" in r else ""), flush=True)
    print("TOTAL per step: fwd %.3f -> %.3f ms, bwd %.3f -> %.3f ms" % (
        T["fwd_unfused"] / 1e3, T["fwd_fused"] / 1e3, T["bwd_unfused"] / 1e3, T["bwd_fused"] / 1e3))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"rows": rows, "total_us": T}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
