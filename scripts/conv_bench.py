#!/usr/bin/env python3
"""Per-layer conv microbenchmark: every distinct conv of ResNet-50/CIFAR at batch B,
HIP implicit-GEMM kernels (fwd / dgrad / wgrad) vs PyTorch's MIOpen convs (NCHW->channels_last
bf16), reported in TFLOP/s.  Interleaved rounds in one process (cdna_hip_programming.md rule 24)."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native  # noqa: E402


def resnet50_convs(B):
    shapes = [(B, 32, 32, 8, 64, 3, 1)]
    cin, hw = 64, 32
    for si, n in enumerate([3, 4, 6, 3]):
        w = 64 * 2 ** si
        for bi in range(n):
            st = 2 if (bi == 0 and si > 0) else 1
            shapes.append((B, hw, hw, cin, w, 1, 1))
            shapes.append((B, hw, hw, w, w, 3, st))
            ohw = hw // st
            shapes.append((B, ohw, ohw, w, 4 * w, 1, 1))
            if bi == 0:
                shapes.append((B, hw, hw, cin, 4 * w, 1, st))
            cin, hw = 4 * w, ohw
    return shapes


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/conv_bench.json")
    a = ap.parse_args()
    assert _native.load()
    dev = torch.device("cuda")
    uniq = {}
    for sh in resnet50_convs(a.batch):
        uniq[sh] = uniq.get(sh, 0) + 1
    rows = []
    tot = {"ours": 0.0, "miopen": 0.0}
    for (N, H, W, C, K, R, st), cnt in uniq.items():
        pad = R // 2
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        y = torch.ops.tfx.conv_fwd(x, w, st, pad, 1)
        gy = torch.randn_like(y)
        dw = torch.zeros(K, R, R, C, device=dev)
        xc = x.permute(0, 3, 1, 2)  # channels_last NCHW view
        wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        gyc = gy.permute(0, 3, 1, 2)
        P, Q = y.shape[1], y.shape[2]
        flops = 2.0 * N * P * Q * K * R * R * C
        r = {"shape": [N, H, W, C, K, R, st], "count": cnt, "gflop": flops / 1e9}
        slots = torch.zeros(64 * 2 * K, device=dev)
        r["fwd_us"] = timeit(lambda: torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots), a.iters)
        r["fwd_nostats_us"] = timeit(lambda: torch.ops.tfx.conv_fwd(x, w, st, pad, 1), a.iters)
        r["dgrad_us"] = timeit(lambda: torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None), a.iters)
        r["wgrad_us"] = timeit(lambda: torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, True), a.iters)
        r["mi_fwd_us"] = timeit(lambda: F.conv2d(xc, wc, stride=st, padding=pad), a.iters)
        r["mi_dgrad_us"] = timeit(lambda: torch.nn.grad.conv2d_input(xc.shape, wc, gyc, stride=st, padding=pad), a.iters)
        r["mi_wgrad_us"] = timeit(lambda: torch.nn.grad.conv2d_weight(xc, wc.shape, gyc, stride=st, padding=pad), a.iters)
        for k in ("fwd", "dgrad", "wgrad"):
            r[k + "_tflops"] = flops / (r[k + "_us"] * 1e-6) / 1e12
            r["mi_" + k + "_tflops"] = flops / (r["mi_" + k + "_us"] * 1e-6) / 1e12
        tot["ours"] += cnt * (r["fwd_us"] + r["dgrad_us"] + r["wgrad_us"])
        tot["miopen"] += cnt * (r["mi_fwd_us"] + r["mi_dgrad_us"] + r["mi_wgrad_us"])
        rows.append(r)
        print(f"{str(r['shape']):34s} x{cnt} {r['gflop']:6.2f}GF | ours fwd {r['fwd_tflops']:6.1f} dgr {r['dgrad_tflops']:6.1f} "
              f"wgr {r['wgrad_tflops']:6.1f} | miopen fwd {r['mi_fwd_tflops']:6.1f} dgr {r['mi_dgrad_tflops']:6.1f} "
              f"wgr {r['mi_wgrad_tflops']:6.1f} TF/s | fwd {r['fwd_us']:.1f}us (no stats {r['fwd_nostats_us']:.1f}) "
              f"dgr {r['dgrad_us']:.1f}us wgr {r['wgrad_us']:.1f}us", flush=True)
    print(f"TOTAL per step (all convs, fwd+dgrad+wgrad): ours {tot['ours']/1e3:.2f} ms, miopen {tot['miopen']/1e3:.2f} ms")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"rows": rows, "total_us": tot}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
