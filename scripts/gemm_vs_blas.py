#!/usr/bin/env python3
"""The framework's implicit-GEMM kernels against the vendor GEMM (hipBLASLt through torch.matmul) on the
GEMMs that are plain GEMMs in both: every 1x1 stride-1 conv of the ResNet-50/CIFAR step at batch B.

Per conv (NHWC x[M = N*H*W][C], w[Ko][C]) and pass, both sides graph-replayed (ITER calls per replay,
best of 3 replays, launch overhead excluded alike):
  fwd    ours conv_fwd (no BN-statistics epilogue)             vs  x[M][C] @ w[Ko][C]^T  -> bf16 [M][Ko]
  dgrad  ours conv_dgrad (no fused BN-backward epilogue)       vs  dy[M][Ko] @ w[Ko][C]  -> bf16 [M][C]
  wgrad  ours conv_wgrad (split-K, f32 atomics into dW)        vs  dy^T[Ko][M] @ x[M][C] -> bf16 [Ko][C]
         (torch writes a bf16 dW, ours an f32 one: the comparison favours torch on output bytes)
plus ours WITH the fused epilogue the model actually runs (conv_fwd_stats / conv_dgrad_bn), whose
work torch would need extra passes for.  Output: one line per (shape, pass) and per-pass totals
weighted by the step's conv counts.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tensorflow_examples_amd.ops import _native  # noqa: E402
from conv_bench import resnet50_convs  # noqa: E402

ITER = 20
NSLOT = 64


def graph_us(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(ITER):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / ITER * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None, help="JSON rows")
    a = ap.parse_args()
    assert _native.load()
    dev = torch.device("cuda")
    print("torch %s, preferred BLAS library: %s" % (torch.__version__, torch.backends.cuda.preferred_blas_library()))
    counts = {}
    for sh in resnet50_convs(a.batch):
        if sh[5] == 1 and sh[6] == 1:
            counts[sh] = counts.get(sh, 0) + 1
    rows = []
    tot = {}
    print("%-26s %-5s %5s %9s %9s %9s %7s %8s" % ("conv [N,H,W,C,Ko]", "pass", "count", "ours us", "blas us",
                                                  "ours+epi", "blas/ours", "ours TF/s"), flush=True)
    for (N, H, W, C, K, R, st), cnt in counts.items():
        M = N * H * W
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).bfloat16()
        gy = torch.randn(N, H, W, K, device=dev).bfloat16()
        dw = torch.zeros(K, 1, 1, C, device=dev)
        x2, w2, gy2 = x.view(M, C), w.view(K, C), gy.view(M, K)
        slots = torch.zeros(NSLOT * 2 * K, device=dev)
        ws = torch.zeros(NSLOT * 2 * C, device=dev)
        save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
        dgam, dbet = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        # numerics once per shape: ours against torch's GEMM (both bf16 in, f32 accumulate)
        yo, yt = torch.ops.tfx.conv_fwd(x, w, 1, 0, 1).view(M, K).float(), (x2 @ w2.t()).float()
        err = ((yo - yt).norm() / yt.norm()).item()
        assert err < 1e-2, ("fwd mismatch", err)
        passes = {
            "fwd": (lambda: torch.ops.tfx.conv_fwd(x, w, 1, 0, 1), lambda: x2 @ w2.t(),
                    lambda: torch.ops.tfx.conv_fwd_stats(x, w, 1, 0, 1, slots)),
            "dgrad": (lambda: torch.ops.tfx.conv_dgrad(gy, w, [N, H, W, C], 1, 0, 1, None), lambda: gy2 @ w2,
                      lambda: torch.ops.tfx.conv_dgrad_bn(gy, w, [N, H, W, C], 1, 0, 1, None, x, save, None, True,
                                                          ws, dgam, dbet)),
            "wgrad": (lambda: torch.ops.tfx.conv_wgrad(gy, x, dw, 1, 0, 1, True), lambda: gy2.t() @ x2, None),
        }
        for name, (ours, blas, epi) in passes.items():
            to, tb = graph_us(ours), graph_us(blas)
            te = graph_us(epi) if epi is not None else None
            tf = 2.0 * M * C * K / (to * 1e-6) / 1e12
            rows.append({"shape": [N, H, W, C, K], "pass": name, "count": cnt, "ours_us": round(to, 2),
                         "blas_us": round(tb, 2), "ours_epi_us": round(te, 2) if te else None, "ours_tflops": round(tf, 1)})
            t = tot.setdefault(name, [0.0, 0.0])
            t[0] += to * cnt
            t[1] += tb * cnt
            print("%-26s %-5s %5d %9.1f %9.1f %9s %7.2f %8.0f" % ([N, H, W, C, K], name, cnt, to, tb,
                                                                 "%.1f" % te if te else "-", tb / to, tf), flush=True)
        del x, w, gy, dw, x2, w2, gy2
    for name, (o, b) in tot.items():
        print("per step, %-5s 1x1 stride-1 convs: ours %7.1f us  blas %7.1f us  (blas/ours %.2f)" % (name, o, b, b / o))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "batch": a.batch, "iter": ITER, "rows": rows,
                       "totals_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
