"""Bucket-readiness timeline of the DP step (ResNet-50, batch 256) on a forced 1-rank RCCL group, and the
modelled exposed all-reduce at N = 8.

For every gradient bucket: its bytes on the wire (f32 or bf16), when its last gradient landed (HIP event
on the compute stream at the moment the grad-ready hook launches the bucket's collective, ms after the
backward started) and the backward's end.  The model for an 8-GPU MI355X node: RCCL runs the buckets one
after another on its stream; a ring all-reduce is bound by one xGMI link per hop,
t(S) = 2 (N-1)/N * S / 153 GB/s; bucket b finishes at max(ready_b, finish_{b-1}) + t(S_b);
the exposed all-reduce is finish_last - backward_end (what the optimizer waits for).

    TFX_DP_FORCE_COLLECTIVE=1 torchrun --nproc-per-node 1 --master-addr 127.0.0.1 scripts/dp_bucket_table.py
Reference: the commented sync-replicas remnant R/distributed/distributed.py:110-113 (no DP there)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.parallel import GradAllReduce, init_distributed  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402

LINK_GBS = 153.0


def ring_ms(nbytes, n=8):
    return 2.0 * (n - 1) / n * nbytes / (LINK_GBS * 1e9) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = init_distributed(device="cuda")
    st, m = build_resnet_cifar(device=dev, depth=a.depth, dtype=torch.bfloat16, seed=0)
    dp = GradAllReduce(st, bucket_bytes=int(a.bucket_mb * (1 << 20)), compress_bf16=a.dtype == "bf16")
    assert dp.force or dp.world > 1, "run with TFX_DP_FORCE_COLLECTIVE=1 (1-rank RCCL group) or >1 ranks"
    opt = MomentumOptimizer(st, 0.0, momentum=0.9)
    tr = ClassifierTrainer(st, m, opt, dp)
    img = torch.randint(0, 256, (a.batch, 32, 32, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (a.batch,), device=dev)
    x = to_model_input(img)
    events = {}
    orig_launch = dp._launch

    def launch(b):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        events.setdefault("ready", {})[b] = e
        return orig_launch(b)

    dp._launch = launch
    orig_bwd = torch.Tensor.backward

    def backward(self, *args, **kw):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig_bwd(self, *args, **kw)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        events["bwd"] = (e0, e1)
        return r

    torch.Tensor.backward = backward
    rows_all = []
    for s in range(a.steps):
        events.clear()
        tr.step(x, lab)
        torch.cuda.synchronize()
        e0, e1 = events["bwd"]
        bwd_ms = e0.elapsed_time(e1)
        rows = []
        for b, e in sorted(events["ready"].items()):
            rows.append((b, e0.elapsed_time(e)))
        rows_all.append((bwd_ms, rows))
    torch.Tensor.backward = orig_bwd
    bwd_ms, rows = rows_all[-1]  # steady state (the last step)
    elem = 2 if a.dtype == "bf16" else 4
    out = []
    fin = 0.0
    for b, ready in rows:
        lo, hi = dp.buckets[b]
        nb = (hi - lo) * elem
        t = ring_ms(nb)
        start = max(ready, fin)
        fin = start + t
        out.append({"bucket": b, "bytes": nb, "vars": len(dp.members[b]), "ready_ms": round(ready, 3),
                    "ring_ms_n8": round(t, 3), "finish_ms_n8": round(fin, 3)})
    exposed = max(0.0, fin - bwd_ms)
    if dist.get_rank() == 0:
        print("ResNet-%d batch %d, %s gradients on the wire, bucket cap %.0f MB, %d buckets" %
              (a.depth, a.batch, a.dtype, a.bucket_mb, len(dp.buckets)))
        print("%6s %10s %5s %10s %12s %14s" % ("bucket", "MB", "vars", "ready_ms", "ring_ms@N8", "finish_ms@N8"))
        for r in out:
            print("%6d %10.2f %5d %10.3f %12.3f %14.3f" % (r["bucket"], r["bytes"] / 2 ** 20, r["vars"], r["ready_ms"],
                                                         r["ring_ms_n8"], r["finish_ms_n8"]))
        print("backward (eager launches) %.3f ms; modelled exposed all-reduce at N=8: %.3f ms "
              "(total ring time %.3f ms)" % (bwd_ms, exposed, sum(r["ring_ms_n8"] for r in out)))
        if a.json:
            with open(a.json, "w") as f:
                json.dump({"depth": a.depth, "batch": a.batch, "dtype": a.dtype, "bucket_mb": a.bucket_mb,
                           "backward_ms": bwd_ms, "exposed_ms_n8": exposed, "buckets": out,
                           "steps": [(bm, rr) for bm, rr in rows_all]}, f, indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
