"""What an 8-rank ring all-reduce costs the graphed ResNet-50 step through CU / memory contention, measured
on ONE MI355X (verdict round 4, item 6).

The round-4 bucket table (profiles/r04_dp) modelled the N = 8 exposure from link time alone: every bucket's
ring finishes before backward ends, so 0 ms exposed.  That ignores that RCCL's kernels occupy CUs beside
backward kernels that each fill the chip.  Here every bucket's collective is replaced, at the same point of
the captured step (its grad-ready hook, a side stream forked there and joined before the optimizer), by
``dp_ring_sim``: B workgroups streaming the bucket for the ring's modelled time 2 (N-1)/N S / 153 GB/s + L
(csrc/kernels/dp_sim.hip).  The step time minus the no-DP step time is the measured contention cost;
B is swept because RCCL's channel count on an MI355X node is not observable on one GPU.

    python scripts/dp_contention.py --blocks 0,8,16,32 --out dp_contention.json
Reference: the sync-replicas remnant R/distributed/distributed.py:110-113 (the reference has no sync DP)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.parallel import GradAllReduce  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402


def timed(tr, x, y, reps=3, n=30):
    best = 1e9
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(n):
            tr.step(x, y)
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / n)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--blocks", default="0,8,16,32")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--link_gbps", type=float, default=153.0)
    ap.add_argument("--latency_us", type=float, default=15.0)
    ap.add_argument("--passes", type=int, default=2, help="read+write sweeps of the bucket per collective "
                    "(2 ~ a ring all-reduce's local traffic); -1 = stream for the whole ring time")
    ap.add_argument("--wires", default="f32,bf16", help="gradient wires to sweep (comma list)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (a.batch, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
    lab = torch.randint(0, 10, (a.batch,), generator=g).to(dev)
    x = to_model_input(img)
    rows = []
    for wire in a.wires.split(","):
        for nb in [int(v) for v in a.blocks.split(",")]:
            if wire == "bf16" and nb == 0:
                continue
            st, m = build_resnet_cifar(device=dev, depth=a.depth, dtype=torch.bfloat16, seed=0)
            dp = None
            if nb > 0:
                dp = GradAllReduce(st, bucket_bytes=int(a.bucket_mb * (1 << 20)), compress_bf16=wire == "bf16",
                                   simulate_ring={"blocks": nb, "ranks": a.ranks, "link_gbps": a.link_gbps,
                                                  "latency_us": a.latency_us, "passes": a.passes})
            tr = ClassifierTrainer(st, m, MomentumOptimizer(st, 0.0, momentum=0.9), dp)
            tr.capture(x, lab)
            ms = timed(tr, x, lab)
            row = {"wire": wire if nb else "none", "blocks": nb, "ms_per_step": ms}
            if dp is not None:
                row["buckets_mb"] = [round(b / 2 ** 20 / (2 if wire == "bf16" else 1), 2) for b in dp.bucket_sizes_bytes]
                row["ring_us"] = [round(dp.sim_ring_us(b // (2 if wire == "bf16" else 1)), 1)
                                  for b in dp.bucket_sizes_bytes]
            rows.append(row)
            print(json.dumps(row), flush=True)
            del tr, dp, st, m
            torch.cuda.empty_cache()
    base = [r["ms_per_step"] for r in rows if r["blocks"] == 0]
    if base:
        for r in rows:
            r["cost_ms"] = r["ms_per_step"] - base[0]
            print("%-5s blocks %3d  %.3f ms/step  (+%.3f ms vs no DP)" % (r["wire"], r["blocks"], r["ms_per_step"],
                                                                         r["cost_ms"]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"config": vars(a), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
