"""Same-process A/B of bench.py's training step under fusion knobs (ops/fusion.py KNOBS): the configs
run interleaved (A B C A B C ...) on ONE GPU so box-to-box variance (~4 % on this pool) cancels.

usage: PYTHONPATH=. python scripts/dev/ab_bench.py [--reps 3] [--steps 30] [--warmup 10]
       --config name:knob=0,knob=1 ...   (default: all fusions on vs each fused 3x3 path off)"""
import argparse
import contextlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import bench  # noqa: E402
from tensorflow_examples_amd.ops import fusion  # noqa: E402

DEFAULT = [
    "fused:",
    "no_c3bwd:fuse_conv3_bwd=0",
    "no_bn_in:defer_bn_in=0",
]


def parse_cfg(s):
    name, _, rest = s.partition(":")
    kv = {}
    for item in filter(None, rest.split(",")):
        k, _, v = item.partition("=")
        kv[k] = bool(int(v))
    return name, kv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", action="append")
    a = ap.parse_args()
    cfgs = [parse_cfg(c) for c in (a.config or DEFAULT)]
    base = {k: fusion.knob(k) for _, kv in cfgs for k in kv}
    res = {name: [] for name, _ in cfgs}
    for rep in range(a.reps):
        for name, kv in cfgs:
            for k, v in base.items():
                fusion.CONFIG.set(k, v)
            for k, v in kv.items():
                fusion.CONFIG.set(k, v)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                bench.run(bench.parse(["--steps", str(a.steps), "--warmup", str(a.warmup)]))
            rec = json.loads(buf.getvalue().strip().splitlines()[-1])
            res[name].append(rec["ms_per_step"])
            print("rep %d %-12s %.3f ms/step" % (rep, name, rec["ms_per_step"]), flush=True)
    for name, v in res.items():
        print("%-12s min %.3f  mean %.3f  all %s" % (name, min(v), sum(v) / len(v), v))


if __name__ == "__main__":
    main()
