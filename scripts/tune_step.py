#!/usr/bin/env python3
"""Validate / re-pick igemm launch configurations inside the graph-replayed ResNet-50 training step.

``scripts/tune_convs.py`` times each conv pass alone, back to back on an otherwise idle chip.  Those
per-conv wins do not all carry into the step (profiles/r05_retune: a whole re-tuned table was 0.5 %
slower in the step), and two convs that reach the same (family, M, N, K) key -- a stride-2 3x3 conv and
the stride-1 3x3 convs after it have the same weight-gradient GEMM shape -- share one entry that the
isolated tuner picked for whichever conv it met first.

This script measures in the step itself.  One eager step under the launch trace lists the (family, M,
N, K) keys the step launches.  Then for each key (coordinate descent, most step time first):

  1. screen: every candidate configuration of the key's family is installed (``igemm_tune_set``), the
     step is re-captured into a HIP graph and ``--screen`` replays are timed;
  2. confirm: the current configuration and the ``--top`` best screened candidates are re-timed in
     ``--rounds`` interleaved rounds of ``--steps`` replays;
  3. a candidate replaces the current configuration only when its median beats the current median by
     more than ``--margin`` AND it is faster in every round.

Accepted changes stay installed for the keys measured after them.  The result is written as a full
table (``--out``; the committed table's rows with the accepted rows replaced / added) plus a report.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_examples_amd.ops import _native, tuning  # noqa: E402

BF16_CANDS = [(t, 0, g, 0) for t in (1, 2, 3) for g in (0, 2, 3)] + [(t, 2, g, 0) for t in (1, 2) for g in (0, 2)]
ATOMIC_CANDS = [(t, k, g, w) for t in (1, 2) for k in (1, 2) for g in (0, 3) for w in (256, 512)]
# --cands ext: the split-K block target off the 256 / 512 grid, ring depth 2, and ks 2 with a 3-deep ring
BF16_EXT = BF16_CANDS + [(1, 2, 3, 0), (2, 2, 3, 0)]
ATOMIC_EXT = [(t, k, g, w) for t in (1, 2) for k in (1, 2) for g in (0, 2, 3) for w in (128, 256, 384, 512, 768, 1024)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--screen", type=int, default=20, help="replays per screened candidate")
    ap.add_argument("--steps", type=int, default=40, help="replays per confirmation measurement")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--top", type=int, default=2)
    ap.add_argument("--margin", type=float, default=0.0015)
    ap.add_argument("--keys", default="", help="only these key indices (comma list, in step-time order)")
    ap.add_argument("--cands", default="base", choices=["base", "ext"])
    ap.add_argument("--min-launches", type=int, default=1, help="skip keys launched fewer times per step")
    ap.add_argument("--families", default="", help="only these family names (comma list)")
    ap.add_argument("--budget-s", type=float, default=900.0, help="stop starting new keys after this long")
    ap.add_argument("--out", default="gpurun_out/tune_step/igemm_step.json")
    ap.add_argument("--report", default="gpurun_out/tune_step/report.json")
    a = ap.parse_args()

    from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_batch
    from tensorflow_examples_amd.optim import MomentumOptimizer
    from tensorflow_examples_amd.train import ClassifierTrainer

    assert _native.load()
    n_loaded = tuning.load()
    with open(tuning.TABLE) as f:
        table = json.load(f)
    cur = {(e["fam"], e["M"], e["N"], e["K"]): (e["tile"], e["ks"], e["gls"], e["want"]) for e in table["entries"]}
    dev = torch.device("cuda")
    torch.manual_seed(0)
    store, model = build_resnet_cifar(device=dev, depth=50, dtype=torch.bfloat16, seed=0)
    opt = MomentumOptimizer(store, 0.1, momentum=0.9, weight_decay=5e-4)
    tr = ClassifierTrainer(store, model, opt, None, fuse_zero_grad=True)
    img = torch.randint(0, 256, (a.batch, 32, 32, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (a.batch,), device=dev)
    x, y = to_model_batch(img, lab, dtype=torch.bfloat16, device=dev)
    for _ in range(3):
        tr.step(x, y)
    torch.cuda.synchronize()

    # the keys the step launches, with their launch counts
    torch.ops.tfx.igemm_tune_trace(True)
    tr.step(x, y)
    torch.cuda.synchronize()
    torch.ops.tfx.igemm_tune_trace(False)
    rows = [tuple(r) for r in torch.ops.tfx.igemm_tune_traced().tolist()]
    counts = {}
    for r in rows:
        counts[r] = counts.get(r, 0) + 1

    def capture():
        tr.graph, tr._static = None, None
        torch.cuda.synchronize()
        tr.capture(x, y, warmup=1)
        torch.cuda.synchronize()

    def timed(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tr.graph.replay()
        s.record()
        for _ in range(n):
            tr.graph.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n * 1e3  # us per step

    def set_cfg(key, cfg):
        if cfg is None:  # back to the heuristic: a table row cannot be removed, so re-load without it
            tuning.clear()
            for k, c in cur.items():
                if k != key:
                    torch.ops.tfx.igemm_tune_set(*k, *c)
        else:
            torch.ops.tfx.igemm_tune_set(*key, *cfg)

    def measure(key, cfg, n):
        set_cfg(key, cfg)
        capture()
        return timed(n)

    # order keys by a one-shot estimate of their share: launches x GEMM work
    keys = sorted(counts, key=lambda k: -counts[k] * k[1] * k[2] * k[3])
    if a.keys:
        keys = [keys[int(i)] for i in a.keys.split(",")]
    keys = [k for k in keys if counts[k] >= a.min_launches]
    if a.families:
        keys = [k for k in keys if tuning.FAMILIES[k[0]] in a.families.split(",")]
    capture()
    base0 = statistics.median(timed(a.steps) for _ in range(3))
    print("table rows %d, step keys %d, baseline %.1f us/step" % (n_loaded, len(keys), base0), flush=True)
    report, changed = [], {}
    t0 = time.time()
    for ki, key in enumerate(keys):
        if time.time() - t0 > a.budget_s:
            print("budget reached after %d keys" % ki, flush=True)
            break
        fam = key[0]
        if a.cands == "ext":
            cands = ATOMIC_EXT if fam in tuning.ATOMIC_FAMILIES else BF16_EXT
        else:
            cands = ATOMIC_CANDS if fam in tuning.ATOMIC_FAMILIES else BF16_CANDS
        now = cur.get(key)
        scr = {}
        for c in cands:
            if c == now:
                continue
            scr[c] = measure(key, c, a.screen)
        ref_scr = measure(key, now, a.screen)
        top = sorted(scr, key=scr.get)[:a.top]
        times = {now: [], **{c: [] for c in top}}
        for _ in range(a.rounds):
            for c in [now] + top:
                times[c].append(measure(key, c, a.steps))
        med = {c: statistics.median(v) for c, v in times.items()}
        best = min(top, key=med.get) if top else None
        win = (best is not None and med[best] < med[now] * (1 - a.margin)
               and all(tb < tn for tb, tn in zip(times[best], times[now])))
        if win:
            cur[key] = best
            changed[key] = best
        set_cfg(key, cur.get(key))
        rec = {"key": list(key), "family": tuning.FAMILIES[fam], "launches": counts[key],
               "current": list(now) if now else None, "current_us": round(med[now], 1),
               "screen_current_us": round(ref_scr, 1),
               "screen": {"%d/%d/%d/%d" % c: round(t, 1) for c, t in sorted(scr.items(), key=lambda kv: kv[1])},
               "confirm": {("%d/%d/%d/%d" % c if c else "auto"): [round(t, 1) for t in v] for c, v in times.items()},
               "accepted": list(best) if win else None}
        report.append(rec)
        print("[%2d] %-11s M=%5d N=%5d K=%6d x%d  current %s %.1f  best %s %.1f %s" % (
            ki, tuning.FAMILIES[fam], key[1], key[2], key[3], counts[key], now, med[now], best,
            med[best] if best else float("nan"), " <- accepted" if win else ""), flush=True)
    capture()
    fin = statistics.median(timed(a.steps) for _ in range(3))
    print("step: %.1f -> %.1f us (%d keys changed)" % (base0, fin, len(changed)), flush=True)

    entries = []
    for e in table["entries"]:
        k = (e["fam"], e["M"], e["N"], e["K"])
        if k in changed:
            e = dict(e)
            e["tile"], e["ks"], e["gls"], e["want"] = changed.pop(k)
            e["pass"] = e.get("pass", "") + " (step-tuned)"
        entries.append(e)
    for k, c in changed.items():
        entries.append({"fam": k[0], "M": k[1], "N": k[2], "K": k[3], "tile": c[0], "ks": c[1], "gls": c[2],
                        "want": c[3], "pass": "step-tuned"})
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"meta": dict(table.get("meta", {}), step_tuned={"baseline_us": round(base0, 1),
                                                                   "final_us": round(fin, 1)}),
                   "entries": entries}, f, indent=1)
    with open(a.report, "w") as f:
        json.dump({"baseline_us": base0, "final_us": fin, "rows": report}, f, indent=1)


if __name__ == "__main__":
    main()
