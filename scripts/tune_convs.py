#!/usr/bin/env python3
"""Measure every igemm launch configuration of every ResNet-50/CIFAR conv and write the winners.

For each distinct conv of the batch-B step and each pass -- forward with the fused BN-statistics
epilogue (conv_fwd_stats), data gradient with the fused BN-backward epilogue where the model uses it
(conv_dgrad_bn: stride 1) or the parity-class data gradient (stride 2), weight gradient (conv_wgrad)
-- the op runs once under a launch trace to learn which kernel families / GEMM shapes it launches,
then every candidate configuration is forced on those families and timed.  Rounds are interleaved
(the auto configuration is re-timed in every round) and the median over rounds decides.  A
candidate replaces the heuristic only when it beats it by more than --margin.

Writes ``tensorflow_examples_amd/tune/igemm_gfx950.json`` (loaded by ops/tuning.py) plus a report.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tensorflow_examples_amd.ops import _native, tuning  # noqa: E402
from conv_bench import resnet50_convs  # noqa: E402

NSLOT = 64
# (tile, ks, gls, want): tile 1 = 128x128, 2 = 128x64, 3 = 256x64
# (deep rings -- gls 4-6, one 4-wave block per CU -- were candidates once and never won: profiles/r05_deep)
BF16_CANDS = [(t, 0, g, 0) for t in (1, 2, 3) for g in (0, 2, 3)] + [(t, 2, g, 0) for t in (1, 2) for g in (0, 2)]
ATOMIC_CANDS = [(t, k, g, w) for t in (1, 2) for k in (1, 2) for g in (0, 3) for w in (256, 512)]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def traced(fn):
    torch.ops.tfx.igemm_tune_trace(True)
    fn()
    torch.cuda.synchronize()
    torch.ops.tfx.igemm_tune_trace(False)
    rows = torch.ops.tfx.igemm_tune_traced().tolist()
    return sorted({tuple(r) for r in rows})


def force(fams, cand):
    torch.ops.tfx.igemm_tune_force(-1, 0, 0, -1, 0)
    if cand is not None:
        for f in fams:
            torch.ops.tfx.igemm_tune_force(f, *cand)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--margin", type=float, default=0.03)
    ap.add_argument("--out", default=tuning.TABLE)
    ap.add_argument("--report", default="gpurun_out/tune_report.json")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad", help="comma list of passes to tune")
    ap.add_argument("--merge", default=None,
                    help="existing table: keep its entries for the passes not tuned now, replace the rest")
    a = ap.parse_args()
    want_passes = set(a.passes.split(","))
    os.environ["TFX_TUNE"] = "0"
    assert _native.load()
    tuning.clear()
    dev = torch.device("cuda")
    uniq = {}
    for sh in resnet50_convs(a.batch):
        uniq[sh] = uniq.get(sh, 0) + 1
    entries, report = [], []
    tot_auto = tot_best = 0.0
    t_start = time.time()
    for (N, H, W, C, K, R, st), cnt in uniq.items():
        pad = R // 2
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        y = torch.ops.tfx.conv_fwd(x, w, st, pad, 1)
        gy = torch.randn_like(y)
        dw = torch.zeros(K, R, R, C, device=dev)
        slots = torch.zeros(NSLOT * 2 * K, device=dev)
        ws = torch.zeros(NSLOT * 2 * C, device=dev)
        save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
        dgam, dbet = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        passes = {
            "fwd": lambda: torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots),
            "dgrad": (lambda: torch.ops.tfx.conv_dgrad_bn(gy, w, list(x.shape), 1, pad, 1, None, x, save, None, True,
                                                           ws, dgam, dbet)) if st == 1 else
                     (lambda: torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None)),
            "wgrad": lambda: torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, True),
        }
        if C == 8:  # the stem: its input needs no gradient, so the model never runs its dgrad
            del passes["dgrad"]
        for name, fn in passes.items():
            if name not in want_passes:
                continue
            launches = traced(fn)
            fams = sorted({r[0] for r in launches})
            atomic = any(f in tuning.ATOMIC_FAMILIES for f in fams)
            cands = ATOMIC_CANDS if atomic else BF16_CANDS
            times = {None: []}
            times.update({c: [] for c in cands})
            for _ in range(a.rounds):
                for c in [None] + cands:
                    force(fams, c)
                    times[c].append(timeit(fn, a.iters))
            force(fams, None)
            med = {c: statistics.median(v) for c, v in times.items()}
            auto = med[None]
            best = min(cands, key=lambda c: med[c])
            use = med[best] < auto * (1 - a.margin)
            tot_auto += auto * cnt
            tot_best += (med[best] if use else auto) * cnt
            rec = {"shape": [N, H, W, C, K, R, st], "count": cnt, "pass": name,
                   "families": [tuning.FAMILIES[f] for f in fams], "launches": launches,
                   "auto_us": round(auto, 2), "best": list(best), "best_us": round(med[best], 2), "used": use,
                   "all": {"%d/%d/%d/%d" % c: round(t, 2) for c, t in med.items() if c is not None}}
            report.append(rec)
            print("%-30s %-5s %-28s auto %7.1f  best %7.1f %s%s" % (
                str([N, H, W, C, K, R, st]), name, ",".join(rec["families"]), auto, med[best], best,
                "  <- used" if use else ""), flush=True)
            if use:
                for fam, M, Nn, Kk in launches:
                    entries.append({"fam": fam, "M": M, "N": Nn, "K": Kk, "tile": best[0], "ks": best[1],
                                    "gls": best[2], "want": best[3], "us": round(med[best], 2),
                                    "auto_us": round(auto, 2), "shape": [N, H, W, C, K, R, st], "pass": name,
                                    "count": cnt})
        del x, w, y, gy, dw
    # a GEMM key reached from two convs keeps the row of the conv launched more often per step: a
    # stride-2 3x3 conv and the stride-1 3x3 convs after it share their weight-gradient key but not
    # their input layout (profiles/r06_tune_step); scripts/tune_step.py re-checks shared keys in the step
    entries.sort(key=lambda e: -e.get("count", 0))
    if a.merge:
        # keep the merged table's entries of the passes not re-tuned now (dgrad_flip rows included)
        with open(a.merge) as f:
            old = json.load(f)["entries"]
        entries += [e for e in old if e.get("pass", "").split(" ")[0] not in want_passes]
    seen, uniq_entries = set(), []
    for e in entries:
        k = (e["fam"], e["M"], e["N"], e["K"])
        if k not in seen:
            seen.add(k)
            uniq_entries.append(e)
    meta = {"device": torch.cuda.get_device_name(0), "batch": a.batch, "iters": a.iters, "rounds": a.rounds,
            "margin": a.margin, "conv_total_auto_us": round(tot_auto, 1), "conv_total_tuned_us": round(tot_best, 1),
            "tuning_seconds": round(time.time() - t_start, 1)}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"meta": meta, "entries": uniq_entries}, f, indent=1)
    os.makedirs(os.path.dirname(a.report) or ".", exist_ok=True)
    with open(a.report, "w") as f:
        json.dump({"meta": meta, "rows": report}, f, indent=1)
    print("conv passes per step: auto %.1f us -> tuned %.1f us (%d table entries)" % (tot_auto, tot_best,
                                                                                   len(uniq_entries)))


if __name__ == "__main__":
    main()
