#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 ``--pmc`` passes (counter_collection.csv files).

usage: python scripts/pmc_summary.py <dir with pass subdirs> [--steps N] [--flops flops.json]

Aggregates every ``*counter_collection.csv`` under the directory (one pass per subdir, each with
its own counter set), sums each counter per kernel name, and derives:

* MFMA busy %  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES-equivalent chip cycles * 1024 SIMDs)
  computed as busy / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs): GRBM_GUI_ACTIVE is summed over the
  8 XCDs (MI355X_MICROARCH.md 'DVFS give-back');
* achieved bf16 TFLOP/s implied by the MFMA busy cycles (1024 FLOP per busy cycle per SIMD for the
  bf16 16x16x32 / 32x32x16 MFMAs) over the kernels' wall time;
* LDS bank-conflict rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* HBM bytes: FETCH_SIZE (KB, reported x2 for gfx950 wide streaming reads -- MICROARCH 'HBM') and
  WRITE_SIZE (KB).
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("(tfx::IgemmArgs)", "")
    n = re.sub(r"^void ", "", n)
    if "igemm" not in n:
        n = re.sub(r"\(.*$", "", n)
    return n[:90]


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    durs = []  # per pass: kernel -> us (each pass runs the same dispatches; keep the least perturbed)
    calls = {}
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        seen, dur, cnt = set(), collections.defaultdict(float), collections.defaultdict(int)
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            d = r["Dispatch_Id"]
            if d not in seen:
                seen.add(d)
                cnt[k] += 1
                if r.get("Start_Timestamp"):
                    dur[k] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3  # us
        durs.append(dur)
        for k, n in cnt.items():
            calls[k] = n
    dur = {k: min(d.get(k, float("inf")) for d in durs) for k in per}
    return per, dur, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    per, dur, calls = load(a.root)
    rows = []
    for k, c in per.items():
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        util = 100.0 * busy / (gui / 8 * 1024) if gui else float("nan")
        us = dur.get(k, 0.0)
        tf = busy * 1024 / (us * 1e-6) / 1e12 if us else float("nan")
        conf = c.get("SQ_LDS_BANK_CONFLICT", float("nan"))
        lds = c.get("SQ_LDS_IDX_ACTIVE", float("nan"))
        conf_pct = 100.0 * conf / lds if lds and lds == lds else float("nan")
        fetch = 2 * c.get("FETCH_SIZE", float("nan")) / 1024  # MB (x2: gfx950 FETCH_SIZE undercount)
        write = c.get("WRITE_SIZE", float("nan")) / 1024
        waves = c.get("SQ_WAVE_CYCLES", float("nan"))
        wait = c.get("SQ_WAIT_ANY", float("nan"))
        rows.append((us, k, calls.get(k, 0), util, tf, conf_pct, fetch, write,
                     100.0 * wait / waves if waves == waves and waves else float("nan"),
                     c.get("SQ_WAIT_INST_LDS", float("nan")) / waves * 100 if waves == waves and waves else float("nan")))
    rows.sort(reverse=True)
    s = a.steps
    print("%9s %6s %7s %8s %7s %9s %9s %6s %6s  %s" % ("us/step", "calls", "mfma%", "TF/s", "ldsC%", "fetchMB",
                                                     "writeMB", "wait%", "ldsW%", "kernel"))
    for us, k, n, util, tf, conf, fetch, write, wait, ldsw in rows[:a.top]:
        print("%9.1f %6d %7.1f %8.1f %7.1f %9.1f %9.1f %6.1f %6.1f  %s" % (us / s, n, util, tf, conf, fetch / s,
                                                                          write / s, wait, ldsw, k))


if __name__ == "__main__":
    main()
