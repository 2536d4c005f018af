#!/usr/bin/env python3
"""One training step of a rocprofv3 kernel trace, in launch order: per kernel its duration, the gap
since the previous kernel ended, grid and VGPRs -- the step is the span between the last two
once-per-step optimizer launches (``opt_kernel``).

usage: python scripts/step_trace.py <run_kernel_trace.csv> [--csv out.csv]"""
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("tfx::", "")
    m = re.match(r"(?:void )?([\w:]+)(<[^()]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:80]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "opt_kernel" in r["Kernel_Name"]]
    a, b = opt[-2] + 1, opt[-1] + 1
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = int(rows[a - 1]["End_Timestamp"])
    tot_k = tot_gap = 0.0
    out = []
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d, g = (e - s) / 1e3, (s - prev_end) / 1e3
        tot_k += d
        tot_gap += max(g, 0)
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        out.append((round((s - t0) / 1e3, 1), round(d, 1), round(g, 1), grid, int(r["VGPR_Count"]),
                    short(r["Kernel_Name"])))
        prev_end = e
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
    print("step span %.1f us: %d kernels, kernel time %.1f us, gaps %.1f us" % (span, len(step), tot_k, tot_gap))
    for o in out:
        print("%8.1f %7.1f %6.1f %6d %4d  %s" % o)


if __name__ == "__main__":
    main()
