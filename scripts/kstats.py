#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv per training step: ms/step per kernel and totals.

usage: python scripts/kstats.py <run_kernel_stats.csv> [steps=7] [top=30]
(bench.py under rocprofv3 with --steps 5 --warmup 2 runs 7 steps.)"""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", "")) if "igemm" not in name else \
        name.replace("(tfx::IgemmArgs)", "")
    return name.replace("void ", "")[:100]


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / steps / 1e6
    groups = {}
    for r in rows:
        n = r["Name"]
        g = "igemm" if "igemm" in n else "bn" if "bn_" in n else "other"
        groups[g] = groups.get(g, 0.0) + float(r["TotalDurationNs"]) / steps / 1e6
    print("kernel time per step: %.3f ms  (%s)" % (tot, ", ".join("%s %.3f" % kv for kv in sorted(groups.items()))))
    for r in rows[:top]:
        print("%7.3f ms %5d calls %8.1f us  %s" % (float(r["TotalDurationNs"]) / steps / 1e6, int(r["Calls"]),
                                                    float(r["AverageNs"]) / 1e3, short(r["Name"])))


if __name__ == "__main__":
    main()
