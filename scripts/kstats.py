#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv per training step: ms/step per kernel and totals.

usage: python scripts/kstats.py <run_kernel_stats.csv> [steps|auto] [top]
       python scripts/kstats.py --renorm <kernel_summary.txt> <old_divisor>

The per-step divisor is derived from the CALL COUNT of a kernel that runs exactly once per
training step (the fused optimizer ``opt_kernel``, else the loss kernel), so it always matches the
profiled run -- warmup, capture warm-ups and replays included -- instead of being assumed.  An
explicit ``steps`` argument is only a cross-check: a mismatch is reported, the derived count wins.
``--renorm`` rescales an older summary that was divided by a wrong step count.
"""
import csv
import re
import sys

# kernels that run exactly once per training step, in order of preference
ANCHORS = ("opt_kernel", "softmax_xent_mean_kernel", "softmax_xent_kernel")


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", "")) if "igemm" not in name else \
        name.replace("(tfx::IgemmArgs)", "")
    return name.replace("void ", "")[:100]


def derive_steps(rows):
    """(steps, anchor name) from the call count of a once-per-step kernel; (None, None) if absent."""
    for a in ANCHORS:
        calls = [int(r["Calls"]) for r in rows if a in r["Name"]]
        if calls:
            return sum(calls), a
    return None, None


def group(name: str) -> str:
    return "igemm" if "igemm" in name else "bn" if "bn_" in name else "other"


def summarize(rows, steps, top):
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / steps / 1e6
    groups = {}
    for r in rows:
        g = group(r["Name"])
        groups[g] = groups.get(g, 0.0) + float(r["TotalDurationNs"]) / steps / 1e6
    launches = sum(int(r["Calls"]) for r in rows) / steps
    out = ["kernel time per step: %.3f ms  (%s); %.0f launches per step" %
           (tot, ", ".join("%s %.3f" % kv for kv in sorted(groups.items())), launches)]
    rows = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:top]:
        out.append("%7.3f ms %5d calls %8.1f us  %s" % (float(r["TotalDurationNs"]) / steps / 1e6, int(r["Calls"]),
                                                       float(r["AverageNs"]) / 1e3, short(r["Name"])))
    return out


def renorm(path, old_div):
    """Rescale an old kernel_summary.txt (ms columns divided by ``old_div``) to the anchor's count."""
    lines = open(path).read().splitlines()
    pat = re.compile(r"^\s*([0-9.]+) ms\s+(\d+) calls\s+([0-9.]+) us\s+(.*)$")
    rows = []
    for ln in lines[1:]:
        m = pat.match(ln)
        if m:
            ms, calls, avg, name = float(m.group(1)), int(m.group(2)), float(m.group(3)), m.group(4)
            rows.append({"Name": name, "Calls": calls, "TotalDurationNs": ms * old_div * 1e6,
                         "AverageNs": avg * 1e3})
    steps, anchor = derive_steps(rows)
    assert steps, "no once-per-step anchor kernel in the summary"
    out = summarize(rows, steps, len(rows))
    out[0] += "  [divisor %d = calls of %s; re-normalised from a summary divided by %d]" % (steps, anchor, old_div)
    return out


def main():
    if sys.argv[1] == "--renorm":
        print("\n".join(renorm(sys.argv[2], int(sys.argv[3]))))
        return
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "auto"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    steps, anchor = derive_steps(rows)
    note = ""
    if steps is None:
        steps = int(want) if want != "auto" else 1
        note = "  [no once-per-step anchor kernel: divisor %d as given]" % steps
    else:
        note = "  [divisor %d = calls of %s]" % (steps, anchor)
        if want != "auto" and int(want) != steps:
            note += " (the %s steps given disagree: the call count wins)" % want
    out = summarize(rows, steps, top)
    out[0] += note
    print("\n".join(out))


if __name__ == "__main__":
    main()
