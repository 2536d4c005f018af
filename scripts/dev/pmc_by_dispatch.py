"""Per (phase, kernel, grid) counter means from rocprofv3 --pmc passes: the shapes of one kernel kept
apart.  A "phase" starts at each dispatch of the --phase kernel with a new grid (scripts/dev/bna_probe.py
runs one shape after another: the bn_apply grid changes with the shape).
usage: python scripts/dev/pmc_by_dispatch.py <dir with pass subdirs> [--phase name] [kernel-substring ...]"""
import collections
import csv
import glob
import os
import re
import sys

args = sys.argv[2:]
phase_k = None
if args[:1] == ["--phase"]:
    phase_k, args = args[1], args[2:]
root, pats = sys.argv[1], args
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    phase, last_grid = 0, None
    for r in rows:
        name = re.sub(r"\(.*$", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
        grid = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
        if phase_k and phase_k in name and grid != last_grid:
            if last_grid is not None:
                phase += 1
            last_grid = grid
        if pats and not any(p in name for p in pats):
            continue
        key = (phase, name[:64], grid)
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[key]["_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cols = ["_us", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
        "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "FETCH_SIZE", "WRITE_SIZE"]
print("%2s %-64s %6s " % ("ph", "kernel", "blocks") + " ".join("%12s" % c.replace("SQ_", "")[:12] for c in cols) + "  wait%  valu/mfma")
for key in sorted(agg):
    d = agg[key]
    m = {c: (sum(d[c]) / len(d[c]) if d.get(c) else float("nan")) for c in cols}
    wait = 100 * m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"] if m["SQ_WAVE_CYCLES"] == m["SQ_WAVE_CYCLES"] else float("nan")
    ratio = m["SQ_ACTIVE_INST_VALU"] / m["SQ_VALU_MFMA_BUSY_CYCLES"] if m["SQ_VALU_MFMA_BUSY_CYCLES"] else float("nan")
    print("%2d %-64s %6d " % key + " ".join("%12.4g" % m[c] for c in cols) + "  %5.1f  %6.2f" % (wait, ratio))
