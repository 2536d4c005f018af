#!/usr/bin/env python3
"""Summarise gpurun_out/pmcc/<pass>_<cfg>_p<i> counter dirs: per config, the igemm kernel's mean
duration and per-dispatch counters, with derived MFMA busy %, stall splits and loads in flight."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcc"
cfgs = sorted({os.path.basename(p).rsplit("_p", 1)[0] for p in glob.glob(os.path.join(root, "*_p1"))})
for cfg in cfgs:
    c = collections.defaultdict(float)
    n = collections.defaultdict(int)
    durs, name = [], ""
    for p in sorted(glob.glob(os.path.join(root, cfg + "_p*", "p_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            if "igemm" not in r["Kernel_Name"]:
                continue
            c[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
    for r in csv.DictReader(open(os.path.join(root, cfg + "_p1", "p_kernel_trace.csv"))):
        if "igemm" in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
            name = r["Kernel_Name"].split("igemm_kernel")[1].split(">")[0] + ">"
            vg = r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"]
    v = {k: c[k] / n[k] for k in c}
    d = sorted(durs)[len(durs) // 2]
    gui = v.get("GRBM_GUI_ACTIVE", 1)
    mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui / 8 * 1024) * 100 if gui else 0
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(f"{cfg:14s} {name:28s} vgpr/agpr/lds {vg}  median {d:6.1f} us  MFMA busy {mf:5.1f}%  "
          f"wait {v.get('SQ_WAIT_ANY', 0) / wc * 100:5.1f}%  wait_inst {v.get('SQ_WAIT_INST_ANY', 0) / wc * 100:5.1f}%  "
          f"active {v.get('SQ_ACTIVE_INST_ANY', 0) / wc * 100:5.1f}% (vmem {v.get('SQ_ACTIVE_INST_VMEM', 0) / wc * 100:4.1f} "
          f"lds {v.get('SQ_ACTIVE_INST_LDS', 0) / wc * 100:4.1f} valu {v.get('SQ_ACTIVE_INST_VALU', 0) / wc * 100:4.1f} "
          f"sca {v.get('SQ_ACTIVE_INST_SCA', 0) / wc * 100:4.1f})  wait_lds {v.get('SQ_WAIT_INST_LDS', 0) / wc * 100:4.1f}%  "
          f"ldsconf {v.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, v.get('SQ_LDS_IDX_ACTIVE', 1)) * 100:4.1f}%  "
          f"vmem_lvl {v.get('SQ_INST_LEVEL_VMEM', 0) / wc:5.2f}  ta_fifo_full {v.get('SQ_VMEM_TA_CMD_FIFO_FULL', 0):.0f} "
          f"lds_fifo_full {v.get('SQ_LDS_CMD_FIFO_FULL', 0):.0f}  L2 hit {v.get('TCC_HIT_sum', 0) / max(1, v.get('TCC_HIT_sum', 0) + v.get('TCC_MISS_sum', 0)) * 100:4.1f}%")
