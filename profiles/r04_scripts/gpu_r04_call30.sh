#!/bin/bash
# Load-path counters (TA / TD / TCP busy and stall, L2 read latency) over the eager bench: one pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_lp
mkdir -p $O
cd $R
timeout -k 10 90 rocprofv3 --list-avail > $O/avail.txt 2>&1; echo "list-avail rc=$?"
grp=$(python3 - "$O/avail.txt" <<'PY'
import re, sys
txt = open(sys.argv[1], errors="replace").read()
names = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", txt))
want = [["TA_TA_BUSY_sum", "TA_TA_BUSY"], ["TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_ADDR_STALLED_BY_TC_CYCLES"],
        ["TD_TD_BUSY_sum", "TD_TD_BUSY"],
        ["TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_LATENCY"], ["TCP_TCC_READ_REQ_sum", "TCP_TCC_READ_REQ"],
        ["TCP_PENDING_STALL_CYCLES_sum", "TCP_PENDING_STALL_CYCLES"], ["GRBM_GUI_ACTIVE"]]
out = []
for alts in want:
    for n in alts:
        if n in names:
            out.append(n)
            break
print(" ".join(out))
PY
)
echo "counters: $grp" | tee $O/group.txt
[ -n "$grp" ] || exit 3
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$O/pmc" -o p -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --no-graph > $O/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc.log; exit $rc; }
python3 scripts/pmc_loadpath.py $O/pmc --steps 3 > $O/loadpath.txt; head -30 $O/loadpath.txt
