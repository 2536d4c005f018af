#!/bin/bash
# Weight gradient as a parallel graph branch of its data gradient: serial vs forked/joined side stream.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_overlap
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u scripts/dev/wgrad_overlap_probe.py > $O/wgrad_overlap_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/wgrad_overlap_probe.txt; exit $rc
