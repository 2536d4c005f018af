#!/bin/bash
# Split-K 1x1 weight gradient: per-block fixed cost vs per-k-tile cost (forced launch config, scaled batch).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_kps
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u scripts/dev/wgrad_kps_probe.py > $O/wgrad_kps_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/wgrad_kps_probe.txt; exit $rc
