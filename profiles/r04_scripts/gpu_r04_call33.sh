#!/bin/bash
# Split-K atomic epilogue cost: the production 1x1 weight-gradient kernel with atomics vs plain stores.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_atomic
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u scripts/dev/splitk_atomic_probe.py > $O/splitk_atomic_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/splitk_atomic_probe.txt; exit $rc
