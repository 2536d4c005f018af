# round-4 call 13: is the run-to-run gradient spread a race or chaos?  Sensitivity of one step to a
# 1e-6 nudge of one BN gamma on the bit-reproducible r2 profile, and the spread with zero-init residuals
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { TFX_FUSION=$1 timeout -k 10 240 python -u scripts/dev/determinism.py --reps 2 ${@:2} >> $O/determinism3.log 2>&1
        rc=$?; echo "det $* rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/determinism3.log; exit $rc; }; }
run r2 --depth 18 --batch 16 --perturb 1e-6
run r2 --depth 50 --batch 64
run r2 --depth 50 --batch 64 --perturb 1e-6
run all --depth 50 --batch 64 --zero-init
run r2 --depth 50 --batch 64 --zero-init --perturb 1e-6
run all --depth 18 --batch 16 --zero-init
grep rep $O/determinism3.log | cut -c1-260
