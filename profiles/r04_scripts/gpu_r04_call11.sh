# round-4 call 11: run-to-run determinism bisection (two identical steps, per-variable gradient
# distance) under the operand / fusion toggles; folded-finalize v3 tests and bench A/B
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in "1 all" "0 all" "1 r2" "1 none" "0 none"; do
  set -- $cfg
  TFX_IGEMM_XT=$1 TFX_FUSION=$2 timeout -k 10 240 python -u scripts/dev/determinism.py --depth 18 --batch 16 \
    >> $O/determinism.log 2>&1
  rc=$?; echo "det XT=$1 FUSION=$2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/determinism.log; exit $rc; }
done
grep -E "rep" $O/determinism.log
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_bn_fold_gpu.py > $O/pytest_call11.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call11.log | head -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
i=0
for v in all -bn_finalize_fold all -bn_finalize_fold; do
  i=$((i+1))
  TFX_FUSION=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c11_$i.log 2>&1
  rc=$?; echo "bench $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c11_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
STEPS="prof" bash scripts/gpu_session.sh || exit $?
