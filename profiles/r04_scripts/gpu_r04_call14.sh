# round-4 call 14: DP / fold tests from the zero-init start; interleaved fold A/B (3 pairs); then the
# launch-table re-measurement (call 10's steps)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests/test_dp_gpu.py tests/test_bn_fold_gpu.py > $O/pytest_call14.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call14.log | head -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
i=0
for v in all -bn_finalize_fold all -bn_finalize_fold all -bn_finalize_fold; do
  i=$((i+1))
  TFX_FUSION=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > $O/bench_c14_$i.log 2>&1
  rc=$?; echo "bench $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c14_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_r04_call10.sh
