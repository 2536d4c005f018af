# round-4 call 22: the example GPU test with its 60-step recipe
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_examples_gpu.py > $O/pytest_call22.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call22.log | head -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
i=0
for v in 4 2 8 1 4 2 8 1; do
  i=$((i+1))
  TFX_BN_VPT=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > $O/bench_c23_$i.log 2>&1
  rc=$?; echo "bench vpt=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c23_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
