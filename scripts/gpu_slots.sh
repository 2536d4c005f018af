set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_bn_slots_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_slots.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_slots.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bn_slots_bench.py > gpurun_out/bn_slots_bench.log 2>&1 || exit 1
cat gpurun_out/bn_slots_bench.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_on$i.log 2>&1 || exit 1
TFX_BN_SLOTS=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_off$i.log 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_o*.log
echo DONE
