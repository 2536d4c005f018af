set -u
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_s2_addend_gpu.py tests/test_resnet_gpu.py tests/test_kernels_gpu.py tests/test_conv_production_gpu.py tests/test_dp_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_s2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_s2.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_s2_on$i.log 2>&1 || exit 1
TFX_S2_ADDEND=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_s2_off$i.log 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_s2_*.log
