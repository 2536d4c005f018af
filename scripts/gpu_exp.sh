set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_igemm_ks2_gpu.py -x -q -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/pytest_ks2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ks2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/tune_convs.py --out gpurun_out/igemm_gfx950.json --report gpurun_out/tune_report.json > gpurun_out/tune.log 2>&1 || { tail -5 gpurun_out/tune.log; exit 1; }
tail -2 gpurun_out/tune.log
cp gpurun_out/igemm_gfx950.json tensorflow_examples_amd/tune/igemm_gfx950.json
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_ks2_$i.log 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ks2_*.log
