set -u
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/pytest_all.log | head -40; exit $rc; }
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_head_$i.log 2>&1 || exit 1
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_head_*.log
