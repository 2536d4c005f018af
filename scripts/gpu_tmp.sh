set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dev/conv3x3_probe.py > gpurun_out/conv3x3_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/conv3x3_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_conv3_fused_gpu.py tests/test_resnet50_train_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log; exit $rc
