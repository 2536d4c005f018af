set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pw_bwd_gpu.py tests/test_pw_fwd_gpu.py tests/test_resnet_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_f1.log 2>&1
rc=$?; echo "f1 rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_f1.log | head -60; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench2.log | cut -c1-200; exit $rc
