set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_conv3_fused_gpu.py tests/test_pw_fwd_gpu.py tests/test_pw_bwd_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; grep -E "FAIL|Error|assert|passed|failed" gpurun_out/pytest_c3.log | head -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
STEPS=prof bash scripts/gpu_session.sh
