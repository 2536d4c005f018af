set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_head_gpu.py tests/test_resnet_gpu.py} -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_head.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_head.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
STEPS="bench prof" bash scripts/gpu_session.sh
