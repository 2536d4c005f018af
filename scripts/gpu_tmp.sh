set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_mlp_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_mlp.log | head -30; exit $rc
