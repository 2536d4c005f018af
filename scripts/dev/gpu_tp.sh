# tests (TESTS) then a kernel-trace profile of bench.py (one gpurun call)
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_tp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_tp.log; [ $rc -eq 0 ] || exit $rc
STEPS="${STEPS:-bench prof}" bash scripts/gpu_session.sh
