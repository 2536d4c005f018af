# tests (TESTS) then a same-box A/B (AB_ARGS) -- one gpurun call
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 800 python scripts/dev/ab_bench.py ${AB_ARGS:-} > gpurun_out/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -6 gpurun_out/ab.txt; exit $rc
