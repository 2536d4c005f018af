set -u
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; exit $rc
