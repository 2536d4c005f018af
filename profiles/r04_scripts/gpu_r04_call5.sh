# round-4 call 5: convergence A/B over 4 seeds (fused vs round-2 layer-wise), new GPU tests, PMC + kernel trace
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_resnet50_train_gpu.py > $O/pytest_call5.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL" $O/pytest_call5.log | head -20; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PROFILES="all r2" SEEDS="2 3 4" TAG=_e3 OUT=$O bash scripts/dev/train_ab.sh || exit $?
STEPS="prof pmc" OUT=$O bash scripts/gpu_session.sh
