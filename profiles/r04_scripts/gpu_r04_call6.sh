# round-4 call 6: convergence with the zero-init-residual + warm-up recipe (4 seeds, fused path), r2 control,
# the synthetic-training test
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 280 --timeout-method thread -p no:cacheprovider \
  "tests/test_resnet50_train_gpu.py::test_resnet50_trains_synthetic_cifar" > $O/pytest_call6.log 2>&1
rc=$?; echo "test rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call6.log | head -5; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PROFILES="all" SEEDS="0 1 2 3 4" TAG=_zi OUT=$O bash scripts/dev/train_ab.sh || exit $?
PROFILES="r2" SEEDS="0 1" TAG=_zi OUT=$O bash scripts/dev/train_ab.sh || exit $?
