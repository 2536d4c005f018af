# round-4 call 9: folded finalize v2 (store-scratch rows, no counter) -- tests, bench A/B, step trace;
# the DP one-rank graph test diagnosis (noise floor vs DP update)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_bn_fold_gpu.py "tests/test_resnet50_train_gpu.py::test_resnet50_fusion_plan" > $O/pytest_call9.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call9.log | head -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for d in "18 16" "50 256"; do
  set -- $d
  DP_DEPTH=$1 DP_BATCH=$2 TFX_DP_FORCE_COLLECTIVE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 scripts/dev/dp_diag.py > $O/dp_diag_$1.log 2>&1
  rc=$?; echo "dp_diag $1 rc=$rc"; grep -E "loss|update rel|worst" $O/dp_diag_$1.log | head -12; [ $rc -eq 0 ] || exit $rc
done
i=0
for v in all -bn_finalize_fold all -bn_finalize_fold; do
  i=$((i+1))
  TFX_FUSION=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c9_$i.log 2>&1
  rc=$?; echo "bench $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c9_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
STEPS="prof" bash scripts/gpu_session.sh || exit $?
