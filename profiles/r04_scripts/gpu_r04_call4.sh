# round-4 call 4: per-variable fused-vs-layer-wise gradient / running-stat diagnostic + state-leak tests
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python scripts/diag_fusion_grads.py --steps 3 \
  --profiles "all;-head_tail;-lazy_bn_bwd;-bn_on_load;-block_boundary_fwd;-conv3_fused_bwd;-stem_kernels" \
  --json $O/diag_fusion.json > $O/diag_fusion.txt 2>&1
rc=$?; echo "diag rc=$rc"; grep -E "^===|^step" $O/diag_fusion.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_resnet50_train_gpu.py::test_resnet50_no_state_leaks_across_steps" > $O/pytest_call4.log 2>&1
rc=$?; echo "leak tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call4.log | head -20
