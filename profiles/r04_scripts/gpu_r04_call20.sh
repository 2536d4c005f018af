# round-4 call 20: conv3x3_bwd_fused with its weight-gradient B fragments prefetched two ahead
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_conv3_fused_gpu.py > $O/pytest_call20.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call20.log | head -20; [ $rc -eq 0 ] || exit 1
STEPS="bench prof" BENCH_REPS="1 2" bash scripts/gpu_session.sh || exit $?
rm -rf $O/prof
grep -E "conv3x3_bwd_fused" $O/kernel_summary.txt
timeout -k 10 600 python -u examples/resnet_cifar.py --depth=50 --epochs=3 --logdir=/tmp/ex_logdir > $O/resnet50_3ep_head.log 2>&1
rc=$?; echo "example rc=$rc"; grep -E "accuracy|images/sec" $O/resnet50_3ep_head.log; [ $rc -eq 0 ] || exit $rc
ls -la /tmp/ex_logdir > $O/ex_logdir_listing.txt; head -40 /tmp/ex_logdir/graph.pbtxt > $O/ex_graph_pbtxt_head.txt
