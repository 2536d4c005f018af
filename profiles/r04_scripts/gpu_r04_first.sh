set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_head.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet50_train_gpu.py \
  "tests/test_char_lstm_dp_gpu.py::test_persistent_lstm_failure_skips_update_and_falls_back" \
  "tests/test_char_lstm_dp_gpu.py::test_persistent_lstm_spin_expiry_raises" > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/pytest_new.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python examples/resnet_cifar.py --depth=50 --epochs=3 --logdir=/tmp/tfx_r04ckpt > gpurun_out/resnet50_3ep_example.log 2>&1
rc=$?; echo "example rc=$rc"; tail -4 gpurun_out/resnet50_3ep_example.log; exit $rc
