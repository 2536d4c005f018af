# round-4 call 8 (+ the call-7 steps: DP depth 50, LSTM protection, launch floor): the folded BN finalize (bn_apply_fin) -- kernel + model tests, bench A/B, step trace
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_bn_fold_gpu.py "tests/test_resnet50_train_gpu.py::test_resnet50_fusion_plan" > $O/pytest_call8.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call8.log | head -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
i=0
for v in all -bn_finalize_fold all -bn_finalize_fold; do
  i=$((i+1))
  TFX_FUSION=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c8_$i.log 2>&1
  rc=$?; echo "bench $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c8_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
STEPS="prof" bash scripts/gpu_session.sh || exit $?
timeout -k 10 120 python -u scripts/launch_floor.py > $O/launch_floor.txt 2>&1
rc=$?; echo "launch_floor rc=$rc"; cat $O/launch_floor.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests/test_dp_gpu.py tests/test_char_lstm_dp_gpu.py > $O/pytest_call7.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|SKIP|^E " $O/pytest_call7.log | head -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
