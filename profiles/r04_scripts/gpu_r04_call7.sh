# round-4 call 7: DP at depth 50 / batch 256 (f32 + bf16 wire), LSTM forced-expiry protection,
# the dependent-launch floor inside a graph
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python -u scripts/launch_floor.py > $O/launch_floor.txt 2>&1
rc=$?; echo "launch_floor rc=$rc"; cat $O/launch_floor.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests/test_dp_gpu.py tests/test_char_lstm_dp_gpu.py > $O/pytest_call7.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|SKIP|^E " $O/pytest_call7.log | head -30; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
