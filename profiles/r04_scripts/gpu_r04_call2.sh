# round-4 call 2: LSTM protection, DP (depth 50 / bf16 wire), bucket table, forced-collective bench A/B,
# fusion-profile training A/B.  Runs from a frozen snapshot (scripts/snap_submit.sh); OUT = merged dir.
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_char_lstm_dp_gpu.py::test_persistent_lstm_failure_skips_update_and_falls_back" \
  "tests/test_char_lstm_dp_gpu.py::test_persistent_lstm_spin_expiry_raises" \
  tests/test_dp_gpu.py > $O/pytest_call2.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL" $O/pytest_call2.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for dt in f32 bf16; do
  TFX_DP_FORCE_COLLECTIVE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 2953$([ $dt = f32 ] && echo 1 || echo 2) scripts/dp_bucket_table.py \
    --dtype $dt --json $O/dp_buckets_$dt.json > $O/dp_buckets_$dt.txt 2>&1
  rc=$?; echo "buckets $dt rc=$rc"; tail -3 $O/dp_buckets_$dt.txt; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
for dt in f32 bf16; do
  TFX_DP_FORCE_COLLECTIVE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 2954$rep bench.py --steps 30 --warmup 5 --allreduce-dtype $dt \
    > $O/bench_dpforce_${dt}_$rep.log 2>&1
  rc=$?; echo "dpforce $dt rep $rep rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_dpforce_${dt}_$rep.log)"
  [ $rc -eq 0 ] || exit $rc
done
done
PROFILES="all r2" SEEDS="0 1" OUT=$O bash scripts/dev/train_ab.sh
