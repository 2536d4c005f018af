# round-4 call 24: two fused-BN 1x1 data-gradient launch-table entries from the training-step-form sweep
# (stage-2 block-1 conv1: 128x128 LDS-DMA ring; stage-4 conv1: 256x64 ring), interleaved bench A/B
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
i=0
for f in cand base cand base cand base; do
  i=$((i+1))
  if [ $f = cand ]; then export TFX_TUNE_FILE=scripts/dev/tune_dgrad_cand.json; else unset TFX_TUNE_FILE; fi
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 > $O/bench_c24_$i.log 2>&1
  rc=$?; echo "bench $f rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c24_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
