# round-4 call 10: re-measure the igemm launch table (fwd, dgrad, wgrad) with the round-4 loaders, then
# an interleaved bench A/B of the new table against the committed one
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cp tensorflow_examples_amd/tune/igemm_gfx950.json $O/tune_old.json
timeout -k 10 900 python -u scripts/tune_convs.py --passes fwd,dgrad,wgrad --merge $O/tune_old.json \
  --out $O/tune_new.json --report $O/tune_report.json > $O/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -3 $O/tune.log; [ $rc -eq 0 ] || exit $rc
i=0
for f in new old new old; do
  i=$((i+1))
  TFX_TUNE_FILE=$O/tune_$f.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c9_$i.log 2>&1
  rc=$?; echo "bench table=$f rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c9_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
