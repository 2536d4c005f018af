# round-4 call 23: vectors per thread of the BN elementwise passes (TFX_BN_VPT), interleaved bench A/B
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
i=0
for v in 4 2 8 1 4 2 8 1; do
  i=$((i+1))
  TFX_BN_VPT=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > $O/bench_c23_$i.log 2>&1
  rc=$?; echo "bench vpt=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c23_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
