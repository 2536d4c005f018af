# round-4 call 27: the stock PyTorch-ROCm comparison re-run on the same box as the native bench (the
# round-1 number was another box), and every conv pass vs MIOpen in isolation
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_native_c27.log 2>&1
rc=$?; echo "native rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_native_c27.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --impl torch --steps 20 --warmup 5 > $O/bench_torch_c27.log 2>&1
rc=$?; echo "torch rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_torch_c27.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/conv_bench.py --out $O/conv_bench_c27.json > $O/conv_bench_c27.log 2>&1
rc=$?; echo "convs rc=$rc"; tail -4 $O/conv_bench_c27.log; [ $rc -eq 0 ] || exit $rc
