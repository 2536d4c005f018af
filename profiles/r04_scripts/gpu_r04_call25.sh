# round-4 call 25: projection shortcut launched right after conv1 (x still hot) -- the model tests that
# exercise the projection blocks' fused backward, then an interleaved bench A/B (TFX_PROJ_EARLY)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 280 --timeout-method thread -p no:cacheprovider \
  tests/test_resnet50_train_gpu.py tests/test_res_bn_sec_gpu.py tests/test_s2_addend_gpu.py tests/test_pw_bwd_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest_call25.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|^E " $O/pytest_call25.log | head -40; [ $rc -eq 0 ] || exit 1
i=0
for v in 1 0 1 0 1 0; do
  i=$((i+1))
  TFX_PROJ_EARLY=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 > $O/bench_c25_$i.log 2>&1
  rc=$?; echo "bench proj_early=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_c25_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
