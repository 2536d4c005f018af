# round-4 call 3: numerics of the new loader kinds (production conv shapes vs fp32), bench, then bisect the
# fused-path training regression (1-epoch runs)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_production_gpu.py tests/test_dgrad_flip_gpu.py > $O/pytest_call3.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -3 $O/pytest_call3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $O/bench_call3.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_call3.log)"; [ $rc -eq 0 ] || exit $rc
EPOCHS=1 SEEDS=0 PROFILES="r2 all" TAG=_e1 OUT=$O bash scripts/dev/train_ab.sh || exit $?
EPOCHS=1 SEEDS=0 PROFILES="all" EXTRA=--nograph TAG=_e1_eager OUT=$O bash scripts/dev/train_ab.sh || exit $?
EPOCHS=1 SEEDS=0 PROFILES="-head_tail -bn_on_load -lazy_bn_bwd -conv3_fused_bwd -stem_kernels -block_boundary_fwd" \
  TAG=_e1 OUT=$O bash scripts/dev/train_ab.sh || exit $?
