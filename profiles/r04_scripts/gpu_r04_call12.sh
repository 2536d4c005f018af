# round-4 call 12: which fusion group makes the "all" profile's step nondeterministic (ResNet-18 b16)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for f in "-stem_kernels" "-bn_finalize_fold" "-lazy_bn_bwd" "r2" "-stem_kernels,-bn_finalize_fold"; do
  TFX_FUSION=$f timeout -k 10 240 python -u scripts/dev/determinism.py --depth 18 --batch 16 --reps 2 \
    >> $O/determinism2.log 2>&1
  rc=$?; echo "det FUSION=$f rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/determinism2.log; exit $rc; }
done
for f in "all" "-bn_finalize_fold"; do
  TFX_FUSION=$f timeout -k 10 240 python -u scripts/dev/determinism.py --depth 50 --batch 64 --reps 2 \
    >> $O/determinism2.log 2>&1
  rc=$?; echo "det r50 FUSION=$f rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/determinism2.log; exit $rc; }
done
grep rep $O/determinism2.log | cut -c1-200
