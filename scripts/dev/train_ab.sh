# ResNet-50 synthetic-CIFAR runs: fusion profiles x seeds (accuracy / loss-curve A/B).
# PROFILES: TFX_FUSION specs (ops/fusion.py); EXTRA: extra example flags; TAG: log-name suffix.
set -u
O=${OUT:-gpurun_out}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for spec in ${PROFILES:-all r2}; do
  for seed in ${SEEDS:-0 1}; do
    log=$O/train_${spec}_s${seed}${TAG:-}.log
    TFX_FUSION=$spec timeout -k 10 300 python examples/resnet_cifar.py --depth=50 --epochs=${EPOCHS:-3} --seed=$seed \
      ${EXTRA:-} > $log 2>&1
    rc=$?; echo "fusion=$spec seed=$seed rc=$rc $(grep 'step .*0 lr' $log | tail -1) $(grep 'test accuracy' $log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
