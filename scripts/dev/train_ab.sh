# ResNet-50 3-epoch synthetic-CIFAR runs: fusion profiles x seeds (accuracy / loss-curve A/B).
set -u
O=${OUT:-gpurun_out}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for spec in ${PROFILES:-all r2}; do
  for seed in ${SEEDS:-0 1}; do
    TFX_FUSION=$spec timeout -k 10 300 python examples/resnet_cifar.py --depth=50 --epochs=${EPOCHS:-3} --seed=$seed \
      > $O/train_${spec}_s$seed.log 2>&1
    rc=$?; echo "fusion=$spec seed=$seed rc=$rc $(grep 'test accuracy' $O/train_${spec}_s$seed.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
