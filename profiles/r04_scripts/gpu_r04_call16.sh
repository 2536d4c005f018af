# round-4 call 16: the fused-BN 1x1 data gradient in its training-step form, every launch configuration
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u scripts/dev/dgrad_bn_sweep.py > $O/dgrad_bn_sweep.txt 2>&1
rc=$?; echo "sweep rc=$rc"; cat $O/dgrad_bn_sweep.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
