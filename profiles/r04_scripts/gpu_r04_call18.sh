# round-4 call 18: HEAD kernel trace + step trace, and the 3-epoch depth-50 example at HEAD
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
STEPS="prof" bash scripts/gpu_session.sh || exit $?
timeout -k 10 600 python -u examples/resnet_cifar.py --depth=50 --epochs=3 --logdir=$O/ex_logdir > $O/resnet50_3ep_head.log 2>&1
rc=$?; echo "example rc=$rc"; grep -E "accuracy|images/sec" $O/resnet50_3ep_head.log; [ $rc -eq 0 ] || exit $rc
ls $O/ex_logdir | head
