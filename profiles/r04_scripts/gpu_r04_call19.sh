# round-4 call 19: HEAD kernel trace + step trace, and the 3-epoch depth-50 example at HEAD (checkpoint
# under /tmp: it exceeds what gpurun copies back; its file list and graph.pbtxt head are kept)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
STEPS="prof" bash scripts/gpu_session.sh || exit $?
rm -rf $O/prof
timeout -k 10 600 python -u examples/resnet_cifar.py --depth=50 --epochs=3 --logdir=/tmp/ex_logdir > $O/resnet50_3ep_head.log 2>&1
rc=$?; echo "example rc=$rc"; grep -E "accuracy|images/sec" $O/resnet50_3ep_head.log; [ $rc -eq 0 ] || exit $rc
ls -la /tmp/ex_logdir > $O/ex_logdir_listing.txt; head -40 /tmp/ex_logdir/graph.pbtxt > $O/ex_graph_pbtxt_head.txt
