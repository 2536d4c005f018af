set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_head.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python examples/resnet_cifar.py --depth=50 --epochs=3 --logdir=/tmp/tfx_r04ckpt > gpurun_out/resnet50_3ep_example.log 2>&1
rc=$?; echo "example rc=$rc"; tail -4 gpurun_out/resnet50_3ep_example.log; exit $rc
