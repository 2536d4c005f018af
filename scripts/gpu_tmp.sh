set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_resnet50_train_gpu.py -k "leak" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_leak.log 2>&1
rc=$?; echo "leak rc=$rc"; tail -3 gpurun_out/pytest_leak.log; [ $rc -eq 0 ] || { grep -E "assert|Error" gpurun_out/pytest_leak.log | head; exit $rc; }
timeout -k 10 900 python -u scripts/convergence_parity.py --steps 300 --batch 128 --repeat 2 \
  --negctl lazy_bn_bwd:0.8,conv3_fused_bwd:0.8,lazy_bn_bwd:0.5 --out gpurun_out/conv_parity.json > gpurun_out/conv_parity.log 2>&1
rc=$?; echo "conv rc=$rc"; grep -E "COMPARE|data|mode" gpurun_out/conv_parity.log | cut -c1-400; exit $rc
