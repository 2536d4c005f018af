set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dev/conv3x3_probe.py > gpurun_out/conv3x3_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/conv3x3_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 \
  scripts/diag_premul_bf16.py > gpurun_out/diag_premul_bf16.txt 2>&1
rc=$?; echo "premul rc=$rc"; grep '{' gpurun_out/diag_premul_bf16.txt; exit $rc
