#!/bin/bash
# The reference's 3-process recipe (R/distributed/distributed.py:7-14) on one node over xGMI: one ps and
# two workers, 50 epochs x 550 batches (synthetic MNIST when MNIST_data is absent).  Logs go to
# gpurun_out/mlp_{ps,worker0,worker1}.log.  Usage: bash scripts/run_mlp_xgmi.sh [extra flags]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P=$(python - <<'PY'
import socket
s = [socket.socket() for _ in range(3)]
for x in s: x.bind(("127.0.0.1", 0))
print(" ".join(str(x.getsockname()[1]) for x in s))
PY
)
set -- $P "$@"
PS=$1; W0=$2; W1=$3; shift 3
ARGS="--ps_hosts=127.0.0.1:$PS --worker_hosts=127.0.0.1:$W0,127.0.0.1:$W1 --device=cuda --transport=xgmi \
  --logs_path=/tmp/mnist_xgmi --ps_exit_after_workers $*"
timeout -k 10 500 python distributed/distributed.py $ARGS --job_name=ps --task_index=0 > gpurun_out/mlp_ps.log 2>&1 &
PSPID=$!
timeout -k 10 500 python distributed/distributed.py $ARGS --job_name=worker --task_index=0 > gpurun_out/mlp_worker0.log 2>&1 &
A=$!
timeout -k 10 500 python distributed/distributed.py $ARGS --job_name=worker --task_index=1 > gpurun_out/mlp_worker1.log 2>&1 &
B=$!
wait $A; ra=$?
wait $B; rb=$?
wait $PSPID; rp=$?
echo "worker0 rc=$ra worker1 rc=$rb ps rc=$rp"
tail -4 gpurun_out/mlp_worker0.log gpurun_out/mlp_worker1.log
[ $ra -eq 0 ] && [ $rb -eq 0 ] && [ $rp -eq 0 ]
