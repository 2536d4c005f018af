set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_dp_gpu.py::test_dp_ring_simulation_leaves_gradients_unchanged" -x -q -p no:cacheprovider --timeout 250 --timeout-method thread > gpurun_out/pytest_dpsim.log 2>&1
rc=$?; echo "dpsim rc=$rc"; tail -3 gpurun_out/pytest_dpsim.log; [ $rc -eq 0 ] || { grep -E "assert|Error" gpurun_out/pytest_dpsim.log | head; exit $rc; }
for p in 2 0; do
timeout -k 10 300 python -u scripts/dp_contention.py --blocks 0,16,32 --passes $p --out gpurun_out/dp_contention_p$p.json > gpurun_out/dp_contention_p$p.log 2>&1
rc=$?; echo "contention passes=$p rc=$rc"; grep "vs no DP" gpurun_out/dp_contention_p$p.log; [ $rc -eq 0 ] || exit $rc
done
