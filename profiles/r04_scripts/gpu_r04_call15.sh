# round-4 call 15: the whole GPU suite, smoke(), and the driver's bench command at HEAD
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
STEPS="tests bench" BENCH_REPS="1 2" bash scripts/gpu_session.sh
