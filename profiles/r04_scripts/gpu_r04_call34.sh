# round-4 call 34: whole GPU suite, smoke and the driver's bench on the rebuilt libtfx_ops.so
set -u
mkdir -p gpurun_out/r04_final
OUT=$PWD/gpurun_out/r04_final STEPS="tests bench" BENCH_REPS="1 2" bash scripts/gpu_session.sh || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r04_final/smoke.log; exit $rc
