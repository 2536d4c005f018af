set -u
R=$GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k sgemm tests/test_sparse_rnn_gpu.py tests/test_mlp_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sg.log; [ $rc -eq 0 ] || exit $rc
for b in 4096 128; do
timeout -k 10 300 python scripts/bench_models.py --model word2vec --batch $b --steps 50 --warmup 10 --graph 2>&1 | tail -1 | cut -c1-220
done
timeout -k 10 300 python scripts/bench_models.py --model word2vec --batch 4096 --steps 50 --warmup 10 --impl torch 2>&1 | tail -1 | cut -c1-220
rm -rf $R/gpurun_out/profw
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profw" -o run -- python3 "$R/scripts/bench_models.py" --model word2vec --batch 4096 --steps 20 --warmup 5 > "$R/gpurun_out/profw.log" 2>&1 || { tail -5 $R/gpurun_out/profw.log; exit 1; }
echo DONE
