#!/bin/bash
# One gpurun session: GPU tests, 1-GPU native bench, stock-torch bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout stops the script (no further GPU work).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
STEPS=${STEPS:-"tests bench torch prof"}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
      ok_or_testfail $rc || exit $rc ;;
    bench)
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_native.log; [ $rc -eq 0 ] || exit $rc ;;
    ab)
      for i in 1 2; do
        TFX_NO_GRADSINK=1 timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_off_$i.log 2>&1 || exit 1
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_on_$i.log 2>&1 || exit 1
      done
      grep -ho '"ms_per_step": [0-9.]*' gpurun_out/ab_*.log ;;
    epibench)
      for v in 1 0; do
        TFX_BN_LAST_ARRIVER=$v timeout -k 10 300 python scripts/epi_bench.py --out gpurun_out/epi_bench_la$v.json > gpurun_out/epi_bench_la$v.log 2>&1 || exit 1
      done
      tail -1 gpurun_out/epi_bench_la*.log ;;
    abks)
      for v in 1 2; do
        TFX_WGRAD_KS=$v timeout -k 10 300 python scripts/conv_bench.py --out gpurun_out/conv_bench_ks$v.json > gpurun_out/conv_bench_ks$v.log 2>&1 || exit 1
      done
      for i in 1 2; do for v in 1 2; do
        TFX_WGRAD_KS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/abks_${v}_$i.log 2>&1 || exit 1
      done; done
      grep TOTAL gpurun_out/conv_bench_ks*.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/abks_*.log ;;
    abfuse)
      for i in 1 2; do
        TFX_FUSE_BN=0 timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/abf_off_$i.log 2>&1 || exit 1
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/abf_on_$i.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/abf_*.log ;;
    abtile)
      for i in 1 2; do
        TFX_TILE_POLICY=0 timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/abt_off_$i.log 2>&1 || exit 1
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/abt_on_$i.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/abt_*.log ;;
    absplit)
      for v in 128 192 256; do
        TFX_SPLITK_BLOCKS=$v timeout -k 10 400 python bench.py --steps 40 --warmup 5 > gpurun_out/abs_$v.log 2>&1 || exit 1
      done
      for v in 128 192 256; do
        TFX_SPLITK_BLOCKS=$v timeout -k 10 400 python bench.py --steps 40 --warmup 5 > gpurun_out/abs2_$v.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/abs*.log ;;
    abwg)
      for v in 128 64; do
        TFX_WGRAD_TILE=$v timeout -k 10 300 python scripts/conv_bench.py --out gpurun_out/conv_bench_wg$v.json > gpurun_out/conv_bench_wg$v.log 2>&1 || exit 1
      done
      for i in 1 2; do for v in 128 64; do
        TFX_WGRAD_TILE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/abwg_${v}_$i.log 2>&1 || exit 1
      done; done
      tail -1 gpurun_out/conv_bench_wg*.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/abwg_*.log ;;
    dpgraph)
      timeout -k 10 400 python -m pytest tests/test_dp_gpu.py -x -q -p no:cacheprovider -k graph > gpurun_out/pytest_dpgraph.log 2>&1
      rc=$?; echo "dpgraph test rc=$rc"; tail -5 gpurun_out/pytest_dpgraph.log; [ $rc -eq 0 ] || exit $rc
      for v in 1 0; do
        TFX_DP_FORCE_COLLECTIVE=1 TFX_DP_GRAPH=$v timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 30 --warmup 5 > gpurun_out/bench_dpforce_g$v.log 2>&1
        rc=$?; echo "dpforce graph=$v rc=$rc"; tail -2 gpurun_out/bench_dpforce_g$v.log; [ $rc -eq 0 ] || exit $rc
      done ;;
    kerneltests)
      timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_kernels.log 2>&1
      rc=$?; echo "kerneltests rc=$rc"; tail -5 gpurun_out/pytest_kernels.log
      [ $rc -eq 0 ] || exit $rc ;;
    graph)
      timeout -k 10 400 python bench.py --steps 20 --warmup 5 --graph > gpurun_out/bench_graph.log 2>&1
      rc=$?; echo "graph rc=$rc"; tail -3 gpurun_out/bench_graph.log; [ $rc -eq 0 ] || exit $rc ;;
    torch)
      timeout -k 10 400 python bench.py --impl torch --steps 20 --warmup 5 > gpurun_out/bench_torch.log 2>&1
      rc=$?; echo "torch rc=$rc"; tail -3 gpurun_out/bench_torch.log; [ $rc -eq 0 ] || exit $rc ;;
    convbench)
      timeout -k 10 400 python scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1
      rc=$?; echo "convbench rc=$rc"; tail -3 gpurun_out/conv_bench.log; [ $rc -eq 0 ] || exit $rc ;;
    bnbench)
      for u in 1; do TFX_BN_RED_U=$u timeout -k 10 200 python scripts/bn_bench.py > gpurun_out/bn_bench_u$u.log 2>&1 || exit 1; done
      echo bnbench done; tail -1 gpurun_out/bn_bench_u*.log ;;
    newtests)
      timeout -k 10 600 python -m pytest tests/test_sparse_rnn_gpu.py -q -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1
      rc=$?; echo "newtests rc=$rc"; tail -8 gpurun_out/pytest_new.log
      ok_or_testfail $rc || exit $rc ;;
    lstm)
      timeout -k 10 300 python -u -m pytest tests/test_sparse_rnn_gpu.py -k lstm -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm.log 2>&1
      rc=$?; echo "lstm tests rc=$rc"; tail -15 gpurun_out/pytest_lstm.log; [ $rc -eq 0 ] || exit $rc
      : > gpurun_out/bench_lstm.jsonl
      for v in "1 0" "1 2"; do set -- $v; for g in "" "--graph"; do
        TFX_LSTM_PERSISTENT=$1 TFX_LSTM_PROTO=$2 timeout -k 10 300 python scripts/bench_models.py --model char_lstm --impl native $g >> gpurun_out/bench_lstm.jsonl 2> gpurun_out/bench_lstm_err.log || { tail -20 gpurun_out/bench_lstm_err.log; exit 1; }
        echo "persistent=$1 proto=$2 $g: $(tail -1 gpurun_out/bench_lstm.jsonl | cut -c1-200)"
      done; done
      TFX_LSTM_PROTO=2 timeout -k 10 300 python -u -m pytest tests/test_sparse_rnn_gpu.py -k "lstm and (persistent or reference)" -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm_proto2.log 2>&1
      rc=$?; echo "lstm proto2 tests rc=$rc"; tail -3 gpurun_out/pytest_lstm_proto2.log; [ $rc -eq 0 ] || exit $rc
      cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_lstm" -o lstm -- python3 "$R/scripts/bench_models.py" --model char_lstm --impl native --graph --steps 20 --warmup 5 > "$R/gpurun_out/prof_lstm.log" 2>&1
      rc=$?; cd "$R"; echo "prof lstm rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    tune)
      timeout -k 10 900 python scripts/tune_convs.py --out gpurun_out/igemm_gfx950.json > gpurun_out/tune.log 2>&1
      rc=$?; echo "tune rc=$rc"; tail -3 gpurun_out/tune.log; [ $rc -eq 0 ] || exit $rc
      for i in 1 2 3; do
        TFX_TUNE=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_tune0_$i.log 2>&1 || exit 1
        TFX_TUNE_FILE=gpurun_out/igemm_gfx950.json timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_tune1_$i.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tune*.log
      TFX_TUNE_FILE=gpurun_out/igemm_gfx950.json timeout -k 10 600 python -u -m pytest tests/test_conv_production_gpu.py tests/test_resnet_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_tuned.log 2>&1
      rc=$?; echo "tuned tests rc=$rc"; tail -3 gpurun_out/pytest_tuned.log; [ $rc -eq 0 ] || exit $rc ;;
    w2v)
      for g in "" "--graph"; do
        timeout -k 10 300 python scripts/bench_models.py --model word2vec --impl native $g >> gpurun_out/bench_w2v.jsonl 2> gpurun_out/bench_w2v_err.log || { tail -20 gpurun_out/bench_w2v_err.log; exit 1; }
      done
      timeout -k 10 300 python scripts/bench_models.py --model word2vec --impl torch >> gpurun_out/bench_w2v.jsonl 2>> gpurun_out/bench_w2v_err.log || exit 1
      cut -c1-200 gpurun_out/bench_w2v.jsonl
      cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_w2v" -o w2v -- python3 "$R/scripts/bench_models.py" --model word2vec --impl native --graph --steps 50 --warmup 10 > "$R/gpurun_out/prof_w2v.log" 2>&1
      rc=$?; cd "$R"; echo "prof w2v rc=$rc"; [ $rc -eq 0 ] || exit $rc
      cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_w2v_torch" -o w2vt -- python3 "$R/scripts/bench_models.py" --model word2vec --impl torch --steps 50 --warmup 10 > "$R/gpurun_out/prof_w2v_torch.log" 2>&1
      rc=$?; cd "$R"; echo "prof w2v torch rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    models)
      : > gpurun_out/bench_models.jsonl
      for spec in "lenet5 native" "lenet5 native --graph" "lenet5 torch" "lenet5 torch --graph" \
                  "word2vec native" "word2vec native --graph" "word2vec torch" \
                  "word2vec native --batch 128 --graph" "word2vec torch --batch 128" \
                  "char_lstm native" "char_lstm native --graph" "char_lstm torch"; do
        set -- $spec
        m=$1; impl=$2; shift 2
        timeout -k 10 300 python scripts/bench_models.py --model $m --impl $impl "$@" >> gpurun_out/bench_models.jsonl 2> gpurun_out/bench_models_err.log
        rc=$?; echo "$spec rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_models_err.log; [ $rc -eq 1 ] || exit $rc; }
      done
      cat gpurun_out/bench_models.jsonl ;;
    glab)
      for v in 3 0; do
        TFX_GLDS=$v timeout -k 10 300 python scripts/conv_bench.py --out gpurun_out/conv_bench_gl$v.json > gpurun_out/conv_bench_gl$v.log 2>&1 || exit 1
      done
      for i in 1 2; do for v in 3 2 0; do
        TFX_GLDS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_gl${v}_$i.log 2>&1 || exit 1
      done; done
      grep TOTAL gpurun_out/conv_bench_gl*.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_gl*.log ;;
    glmode)
      for i in 1 2 3; do for v in def 0; do
        if [ $v = def ]; then timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_glm${v}_$i.log 2>&1 || exit 1
        else TFX_GLDS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_glm${v}_$i.log 2>&1 || exit 1; fi
      done; done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_glm*.log ;;
    mlp)
      # SURVEY §7.2 minimum slice: 1 ps + 1 worker on the GPU, full 50 x 550, tcp vs xgmi transport
      for tr in xgmi tcp; do
        P=$((29700 + RANDOM % 200)); W=$((P + 1))
        A="--ps_hosts=127.0.0.1:$P --worker_hosts=127.0.0.1:$W --device=cuda --logs_path=$R/gpurun_out/mnist_$tr --ps_exit_after_workers --transport=$tr"
        timeout -k 10 400 python distributed/distributed.py $A --job_name=ps --task_index=0 > gpurun_out/mlp_ps_$tr.log 2>&1 &
        PSPID=$!
        timeout -k 10 400 python distributed/distributed.py $A --job_name=worker --task_index=0 > gpurun_out/mlp_worker_$tr.log 2>&1
        rc=$?; wait $PSPID; echo "mlp $tr rc=$rc"; tail -4 gpurun_out/mlp_worker_$tr.log; [ $rc -eq 0 ] || exit $rc
      done ;;
    diagrccl)
      for d in 18 50; do
        RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 TFX_DP_FORCE_COLLECTIVE=1 \
          timeout -k 10 300 python scripts/diag_dp_rccl.py $d > gpurun_out/diag_rccl_$d.log 2>&1
        rc=$?; echo "diagrccl $d rc=$rc"; grep -v amdgpu.ids gpurun_out/diag_rccl_$d.log | tail -40; [ $rc -eq 0 ] || exit $rc
      done ;;
    labn)
      for i in 1 2 3; do for v in 1 0; do
        TFX_BN_LAST_ARRIVER=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_la${v}_$i.log 2>&1 || exit 1
      done; done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_la*.log ;;
    diagdp)
      for d in 50 18; do
        timeout -k 10 300 python scripts/diag_dp.py $d > gpurun_out/diag_dp_$d.log 2>&1
        rc=$?; echo "diagdp $d rc=$rc"; cat gpurun_out/diag_dp_$d.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
      done ;;
    hostin)
      for i in 1 2; do
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_dev_$i.log 2>&1 || exit 1
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 --host-input > gpurun_out/bench_hostin_$i.log 2>&1 || exit 1
      done
      grep -ho '"ms_per_step": [0-9.]*' gpurun_out/bench_dev_*.log gpurun_out/bench_hostin_*.log ;;
    hostin2)
      timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_pipeline.log 2>&1
      rc=$?; echo "pipeline tests rc=$rc"; tail -12 gpurun_out/pytest_pipeline.log; [ $rc -eq 0 ] || exit $rc
      for i in 1 2; do
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_dev_$i.log 2>&1 || exit 1
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 --host-input zerocopy > gpurun_out/bench_hostzc_$i.log 2>&1 || exit 1
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 --host-input copy > gpurun_out/bench_hostcp_$i.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_dev_*.log gpurun_out/bench_hostzc_*.log gpurun_out/bench_hostcp_*.log
      export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/prof_hostcp" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --host-input copy > gpurun_out/prof_hostcp.log 2>&1
      rc=$?; echo "prof hostcp rc=$rc"; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_hostzc" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --host-input zerocopy > gpurun_out/prof_hostzc.log 2>&1
      rc=$?; echo "prof hostzc rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    eager)
      for i in 1 2; do
        timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-graph > gpurun_out/bench_eager_$i.log 2>&1 || exit 1
      done
      for v in 0 1; do
        TFX_DP_FORCE_COLLECTIVE=1 TFX_DP_GRAPH=$v timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 30 --warmup 5 > gpurun_out/bench_dpforce_g$v.log 2>&1
        rc=$?; echo "dpforce graph=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_dpforce_g$v.log; exit $rc; }
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_eager_*.log gpurun_out/bench_dpforce_g*.log
      export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_eager" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-graph > gpurun_out/prof_eager.log 2>&1
      rc=$?; echo "prof eager rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    dpprof)
      export TMPDIR=/tmp
      for v in 0 1; do
        RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$v TFX_DP_FORCE_COLLECTIVE=1 TFX_DP_GRAPH=$v \
          timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_dp$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > gpurun_out/prof_dp$v.log 2>&1
        rc=$?; echo "prof dp graph=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_dp$v.log; exit $rc; }
      done ;;
    retune)
      timeout -k 10 1000 python scripts/tune_convs.py --passes fwd,dgrad --merge tensorflow_examples_amd/tune/igemm_gfx950.json --out gpurun_out/igemm_gfx950.json --report gpurun_out/tune_report_fd.json > gpurun_out/tune_fd.log 2>&1
      rc=$?; echo "tune rc=$rc"; tail -40 gpurun_out/tune_fd.log; [ $rc -eq 0 ] || exit $rc
      for i in 1 2 3; do
        timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_rt0_$i.log 2>&1 || exit 1
        TFX_TUNE_FILE=gpurun_out/igemm_gfx950.json timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_rt1_$i.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_rt*.log ;;
    tunebig)
      timeout -k 10 900 python scripts/tune_convs.py --passes wgrad --merge tensorflow_examples_amd/tune/igemm_gfx950.json --out gpurun_out/igemm_gfx950.json --report gpurun_out/tune_report_big.json > gpurun_out/tune_big.log 2>&1
      rc=$?; echo "tune rc=$rc"; tail -25 gpurun_out/tune_big.log; [ $rc -eq 0 ] || exit $rc
      for i in 1 2 3; do
        timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_tb0_$i.log 2>&1 || exit 1
        TFX_TUNE_FILE=gpurun_out/igemm_gfx950.json timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_tb1_$i.log 2>&1 || exit 1
      done
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tb*.log ;;
    pmcbench)
      # PMC passes over a short eager bench (each pass its own run; <= 8 SQ, 4 TCC, 2 GRBM counters)
      export TMPDIR=/tmp
      i=0
      for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum" \
                 "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$R/gpurun_out/pmc/p$i" -o p -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-graph > gpurun_out/pmc_p$i.log 2>&1
        rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_p$i.log; exit $rc; }
      done
      python scripts/pmc_summary.py gpurun_out/pmc --steps 3 > gpurun_out/pmc_summary.txt; head -45 gpurun_out/pmc_summary.txt ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo ALL_DONE
