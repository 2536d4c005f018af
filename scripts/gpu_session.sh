#!/bin/bash
# One gpurun session, as named steps (STEPS="tests bench prof ..."): every GPU step runs under its
# own time limit and the steps are chained -- a crash, abort or time-out ends the session (no further
# GPU work), a failing test does not.  Output under $O/; copy what is worth keeping to profiles/.
#   tests    pytest -m gpu (the whole GPU suite, one process)
#   smoke    __graft_entry__.smoke() (the driver's round-end smoke)
#   bench    bench.py --steps 20 --warmup 5 (the driver's 1-GPU command)
#   prof     rocprofv3 --kernel-trace --stats over a short bench, summarised by scripts/kstats.py
#   pmc      PMC passes (MFMA busy, LDS conflicts, HBM bytes) over an eager bench, one run per pass
#   convs    scripts/conv_bench.py (every ResNet-50 conv pass in isolation)
#   models   scripts/bench_models.py (LeNet-5, word2vec, char-LSTM; native graphed and stock PyTorch)
#   dpforce  the DP step on a 1-rank RCCL group under torch.distributed.run, graphed and eager
set -u
# R = the tree to run (cwd: the repo root, or the frozen .snap copy of scripts/snap_submit.sh);
# O = where results go (OUT, default R/gpurun_out -- gpurun merges $GRAFT_REPO_ROOT/gpurun_out back)
R=$(pwd)
O=${OUT:-$R/gpurun_out}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
STEPS=${STEPS:-"tests bench prof"}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
        ${PYTEST_EXTRA:-} > $O/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      for i in ${BENCH_REPS:-1}; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1
        rc=$?; echo "bench rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log; [ $rc -eq 0 ] || exit $rc
      done ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
        python3 "$R/bench.py" --steps 5 --warmup 2 > $O/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof.log; exit $rc; }
      f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
      python scripts/kstats.py "$f" auto 60 > $O/kernel_summary.txt; head -25 $O/kernel_summary.txt
      kt=$(find $O/prof -name '*kernel_trace.csv' | head -1)
      python scripts/step_trace.py "$kt" > $O/step_trace.txt; head -1 $O/step_trace.txt ;;
    pmc)
      i=0
      for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum" \
                 "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$O/pmc/p$i" -o p -- \
          python3 "$R/bench.py" --steps 2 --warmup 1 --no-graph > $O/pmc_p$i.log 2>&1
        rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_p$i.log; exit $rc; }
      done
      python scripts/pmc_summary.py $O/pmc --steps 3 > $O/pmc_summary.txt; head -45 $O/pmc_summary.txt ;;
    convs)
      timeout -k 10 400 python scripts/conv_bench.py --out $O/conv_bench.json > $O/conv_bench.log 2>&1
      rc=$?; echo "convs rc=$rc"; tail -3 $O/conv_bench.log; [ $rc -eq 0 ] || exit $rc ;;
    models)
      : > $O/bench_models.jsonl
      for spec in "lenet5 --graph" "lenet5 --graph --impl torch" "word2vec --graph --batch 128" \
                  "word2vec --graph --batch 4096" "word2vec --impl torch --batch 4096" "char_lstm --graph" \
                  "char_lstm --impl torch"; do
        timeout -k 10 300 python scripts/bench_models.py --model $spec >> $O/bench_models.jsonl 2>> $O/bench_models.err
        rc=$?; echo "models [$spec] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_models.err; exit $rc; }
      done
      cat $O/bench_models.jsonl ;;
    dpforce)
      for v in 1 0; do
        TFX_DP_FORCE_COLLECTIVE=1 TFX_DP_GRAPH=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2951$v bench.py --steps 20 --warmup 5 \
          > $O/bench_dpforce_g$v.log 2>&1
        rc=$?; echo "dpforce graph=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_dpforce_g$v.log; exit $rc; }
      done
      grep -o '"ms_per_step": [0-9.]*' $O/bench_dpforce_g*.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo ALL_DONE
