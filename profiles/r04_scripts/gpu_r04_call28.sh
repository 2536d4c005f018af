# round-4 call 28: DP bucket size on the forced 1-rank RCCL step (graphed): launch/overlap overhead only
# (the N=8 link time is modelled in profiles/r04_dp)
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
i=0
for mb in 8 16 32 64 128 32; do
  i=$((i+1))
  TFX_DP_FORCE_COLLECTIVE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 2960$i bench.py --steps 30 --warmup 5 --bucket-mb $mb > $O/bench_bucket_$i.log 2>&1
  rc=$?; echo "bucket ${mb}MB rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_bucket_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
