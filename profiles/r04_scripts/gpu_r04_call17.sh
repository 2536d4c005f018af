# round-4 call 17: cost of the slot-reduction tail blocks in weight-gradient launches
set -u
O=${OUT:-gpurun_out}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dev/wgrad_sr_probe.py > $O/wgrad_sr_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids $O/wgrad_sr_probe.txt; [ $rc -eq 0 ] || exit $rc
