#!/bin/bash
# Submit one gpurun call; resubmit ONLY when gpurun reports exit 3 (no GPU slot/box free: nothing ran,
# nothing charged).  Any other exit (including a failing GPU step) ends the loop.
# usage: scripts/gpurun_retry.sh <out.txt> <timeout> <command...>
out=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy" "$out"; then echo "rc=$rc" >> "$out"; exit $rc; fi
  sleep 90
done
