#!/bin/bash
# Freeze the working tree into .snap/ and submit ONE gpurun call that runs <script> from that frozen
# copy, so edits made while the call waits for a box cannot leak into it.  The script gets
# OUT=$GRAFT_REPO_ROOT/gpurun_out (merged back by gpurun) and runs with cwd = the frozen copy.
# usage: scripts/snap_submit.sh <out.txt> <timeout_s> <script relative to repo> [env assignments...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
out=$1; to=$2; script=$3; shift 3
rm -rf "$R/.snap"
mkdir -p "$R/.snap"
(cd "$R" && tar --exclude=./.git --exclude=./.snap --exclude=./gpurun_out --exclude=./profiles --exclude=./build \
   --exclude='__pycache__' -cf - .) | (cd "$R/.snap" && tar -xf -)
envs="$*"
cmd="cd .snap && env OUT=\$GRAFT_REPO_ROOT/gpurun_out $envs bash $script"
exec "$R/scripts/gpurun_retry.sh" "$out" "$to" "$cmd"
