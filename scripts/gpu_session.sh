#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time limit and the
# sequence stops at the first crash / abort / timeout (exit codes other than 0 and 1).
# Usage: scripts/gpu_session.sh <name> "<cmd1>" "<cmd2>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1; shift
out=gpurun_out/$name
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a "$out/steps.log"
  start=$(date +%s)
  bash -c "$cmd" > "$out/step$i.log" 2>&1
  rc=$?
  echo "=== step $i rc=$rc ($(( $(date +%s) - start )) s)" | tee -a "$out/steps.log"
  tail -n 25 "$out/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $i exited $rc" | tee -a "$out/steps.log"
    exit $rc
  fi
done
