#!/usr/bin/env bash
# Order-balanced A/B at config 3: previous build (ab/base.so), the tree's libpekf.so (default schedule
# at this size), and the tree's libpekf.so with the PIN schedule forced (PEKF_RUN_PIN=1).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2"
run() { echo "== $1 $2"; PEKF_LIB=$1 PEKF_RUN_PIN=$2 timeout -k 10 200 $B 2>&1 >/dev/null | grep "timed:" || exit $?; }
L=poseestimationkf_amd/libpekf.so
for r in 1 2; do
  run ab/base.so auto; run $L auto; run $L 1; run $L 1; run $L auto; run ab/base.so auto
done
