#!/usr/bin/env bash
# PIN schedule (small batches): GPU suite, then same-box A/B of the previous build (ab/base.so) against
# the tree's libpekf.so at config 2 (PIN auto-selected) and config 3 (default schedule, unchanged ISA).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pin2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--batch 65536" timeout -k 10 300 scripts/ab_libs.sh ab/base.so poseestimationkf_amd/libpekf.so 2>&1 | tee $O/ab_c2.txt || exit $?
timeout -k 10 400 scripts/ab_libs.sh ab/base.so poseestimationkf_amd/libpekf.so 2>&1 | tee $O/ab_c3.txt || exit $?
timeout -k 10 300 python3 bench.py --batch 65536 --cpu-baseline none > $O/bench_c2.json || exit $?
