#!/usr/bin/env bash
# GPU check of the rank-1 Wahba handling: its tests, the whole GPU suite, and same-box A/Bs of the
# library before (ab/deg_base.so) and after (ab/deg_new3.so) on the headline, the fused front-end +
# filter kernel and the kernels beside the headline.  Output under gpurun_out/deg/.
set -u
mkdir -p gpurun_out/deg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_degenerate_samples.py > gpurun_out/deg/tests_degenerate.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/deg/tests_gpu.log 2>&1 || exit $?
timeout -k 10 700 scripts/ab_abba.sh ab/deg_base.so ab/deg_new3.so > gpurun_out/deg/ab_c3.log 2>&1 || exit $?
REPS=6 timeout -k 10 400 scripts/ab_live.sh ab/deg_base.so ab/deg_new3.so > gpurun_out/deg/ab_live.log 2>&1 || exit $?
timeout -k 10 600 scripts/ab_aux.sh ab/deg_base.so ab/deg_new3.so > gpurun_out/deg/ab_aux.log 2>&1 || exit $?
