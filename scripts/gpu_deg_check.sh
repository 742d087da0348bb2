#!/usr/bin/env bash
# GPU check of the rank-1 Wahba handling: its tests, then the whole GPU suite.  Output under gpurun_out/deg/.
set -u
mkdir -p gpurun_out/deg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_degenerate_samples.py > gpurun_out/deg/tests_degenerate.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/deg/tests_gpu.log 2>&1 || exit $?
