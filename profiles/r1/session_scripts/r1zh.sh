#!/usr/bin/env bash
# refresh of the side configurations and the aux-kernel trace for the current build
exec scripts/gpu_session.sh r1zh \
 "timeout -k 10 400 python bench.py --batch 65536 --cpu-baseline none > gpurun_out/r1zh/bench_c2_f64.json" \
 "timeout -k 10 400 python bench.py --missing --cpu-baseline none > gpurun_out/r1zh/bench_c5_f64.json" \
 "timeout -k 10 400 python bench.py --precision mixed --cpu-baseline none > gpurun_out/r1zh/bench_c3_mixed.json"
