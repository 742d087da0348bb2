#!/usr/bin/env bash
# RK4 normalisation without rsqrt for IMU-rate steps: parity suite, then same-box A/B against the 360-VALU build
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zg \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zg/v360_1.json" \
 "timeout -k 10 300 $B > gpurun_out/r1zg/v357_1.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zg/v360_2.json" \
 "timeout -k 10 300 $B > gpurun_out/r1zg/v357_2.json" \
 "timeout -k 10 400 python bench.py > gpurun_out/r1zg/bench_c3_f64.json"
